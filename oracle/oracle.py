"""ctypes binding of the CPU oracle (oracle/libkcnn_oracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the *checker*; the product (libkcnn.so) never
touches it.  PARITY UNPINNED: see kcnn_oracle.h.

Matrices are numpy float32 arrays, 2-D, row-contiguous (a row stride larger
than the column count is allowed, mirroring Kaldi's pitched CuMatrix).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libkcnn_oracle.so")


class OrcMat(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_float)),
                ("rows", ctypes.c_int32), ("cols", ctypes.c_int32),
                ("stride", ctypes.c_int32)]


class OrcConv(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "in_height", "in_width", "in_channel", "in_pad_height", "in_pad_width",
        "kernel_height", "kernel_width", "stride", "group", "out_height",
        "out_width")] + [
        ("learning_rate", ctypes.c_float), ("weight_decay", ctypes.c_float),
        ("momentum", ctypes.c_float), ("W", OrcMat),
        ("b", ctypes.POINTER(ctypes.c_float)), ("prev", OrcMat)]


class OrcPool(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "in_height", "in_width", "in_channel", "pool_height_dim",
        "pool_width_dim", "pool_channel_dim", "overlap", "overlap2D")]


class OrcFC(ctypes.Structure):
    _fields_ = [("input_dim", ctypes.c_int32), ("output_dim", ctypes.c_int32),
                ("learning_rate", ctypes.c_float),
                ("weight_decay", ctypes.c_float), ("momentum", ctypes.c_float),
                ("W", OrcMat), ("b", ctypes.POINTER(ctypes.c_float)),
                ("prev", OrcMat)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            # test infrastructure: build the checker on first use (gcc only)
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.dirname(_LIB_PATH)], check=True)
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_last_error.restype = ctypes.c_char_p
    return _lib


class OracleError(RuntimeError):
    pass


def _chk(rc):
    if rc != 0:
        raise OracleError(lib().orc_last_error().decode())


def mat(a: np.ndarray) -> OrcMat:
    assert a.dtype == np.float32 and a.ndim == 2, (a.dtype, a.ndim)
    assert a.strides[1] == 4, "rows must be contiguous"
    rows, cols = a.shape
    stride = a.strides[0] // 4 if rows > 1 else max(cols, 1)
    return OrcMat(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), rows, cols,
                  stride)


def fptr(v: np.ndarray):
    assert v.dtype == np.float32 and v.flags.c_contiguous
    return v.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class accum:
    """Context manager selecting the oracle's reduction precision.

    0 = float sequential (reference BLAS stand-in), 1 = double accumulation
    (fp64 truth), 2 = sum of |a*b| (error-bound scale)."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        self.prev = lib().orc_get_accum_mode()
        lib().orc_set_accum_mode(self.mode)

    def __exit__(self, *a):
        lib().orc_set_accum_mode(self.prev)


def set_threads(n: int):
    lib().orc_set_num_threads(int(n))


def openblas_path():
    """numpy's bundled OpenBLAS (the CBLAS class upstream Kaldi links), or None."""
    import glob
    d = os.path.join(os.path.dirname(np.__file__), "..", "numpy.libs")
    hits = sorted(glob.glob(os.path.join(d, "libscipy_openblas64_*.so")))
    return os.path.abspath(hits[0]) if hits else None


def use_blas(on: bool = True) -> str | None:
    """Mode-0 GEMMs through OpenBLAS sgemm (CPU-baseline timing) or, with
    on=False, the sequential-k loops (the parity tests' reference order).
    Returns the library used."""
    path = openblas_path() if on else None
    if on and path is None:
        raise OracleError("numpy's OpenBLAS not found")
    _chk(lib().orc_use_blas(path.encode() if path else None))
    return path


# --- CuMatrixBase extensions ------------------------------------------------

def conv2d(x, k, H, W, C, kh, kw, G, concat=True, out=None):
    oh, ow = H - kh + 1, W - kw + 1
    if out is None:
        shape = (x.shape[0], oh * ow * G) if concat else (oh * ow * x.shape[0], G)
        out = np.zeros(shape, np.float32)
    _chk(lib().orc_conv2d(ctypes.byref(mat(x)), ctypes.byref(mat(k)), H, W, C,
                          kh, kw, G, ctypes.byref(mat(out)), int(concat)))
    return out


def add_mat_rep_vec(m, vec, rep):
    _chk(lib().orc_add_mat_rep_vec(ctypes.byref(mat(m)), fptr(vec), vec.shape[0], rep))
    return m


def flip_mat(m, kh, kw, C, G):
    flip = np.zeros((kh * kw * G, C), np.float32)
    _chk(lib().orc_flip_mat(ctypes.byref(mat(m)), kh, kw, C, G, ctypes.byref(mat(flip))))
    return flip


def padding_zero(m, H, W, C, kh, kw):
    ph, pw = H + 2 * (kh - 1), W + 2 * (kw - 1)
    out = np.zeros((m.shape[0], ph * pw * C), np.float32)
    _chk(lib().orc_padding_zero(ctypes.byref(mat(m)), H, W, C, kh, kw,
                                ctypes.byref(mat(out))))
    return out


def tp_block(m, C, bs):
    out = np.zeros((C, m.shape[0] * bs), np.float32)
    _chk(lib().orc_tp_block(ctypes.byref(mat(m)), C, bs, ctypes.byref(mat(out))))
    return out


def tp_inside_block(m, G, bs):
    out = np.zeros((bs * m.shape[0], G), np.float32)
    _chk(lib().orc_tp_inside_block(ctypes.byref(mat(m)), G, bs, ctypes.byref(mat(out))))
    return out


def mod_permute_row(m, C, bs):
    out = np.zeros_like(m)
    _chk(lib().orc_mod_permute_row(ctypes.byref(mat(m)), C, bs, ctypes.byref(mat(out))))
    return out


def mod_permute_channel(comp, comp_idx, num_component, H, W, container, to_container):
    _chk(lib().orc_mod_permute_channel(ctypes.byref(mat(comp)), comp_idx, num_component,
                                       H, W, ctypes.byref(mat(container)),
                                       int(bool(to_container))))
    return container if to_container else comp


def maxpool_prop(x, H, W, ph, pw, pc, out_dim, overlap=False, overlap2D=False):
    out = np.zeros((x.shape[0], out_dim), np.float32)
    _chk(lib().orc_maxpool_prop(ctypes.byref(mat(x)), H, W, ph, pw, pc,
                                int(overlap), int(overlap2D), ctypes.byref(mat(out))))
    return out


def maxpool_backprop(x, y, dy, H, W, ph, pw, pc, overlap=False, overlap2D=False):
    dx = np.zeros_like(x)
    _chk(lib().orc_maxpool_backprop(ctypes.byref(mat(x)), ctypes.byref(mat(y)),
                                    ctypes.byref(mat(dy)), ctypes.byref(mat(dx)),
                                    H, W, ph, pw, pc, int(overlap), int(overlap2D)))
    return dx


def gemm(alpha, A, tA, B, tB, beta, C):
    _chk(lib().orc_gemm(ctypes.c_float(alpha), ctypes.byref(mat(A)), int(tA),
                        ctypes.byref(mat(B)), int(tB), ctypes.c_float(beta),
                        ctypes.byref(mat(C))))
    return C


# --- components -----------------------------------------------------------------

@dataclass
class Conv:
    """ConvolutionComponent state (nnet-component-nnet0.h:123-145)."""
    in_height: int
    in_width: int
    in_channel: int
    kernel_height: int
    kernel_width: int
    group: int
    in_pad_height: int = 0
    in_pad_width: int = 0
    learning_rate: float = 0.02
    weight_decay: float = 0.0002
    momentum: float = 0.9
    W: np.ndarray = None
    b: np.ndarray = None
    prev: np.ndarray = None
    _keep: list = field(default_factory=list, repr=False)

    @property
    def out_height(self):
        return self.in_height + 2 * self.in_pad_height - self.kernel_height + 1

    @property
    def out_width(self):
        return self.in_width + 2 * self.in_pad_width - self.kernel_width + 1

    @property
    def input_dim(self):
        return self.in_height * self.in_width * self.in_channel

    @property
    def output_dim(self):
        return self.out_height * self.out_width * self.group

    def _c(self) -> OrcConv:
        kd = self.kernel_height * self.kernel_width * self.in_channel
        if self.W is None:
            self.W = np.zeros((kd, self.group), np.float32)
        if self.b is None:
            self.b = np.zeros(self.group, np.float32)
        if self.prev is None:
            self.prev = np.zeros_like(self.W)
        s = OrcConv(self.in_height, self.in_width, self.in_channel,
                    self.in_pad_height, self.in_pad_width, self.kernel_height,
                    self.kernel_width, 1, self.group, self.out_height,
                    self.out_width, self.learning_rate, self.weight_decay,
                    self.momentum, mat(self.W), fptr(self.b), mat(self.prev))
        return s

    def flip_branch(self) -> bool:
        return bool(lib().orc_conv_flip_branch(ctypes.byref(self._c())))

    def propagate(self, x):
        out = np.zeros((x.shape[0], self.output_dim), np.float32)
        _chk(lib().orc_conv_propagate(ctypes.byref(self._c()), ctypes.byref(mat(x)),
                                      ctypes.byref(mat(out))))
        return out

    def backprop(self, x, dy, update=True):
        dx = np.zeros((dy.shape[0], self.input_dim), np.float32)
        _chk(lib().orc_conv_backprop(ctypes.byref(self._c()), ctypes.byref(mat(x)),
                                     ctypes.byref(mat(dy)), ctypes.byref(mat(dx)),
                                     int(update)))
        return dx

    def gradient(self, x, dy):
        kd = self.kernel_height * self.kernel_width * self.in_channel
        gW = np.zeros((kd, self.group), np.float32)
        gb = np.zeros(self.group, np.float32)
        _chk(lib().orc_conv_gradient(ctypes.byref(self._c()), ctypes.byref(mat(x)),
                                     ctypes.byref(mat(dy)), ctypes.byref(mat(gW)),
                                     fptr(gb)))
        return gW, gb

    def apply(self, gW, gb, num_sample):
        _chk(lib().orc_conv_apply(ctypes.byref(self._c()), ctypes.byref(mat(gW)),
                                  fptr(gb), int(num_sample)))


@dataclass
class Pool:
    in_height: int
    in_width: int
    in_channel: int
    pool_height_dim: int = 1
    pool_width_dim: int = 1
    pool_channel_dim: int = 1
    overlap: bool = False
    overlap2D: bool = False

    def _c(self):
        return OrcPool(self.in_height, self.in_width, self.in_channel,
                       self.pool_height_dim, self.pool_width_dim,
                       self.pool_channel_dim, int(self.overlap), int(self.overlap2D))

    @property
    def input_dim(self):
        return self.in_height * self.in_width * self.in_channel

    @property
    def output_dim(self):
        return lib().orc_pool_output_dim(ctypes.byref(self._c()))

    def propagate(self, x):
        return maxpool_prop(x, self.in_height, self.in_width, self.pool_height_dim,
                            self.pool_width_dim, self.pool_channel_dim,
                            self.output_dim, self.overlap, self.overlap2D)

    def backprop(self, x, y, dy):
        return maxpool_backprop(x, y, dy, self.in_height, self.in_width,
                                self.pool_height_dim, self.pool_width_dim,
                                self.pool_channel_dim, self.overlap, self.overlap2D)


@dataclass
class FC:
    input_dim: int
    output_dim: int
    learning_rate: float = 0.02
    weight_decay: float = 0.0002
    momentum: float = 0.9
    W: np.ndarray = None
    b: np.ndarray = None
    prev: np.ndarray = None

    def _c(self):
        if self.W is None:
            self.W = np.zeros((self.output_dim, self.input_dim), np.float32)
        if self.b is None:
            self.b = np.zeros(self.output_dim, np.float32)
        if self.prev is None:
            self.prev = np.zeros_like(self.W)
        return OrcFC(self.input_dim, self.output_dim, self.learning_rate,
                     self.weight_decay, self.momentum, mat(self.W), fptr(self.b),
                     mat(self.prev))

    def propagate(self, x):
        out = np.zeros((x.shape[0], self.output_dim), np.float32)
        _chk(lib().orc_fc_propagate(ctypes.byref(self._c()), ctypes.byref(mat(x)),
                                    ctypes.byref(mat(out))))
        return out

    def backprop(self, x, dy, update=True):
        dx = np.zeros((dy.shape[0], self.input_dim), np.float32)
        _chk(lib().orc_fc_backprop(ctypes.byref(self._c()), ctypes.byref(mat(x)),
                                   ctypes.byref(mat(dy)), ctypes.byref(mat(dx)),
                                   int(update)))
        return dx

    def gradient(self, x, dy):
        gW = np.zeros((self.output_dim, self.input_dim), np.float32)
        gb = np.zeros(self.output_dim, np.float32)
        _chk(lib().orc_fc_gradient(ctypes.byref(self._c()), ctypes.byref(mat(x)),
                                   ctypes.byref(mat(dy)), ctypes.byref(mat(gW)),
                                   fptr(gb)))
        return gW, gb

    def apply(self, gW, gb, num_sample):
        _chk(lib().orc_fc_apply(ctypes.byref(self._c()), ctypes.byref(mat(gW)),
                                fptr(gb), int(num_sample)))


# ---- upstream nnet2 components either side of the path --
@dataclass
class ReLU:
    """RectifiedLinearComponent (nnet2/nnet-component.cc:799-827) with its
    NonlinearComponent stats (fp64 value_sum / deriv_sum, count)."""
    dim: int
    value_sum: np.ndarray = None
    deriv_sum: np.ndarray = None
    count: float = 0.0

    def propagate(self, x):
        out = np.zeros_like(x)
        _chk(lib().orc_relu_propagate(ctypes.byref(mat(x)), ctypes.byref(mat(out))))
        return out

    def backprop(self, y, dy, update=True):
        dx = np.zeros_like(dy)
        if update and self.value_sum is None:
            self.value_sum = np.zeros(self.dim, np.float64)
            self.deriv_sum = np.zeros(self.dim, np.float64)
        cnt = ctypes.c_double(self.count)
        dp = ctypes.POINTER(ctypes.c_double)
        vs = self.value_sum.ctypes.data_as(dp) if update else None
        ds = self.deriv_sum.ctypes.data_as(dp) if update else None
        _chk(lib().orc_relu_backprop(ctypes.byref(mat(y)), ctypes.byref(mat(dy)),
                                     ctypes.byref(mat(dx)), vs, ds, ctypes.byref(cnt)))
        self.count = cnt.value
        return dx


@dataclass
class Splice:
    """SpliceComponent (nnet2/nnet-component.cc:2524-2866); one output frame
    per chunk by default, i.e. chunks of len(context) input frames."""
    input_dim: int
    context: tuple
    const_dim: int = 0

    @property
    def output_dim(self):
        return (self.input_dim - self.const_dim) * len(self.context) + self.const_dim

    def _geom(self, num_chunks, out_cs):
        ctx = list(self.context)
        in_cs = out_cs + ctx[-1] - ctx[0]
        c = (ctypes.c_int * len(ctx))(*ctx)
        # offsets as the runtime builds them: input chunk from 0, output chunk
        # starting at -context[0]
        return num_chunks, 0, in_cs, -ctx[0], out_cs, c, len(ctx), self.const_dim

    def propagate(self, x, num_chunks=None, out_cs=1):
        ctx = list(self.context)
        in_cs = out_cs + ctx[-1] - ctx[0]
        num_chunks = num_chunks or x.shape[0] // in_cs
        out = np.zeros((num_chunks * out_cs, self.output_dim), np.float32)
        _chk(lib().orc_splice_propagate(ctypes.byref(mat(x)), ctypes.byref(mat(out)),
                                        *self._geom(num_chunks, out_cs)))
        return out

    def propagate_offsets(self, x, in_offsets, out_offsets, num_chunks):
        """Propagate with explicit chunk offset lists (upstream ChunkInfo with
        an offsets_ vector: gapped contexts deeper in a stack)."""
        io = (ctypes.c_int * len(in_offsets))(*in_offsets)
        oo = (ctypes.c_int * len(out_offsets))(*out_offsets)
        ctx = (ctypes.c_int * len(self.context))(*self.context)
        out = np.zeros((num_chunks * len(out_offsets), self.output_dim), np.float32)
        _chk(lib().orc_splice_propagate_offsets(
            ctypes.byref(mat(x)), ctypes.byref(mat(out)), num_chunks, io, len(in_offsets),
            oo, len(out_offsets), ctx, len(self.context), self.const_dim))
        return out

    def backprop_offsets(self, dy, in_offsets, out_offsets, num_chunks):
        io = (ctypes.c_int * len(in_offsets))(*in_offsets)
        oo = (ctypes.c_int * len(out_offsets))(*out_offsets)
        ctx = (ctypes.c_int * len(self.context))(*self.context)
        dx = np.zeros((num_chunks * len(in_offsets), self.input_dim), np.float32)
        _chk(lib().orc_splice_backprop_offsets(
            ctypes.byref(mat(dy)), ctypes.byref(mat(dx)), num_chunks, io, len(in_offsets),
            oo, len(out_offsets), ctx, len(self.context), self.const_dim))
        return dx

    def backprop(self, dy, num_chunks=None, out_cs=1):
        ctx = list(self.context)
        in_cs = out_cs + ctx[-1] - ctx[0]
        num_chunks = num_chunks or dy.shape[0] // out_cs
        dx = np.zeros((num_chunks * in_cs, self.input_dim), np.float32)
        _chk(lib().orc_splice_backprop(ctypes.byref(mat(dy)), ctypes.byref(mat(dx)),
                                       *self._geom(num_chunks, out_cs)))
        return dx


def chunk_offsets(contexts, out_frames=1):
    """Upstream nnet2 Nnet::ComputeChunkInfo for a stack whose components have
    the given Context() lists: walking back from the last output (out_frames
    consecutive offsets), each component's input offsets are the sorted set
    of output offset + context; the network input is made contiguous
    (MakeOffsetsContiguous); everything shifted so the first offset is 0.
    Returns one ascending offset list per chunk info (len(contexts) + 1)."""
    offs = [None] * (len(contexts) + 1)
    offs[-1] = list(range(out_frames))
    for k in range(len(contexts) - 1, -1, -1):
        offs[k] = sorted({o + c for o in offs[k + 1] for c in contexts[k]})
    offs[0] = list(range(offs[0][0], offs[0][-1] + 1))
    shift = -offs[0][0]
    return [[o + shift for o in lst] for lst in offs]
