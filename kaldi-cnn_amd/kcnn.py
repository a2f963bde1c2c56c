"""kcnn -- Python host binding of libkcnn.so (the MI355X build of kaldi-cnn's
nnet2 CNN hot path).

Mirrors the reference's interfaces with the same names and argument meaning:

  * ``Mat*`` functions  = ``CuMatrixBase<float>::{Conv2D, AddMatRepVec,
    FlipMat, PaddingZero, TpBlock, TpInsideBlock, ModPermuteRow,
    Maxpool_prop, Maxpool_backprop}`` (reference cudamatrix/cu-matrix.h:451-480)
  * ``Component``       = nnet2 ``Component`` / ``UpdatableComponent`` as the
    nnet0 components implement them (nnet0/nnet-component-nnet0.h:23-232),
    created with ``Component.NewFromString`` (nnet2/nnet-component.cc:124-136)
  * ``Nnet``            = a component stack run NnetUpdater-style.

Matrices are 2-D float32 CUDA tensors with unit column stride (any row
stride); they are handed to the C++ library as raw device pointers + MatrixDim
on torch's current stream.  PyTorch is plumbing here (device memory, streams,
torch.distributed); every computation runs in libkcnn.so's HIP kernels.  There
is no fallback: if the library or a GPU is missing, calls raise.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# KCNN_LIB: an alternative build of the same library (e.g. the phase-timing
# build, `make -C kaldi-cnn_amd timing`)
LIB_PATH = os.environ.get("KCNN_LIB") or os.path.join(_HERE, "libkcnn.so")
INCLUDE_DIR = os.path.join(os.path.dirname(_HERE), "include")


class KcnnError(RuntimeError):
    """A KALDI_ASSERT / KALDI_ERR / HIP error raised inside libkcnn.so."""


class MatrixDim(ctypes.Structure):
    _fields_ = [("rows", ctypes.c_int32), ("cols", ctypes.c_int32),
                ("stride", ctypes.c_int32)]

    def __repr__(self):
        return f"MatrixDim({self.rows}, {self.cols}, {self.stride})"


_lib = None


def lib():
    """The loaded libkcnn.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles libamdhip64.so.7 (same
        # SONAME as /opt/rocm's); loading torch first makes libkcnn.so bind
        # to that already-loaded runtime instead of a second copy.
        import torch  # noqa: F401
        if not os.path.exists(LIB_PATH):
            raise KcnnError(f"{LIB_PATH} not built (run `make -C kaldi-cnn_amd` "
                            "or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.kcnn_last_error.restype = ctypes.c_char_p
        L.kcnn_version.restype = ctypes.c_char_p
        if hasattr(L, "kcnn_device_malloc_calls"):  # (absent from pre-r05 builds)
            L.kcnn_device_malloc_calls.restype = ctypes.c_ulonglong
        for name in ("kcnn_component_new_from_string", "kcnn_component_read",
                     "kcnn_component_copy"):
            getattr(L, name).restype = ctypes.c_void_p
        L.kcnn_component_new_from_string.argtypes = [ctypes.c_char_p]
        L.kcnn_component_read.argtypes = [ctypes.c_char_p]
        L.kcnn_component_copy.argtypes = [ctypes.c_void_p]
        L.kcnn_component_free.argtypes = [ctypes.c_void_p]
        L.kcnn_component_learning_rate.restype = ctypes.c_float
        L.kcnn_nnet_new.restype = ctypes.c_void_p
        L.kcnn_nnet_new.argtypes = [ctypes.c_char_p]
        L.kcnn_nnet_free.argtypes = [ctypes.c_void_p]
        L.kcnn_nnet_component.restype = ctypes.c_void_p
        L.kcnn_nnet_component.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.kcnn_set_stream.argtypes = [ctypes.c_void_p]
        L.kcnn_set_randn_seed.argtypes = [ctypes.c_uint64]
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise KcnnError(lib().kcnn_last_error().decode(errors="replace"))
    return rc


def declared_symbols():
    """Function names declared in include/*.h (the exported C-ABI)."""
    import re
    names = []
    for fn in sorted(os.listdir(INCLUDE_DIR)):
        if not fn.endswith(".h"):
            continue
        src = open(os.path.join(INCLUDE_DIR, fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"\b((?:hipF|kcnn)_[A-Za-z0-9_]+)\s*\(", src)
    return sorted(set(names))


# ---------------------------------------------------------------------------
# device / stream
_initialized_device = None


def init(device: int = 0):
    """CuDevice::SelectGpuId + bind the library to torch's current stream."""
    global _initialized_device
    import torch
    if not torch.cuda.is_available():
        raise KcnnError("no GPU: the kcnn product path has no CPU fallback")
    torch.cuda.set_device(device)
    check(lib().kcnn_init(device))
    sync_stream()
    _initialized_device = device


def sync_stream():
    """Launch subsequent kernels on torch's current stream."""
    import torch
    check(lib().kcnn_set_stream(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))


def _ensure_init():
    if _initialized_device is None:
        import torch
        init(torch.cuda.current_device() if torch.cuda.is_available() else 0)


def set_literal_path(on: bool):
    check(lib().kcnn_set_literal_path(int(bool(on))))


def set_profiling(on: bool):
    check(lib().kcnn_set_profiling(int(bool(on))))


def set_fusion(mode):
    """kcnn_nnet runtime: fuse Conv -> Maxpool (see kcnn.h).  0 / False: off;
    1 / True: on, the conv output not stored; 2: on, the conv output stored."""
    check(lib().kcnn_set_fusion(int(mode)))


def device_malloc_calls() -> int:
    """CuDevice::Malloc calls so far (kcnn_device_malloc_calls)."""
    return int(lib().kcnn_device_malloc_calls())


def conv_fix_counts(reset=False):
    """(f16x3 implicit-GEMM calls, tiles, elements recomputed by its fp32
    fix-ups) since the last reset (kcnn_conv_fix_counts)."""
    if not hasattr(lib(), "kcnn_conv_fix_counts"):  # (absent from pre-r06 builds)
        return None
    out = (ctypes.c_ulonglong * 3)()
    check(lib().kcnn_conv_fix_counts(out, int(bool(reset))))
    return tuple(int(v) for v in out)


def profile_string() -> str:
    buf = ctypes.create_string_buffer(1 << 16)
    check(lib().kcnn_profile_string(buf, len(buf)))
    return buf.value.decode()


def set_gemm_mode(mode: int):
    """AddMatMat's fp32 product: 0 = rocBLAS sgemm, 1 = bf16x6 split kernel,
    2 = f16x3 split kernel (default)."""
    check(lib().kcnn_set_gemm_mode(int(mode)))


def set_kernel_family(name: str, value: int):
    """Kernel-family selector (kcnn.h): "fwd_x6" (2 f16x3 / 1 bf16x6 / 0),
    "bwd_x6", "igemm_x6", "wgrad_x6" (2 wide / 1 / 0) or "gemm" (2 f16x3 /
    1 bf16x6 / 0 rocBLAS); 0 = the fp32-MFMA kernels."""
    check(lib().kcnn_set_kernel_family(name.encode(), int(value)))


def get_kernel_family(name: str) -> int:
    v = lib().kcnn_get_kernel_family(name.encode())
    if v < 0:
        raise KcnnError(f"unknown kernel family {name!r}")
    return v


def gemm(a, b, c, trans_a=False, trans_b=False, alpha=1.0, beta=0.0):
    """c = alpha * op(a) op(b) + beta * c (CuMatrixBase::AddMatMat) on torch
    fp32 device matrices with contiguous rows."""
    m, n = c.shape
    am, k = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    bk, bn = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if am != m or bk != k or bn != n:
        raise KcnnError(f"gemm: op(a) {am}x{k}, op(b) {bk}x{bn} do not make c {m}x{n}")
    for t in (a, b, c):
        dim(t)
    check(lib().kcnn_gemm(int(bool(trans_a)), int(bool(trans_b)), m, n, k,
                          ctypes.c_float(alpha), ctypes.c_void_p(a.data_ptr()), a.stride(0),
                          ctypes.c_void_p(b.data_ptr()), b.stride(0), ctypes.c_float(beta),
                          ctypes.c_void_p(c.data_ptr()), c.stride(0)))


def split_planes(x):
    """fp32 [rows x cols] device matrix -> int16 tensor [3, rows, cols'] of its
    bf16 planes h, m, l (x = h + m + l exactly); cols' = cols rounded up to 8."""
    import torch
    rows, cols = x.shape
    ldp = (cols + 7) // 8 * 8
    out = torch.zeros((3, rows, ldp), dtype=torch.int16, device=x.device)
    check(lib().kcnn_split_planes(ctypes.c_void_p(x.data_ptr()), rows, cols, x.stride(0),
                                  ctypes.c_void_p(out.data_ptr()), ldp,
                                  ctypes.c_int64(rows * ldp)))
    return out


def gemm_planes(ap, bp, c, k, trans_a=False, trans_b=False, alpha=1.0, beta=0.0):
    """kcnn_gemm from split_planes() operands; c fp32 [m x n]."""
    m, n = c.shape
    check(lib().kcnn_gemm_planes(int(bool(trans_a)), int(bool(trans_b)), m, n, k,
                                 ctypes.c_float(alpha), ctypes.c_void_p(ap.data_ptr()),
                                 ap.stride(1), ctypes.c_int64(ap.stride(0)),
                                 ctypes.c_void_p(bp.data_ptr()), bp.stride(1),
                                 ctypes.c_int64(bp.stride(0)), ctypes.c_float(beta),
                                 ctypes.c_void_p(c.data_ptr()), c.stride(0)))


def reset_profile():
    check(lib().kcnn_reset_profile())


def set_randn_seed(seed: int):
    lib().kcnn_set_randn_seed(ctypes.c_uint64(seed))


def synchronize():
    check(lib().kcnn_synchronize())


def dim(t) -> MatrixDim:
    assert t.dim() == 2, "matrices are 2-D"
    assert t.dtype.is_floating_point and t.element_size() == 4, t.dtype
    assert t.is_cuda, "device tensors only"
    assert t.shape[1] <= 1 or t.stride(1) == 1, "rows must be contiguous"
    stride = t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1)
    return MatrixDim(t.shape[0], t.shape[1], stride)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def empty(rows, cols, device=None):
    import torch
    return torch.empty((rows, cols), dtype=torch.float32,
                       device=device or "cuda")


def zeros(rows, cols, device=None):
    import torch
    return torch.zeros((rows, cols), dtype=torch.float32,
                       device=device or "cuda")


# ---------------------------------------------------------------------------
# CuMatrixBase extension methods (cu-matrix.h:451-480)

def Conv2D(this, kernel, in_height, in_width, in_channel, kernel_height,
           kernel_width, group, out=None, concat=True):
    _ensure_init()
    oh, ow = in_height - kernel_height + 1, in_width - kernel_width + 1
    if out is None:
        out = (empty(this.shape[0], oh * ow * group) if concat
               else empty(oh * ow * this.shape[0], group))
    check(lib().kcnn_mat_conv2d(ptr(this), dim(this), ptr(kernel), dim(kernel),
                                in_height, in_width, in_channel, kernel_height,
                                kernel_width, group, ptr(out), dim(out),
                                int(concat)))
    return out


def AddMatRepVec(this, vec, rep):
    _ensure_init()
    check(lib().kcnn_mat_add_mat_rep_vec(ptr(this), dim(this), ptr(vec),
                                         vec.numel(), rep))
    return this


def FlipMat(this, kernel_height, kernel_width, in_channel, group, flip=None):
    _ensure_init()
    if flip is None:
        flip = zeros(kernel_height * kernel_width * group, in_channel)
    check(lib().kcnn_mat_flip_mat(ptr(this), dim(this), kernel_height,
                                  kernel_width, in_channel, group, ptr(flip),
                                  dim(flip)))
    return flip


def PaddingZero(this, orig_height, orig_width, orig_channel, kernel_height,
                kernel_width, padmat=None):
    _ensure_init()
    ph, pw = orig_height + 2 * (kernel_height - 1), orig_width + 2 * (kernel_width - 1)
    if padmat is None:
        padmat = zeros(this.shape[0], ph * pw * orig_channel)
    check(lib().kcnn_mat_padding_zero(ptr(this), dim(this), orig_height,
                                      orig_width, orig_channel, kernel_height,
                                      kernel_width, ptr(padmat), dim(padmat)))
    return padmat


def TpBlock(this, in_channel, block_size, out=None):
    _ensure_init()
    if out is None:
        out = zeros(in_channel, this.shape[0] * block_size)
    check(lib().kcnn_mat_tp_block(ptr(this), dim(this), in_channel, block_size,
                                  ptr(out), dim(out)))
    return out


def TpInsideBlock(this, group, block_size, out=None):
    _ensure_init()
    if out is None:
        out = zeros(block_size * this.shape[0], group)
    check(lib().kcnn_mat_tp_inside_block(ptr(this), dim(this), group,
                                         block_size, ptr(out), dim(out)))
    return out


def ModPermuteRow(this, in_channel, block_size, out=None):
    _ensure_init()
    if out is None:
        out = zeros(this.shape[0], this.shape[1])
    check(lib().kcnn_mat_mod_permute_row(ptr(this), dim(this), in_channel,
                                         block_size, ptr(out), dim(out)))
    return out


def ModPermuteChannel(this, comp_idx, num_component, in_height, in_width,
                      container, from_comp_to_container):
    """conv2D.cc:685-727; writes `container` (or `this` when
    from_comp_to_container is False)."""
    _ensure_init()
    check(lib().kcnn_mat_mod_permute_channel(
        ptr(this), dim(this), comp_idx, num_component, in_height, in_width,
        ptr(container), dim(container), int(bool(from_comp_to_container))))
    return container if from_comp_to_container else this


def Maxpool_prop(this, in_height, in_width, pool_height_dim, pool_width_dim,
                 pool_channel_dim, overlap, overlap2D, out):
    _ensure_init()
    check(lib().kcnn_mat_maxpool_prop(ptr(this), dim(this), in_height, in_width,
                                      pool_height_dim, pool_width_dim,
                                      pool_channel_dim, int(overlap),
                                      int(overlap2D), ptr(out), dim(out)))
    return out


def Maxpool_backprop(this, out_value, out_deriv, in_deriv, in_height, in_width,
                     pool_height_dim, pool_width_dim, pool_channel_dim,
                     overlap=False, overlap2D=False):
    _ensure_init()
    check(lib().kcnn_mat_maxpool_backprop(
        ptr(this), dim(this), ptr(out_value), dim(out_value), ptr(out_deriv),
        dim(out_deriv), ptr(in_deriv), dim(in_deriv), in_height, in_width,
        pool_height_dim, pool_width_dim, pool_channel_dim, int(overlap),
        int(overlap2D)))
    return in_deriv


# ---------------------------------------------------------------------------
# Components

PARAM_LINEAR, PARAM_BIAS, PARAM_PREV_GRAD = 0, 1, 2


class Component:
    """Handle on an nnet2 component living in libkcnn.so."""

    def __init__(self, handle, owned=True, keep=None):
        if not handle:
            raise KcnnError(lib().kcnn_last_error().decode(errors="replace"))
        self._h = ctypes.c_void_p(handle)
        self._owned = owned
        self._keep = keep  # keeps an owning Nnet alive for borrowed handles

    @classmethod
    def NewFromString(cls, initializer_line: str) -> "Component":
        _ensure_init()
        return cls(lib().kcnn_component_new_from_string(initializer_line.encode()))

    @classmethod
    def ReadNew(cls, path: str) -> "Component":
        _ensure_init()
        return cls(lib().kcnn_component_read(str(path).encode()))

    def Write(self, path: str, binary: bool = True):
        check(lib().kcnn_component_write(self._h, str(path).encode(), int(binary)))

    def Copy(self) -> "Component":
        return Component(lib().kcnn_component_copy(self._h))

    def __del__(self):
        try:
            if getattr(self, "_owned", False) and self._h:
                lib().kcnn_component_free(self._h)
                self._h = None
        except Exception:
            pass

    def _str(self, fn) -> str:
        buf = ctypes.create_string_buffer(4096)
        check(fn(self._h, buf, len(buf)))
        return buf.value.decode()

    def SplitGradient(self) -> bool:
        """Whether kcnn_dp may compute this layer's gradient apart from its
        data gradient (mode 3 then mode 2): not for a convolution, whose
        fused backward makes both from one pass over its output derivative."""
        return self.Type() != "ConvolutionComponent"

    def Type(self) -> str:
        return self._str(lib().kcnn_component_type)

    def Info(self) -> str:
        return self._str(lib().kcnn_component_info)

    def InputDim(self) -> int:
        return lib().kcnn_component_input_dim(self._h)

    def OutputDim(self) -> int:
        return lib().kcnn_component_output_dim(self._h)

    def BackpropNeedsInput(self) -> bool:
        return bool(lib().kcnn_component_backprop_needs_input(self._h))

    def BackpropNeedsOutput(self) -> bool:
        return bool(lib().kcnn_component_backprop_needs_output(self._h))

    def Context(self):
        """Component::Context(): frame offsets read per output frame."""
        buf = (ctypes.c_int * 256)()
        n = lib().kcnn_component_context(self._h, buf, 256)
        if n < 0:
            check(1)
        return list(buf[:n])

    def _span(self):
        ctx = self.Context()
        return ctx[-1] - ctx[0]

    def Propagate(self, inp, out=None, num_chunks=None):
        """num_chunks defaults to one output frame per chunk (the input chunk
        is that frame widened by Context(): SpliceComponent)."""
        span = self._span()
        if num_chunks is None:
            num_chunks = inp.shape[0] // (span + 1)
        if out is None:
            out = empty(inp.shape[0] - num_chunks * span, self.OutputDim())
        check(lib().kcnn_component_propagate(self._h, ptr(inp), dim(inp),
                                             ptr(out), dim(out), num_chunks))
        return out

    def NonlinearStats(self):
        """(value_sum, deriv_sum, count) of a NonlinearComponent (fp64)."""
        import numpy as np
        n = self.InputDim()
        vs, ds = np.zeros(n, np.float64), np.zeros(n, np.float64)
        cnt = ctypes.c_double()
        k = ctypes.c_int()
        check(lib().kcnn_component_nonlinear_stats(
            self._h, vs.ctypes.data_as(ctypes.c_void_p), ds.ctypes.data_as(ctypes.c_void_p),
            n, ctypes.byref(k), ctypes.byref(cnt)))
        return vs[:k.value], ds[:k.value], cnt.value

    def Backprop(self, in_value, out_value, out_deriv, in_deriv=None,
                 update=True, num_chunks=None, need_in_deriv=True):
        span = self._span()
        if num_chunks is None:
            num_chunks = out_deriv.shape[0]
        if in_deriv is None and need_in_deriv:
            in_deriv = empty(out_deriv.shape[0] + num_chunks * span, self.InputDim())
        if out_value is None:
            out_value = out_deriv  # dummy when BackpropNeedsOutput() is false
        if in_value is None:
            in_value = in_deriv if in_deriv is not None else out_deriv
        idim = dim(in_deriv) if in_deriv is not None else MatrixDim(0, 0, 0)
        check(lib().kcnn_component_backprop(
            self._h, ptr(in_value), dim(in_value), ptr(out_value),
            dim(out_value), ptr(out_deriv), dim(out_deriv), ptr(in_deriv), idim,
            num_chunks, int(update)))
        return in_deriv

    # parameters
    def ParamDim(self, which):
        r, c = ctypes.c_int(), ctypes.c_int()
        check(lib().kcnn_component_param_dim(self._h, which, ctypes.byref(r),
                                             ctypes.byref(c)))
        return r.value, c.value

    def GetParam(self, which):
        r, c = self.ParamDim(which)
        t = empty(r, c)
        check(lib().kcnn_component_get_param(self._h, which, ptr(t), dim(t)))
        return t if which != PARAM_BIAS else t.view(-1)

    def SetParam(self, which, value):
        r, c = self.ParamDim(which)
        v = value.reshape(r, c).contiguous().float()
        check(lib().kcnn_component_set_param(self._h, which, ptr(v), dim(v)))

    def LinearParams(self):
        return self.GetParam(PARAM_LINEAR)

    def BiasParams(self):
        return self.GetParam(PARAM_BIAS)

    def PrevGrad(self):
        return self.GetParam(PARAM_PREV_GRAD)

    def LearningRate(self) -> float:
        return lib().kcnn_component_learning_rate(self._h)

    def SetLearningRate(self, lr: float):
        check(lib().kcnn_component_set_learning_rate(self._h, ctypes.c_float(lr)))

    def DotProduct(self, other) -> float:
        out = ctypes.c_float()
        check(lib().kcnn_component_dot_product(self._h, other._h, ctypes.byref(out)))
        return out.value

    def SetZero(self, treat_as_gradient: bool):
        check(lib().kcnn_component_set_zero(self._h, int(treat_as_gradient)))

    def Scale(self, s: float):
        check(lib().kcnn_component_scale(self._h, ctypes.c_float(s)))

    def Add(self, alpha: float, other):
        check(lib().kcnn_component_add(self._h, ctypes.c_float(alpha), other._h))

    def PerturbParams(self, stddev: float):
        check(lib().kcnn_component_perturb_params(self._h, ctypes.c_float(stddev)))

    def NumGradientParams(self) -> int:
        return lib().kcnn_component_num_gradient_params(self._h)

    def ComputeGradient(self, in_value, out_deriv, grad=None):
        import torch
        if grad is None:
            grad = torch.empty(self.NumGradientParams(), dtype=torch.float32,
                               device="cuda")
        check(lib().kcnn_component_compute_gradient(
            self._h, ptr(in_value), dim(in_value), ptr(out_deriv),
            dim(out_deriv), ptr(grad)))
        return grad

    def BackpropGradient(self, in_value, out_deriv, in_deriv=None, grad=None,
                         want_in_deriv=True):
        """Backprop (no update) + ComputeGradient in one call; returns
        (in_deriv or None, grad)."""
        import torch
        if grad is None:
            grad = torch.empty(self.NumGradientParams(), dtype=torch.float32,
                               device="cuda")
        if in_deriv is None and want_in_deriv:
            in_deriv = empty(in_value.shape[0], self.InputDim())
        check(lib().kcnn_component_backprop_gradient(
            self._h, ptr(in_value), dim(in_value), ptr(out_deriv),
            dim(out_deriv), ptr(in_deriv) if in_deriv is not None else None,
            dim(in_deriv) if in_deriv is not None else MatrixDim(0, 0, 0),
            ptr(grad)))
        return in_deriv, grad

    def ApplyGradient(self, grad, num_sample: int):
        check(lib().kcnn_component_apply_gradient(self._h, ptr(grad), int(num_sample)))

    def FlipKernelBranch(self) -> bool:
        rc = lib().kcnn_component_conv_flip_branch(self._h)
        if rc < 0:
            check(rc)
        return bool(rc)


class Nnet:
    """A stack of components run like upstream nnet2's NnetUpdater."""

    def __init__(self, config: str):
        _ensure_init()
        h = lib().kcnn_nnet_new(config.encode())
        if not h:
            raise KcnnError(lib().kcnn_last_error().decode(errors="replace"))
        self._h = ctypes.c_void_p(h)
        n = lib().kcnn_nnet_num_components(self._h)
        self.components = [Component(lib().kcnn_nnet_component(self._h, i),
                                     owned=False, keep=self) for i in range(n)]

    def __del__(self):
        try:
            if self._h:
                lib().kcnn_nnet_free(self._h)
                self._h = None
        except Exception:
            pass

    def NumComponents(self):
        return len(self.components)

    def Propagate(self, inp):
        self._input = inp  # the library borrows it until Backprop
        check(lib().kcnn_nnet_propagate(self._h, ptr(inp), dim(inp)))

    def Output(self, i=-2):
        """Layer i's output as a torch view (i = -2: the last layer)."""
        import torch
        if i == -2:
            i = self.NumComponents() - 1
        p = ctypes.c_void_p()
        d = MatrixDim()
        check(lib().kcnn_nnet_output(self._h, i, ctypes.byref(p), ctypes.byref(d)))
        return _device_view(p.value, d)

    def InputDeriv(self, i):
        """d(input of component i) from the last backprop, as a torch view."""
        p = ctypes.c_void_p()
        d = MatrixDim()
        check(lib().kcnn_nnet_input_deriv(self._h, i, ctypes.byref(p), ctypes.byref(d)))
        return _device_view(p.value, d)

    def BackpropComponent(self, i, out_deriv=None, mode=0, grad=None,
                          skip_first_dx=True):
        od = out_deriv
        odim = dim(od) if od is not None else MatrixDim(0, 0, 0)
        check(lib().kcnn_nnet_backprop_component(self._h, i, ptr(od), odim, mode,
                                                 ptr(grad), int(skip_first_dx)))

    def BackpropSplit(self, i, out_deriv, grad, skip_first_dx, between):
        """kcnn_nnet_backprop_split: affine layer i's gradient into grad,
        then between() (e.g. the gradient's all-reduce is started there),
        then its input derivative; one statistics pass for both GEMMs."""
        err = []

        def cb(_ctx):
            try:
                between()
            except BaseException as e:  # noqa: BLE001 -- re-raised below
                err.append(e)
        fn = ctypes.CFUNCTYPE(None, ctypes.c_void_p)(cb)
        od = out_deriv
        odim = dim(od) if od is not None else MatrixDim(0, 0, 0)
        rc = lib().kcnn_nnet_backprop_split(self._h, i, ptr(od), odim, ptr(grad),
                                            int(skip_first_dx), fn, None)
        if err:
            raise err[0]
        check(rc)

    def Backprop(self, out_deriv, skip_first_dx=False):
        """The whole backward in one kcnn_nnet_backprop call; with
        skip_first_dx, one kcnn_nnet_backprop_component call per layer."""
        if not skip_first_dx:
            check(lib().kcnn_nnet_backprop(self._h, ptr(out_deriv), dim(out_deriv)))
            return
        for i in reversed(range(self.NumComponents())):
            self.BackpropComponent(i, out_deriv, 0, None, skip_first_dx)


def _device_view(addr, d: MatrixDim):
    """A torch tensor aliasing library-owned device memory (read-mostly)."""
    import torch
    if d.rows == 0 or d.cols == 0:
        return torch.empty((d.rows, d.cols), dtype=torch.float32, device="cuda")
    nbytes = ((d.rows - 1) * d.stride + d.cols) * 4

    class _Arr:
        __cuda_array_interface__ = {
            "shape": (nbytes // 4,), "typestr": "<f4", "data": (addr, False),
            "version": 2, "strides": None}

    flat = torch.as_tensor(_Arr(), device="cuda")
    return flat.as_strided((d.rows, d.cols), (d.stride, 1))
