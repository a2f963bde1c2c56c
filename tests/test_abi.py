"""The drop-in boundary without a GPU: libkcnn.so (the C-ABI of include/*.h)
loads, exports every declared entry point, and fails loudly -- with an error
code and message, never a silent CPU fallback -- when no GPU is present."""
import ctypes
import os
import subprocess

import pytest
import torch

import kcnn

HAVE_GPU = torch.cuda.is_available()


def _lib():
    if not os.path.exists(kcnn.LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.dirname(kcnn.LIB_PATH), "-j8"],
                       check=True)
    return kcnn.lib()


def test_declared_symbols_parsed():
    names = kcnn.declared_symbols()
    # the reference's cudaF_* operator set (cnsl-cu-kernels.h:22-70) minus
    # launch geometry, the fused conv passes, and the component/nnet C-ABI
    for must in ("hipF_span_row_to_convmat", "hipF_convmat_to_out", "hipF_add_mat_rep_vec",
                 "hipF_flip_mat", "hipF_pad_zero", "hipF_tp_block", "hipF_tp_inside_block",
                 "hipF_mod_permute_row", "hipF_copy_rows_at", "hipF_maxpool_prop",
                 "hipF_maxpool_backprop", "hipF_conv2d", "hipF_conv2d_wgrad",
                 "hipF_conv2d_dgrad", "hipF_conv2d_backward", "hipF_momentum_update",
                 "kcnn_component_new_from_string", "kcnn_component_propagate",
                 "kcnn_component_backprop", "kcnn_component_backprop_gradient",
                 "kcnn_nnet_backprop_component"):
        assert must in names, must
    assert len(names) >= 60


def test_library_exports_every_declared_symbol():
    L = _lib()
    missing = [n for n in kcnn.declared_symbols() if not hasattr(L, n)]
    assert not missing, f"declared in include/*.h but not exported: {missing}"


def test_no_cuda_or_compat_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", kcnn.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = [l.split()[-1] for l in out.splitlines() if " T " in l]
    assert not [s for s in exported if s.startswith(("cuda", "cublas", "nccl"))]


def test_version_and_host_selftest():
    L = _lib()
    assert L.kcnn_version().decode().startswith("kcnn")
    assert L.kcnn_selftest_fastdiv() == 0        # host-side index arithmetic


@pytest.mark.skipif(HAVE_GPU, reason="checks the no-GPU failure path")
def test_fails_loudly_without_gpu():
    L = _lib()
    assert L.kcnn_init(0) != 0
    msg = L.kcnn_last_error().decode()
    assert msg, "no error message"
    with pytest.raises(kcnn.KcnnError, match="no GPU"):
        kcnn.init(0)
    # parameters live in device memory: constructing an updatable component
    # is an error, not a host fallback
    h = L.kcnn_component_new_from_string(
        b"ConvolutionComponent in-height=4 in-width=4 in-channel=1 kernel-height=2 "
        b"kernel-width=2 stride=1 group=2 out-height=3 out-width=3 learning-rate=0.1")
    assert not h
    assert L.kcnn_last_error().decode()


def test_missing_library_raises(monkeypatch):
    monkeypatch.setattr(kcnn, "_lib", None)
    monkeypatch.setattr(kcnn, "LIB_PATH", "/nonexistent/libkcnn.so")
    with pytest.raises(kcnn.KcnnError, match="not built"):
        kcnn.lib()


# the documented run-time switches of the product library (kcnn-knobs.h):
# kernel-family selectors plus fusion, literal replay, profiling and logging.
# Experiment knobs are read only by the `make timing` build.
DOCUMENTED_ENV = {"KCNN_FWD_X6", "KCNN_BWD_X6", "KCNN_IGEMM_X6", "KCNN_WGRAD_X6",
                  "KCNN_GEMM", "KCNN_FUSE", "KCNN_LITERAL", "KCNN_PROFILE", "KCNN_QUIET"}


def test_product_library_reads_only_documented_switches():
    _lib()
    out = subprocess.run(["strings", kcnn.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    env = {l for l in out.split() if l.startswith("KCNN_") and l.isupper()}
    assert env <= DOCUMENTED_ENV, f"undocumented switches: {sorted(env - DOCUMENTED_ENV)}"


def test_kernel_family_selectors():
    _lib()
    defaults = {"fwd_x6": 2, "bwd_x6": 1, "igemm_x6": 2, "wgrad_x6": 2, "gemm": 2}
    for name, d in defaults.items():
        if not os.environ.get("KCNN_" + name.upper()):
            assert kcnn.get_kernel_family(name) == d, name
    try:
        kcnn.set_kernel_family("wgrad_x6", 1)
        assert kcnn.get_kernel_family("wgrad_x6") == 1
        kcnn.set_kernel_family("gemm", 0)
        assert kcnn.get_kernel_family("gemm") == 0
        kcnn.set_kernel_family("igemm_x6", 3)  # f16x3 for every shape
        assert kcnn.get_kernel_family("igemm_x6") == 3
        with pytest.raises(kcnn.KcnnError, match="out of range"):
            kcnn.set_kernel_family("igemm_x6", 4)
        with pytest.raises(kcnn.KcnnError, match="out of range"):
            kcnn.set_kernel_family("bwd_x6", 2)
        with pytest.raises(kcnn.KcnnError, match="unknown"):
            kcnn.set_kernel_family("no_such_family", 0)
        with pytest.raises(kcnn.KcnnError):
            kcnn.get_kernel_family("no_such_family")
    finally:
        for name, d in defaults.items():
            kcnn.set_kernel_family(name, d)
