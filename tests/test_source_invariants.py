"""Source-level invariants of the HIP kernels (CPU only, no build needed).

LDS-DMA (`__builtin_amdgcn_raw_ptr_buffer_load_lds`) writes LDS behind the
compiler's back, so the barrier that publishes its data must wait for the
wave's vector-memory loads first.  That wait + barrier exists in one place,
`x6::publish_dma()` (src/cnslmat/lds-dma.h); these checks keep it that way:
LDS-DMA appears only in the known kernel files, each of them publishes
through the helper, and no hand-rolled vmcnt wait + barrier pair remains.
"""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "kaldi-cnn_amd", "src")
DMA_FILES = {"cnslmat/cnsl-conv-x6.hip", "cnslmat/cnsl-conv-frame.hip",
             "kaldi-lite/cu-gemm-x6.hip"}


def sources():
    for p in sorted(glob.glob(os.path.join(SRC, "*", "*.hip")) +
                    glob.glob(os.path.join(SRC, "*", "*.h"))):
        yield os.path.relpath(p, SRC), open(p).read()


def strip_comments(text):
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def test_lds_dma_only_in_known_kernels():
    users = {name for name, text in sources()
             if "raw_ptr_buffer_load_lds" in strip_comments(text)}
    assert users == DMA_FILES, users


def test_lds_dma_kernels_publish_through_the_helper():
    for name, text in sources():
        code = strip_comments(text)
        if name in DMA_FILES:
            assert "publish_dma()" in code, f"{name}: LDS-DMA without publish_dma()"
        if name == "cnslmat/lds-dma.h":
            continue
        # no hand-rolled vmcnt(0) wait directly followed by a barrier
        pair = re.search(r"s_waitcnt\(0x0F70\)\s*;\s*__syncthreads\(\)", code)
        assert not pair, f"{name}: raw vmcnt wait + barrier, use x6::publish_dma()"
        assert "wait_dma()" not in code.replace("publish_dma()", ""), \
            f"{name}: wait_dma() outside publish_dma()"
