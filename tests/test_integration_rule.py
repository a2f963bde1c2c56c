"""INTEGRATION.md's build rule for a Kaldi tree names every translation unit
of libkcnn.so: linking exactly the objects it lists (as built by
`make -C kaldi-cnn_amd`) into a shared library with --no-undefined must
succeed.  CPU only: hipcc links the gfx950 objects without a GPU."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kaldi-cnn_amd")


def rule_units():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = text[text.index("ifeq ($(ROCM), true)"):text.index("endif")]
    units = []
    for var in ("KCNN_HIP", "KCNN_CC"):
        m = re.search(var + r"\s*=\s*((?:[^\n]*\\\n)*[^\n]*)", block)
        assert m, var
        units += m.group(1).replace("\\\n", " ").split()
    return units


def test_rule_lists_every_makefile_unit():
    mk = open(os.path.join(PKG, "Makefile")).read()
    srcs = re.findall(r"src/([\w/-]+)\.(?:hip|cc)", mk[:mk.index("OBJ :=")])
    assert sorted(rule_units()) == sorted(set(srcs))


def test_rule_links_without_undefined_symbols(tmp_path):
    subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    objs = [os.path.join(PKG, "build", u + ".o") for u in rule_units()]
    missing = [o for o in objs if not os.path.exists(o)]
    assert not missing, missing
    out = tmp_path / "libkcnn_rule.so"
    r = subprocess.run(["/opt/rocm/bin/hipcc", *objs, "-shared", "-Wl,--no-undefined",
                        "-L/opt/rocm/lib", "-lamdhip64", "-lrocblas", "-o", str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
