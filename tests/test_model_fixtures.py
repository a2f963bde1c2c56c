"""Kaldi binary model files (byte-compatible model I/O).

tests/golden/models/*.bin are encoded by tests/kaldi_binary.py -- an encoder
written from Kaldi's binary format definition and the reference's token
sequences, independent of the C++ kaldi-lite I/O -- by
scripts/make_model_fixtures.py.  The reference ships no model files of its
own, so these are the pin.  CPU: the fixtures are what the encoder produces
for the stored parameters.  GPU: Component::ReadNew parses each file into the
stored parameters and Write reproduces it byte for byte.
"""
import os

import numpy as np
import pytest

import kaldi_binary as KB

MODELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "models")
KINDS = ["conv", "maxpool", "fc", "relu", "splice"]


def _params(kind):
    z = np.load(os.path.join(MODELS, f"{kind}.npz"))
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("kind", KINDS)
def test_fixture_matches_spec_encoder(kind):
    data = open(os.path.join(MODELS, f"{kind}.bin"), "rb").read()
    assert data == KB.encode(kind, _params(kind))
    assert data.startswith(b"\x00B<")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_read_new_and_write_are_byte_compatible(kc, tmp_path, kind):
    from _util import host
    path = os.path.join(MODELS, f"{kind}.bin")
    p = _params(kind)
    c = kc.Component.ReadNew(path)
    if kind in ("conv", "fc"):
        np.testing.assert_array_equal(host(c.LinearParams()), p["linear"])
        np.testing.assert_array_equal(host(c.BiasParams()), p["b"])
        np.testing.assert_array_equal(host(c.PrevGrad()), p["prev"])
        assert c.LearningRate() == np.float32(p["lr"])
    elif kind == "maxpool":
        assert c.InputDim() == p["input_dim"] and c.OutputDim() == p["output_dim"]
    elif kind == "relu":
        vs, ds, cnt = c.NonlinearStats()
        np.testing.assert_array_equal(vs, p["value_sum"])
        np.testing.assert_array_equal(ds, p["deriv_sum"])
        assert cnt == p["count"]
    else:
        assert c.Context() == list(p["context"])
        assert c.InputDim() == p["input_dim"]
    out = tmp_path / f"{kind}.bin"
    c.Write(out, True)
    assert open(out, "rb").read() == open(path, "rb").read()
