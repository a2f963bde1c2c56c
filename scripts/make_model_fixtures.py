"""Generate tests/golden/models/: Kaldi binary model files of each component,
encoded by tests/kaldi_binary.py from the format definition, plus the
parameters they hold (.npz).  The GPU test reads them through
Component::ReadNew and requires Write to reproduce them byte for byte.

  python scripts/make_model_fixtures.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kaldi_binary as KB  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "models")


def main():
    os.makedirs(OUT, exist_ok=True)
    r = np.random.default_rng(20261016)
    f = lambda *s: r.standard_normal(s).astype(np.float32)  # noqa: E731
    H, W, C, kh, kw, G, ph, pw = 8, 9, 3, 3, 2, 5, 1, 0
    oh, ow = H + 2 * ph - kh + 1, W + 2 * pw - kw + 1
    fixtures = {
        "conv": dict(H=H, W=W, C=C, kh=kh, kw=kw, stride=1, ph=ph, pw=pw, G=G, oh=oh, ow=ow,
                     lr=0.02, wd=0.0005, m=0.9, linear=f(kh * kw * C, G), b=f(G),
                     prev=f(kh * kw * C, G) * 0.01),
        "maxpool": dict(input_dim=6 * 4 * 8, H=6, W=4, C=8, output_dim=3 * 2 * 4, ph=2, pw=2,
                        pc=2, overlap=False, overlap2D=False),
        "fc": dict(lr=0.01, linear=f(7, 20), b=f(7), wd=0.0005, m=0.5, prev=f(7, 20) * 0.01),
        "relu": dict(dim=6, value_sum=r.standard_normal(6) * 100, deriv_sum=np.arange(6.0),
                     count=17.0),
        "splice": dict(input_dim=13, context=np.array([-2, -1, 0, 1], np.int32), const_dim=3),
    }
    for kind, p in fixtures.items():
        with open(os.path.join(OUT, f"{kind}.bin"), "wb") as fh:
            fh.write(KB.encode(kind, p))
        np.savez(os.path.join(OUT, f"{kind}.npz"), **{k: np.asarray(v) for k, v in p.items()})
        print(kind, os.path.getsize(os.path.join(OUT, f"{kind}.bin")), "bytes")


if __name__ == "__main__":
    main()
