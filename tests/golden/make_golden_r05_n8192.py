#!/usr/bin/env python3
"""The reference RHS pin at the N = 8192 stress size (BASELINE configs[4],
the 32x16x16 grid of SURVEY.md 8(d)), from the reference itself.  Run in the
build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_r05_n8192.py /root/reference

Same stand-ins as make_golden.py / make_golden_r05.py.  Writes
tests/golden/reference_r05_n8192.npz: the reference's own
``KuramotoJAX.dynamics`` (env.py:252-256: fmod, the direct N^2
sin(theta_j - theta_i) sum, float32 arguments) on three float32 states, with
the oscillator coordinates and the SHA-1 of the reference's float32 alpha
(alpha itself, 256 MB, is rebuilt by the test from the coordinates and checked
against the digest).  Only data is written."""
from __future__ import annotations

import contextlib
import hashlib
import io
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def main(ref_root: str) -> None:
    solver = mg.OracleSolve()
    tmp = tempfile.mkdtemp(prefix="kura_stubs_")
    mg._write_stubs(tmp, solver)
    sys.path.insert(0, tmp)
    sys.path.insert(0, ref_root)
    import environment.utils as U   # noqa: E402
    import environment.env as E     # noqa: E402

    n = 8192
    rng = np.random.default_rng(8192)
    with contextlib.redirect_stdout(io.StringIO()):
        np.random.seed(228)
        r = U.generate_w0_with_locus(n, [32, 16, 16], 0.1, locus_center=[4, 4, 4], locus_size=0.55, wmuL=17,
                                     wsdL=1, show=False)
        kj = E.KuramotoJAX(n, 0.52, [32, 16, 16], np.asarray(r[0]).copy(), np.asarray(r[1]), np.asarray(r[2]),
                           [[4, 3, 4]], [[1, 1, 1]], 0.1, spatial_kernel="cos", electrode_amps=[0.0],
                           electrode_prc_type="dummy")
        ys = np.concatenate([rng.uniform(0, 6000, (2, n)), rng.uniform(0, 2 * np.pi, (1, n))]).astype(np.float32)
        a32 = np.asarray(kj.alpha, np.float32)
        pulse = (np.asarray(kj.dbs.conductances[0]) * 3.7).astype(np.float32)
        args = (np.asarray(kj.w0, np.float32), np.float32(0.52 / n), n, a32, pulse)
        f = np.stack([np.asarray(kj.dynamics(0.0, y, args), np.float32) for y in ys])
    fx = dict(y=ys, pulse=pulse, w0=args[0], f=f, coords=np.asarray(r[1], np.float64),
              alpha_sha1=np.frombuffer(hashlib.sha1(a32.tobytes()).digest(), np.uint8))
    path = os.path.join(HERE, "reference_r05_n8192.npz")
    np.savez_compressed(path, **{f"rhs_n8192_{k}": v for k, v in fx.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
