#!/usr/bin/env python3
"""Golden vectors for the episode envelope statistics from the reference itself.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_envelope.py /root/reference

Imports environment/utils.py (absent packages replaced by the inert stand-ins
of make_golden.py) and evaluates calc_envelope (utils.py:835-836) on the
seeded episode-length signals of make_golden_eval.signals() plus short/odd
edge cases, then the statistics custom_callbacks.py:28-31 logs for it
(np.mean, np.std(ddof=1), np.sum -- restated here: the callback class needs
stable_baselines3's logger).  Writes data only, to
tests/golden/reference_envelope_golden.npz.
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def edge_signals():
    """Short, odd and even lengths (n = 1, 2, 3, 64, 255, 1000)."""
    rng = np.random.default_rng(7)
    return [rng.standard_normal(n).astype(np.float32) for n in (1, 2, 3, 64, 255, 1000)]


def main(ref_root):
    from make_golden import _write_stubs
    from make_golden_eval import signals
    tmp = tempfile.mkdtemp(prefix="kura_stubs_env_")
    _write_stubs(tmp, solve=None)
    sys.path.insert(0, tmp)
    sys.path.insert(0, ref_root)
    import environment.utils as U  # noqa: E402
    sig = signals() + edge_signals()
    stats = []
    for x in sig:
        e = U.calc_envelope(x)
        sd = np.std(e, ddof=1) if len(e) > 1 else np.nan
        stats.append([np.mean(e), sd, np.sum(e)])
    out = {"env_stats": np.asarray(stats, np.float64), "env_dtype": np.array(str(U.calc_envelope(sig[0]).dtype))}
    path = os.path.join(HERE, "reference_envelope_golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, out["env_stats"], out["env_dtype"])


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
