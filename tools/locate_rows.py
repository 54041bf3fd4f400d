#!/usr/bin/env python3
"""Offline half of the round-3 codegen investigation (CPU only).

Given the reset state of a good and a miscompiled build (tools/dump_reset.py),
find, for every wrong env, which of the oracle's dense-output rows of the
reset transient (arange(0, 200, 0.05), oracle_solve_rows) each wrong value
equals.  A wrong final state that equals an earlier saved row tells which
save round / pass the store was executed in.
Usage: locate_rows.py DIR ENV N B good.npz bad.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import ko, make_case  # noqa: E402


def main():
    d, name, N, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    good = np.load(os.path.join(d, sys.argv[5]))
    bad = np.load(os.path.join(d, sys.argv[6]))
    cfg, alpha, omega, gs, gr, th0, ct, st, _ = make_case(name, N, B)
    o = ko.Oracle(cfg, alpha)
    o.set_env_params(omega, gs, gr)
    o.set_spectral(ct, st)
    o.reset(th0)
    ref = o.state()
    print("good == oracle:", np.array_equal(good["y"], ref["y"]), np.array_equal(good["ring"], ref["ring"]))
    wrong = sorted(set(np.argwhere(bad["y"] != ref["y"])[:, 0].tolist()))
    print("wrong envs (y):", wrong)
    print("wrong envs (ring):", sorted(set(np.argwhere(bad["ring"] != ref["ring"])[:, 0].tolist())))
    print("t equal:", np.array_equal(bad["t"], ref["t"]), "stats good", good["stats"][:4], "bad", bad["stats"][:4])
    ts = ko.arange(0.0, cfg.transient_len, cfg.dt)
    for b in wrong[:4]:
        rows, _ = o.solve_rows(omega[b], None, ts, th0[b])
        assert np.array_equal(rows[-1], ref["y"][b])
        yb = bad["y"][b]
        nbad = int(np.sum(yb != ref["y"][b]))
        # exact per-element matches against every row
        hits = (rows == yb[None, :]).sum(axis=1)
        top = np.argsort(-hits)[:5]
        print(f"env {b}: {nbad}/{N} elements wrong; best-matching rows {[(int(r), int(hits[r])) for r in top]}")
        # per element: the row index each wrong element equals (if unique)
        idx = [np.flatnonzero(rows[:, i] == yb[i]) for i in range(N)]
        rr = [int(x[-1]) for x in idx if len(x)]
        if rr:
            u, c = np.unique(rr, return_counts=True)
            print("   rows matched per element (row: count):", dict(zip(u[-8:].tolist(), c[-8:].tolist())))
        wr = bad["ring"][b]
        rr_ = ref["ring"][b]
        nd = np.flatnonzero(wr != rr_)
        print(f"   ring: {len(nd)} of {len(wr)} samples differ; first {nd[:5].tolist()}")


if __name__ == "__main__":
    main()
