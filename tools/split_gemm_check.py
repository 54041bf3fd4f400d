"""Check tools/split_gemm_bench's split_stream outputs (workgroup 0, dumped by
`./tools/split_gemm_bench 50 dump.bin`) against the oracle's exact model of
the bf16 MFMA accumulation chained over the split GEMM
(oracle_split_bf16_chain): the twin property of DESIGN.md section 9 at the
scale of a whole coupling GEMM (1024-deep, 384 chained MFMA dots per output).

    python tools/split_gemm_check.py gpurun_out/split_gemm_wg0.bin [n_outputs]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import kura_oracle as ko  # noqa: E402  (checker only)

N, TPW, NT = 1024, 4, 512
GX, GY, GZ = 16, 8, 8


def operand(row, k, w):
    """split_gemm_bench.hip operand(): 32-bit hash -> [-1, 1)"""
    h = (np.uint32(row) * np.uint32(N) + np.uint32(k)) * np.uint32(2654435761) + np.uint32(w) * np.uint32(40503)
    h = h.astype(np.uint32)
    h ^= h >> np.uint32(15)
    h = (h * np.uint32(2246822519)).astype(np.uint32)
    h ^= h >> np.uint32(13)
    return ((h & np.uint32(0xFFFF)).astype(np.float32) / np.float32(32768.0) - np.float32(1.0)).astype(np.float32)


def bf16_rne(v):
    u = np.asarray(v, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf2f(h):
    return (np.asarray(h, np.uint32) << 16).view(np.float32)


def split3(v):
    v = np.asarray(v, np.float32)
    h1 = bf16_rne(v)
    r1 = (v - bf2f(h1)).astype(np.float32)
    h2 = bf16_rne(r1)
    h3 = bf16_rne((r1 - bf2f(h2)).astype(np.float32))
    return np.stack([h1, h2, h3], axis=-2)   # (..., 3, K)


def alpha_matrix():
    dz, dx, dy = np.meshgrid(np.arange(GZ), np.arange(GX), np.arange(GY), indexing="ij")
    T = np.cos(0.1 * np.sqrt((dx * dx + dy * dy + dz * dz).astype(np.float64))).astype(np.float32)  # [dz][dx][dy]
    n = np.arange(N)
    y, x, z = n % GY, (n // GY) % GX, n // (GX * GY)
    return T[np.abs(z[:, None] - z[None, :]), np.abs(x[:, None] - x[None, :]), np.abs(y[:, None] - y[None, :])]


def main():
    got = np.fromfile(sys.argv[1], np.float32)
    assert got.size == NT * TPW * 16, got.size
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else got.size
    alpha = alpha_matrix()                      # [k][col]
    k = np.arange(N)
    X = np.stack([operand(r, k, 0) for r in range(32)])   # [row][k]
    xs = split3(X)                              # (32, 3, K)
    as_ = split3(alpha.T.copy())                # (col, 3, K)
    idx = np.arange(got.size)[:limit]
    r, t, tid = idx % 16, (idx // 16) % TPW, idx // (16 * TPW)
    lane, wave = tid % 64, tid // 64
    row = (r % 4) + 8 * (r // 4) + 4 * (lane >> 5)
    col = (wave * TPW + t) * 32 + (lane & 31)
    want = ko.split_bf16_chain(xs[row], as_[col])
    bad = np.flatnonzero(got[idx].view(np.uint32) != want.view(np.uint32))
    print(f"split_stream vs oracle_split_bf16_chain: {len(bad)} of {len(idx)} outputs differ")
    for b in bad[:5]:
        print(f"  row {row[b]} col {col[b]}: gpu {got[b]!r} oracle {want[b]!r}")
    return 1 if len(bad) else 0


if __name__ == "__main__":
    sys.exit(main())
