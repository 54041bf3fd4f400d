#!/bin/bash
# r03h: reward-tail fix (WinView::at inlined), float64 reward_n actions: GPU suite + K1w/K1 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03h
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1w.json 2> $O/bench_k1w.err &&
KURA_KERNEL=k1 timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1.json 2> $O/bench_k1.err &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "rc=$?"
