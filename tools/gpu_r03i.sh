#!/bin/bash
# r03i: K1t (team-overlapped solver) first GPU run: parity suite, bench, phase stamps K1t vs K1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03i
mkdir -p $O
cd $R
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 100 --timeout-method thread -k "env0 or n1024" > $O/gpu_quick.log 2>&1 &&
timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1t.json 2> $O/bench_k1t.err &&
timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1t_step.json 2> $O/stamps_k1t_step.err &&
KURA_KERNEL=k1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1_step.json 2> $O/stamps_k1_step.err &&
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "rc=$?"
