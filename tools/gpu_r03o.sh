#!/bin/bash
# r03o: LDS-staged twiddles in the reward tail: parity subset, bench, stamps (step, reset)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03o
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_configs.py tests/test_boundary_r03.py tests/test_gpu_parity.py tests/test_debug_build.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_quick.log 2>&1 &&
timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1.json 2> $O/bench_k1.err &&
timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1_step.json 2> $O/stamps_k1_step.err &&
MODE=reset timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1_reset.json 2> $O/stamps_k1_reset.err
echo "rc=$?"
