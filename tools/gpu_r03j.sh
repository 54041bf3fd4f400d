#!/bin/bash
# r03j: bbpow_multi reward tail; K1t vs K1 bench; phase stamps (+ stage-input sub-phases)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03j
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py tests/test_boundary_r03.py tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread > $O/gpu_quick.log 2>&1 &&
timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1t.json 2> $O/bench_k1t.err &&
KURA_KERNEL=k1 timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1.json 2> $O/bench_k1.err &&
timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1t_step.json 2> $O/stamps_k1t_step.err &&
KURA_KERNEL=k1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1_step.json 2> $O/stamps_k1_step.err &&
SI=1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_si_k1t_step.json 2> $O/stamps_si_k1t_step.err &&
SI=1 KURA_KERNEL=k1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_si_k1_step.json 2> $O/stamps_si_k1_step.err
echo "rc=$?"
