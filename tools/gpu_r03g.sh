#!/bin/bash
# r03g: phase breakdown of K1w vs K1 (KURA_STAMPS build), boundary tests re-run
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03g
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1w_step.json 2> $O/stamps_k1w_step.err &&
MODE=reset timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1w_reset.json 2> $O/stamps_k1w_reset.err &&
KURA_KERNEL=k1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1_step.json 2> $O/stamps_k1_step.err &&
timeout -k 10 400 python3 -u -m pytest tests/test_boundary_r03.py -m gpu -v --timeout 150 --timeout-method thread > $O/boundary.log 2>&1
echo "rc=$?"
