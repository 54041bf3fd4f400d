#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03m
mkdir -p $O
cd $R
timeout -k 10 200 ./tools/overlap_bench2 > $O/overlap6.txt 2>&1 &&
MODE=reset KURA_KERNEL=k1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_k1_reset.json 2> $O/stamps_k1_reset.err &&
MODE=reset KURA_KERNEL=k1 SI=1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/stamps_si_k1_reset.json 2> $O/stamps_si_k1_reset.err
echo "rc=$?"
