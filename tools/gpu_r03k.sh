#!/bin/bash
# r03k: packed-f32 vs MFMA co-issue microbench; K1t / K1 built without SLP packing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03k
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/overlap_bench > $O/overlap.txt 2>&1 &&
KURA_LIB=$R/dbs-gym_amd/csrc/libkura_noslp.so timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1t_noslp.json 2> $O/bench_k1t_noslp.err &&
KURA_LIB=$R/dbs-gym_amd/csrc/libkura_noslp.so KURA_KERNEL=k1 timeout -k 10 240 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/bench_k1_noslp.json 2> $O/bench_k1_noslp.err
echo "rc=$?"
