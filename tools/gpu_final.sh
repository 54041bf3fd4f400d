#!/bin/bash
# Validation of a final tree on a fresh box (via gpurun): GPU suite, smoke,
# the default bench line (as the driver runs it), the --gpus 2 launcher
# rehearsal on one device (gloo; default and env2 random-K shapes), the
# N=8192 stress lines, the rocprofv3 trace + FETCH/WRITE/clock passes and the
# SQ/SQC/TA counter passes, and the phase stamps (KURA_STAMPS build).  Each step has its own time limit; the first
# failure ends the script.
#   bash tools/gpu_final.sh <tag> [quick]     (quick: skip the stress lines and counter passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-final}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python3 bench.py --gpus 2 --share-device --dist-backend gloo --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_2rank.json 2> $O/bench_2rank.err &&
timeout -k 10 300 python3 bench.py --gpus 2 --share-device --dist-backend gloo --config env2 --random-k --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_2rank_env2.json 2> $O/bench_2rank_env2.err || exit 1
tail -2 $O/gpu_tests.log; cat $O/smoke.log | tail -1
[ "$2" = "quick" ] && { echo QUICKDONE; exit 0; }
timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_stress128.json 2> $O/bench_stress128.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --steps 4 --warmup 2 --cpu-seconds 0 > $O/bench_stress1024.json 2> $O/bench_stress1024.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --coupling f32 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_stress128_f32.json 2> $O/bench_stress128_f32.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --coupling f32 --steps 4 --warmup 2 --cpu-seconds 0 > $O/bench_stress1024_f32.json 2> $O/bench_stress1024_f32.err &&
bash tools/rocprof_run.sh ${T}_prof > $O/rocprof.log 2>&1 &&
bash tools/pmc_pass.sh ${T}_pmc > $O/pmc.log 2>&1 &&
timeout -k 10 300 python3 tools/phase_stamps.py > $O/stamps_step.json 2> $O/stamps_step.err
echo "rc=$?"
