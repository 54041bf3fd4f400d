#!/bin/bash
# Round-3 validation of the final tree on a fresh box: GPU suite, smoke, the
# default bench line (as the driver runs it), the rocprofv3 trace of 60
# steady launches + FETCH/WRITE/GRBM passes, SQ/SQC counter passes, and the
# N=8192 stress lines (strong form: 128 envs per GPU, parts of 256; weak form).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03_final2}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_stress128.json 2> $O/bench_stress128.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --steps 4 --warmup 2 --cpu-seconds 0 > $O/bench_stress1024.json 2> $O/bench_stress1024.err &&
bash tools/rocprof_run.sh ${T}_prof > $O/rocprof.log 2>&1 &&
bash tools/pmc_pass.sh ${T}_pmc > $O/pmc.log 2>&1
echo "rc=$?"
