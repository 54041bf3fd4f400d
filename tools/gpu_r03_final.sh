#!/bin/bash
# Round-3 validation of the production build on a fresh box: GPU suite,
# smoke, the default bench line (as the driver runs it), the rocprofv3 trace
# of 60 steady launches + FETCH/WRITE/GRBM passes, and SQ/SQC counter passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r03_final}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err &&
bash tools/rocprof_run.sh ${T}_prof > $O/rocprof.log 2>&1 &&
bash tools/pmc_pass.sh ${T}_pmc > $O/pmc.log 2>&1
echo "rc=$?"
