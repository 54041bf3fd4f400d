#!/bin/bash
# Round-6 first box: GPU suite + headline bench of the rebuilt tree, then the
# rocprofv3 trace + FETCH/WRITE/clock passes of both N=8192 forms (BASELINE
# configs[4]) with /proc/self/maps dumped at exit (exit-fault attribution).
#   [TESTS='tests/a.py tests/b.py'] bash tools/gpu_r06a.sh <tag> [noprof|notests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r06a}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ "$2" != "notests" ]; then
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
fi
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cat $O/bench_default.json
[ "$2" = "noprof" ] && exit 0
TRACE_STEPS=8 bash tools/rocprof_run.sh ${T}/prof_weak --osc 8192 --envs 1024 > $O/prof_weak.log 2>&1 || { echo "weak rc=$?"; exit 1; }
echo "weak ok"
TRACE_STEPS=20 bash tools/rocprof_run.sh ${T}/prof_strong --osc 8192 --envs 128 > $O/prof_strong.log 2>&1
echo "strong rc=$?"
