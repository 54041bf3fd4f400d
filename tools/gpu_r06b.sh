#!/bin/bash
# Round-6 box: HEAD validation (GPU suite, smoke, default bench line) and then
# the same-box A/B of prebuilt libraries (KURA_LIB): parity tests of each
# candidate first, then alternating benches (step + warm reset).
#   bash tools/gpu_r06b.sh <tag> <base.so> "<cand.so> [cand2.so ...]" [benchsets]
# (SKIP_HEAD=1 skips the HEAD validation; ROUNDS=n A/B rounds, default 2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r06b}; BASE=$2; CANDS=$3
SETS=${4:-"--reset-reps 3"}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
if [ -z "$SKIP_HEAD" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
fi
LIBS="lib:$BASE"
for CAND in $CANDS; do
  n=$(basename $CAND .so)
  KURA_LIB=$R/$CAND timeout -k 10 900 python3 -u -m pytest ${CAND_TESTS:-tests/test_gpu_parity.py tests/test_gpu_gates.py tests/test_gpu_transient.py tests/test_gpu_configs.py} -m gpu -v --timeout 200 --timeout-method thread > $O/cand_tests_$n.log 2>&1 || { tail -30 $O/cand_tests_$n.log; exit 1; }
  tail -1 $O/cand_tests_$n.log
  LIBS="$LIBS lib:$CAND"
done
bash tools/gpu_session.sh $T/ab none "$SETS" $LIBS || exit 1
cat $O/ab/summary.txt
