#!/bin/bash
# One parameterised GPU session (run through gpurun): GPU tests, then
# same-box A/B benches of several trees, alternating, each step under its own
# time limit; the first failing step ends the script.
#   bash tools/gpu_session.sh TAG TESTS BENCHSETS TREE...
#     TESTS      "all" (tests -m gpu), "none", or pytest node ids/files
#     BENCHSETS  ';'-separated bench.py argument lists ("" = default line)
#     TREE       "." (this tree) or a directory holding another tree (ab/r3)
# Output: gpurun_out/TAG/{tests.log, bench_<tree>_<set>_<round>.json, summary.txt}
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TESTS=$2; SETS=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "$TESTS" != "none" ]; then
  [ "$TESTS" = "all" ] && TESTS="tests"
  timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit $rc; }
fi
IFS=';' read -ra SETV <<< "$SETS"
for round in $(seq 1 ${ROUNDS:-2}); do
  for tree in "$@"; do
    # "lib:<path>": this tree with another build of libkura (KURA_LIB)
    lib=""; t=$tree
    case $tree in lib:*) lib=${tree#lib:}; t=.;; esac
    tn=$(basename $(cd $t && pwd)); [ "$t" = "." ] && tn=head
    [ -n "$lib" ] && tn=$(basename $lib .so)
    si=0
    for set in "${SETV[@]}"; do
      f=$O/bench_${tn}_${si}_${round}.json
      (cd $t && KURA_LIB=${lib:+$R/$lib} timeout -k 10 300 python3 bench.py $set --cpu-seconds 0 > $f 2> ${f%.json}.err) || { echo "bench $tn [$set] failed"; exit 1; }
      python3 -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);print('$tn','[$set]','r$round',round(d['value']),round(d['ms_per_step'],4),round(d['roofline']['frac'],4),round(d['roofline']['avg_kernel_ms'],4),round(d['extra'].get('reset_ms_warm') or d['extra'].get('reset_ms',0),1))" | tee -a $O/summary.txt
      si=$((si+1))
    done
  done
done
echo ALLDONE
