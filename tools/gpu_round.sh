# One gpurun call: GPU test suite, smoke, headline bench, then optional
# diagnostics.  Usage (via gpurun): bash tools/gpu_round.sh <tag> [diag] [prof]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
cat $O/bench.json
if [ "$2" = "diag" ]; then bash tools/diag_r02a.sh $TAG/diag; fi
if [ "$3" = "prof" ]; then bash tools/rocprof_run.sh $TAG/prof; fi
echo ALLDONE
