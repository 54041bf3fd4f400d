# deferred split-group LFP totals: split + debug-build GPU tests, then the
# split-group A/B against the previous build (ring 8)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r03q; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_split.py tests/test_debug_build.py -v --timeout 150 --timeout-method thread > $O/split_tests.log 2>&1; rc=$?
tail -3 $O/split_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_xl_ab.sh r03q_ab libkura.so libkura_ring8.so libkura.so
