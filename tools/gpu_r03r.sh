# save-pass half-tile prefetch: headline/reset A/B against the previous build
# (sv0), a split-group probe + strong line, then the whole GPU suite
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r03r; mkdir -p $O
bash tools/gpu_multi_ab.sh r03r libkura_sv0.so libkura.so libkura_sv0.so libkura.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
bash tools/gpu_xl_ab.sh r03r_xl libkura.so > $O/xl.txt 2>&1 || { cat $O/xl.txt; exit 1; }
cat $O/xl.txt
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
exit $rc
