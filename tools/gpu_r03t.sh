# FSAL by slot renaming: headline/reset A/B against the current build (base),
# then the whole GPU suite (and the KURA_DEBUG build) with the renaming build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r03t; mkdir -p $O; C=dbs-gym_amd/csrc
bash tools/gpu_multi_ab.sh r03t libkura_base.so libkura_fsal.so libkura_base.so libkura_fsal.so > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
cp $C/libkura_fsal.so $C/libkura.so && cp $C/libkura_debug_fsal.so $C/libkura_debug.so &&
PART=256 timeout -k 10 200 python3 -u tools/parity_probe.py env0 2048 19 3 rand > $O/probe_xl.txt 2>&1 && grep -c "all equal" $O/probe_xl.txt &&
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
exit $rc
