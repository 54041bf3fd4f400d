# split-group phase stamps (chunk-barrier slot), then the headline A/B of the
# main-GEMM ring variants (KURA_G_RING=2/4 with the A fragment one block ahead)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/stamps_xl.sh > gpurun_out/stamps_xl.txt 2>&1 || { echo "stamps rc=$?"; exit 1; }
cat gpurun_out/stamps_xl.txt
bash tools/gpu_multi_ab.sh r03p libkura.so libkura_g2.so libkura_g4.so libkura.so
