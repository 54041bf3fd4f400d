# OFF solve keeps the ON solve omega record (KURA_OFF_KEEPS_W): A/B against the current build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/gpu_multi_ab.sh r03w libkura_base.so libkura_offw.so libkura_base.so libkura_offw.so libkura.so
