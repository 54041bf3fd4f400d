# wave-parallel control loops (step size / any-active, save rounds / FSAL mode): A/B against the current build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/gpu_multi_ab.sh r03u libkura_base.so libkura_par.so libkura_base.so libkura_par.so libkura_base.so libkura_par.so
