# save-pass half-tile prefetch: headline/reset A/B against the previous build (sv0)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/gpu_multi_ab.sh r03s libkura_sv0.so libkura.so libkura_sv0.so libkura.so
