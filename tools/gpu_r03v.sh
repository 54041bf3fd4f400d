# epilogue omega/pulse loads issued before the GEMM (KURA_EPI_PREFETCH): A/B against the current build
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash tools/gpu_multi_ab.sh r03v libkura_base.so libkura_epi.so libkura_base.so libkura_epi.so libkura.so
