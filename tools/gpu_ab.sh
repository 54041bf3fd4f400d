#!/bin/bash
# same-box A/B of the step kernel: libkura_base.so (before) vs libkura.so (after), alternating, + parity subset
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-ab}
mkdir -p $O
cd $R
L=$R/dbs-gym_amd/csrc
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_quick.log 2>&1 &&
for i in 1 2; do
  KURA_LIB=$L/libkura_base.so timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/base_$i.json 2> $O/base_$i.err &&
  timeout -k 10 200 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 0 > $O/new_$i.json 2> $O/new_$i.err || exit 1
done
echo "rc=$?"
