#!/bin/bash
# Exit-fault attribution for rocprofv3-traced split-group runs (VERDICT r05
# next #1): the N=8192 strong form unprofiled with the cooperative launch and
# with KURA_XL_LAUNCH=plain (same kernel, ordinary queue; A/B, 3 rounds), then
# the rocprofv3 trace + PMC passes of both N=8192 forms with the plain launch.
# Stops at the first failing step.   bash tools/gpu_r06_xlprobe.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r06d}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --steps 20 --warmup 2 --cpu-seconds 0 > $O/ab_coop_$r.json 2> $O/ab_coop_$r.err || exit 1
  KURA_XL_LAUNCH=plain timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --steps 20 --warmup 2 --cpu-seconds 0 > $O/ab_plain_$r.json 2> $O/ab_plain_$r.err || exit 1
  echo "round $r: coop $(python3 -c "import json;print(json.load(open('$O/ab_coop_$r.json'))['value'])") plain $(python3 -c "import json;print(json.load(open('$O/ab_plain_$r.json'))['value'])")"
done
KURA_XL_LAUNCH=plain TRACE_STEPS=20 bash tools/rocprof_run.sh $T/prof_strong --osc 8192 --envs 128 > $O/prof_strong.log 2>&1 || { echo "strong rc=$?"; exit 1; }
echo "strong ok"
KURA_XL_LAUNCH=plain TRACE_STEPS=8 bash tools/rocprof_run.sh $T/prof_weak --osc 8192 --envs 1024 > $O/prof_weak.log 2>&1 || { echo "weak rc=$?"; exit 1; }
echo "weak ok"
