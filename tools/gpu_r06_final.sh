#!/bin/bash
# Round-6 final evidence on one box (via gpurun), in parts that fit one call:
#   bash tools/gpu_r06_final.sh <tag> prof    -- N=8192 stress bench lines, rocprofv3 trace + FETCH/WRITE/clock
#                                               of the headline, SQ/TA counter passes, board power, full CPU baseline
#   bash tools/gpu_r06_final.sh <tag> stress  -- rocprofv3 trace + FETCH/WRITE/clock of both N=8192 forms
#                                               (plain launch: profiles/r06_exit_fault_attribution.txt)
# Each step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r06f}; O=$R/gpurun_out/$T
mkdir -p $O
cd $R
case "$2" in
prof)
  timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_stress128.json 2> $O/bench_stress128.err &&
  timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --steps 4 --warmup 2 --cpu-seconds 0 > $O/bench_stress1024.json 2> $O/bench_stress1024.err &&
  bash tools/rocprof_run.sh $T/prof --reset-reps 2 > $O/rocprof.log 2>&1 &&
  bash tools/pmc_pass.sh $T/pmc > $O/pmc.log 2>&1 &&
  bash tools/power_probe.sh $T/power_bf16 --steps 10000 > $O/power.log 2>&1 &&
  timeout -k 10 400 python3 tools/cpu_baseline_full.py > $O/cpu_baseline_full.json 2> $O/cpu_baseline_full.err
  echo "rc=$?";;
stress)
  KURA_XL_LAUNCH=plain TRACE_STEPS=20 bash tools/rocprof_run.sh $T/prof_s128 --osc 8192 --envs 128 > $O/rocprof_s128.log 2>&1 &&
  KURA_XL_LAUNCH=plain TRACE_STEPS=8 bash tools/rocprof_run.sh $T/prof_s1024 --osc 8192 --envs 1024 > $O/rocprof_s1024.log 2>&1
  echo "rc=$?";;
*) echo "usage: $0 <tag> prof|stress"; exit 2;;
esac
