# round-2 evidence: rocprof trace/PMC/clock of the headline bench, then one
# bench line per BASELINE config (via gpurun): bash tools/gpu_configs_bench.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cfg}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/rocprof_run.sh $TAG/prof
B="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0"
$B --config env1 > $O/env1_r1.json 2> $O/env1_r1.err
$B --config env1 --reward temp_const_action > $O/env1_r2.json 2> $O/env1_r2.err
$B --config env0 --reward bbpow_threth_action > $O/env0_r3.json 2> $O/env0_r3.err
$B --config env2 --random-k > $O/env2_rk.json 2> $O/env2_rk.err
for f in env1_r1 env1_r2 env0_r3 env2_rk; do
  python -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['frac'],4))"
done
echo ALLDONE
