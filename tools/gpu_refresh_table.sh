# One bench line per BASELINE config, the stress config in both forms and the
# episode-inclusive rate, for the current build (via gpurun):
#   bash tools/gpu_refresh_table.sh <tag>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-tab}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0"
$B > $O/env0_r1.json 2> $O/env0_r1.err
$B --coupling f32 > $O/env0_r1_f32.json 2> $O/env0_r1_f32.err
$B --config env1 > $O/env1_r1.json 2> $O/env1_r1.err
$B --config env1 --reward temp_const_action > $O/env1_r2.json 2> $O/env1_r2.err
$B --config env0 --reward bbpow_threth_action > $O/env0_r3.json 2> $O/env0_r3.err
$B --config env2 --random-k > $O/env2_rk.json 2> $O/env2_rk.err
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --osc 8192 --envs 1024 > $O/stress_weak.json 2> $O/stress_weak.err
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --osc 8192 --envs 128 > $O/stress_strong.json 2> $O/stress_strong.err
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --episode > $O/episode.json 2> $O/episode.err
for f in env0_r1 env0_r1_f32 env1_r1 env1_r2 env0_r3 env2_rk stress_weak stress_strong episode; do
  python -c "import json;d=json.loads(open('$O/$f.json').readline());print('$f', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['frac'],4), d['dtype'], d.get('extra',{}).get('episode',{}).get('episode_vs_steady'))"
done
echo ALLDONE
