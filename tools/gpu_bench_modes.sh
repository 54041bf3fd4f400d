# bench.py modes on one GPU (via gpurun): default line (with the CPU baseline),
# episode-inclusive run, strong-scaling stress form (N=8192, 1024 global envs).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-modes}
mkdir -p $O
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err
cat $O/bench_default.json
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --episode > $O/bench_episode.json 2> $O/bench_episode.err
cat $O/bench_episode.json
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --episode --episode-steps 1111 --episode-metrics > $O/bench_episode_metrics.json 2> $O/bench_episode_metrics.err
cat $O/bench_episode_metrics.json
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --cpu-seconds 0 --osc 8192 --global-envs 1024 > $O/bench_stress_strong.json 2> $O/bench_stress_strong.err
cat $O/bench_stress_strong.json
echo ALLDONE
