#!/bin/bash
# Whole-episode benches: env2 (drift events, per-env K,
# its resets' host draws) and env0 for comparison, 4096 envs per GPU, one
# 5555-step episode through KuraVectorEnv each, autoreset at its end.
#   bash tools/gpu_episode.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-episode}
mkdir -p $O
cd $R
timeout -k 10 400 python3 bench.py --config env2 --random-k --episode --steps 10 --warmup 2 --cpu-seconds 0 > $O/env2_episode.json 2> $O/env2_episode.err || exit 1
timeout -k 10 400 python3 bench.py --config env0 --episode --steps 10 --warmup 2 --cpu-seconds 0 > $O/env0_episode.json 2> $O/env0_episode.err || exit 1
for f in env2 env0; do python3 -c "import json;d=json.load(open('$O/${f}_episode.json'));e=d['extra']['episode'];print('$f',round(d['value']),round(e['value']),round(e['episode_vs_steady'],4),e['boundary'],round(e['boundary_frac'] or 0,4))"; done
