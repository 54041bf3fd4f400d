#!/bin/bash
# rocprofv3 kernel trace + stats of the N=8192 stress config (BASELINE configs[4])
# in the default coupling (AUTO = BF16X3): strong form (128 envs, parts of 256)
# and weak form (1024 envs, parts of 1024).  bash tools/rocprof_stress.sh <outname>
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof_stress}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/strong -o run -- \
    python3 $R/bench.py --osc 8192 --envs 128 --steps 20 --warmup 2 --cpu-seconds 0 > $O/bench_strong.json 2> $O/strong.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/weak -o run -- \
    python3 $R/bench.py --osc 8192 --envs 1024 --steps 6 --warmup 2 --cpu-seconds 0 > $O/bench_weak.json 2> $O/weak.err
echo DONE
