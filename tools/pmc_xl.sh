# HBM/L2 counters of the split-group stress step (N=8192, 128 envs, parts of 256), via gpurun
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_xl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --osc 8192 --envs 128"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/b1.json 2> $O/f.err
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2 -o run -- $B > $O/b2.json 2> $O/l.err
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $B > $O/b3.json 2> $O/t.err
echo DONE
