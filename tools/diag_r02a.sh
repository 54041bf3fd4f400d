# round-2 diagnostics (run via gpurun): phase stamps of reset and step, L2
# hit/miss pass of the bench.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-diag_a}
mkdir -p $O
cd $R
MODE=reset timeout -k 10 200 python3 -u tools/phase_stamps.py > $O/stamps_reset.json 2> $O/stamps_reset.err
timeout -k 10 200 python3 -u tools/phase_stamps.py > $O/stamps_step.json 2> $O/stamps_step.err
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/l2 -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_l2.json 2> $O/l2.err
echo DONE
