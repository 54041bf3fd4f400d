# instruction-cache counters of the step kernel (via gpurun): does the solver's
# code footprint (~200 KB) thrash the SQC instruction cache?
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmc_ic}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -i -E "icache|ifetch|WAIT_INST|INST_LEVEL|INSTS_VALU\b|SQC_" $O/avail.txt | head -60 > $O/avail_grep.txt || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/ic -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_ic.json 2> $O/ic.err
echo DONE
