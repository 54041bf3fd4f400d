# rocprofv3 evidence for the bench kernel (run on the GPU box via gpurun):
#   bash tools/rocprof_run.sh <outname>
# 1) kernel trace + stats of a short bench run (average kernel duration must
#    agree with bench.py's HIP-event figure);
# 2) FETCH_SIZE and 3) WRITE_SIZE in separate --pmc passes (MI355X guide: the
#    two do not fit one TCC pass; FETCH_SIZE is doubled for 16 B/lane loads);
# 4) GRBM_GUI_ACTIVE: effective shader clock under the kernel (MI355X guide,
#    'DVFS give-back': GRBM_GUI_ACTIVE / 8 XCDs / dispatch time).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --steps 60 --warmup 3 --cpu-seconds 0 > $O/bench_trace.json 2> $O/trace.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_fetch.json 2> $O/fetch.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_write.json 2> $O/write.err
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/clock -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_clock.json 2> $O/clock.err
echo DONE
