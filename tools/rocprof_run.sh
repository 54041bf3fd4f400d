# rocprofv3 evidence for a bench workload (run on the GPU box via gpurun):
#   bash tools/rocprof_run.sh <outname> [bench args ...]
# (no bench args = the headline workload, BASELINE configs[1]; e.g.
#  `--osc 8192 --envs 128` = the strong form of configs[4])
# 1) kernel trace + stats of a short bench run (average kernel duration must
#    agree with bench.py's HIP-event figure);
# 2) FETCH_SIZE and 3) WRITE_SIZE in separate --pmc passes (MI355X guide: the
#    two do not fit one TCC pass; FETCH_SIZE is doubled for 16 B/lane loads);
# 4) GRBM_GUI_ACTIVE: effective shader clock under the kernel (MI355X guide,
#    'DVFS give-back': GRBM_GUI_ACTIVE / 8 XCDs / dispatch time).
# TRACE_STEPS (default 60) timed steps in the traced run; 3 in each PMC pass.
# Every profiled process dumps /proc/self/maps at exit (bench.py
# KURA_EXIT_MAPS) so an exit-time fault can be attributed to a library.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof}
shift || true
TS=${TRACE_STEPS:-60}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ulimit -c 0
KURA_EXIT_MAPS=$O/maps_trace.txt timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --steps $TS --warmup 3 --cpu-seconds 0 "$@" > $O/bench_trace.json 2> $O/trace.err
KURA_EXIT_MAPS=$O/maps_fetch.txt timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > $O/bench_fetch.json 2> $O/fetch.err
KURA_EXIT_MAPS=$O/maps_write.txt timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > $O/bench_write.json 2> $O/write.err
KURA_EXIT_MAPS=$O/maps_clock.txt timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/clock -o run -- \
    python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > $O/bench_clock.json 2> $O/clock.err
echo DONE
