# Round 3: full GPU suite on the K1w build, bench K1w vs K1 (same box), rocprofv3
# evidence of the K1w headline (trace of 60 launches, FETCH/WRITE/GRBM passes).
set -e
O=gpurun_out/r03f; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || true
grep -E "FAILED|passed|failed" $O/gpu_tests.log | tail -20
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $O/bench_k1w.json 2> $O/bench_k1w.err
KURA_KERNEL=k1 timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $O/bench_k1.json 2> $O/bench_k1.err
python3 -c "
import json
for k in ('k1w','k1'):
    d=json.loads(open('$O/bench_'+k+'.json').read().strip().splitlines()[-1]); print(k, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'], d['extra'].get('reset_ms'))
"
bash tools/rocprof_run.sh r03f_prof > $O/rocprof.log 2>&1
tail -2 $O/rocprof.log
