# Round 3: first run of the one-wave-per-SIMD kernels (K1w/K2w): GPU suite,
# smoke, bench (K1w) and the K1 A/B on the same box.
set -e
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $O/bench_k1w.json 2> $O/bench_k1w.err
KURA_KERNEL=k1 timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $O/bench_k1.json 2> $O/bench_k1.err
python3 -c "
import json
for k in ('k1w','k1'):
    d=json.loads(open('$O/bench_'+k+'.json').read().strip().splitlines()[-1]); print(k, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'], d['extra'].get('reset_ms'))
"
