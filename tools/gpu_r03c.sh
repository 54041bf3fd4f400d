# Round 3: K1w first-difference probes vs the oracle, then the GPU suite and
# the K1w / K1 benches on the same box.
set -e
O=gpurun_out/r03c; mkdir -p $O; : > $O/probe.txt
for cfg in "env0 256 16 2 rand" "env0 1024 16 2 rand" "env1 1024 19 2 rand"; do
  echo "== $cfg" >> $O/probe.txt
  timeout -k 10 120 python3 -u tools/parity_probe.py $cfg >> $O/probe.txt 2>&1
done
grep -v amdgpu.ids $O/probe.txt
if grep -q "differs\|False" $O/probe.txt; then exit 1; fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || true
grep -E "FAILED|passed|failed" $O/gpu_tests.log | tail -30
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $O/bench_k1w.json 2> $O/bench_k1w.err
KURA_KERNEL=k1 timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $O/bench_k1.json 2> $O/bench_k1.err
python3 -c "
import json
for k in ('k1w','k1'):
    d=json.loads(open('$O/bench_'+k+'.json').read().strip().splitlines()[-1]); print(k, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel'], d['extra'].get('reset_ms'))
"
