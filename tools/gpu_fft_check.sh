set -e
O=gpurun_out/fft1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eval_metric.py tests/test_sb3_adapter.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/metric_bench.py 512 105545 > $O/mb512.json 2>&1; cat $O/mb512.json
timeout -k 10 300 python tools/metric_bench.py 4096 105545 > $O/mb4096.json 2>&1; cat $O/mb4096.json
