# stamps (reset + step), bench, parity subset -- one gpurun call
#   bash tools/quick_perf.sh <outdir-name>
set -e
O=gpurun_out/${1:-qp}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_split.py tests/test_vec_env_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || (tail -30 $O/tests.log; exit 1)
tail -2 $O/tests.log
MODE=reset timeout -k 10 200 python3 -u tools/phase_stamps.py > $O/stamps_reset.json 2>/dev/null
timeout -k 10 200 python3 -u tools/phase_stamps.py > $O/stamps_step.json 2>/dev/null
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 > $O/bench.json 2>$O/bench.err
python3 tools/show_qp.py $O
