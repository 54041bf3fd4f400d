# split-group parts (256/512/1024) on the GPU: parity tests, then the stress
# config in its weak (1024 envs/GPU) and strong (128 envs/GPU) forms.
set -e
O=gpurun_out/${1:-split}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for part in 1024 512 256; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --osc 8192 --envs 128 --part-osc $part > $O/stress128_p$part.json 2> $O/stress128_p$part.err
  python -c "import json;d=json.load(open('$O/stress128_p$part.json'));print($part, d['value'], d['roofline']['frac'], d['extra']['reset_ms'])"
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --osc 8192 --envs 1024 > $O/stress1024.json 2> $O/stress1024.err
python -c "import json;d=json.load(open('$O/stress1024.json'));print('1024 envs', d['value'], d['roofline']['frac'], d['config'])"
