#!/bin/bash
# HEAD refresh on a fresh box (via gpurun): GPU suite, smoke, the default bench,
# the N=8192 stress lines in both arithmetics (AUTO = BF16X3), env1, the SQ/SQC/TA
# counter passes and the phase stamps (prebuilt KURA_STAMPS library).  Each step
# has its own time limit; the first failure ends the script.
set -o pipefail
O=gpurun_out/${1:-r05_refresh}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_stress128.json 2> $O/bench_stress128.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --steps 4 --warmup 2 --cpu-seconds 0 > $O/bench_stress1024.json 2> $O/bench_stress1024.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 128 --coupling f32 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_stress128_f32.json 2> $O/bench_stress128_f32.err &&
timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --coupling f32 --steps 4 --warmup 2 --cpu-seconds 0 > $O/bench_stress1024_f32.json 2> $O/bench_stress1024_f32.err &&
timeout -k 10 300 python3 bench.py --config env1 --reward temp_const_action --steps 20 --warmup 3 --cpu-seconds 0 > $O/bench_env1.json 2> $O/bench_env1.err &&
tail -2 $O/gpu_tests.log &&
bash tools/pmc_pass.sh ${1:-r05_refresh}_pmc > $O/pmc.log 2>&1 &&
timeout -k 10 300 python3 tools/phase_stamps.py > $O/stamps_step.json 2> $O/stamps_step.err
echo "rc=$?"
