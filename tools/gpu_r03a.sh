# Round 3, first GPU call: baseline of the round-2 kernel on this round's box
# (GPU suite, bench) + the bit-select variant's reset state for the offline
# codegen investigation (tools/locate_rows.py).
set -e
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 150 python3 -u tools/dump_reset.py env1 1024 19 libkura.so libkura_bitsel.so > $O/dump.log 2>&1
mv gpurun_out/dump_*.npz $O/
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 > $O/bench.json 2> $O/bench.err
tail -3 $O/gpu_tests.log; cat $O/bench.json
