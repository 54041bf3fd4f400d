#!/bin/bash
# Board power and clocks under a long steady bench (run on the GPU box via
# gpurun): amd-smi samples once a second while bench.py steps (read-only
# queries; the GPU settings are not touched).  Is the step bound by the
# board's power limit?  bash tools/power_probe.sh <outdir> [bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-power}; shift
mkdir -p $O
cd $R
timeout -k 5 20 amd-smi static --limit --json > $O/limits.json 2> $O/limits.err || true
timeout -k 5 20 amd-smi metric --power --clock --temperature --json > $O/idle.json 2> $O/idle.err || true
timeout -k 10 240 python3 bench.py --cpu-seconds 0 "$@" > $O/bench.json 2> $O/bench.err &
pid=$!
sleep 8   # past the import, setup and reset
for i in $(seq 1 12); do
  kill -0 $pid 2>/dev/null || break
  timeout -k 5 10 amd-smi metric --power --clock --temperature --json >> $O/samples.jsonl 2>> $O/samples.err || true
  echo "sample $i"
  sleep 1
done
wait $pid
echo "bench rc=$?"
