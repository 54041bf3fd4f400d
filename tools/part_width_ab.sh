set -o pipefail
O=gpurun_out/r05_parts; mkdir -p $O
for p in 1024 512 256; do
  timeout -k 10 300 python3 bench.py --osc 8192 --envs 1024 --part-osc $p --steps 4 --warmup 2 --cpu-seconds 0 > $O/w_$p.json 2> $O/w_$p.err || exit 1
done
for p in 1024 512; do
  timeout -k 10 300 python3 bench.py --osc 8192 --envs 2048 --part-osc $p --steps 3 --warmup 1 --cpu-seconds 0 > $O/w2048_$p.json 2> $O/w2048_$p.err || exit 1
done
echo rc=0
