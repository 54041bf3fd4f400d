# GPU vs oracle first-difference probe over a few configurations (via gpurun):
#   bash tools/probe_parts.sh "PART ENV N B STEPS ACT" ...   (PART 0 = default)
set -e
O=gpurun_out/probe; mkdir -p $O; : > $O/p.txt
for cfg in "$@"; do
  set -- $cfg
  echo "== part=$1 $2 N=$3 B=$4 steps=$5 act=$6" >> $O/p.txt
  PART=$1 timeout -k 10 120 python3 -u tools/parity_probe.py $2 $3 $4 $5 $6 >> $O/p.txt 2>&1
done
grep -v amdgpu.ids $O/p.txt
