set -e
O=gpurun_out/probe_swap2; mkdir -p $O; : > $O/p.txt
for lib in libkura_v1.so; do
for cfg in "env0 1024 16 2 rand"; do
  echo "== $lib $cfg" >> $O/p.txt
  timeout -k 10 120 python3 -u tools/parity_probe.py $cfg $PWD/dbs-gym_amd/csrc/$lib >> $O/p.txt 2>&1
done; done
grep -v amdgpu.ids $O/p.txt
