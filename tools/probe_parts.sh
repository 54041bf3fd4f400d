set -e
O=gpurun_out/probe_parts3; mkdir -p $O; : > $O/p.txt
for lib in libkura.so; do
  echo "== $lib part 256 env0 2048 16 3 off" >> $O/p.txt
  PART=256 timeout -k 10 120 python3 -u tools/parity_probe.py env0 2048 16 3 off $PWD/dbs-gym_amd/csrc/$lib >> $O/p.txt 2>&1
done
grep -v amdgpu.ids $O/p.txt
