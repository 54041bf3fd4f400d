# Round 3: the store-data hazard, tested.  Same source, two builds that differ
# only in the record stores' offset form: SGPR soffset (LLVM inserts no wait
# states after such MUBUF stores) vs VGPR offset + soffset 0 (LLVM guards the
# store-data hazard).  Record-level K1 vs K1w comparison and oracle probes.
set -e
O=gpurun_out/r03e; mkdir -p $O; : > $O/probe.txt
for lib in libkura_sgprsoff.so libkura.so; do
  echo "##### $lib" >> $O/probe.txt
  LIB=$lib timeout -k 10 200 python3 -u tools/record_probe.py env0 1024 16 4 >> $O/probe.txt 2>&1 || true
  for cfg in "env0 256 16 2 rand" "env0 1024 16 2 rand" "env1 1024 19 2 rand"; do
    echo "== $cfg" >> $O/probe.txt
    timeout -k 10 120 python3 -u tools/parity_probe.py $cfg $PWD/dbs-gym_amd/csrc/$lib >> $O/probe.txt 2>&1 || true
  done
done
grep -v amdgpu.ids $O/probe.txt
