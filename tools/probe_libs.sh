# first-difference probe of several library builds on one configuration (via gpurun):
#   bash tools/probe_libs.sh "ENV N B STEPS ACT" lib1.so lib2.so ...
set -e
O=gpurun_out/probe_libs; mkdir -p $O; : > $O/p.txt
cfg=$1; shift
for lib in "$@"; do
  echo "== $lib $cfg" >> $O/p.txt
  timeout -k 10 150 python3 -u tools/parity_probe.py $cfg $PWD/dbs-gym_amd/csrc/$lib >> $O/p.txt 2>&1
done
grep -v amdgpu.ids $O/p.txt
