# Round 3: record-level localisation of the K1w env-slot divergence.
set -e
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python3 -u tools/record_probe.py env0 1024 16 8 > $O/record_probe.txt 2>&1 || true
grep -v amdgpu.ids $O/record_probe.txt
