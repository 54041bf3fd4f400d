# env1/R2: serial filter load blocks of 16 (production) vs 32 / 64 samples (KURA_R2_BLK)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r03y; mkdir -p $O; C=dbs-gym_amd/csrc
cp $C/libkura.so $C/libkura_orig.so
for lib in libkura_base.so libkura_b32.so libkura_b64.so libkura_base.so libkura_b32.so libkura_b64.so; do
  timeout -k 10 150 python3 -u tools/parity_probe.py env1 1024 19 3 rand $R/$C/$lib > $O/probe_${lib%.so}.txt 2>&1 || exit 1
  grep -q "all equal" $O/probe_${lib%.so}.txt || { echo "$lib MISMATCH"; continue; }
  cp $C/$lib $C/libkura.so
  timeout -k 10 300 python3 bench.py --config env1 --reward temp_const_action --steps 10 --warmup 3 --cpu-seconds 0 > $O/bench_${lib%.so}.json 2> $O/bench_${lib%.so}.err || exit 1
  python3 -c "import json;d=json.loads(open('$O/bench_${lib%.so}.json').readline());print('$lib',round(d['value']),round(d['ms_per_step'],4),round(d['roofline']['frac'],4))"
done
cp $C/libkura_orig.so $C/libkura.so
echo ALLDONE
