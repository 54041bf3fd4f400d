# Split-group (N > 1024) A/B of several library builds on one box (via gpurun):
#   bash tools/gpu_xl_ab.sh <tag> libA.so libB.so ...
# Per build: parity probes vs the oracle (N=2048 parts of 256 and 512,
# N=8192 parts of 256), then the strong-form stress line (N=8192 x 128 envs,
# parts of 256) and the weak-form one (N=8192 x 1024 envs, parts of 1024).
# A probe mismatch skips that build's benches; a crash/abort/time limit ends
# the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R; C=dbs-gym_amd/csrc
cp $C/libkura.so $C/libkura_orig.so
cp $C/libkura.so $C/libkura_prod.so
for lib in "$@"; do
  [ $lib = libkura.so ] && lib=libkura_prod.so
  P=$O/probe_${lib%.so}.txt; : > $P
  for cfg in "256 env0 2048 19 3 rand" "512 env1 2048 19 3 rand" "256 env0 8192 16 2 rand"; do
    set -- $cfg
    PART=$1 timeout -k 10 200 python3 -u tools/parity_probe.py $2 $3 $4 $5 $6 $R/$C/$lib >> $P 2>&1; rc=$?
    [ $rc -eq 0 ] || { echo "$lib probe rc=$rc"; tail -5 $P; exit $rc; }
  done
  n=$(grep -c "all equal" $P)
  if [ "$n" != 3 ]; then echo "$lib MISMATCH ($n/3 equal)"; continue; fi
  [ $lib = libkura.so ] || cp $C/$lib $C/libkura.so
  for mode in "strong --envs 128 --steps 10" "p512 --envs 128 --part-osc 512 --steps 10" "weak --envs 1024 --steps 4"; do
    set -- $mode; m=$1; shift
    timeout -k 10 300 python3 bench.py --osc 8192 "$@" --warmup 2 --cpu-seconds 0 > $O/bench_${lib%.so}_$m.json 2> $O/bench_${lib%.so}_$m.err; rc=$?
    [ $rc -eq 0 ] || { echo "$lib bench $m rc=$rc"; tail -3 $O/bench_${lib%.so}_$m.err; exit $rc; }
    python3 -c "import json;d=json.loads(open('$O/bench_${lib%.so}_$m.json').readline());print('$lib','$m',d['value'],d['ms_per_step'],d['roofline']['frac'])"
  done
done
cp $C/libkura_orig.so $C/libkura.so
echo ALLDONE
