# Parity probe + bench of several library builds on one box (via gpurun):
#   bash tools/gpu_multi_ab.sh <tag> libA.so libB.so ...
# Each build is probed against the oracle first; a probe mismatch skips its
# bench.  A crash/abort/time limit ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R; C=dbs-gym_amd/csrc
cp $C/libkura.so $C/libkura_orig.so
for lib in "$@"; do
  timeout -k 10 150 python3 -u tools/parity_probe.py env1 1024 19 3 rand $R/$C/$lib > $O/probe_${lib%.so}.txt 2>&1; rc=$?
  [ $rc -eq 0 ] || { echo "$lib probe rc=$rc"; cat $O/probe_${lib%.so}.txt | tail -5; exit $rc; }
  if ! grep -q "all equal" $O/probe_${lib%.so}.txt; then echo "$lib MISMATCH"; continue; fi
  # (libkura.so itself: the production build saved above, not whatever was copied over it last)
  if [ $lib = libkura.so ]; then cp $C/libkura_orig.so $C/libkura.so; else cp $C/$lib $C/libkura.so; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_${lib%.so}.json 2> $O/bench_${lib%.so}.err; rc=$?
  [ $rc -eq 0 ] || { echo "$lib bench rc=$rc"; exit $rc; }
  python3 -c "import json;d=json.loads(open('$O/bench_${lib%.so}.json').readline());print('$lib',d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms'],d['extra']['reset_ms'])"
done
cp $C/libkura_orig.so $C/libkura.so
echo ALLDONE
