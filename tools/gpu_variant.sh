# A/B of the production library against one variant build, one gpurun call:
#   bash tools/gpu_variant.sh <tag> <variant.so> ["ENV N B STEPS ACT" probe config]
# 1) first-difference probe of both builds, 2) GPU suite + bench of the
# production build, 3) the same with the variant copied over libkura.so (the
# box's tree is a scratch copy).  A test failure (pytest rc 1) does not stop
# the script; a crash, abort or time limit does.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}; VAR=$2; CFG=${3:-"env1 1024 19 3 rand"}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
C=dbs-gym_amd/csrc
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
for lib in libkura.so $VAR; do
  echo "== $lib $CFG" >> $O/probe.txt
  timeout -k 10 150 python3 -u tools/parity_probe.py $CFG $R/$C/$lib >> $O/probe.txt 2>&1; rc=$?
  ok $rc || { echo "probe rc=$rc"; exit $rc; }
done
grep -v amdgpu.ids $O/probe.txt
cp $C/libkura.so $O/../libkura_prod_backup.so 2>/dev/null
for v in prod var; do
  if [ $v = var ]; then cp $C/$VAR $C/libkura.so; fi
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?
  tail -3 $O/tests_$v.log
  ok $rc || { echo "tests rc=$rc"; exit $rc; }
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_$v.json 2> $O/bench_$v.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
  python3 -c "import json;d=json.loads(open('$O/bench_$v.json').readline());print('$v',d['value'],d['ms_per_step'],d['roofline']['frac'])"
done
rm -f $O/../libkura_prod_backup.so
echo ALLDONE
