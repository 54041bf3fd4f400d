# Same-box bench A/B of library builds (bench only, alternating):
#   bash tools/gpu_ab_bench.sh <tag> libA.so libB.so [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; A=$2; B=$3; N=${4:-2}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R; C=dbs-gym_amd/csrc
cp $C/libkura.so $C/libkura_orig.so
for i in $(seq 1 $N); do
  for lib in $A $B; do
    cp $C/$lib $C/libkura.so
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/bench_${lib%.so}_$i.json 2> $O/bench_${lib%.so}_$i.err; rc=$?
    [ $rc -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
    python3 -c "import json;d=json.loads(open('$O/bench_${lib%.so}_$i.json').readline());print('$lib',$i,d['value'],d['ms_per_step'],d['roofline']['avg_kernel_ms'])"
  done
done
cp $C/libkura_orig.so $C/libkura.so
echo ALLDONE
