set -e
O=gpurun_out/stamps_B; mkdir -p $O
for B in 4096 1024 256 64; do
  ENVS=$B timeout -k 10 200 python3 -u tools/phase_stamps.py > $O/step_$B.json 2>/dev/null
done
python3 - <<'PY'
import json
for B in (4096, 1024, 256, 64):
    d=json.load(open(f"gpurun_out/stamps_B/step_{B}.json"))
    pw=d["per_wave"]
    print(B, round(d["ms_per_launch"],3), {k: round(sum(v[4:])/4/1e3) for k,v in pw.items() if k in ("stage_input","gemm","epilogue","post_err","save_loadwait","save_compute","post_fsal","barrier1")})
PY
