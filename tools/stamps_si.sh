# stage-input sub-phase stamps (KURA_STAMPS_SI build: no record prefetch)
set -e
O=gpurun_out/stamps_si; mkdir -p $O
for B in 64 4096; do
  SI=1 ENVS=$B timeout -k 10 200 python3 -u tools/phase_stamps.py > $O/si_$B.json 2>$O/si_$B.err
done
python3 - <<'PY'
import json
for B in (64, 4096):
    d=json.load(open(f"gpurun_out/stamps_si/si_{B}.json"))
    pw=d["per_wave"]
    print(B, round(d["ms_per_launch"],3), {k: round(sum(v[4:])/4/1e3) for k,v in pw.items() if k in ("stage_input","gemm","si_load","si_compute","si_lds","si_misc","barrier1")})
PY
