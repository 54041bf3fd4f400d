# phase stamps of the split-group step at N=8192: 1024 envs (parts of 1024)
# and 128 envs (auto parts of 256) -- via gpurun
set -e
O=gpurun_out/stamps_xl; mkdir -p $O
OSC=8192 ENVS=1024 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/xl_1024.json 2>$O/xl_1024.err
OSC=8192 ENVS=128 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/xl_128.json 2>$O/xl_128.err
python3 - <<'PY'
import json
for B in (1024, 128):
    d=json.load(open(f"gpurun_out/stamps_xl/xl_{B}.json"))
    pw=d["per_wave"]
    tot=sum(sum(v[4:])/4 for v in pw.values())
    print(B, round(d["ms_per_launch"],2), 'total', round(tot/1e6,2), {k: round(sum(v[4:])/4/1e6,3) for k,v in pw.items() if sum(v[4:])/4 > 0.01*tot})
PY
