# phase stamps of env1 with R1 and with R2 (same build): where the R2 step spends its extra time
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=$R/gpurun_out/r03x; mkdir -p $O
CFG=env1 timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/env1_r1.json 2> $O/env1_r1.err &&
CFG=env1 REWARD=temp_const_action timeout -k 10 300 python3 -u tools/phase_stamps.py > $O/env1_r2.json 2> $O/env1_r2.err &&
python3 - <<'PY'
import json
a=json.load(open("gpurun_out/r03x/env1_r1.json")); b=json.load(open("gpurun_out/r03x/env1_r2.json"))
print("ms", a["ms_per_launch"], b["ms_per_launch"])
for k in a["cycles_per_step_per_wave"]:
    x, y = a["cycles_per_step_per_wave"][k], b["cycles_per_step_per_wave"][k]
    if max(x, y) > 20000: print(k, x, y, y - x)
PY
