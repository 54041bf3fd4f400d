import json, sys
d0 = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/qp"
for f in ("stamps_reset.json", "stamps_step.json"):
    try:
        d = json.load(open(f"{d0}/{f}"))
    except Exception as e:
        print(f, e); continue
    print(d["mode"], round(d["ms_per_launch"], 2))
    pw = d["per_wave"]
    for k in pw:
        print("   %-14s %12d %12d" % (k, sum(pw[k][:4]) / 4, sum(pw[k][4:]) / 4))
b = json.load(open(f"{d0}/bench.json"))
print("bench", round(b["value"]), "ms", round(b["ms_per_step"], 3), "frac", round(b["roofline"]["frac"], 4), "reset_ms", round(b["extra"]["reset_ms"], 1))
