#!/usr/bin/env python3
"""Transcribe the paper's DBS-OFF / HF-DBS rows from the reference's
data/kur-table-metrics.xlsx (sheet "Experiment_for_paper", rows 4-5) into
tests/golden/paper_anchors.json.  Run in the build container only:

    python tests/golden/make_paper_anchors.py /root/reference

openpyxl is not installed; an .xlsx is a zip of XML parts, read here with the
standard library (shared strings + sheet1 cells).  Only the numbers are
written."""
import json
import os
import re
import sys
import xml.etree.ElementTree as ET
import zipfile

HERE = os.path.dirname(os.path.abspath(__file__))
NS = {"m": "http://schemas.openxmlformats.org/spreadsheetml/2006/main"}


def cells(path):
    z = zipfile.ZipFile(path)
    ss = ["".join(t.text or "" for t in si.iter("{%s}t" % NS["m"]))
          for si in ET.fromstring(z.read("xl/sharedStrings.xml")).findall("m:si", NS)]
    sheets = ET.fromstring(z.read("xl/workbook.xml")).find("m:sheets", NS)
    assert sheets[0].get("name") == "Experiment_for_paper"
    out = {}
    for row in ET.fromstring(z.read("xl/worksheets/sheet1.xml")).find("m:sheetData", NS):
        for c in row:
            v = c.find("m:v", NS)
            if v is None:
                continue
            out[c.get("r")] = ss[int(v.text)] if c.get("t") == "s" else v.text
    return out


def mean_sd(s):
    m = re.fullmatch(r"\s*([0-9.]+)\s*\(([0-9.]+)\)\s*", s)
    return float(m.group(1)), float(m.group(2))


def main(ref):
    c = cells(os.path.join(ref, "data", "kur-table-metrics.xlsx"))
    # bbpow columns of Reward #1 per env: B (env0), H (env1), N (env2); energy C, I, O
    cols = {"env0": ("B", "C"), "env1": ("H", "I"), "env2": ("N", "O")}
    assert c["A4"] == "DBS OFF" and c["A5"] == "HF-DBS", (c["A4"], c["A5"])
    out = {"source": "data/kur-table-metrics.xlsx, sheet Experiment_for_paper, rows 4 (DBS OFF) and 5 (HF-DBS); "
                     "beta-band power x1e-3 as mean (sd) over the 5 eval envs; energy = sum |a| per env",
           "anchors": {}}
    for env, (cb, ce) in cols.items():
        off, hf = mean_sd(c[cb + "4"]), mean_sd(c[cb + "5"])
        out["anchors"][env] = {"off": {"mean": off[0] * 1e-3, "sd": off[1] * 1e-3, "energy": float(c[ce + "4"])},
                               "hf": {"mean": hf[0] * 1e-3, "sd": hf[1] * 1e-3,
                                      "energy": mean_sd(c[ce + "5"])[0]}}
    path = os.path.join(HERE, "paper_anchors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
