"""Per-dtype clock and MFMA busy of the fused stem from tools/dtype_clock.sh.

    python tools/dtype_clock.py gpurun_out/dtype_clock
"""
import csv
import json
import sys
from pathlib import Path

root = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dtype_clock")
res = {}
for dt in ("bf16", "fp16"):
    d = root / dt
    cc = list(csv.DictReader(open(d / "run_counter_collection.csv")))
    per = {}
    for r in cc:
        if "stem224_fused" not in r["Kernel_Name"]:
            continue
        e = per.setdefault(r["Dispatch_Id"], {})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
        e["_dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows = []
    for did, m in per.items():
        if "GRBM_GUI_ACTIVE" not in m or m["_dur"] <= 0:
            continue
        dur = m["_dur"]
        cyc = m["GRBM_GUI_ACTIVE"] / 8
        rows.append((dur, cyc / dur, m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * cyc)))
    n = len(rows)
    res[dt] = {"dispatches": n, "mean_us": round(sum(r[0] for r in rows) / n / 1e3, 2),
               "clock_ghz": round(sum(r[1] for r in rows) / n, 3), "mfma_busy": round(sum(r[2] for r in rows) / n, 4)}
print(json.dumps(res))
