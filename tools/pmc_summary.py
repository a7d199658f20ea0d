"""Summarise rocprofv3 --pmc CSVs per kernel (mean over dispatches)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(root.glob("p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = k.replace("void fac::", "").split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(vals.items(), key=lambda kv: -sum(kv[1].get("SQ_BUSY_CYCLES", [0]))):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    line = f"{k[:60]:60s}"
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        line += f" wait={m.get('SQ_WAIT_ANY', 0) / wc:5.2f} waitinst={m.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} active={m.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f}"
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        line += f" mfma_util={100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] * 1024):5.1f}%"
    if "SQ_LDS_IDX_ACTIVE" in m and m["SQ_LDS_IDX_ACTIVE"]:
        line += f" ldsconf={m.get('SQ_LDS_BANK_CONFLICT', 0) / m['SQ_LDS_IDX_ACTIVE']:5.2f}"
    if "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"]:
        line += f" valu/mfma={m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:5.2f} lds/mfma={m.get('SQ_INSTS_LDS', 0) / m['SQ_INSTS_MFMA']:5.2f} salu/mfma={m.get('SQ_INSTS_SALU', 0) / m['SQ_INSTS_MFMA']:5.2f}"
    print(line)
