"""Per-layer SQ counter table from tools/archive/conv_pmc.sh output (gpurun_out/cpmc)."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/cpmc"
layers = sorted({p.split("/")[-1].split("_")[0] for p in glob.glob(f"{root}/l*_p*") if not p.endswith(".log")})
for L in layers:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{root}/{L}_p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "conv3x3" in r["Kernel_Name"] or "conv112" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    g = m.get("GRBM_GUI_ACTIVE", 1) / 8  # cycles (counter summed over 8 XCDs)
    pr = lambda k, d: m.get(k, 0) / d
    print(f"{L}: cycles {g:.0f}  MFMA busy {pr('SQ_VALU_MFMA_BUSY_CYCLES', g * 1024):.2f}  "
          f"LDS active/CU {pr('SQ_LDS_IDX_ACTIVE', g * 256):.2f}  bank-confl/LDS-active {pr('SQ_LDS_BANK_CONFLICT', m.get('SQ_LDS_IDX_ACTIVE', 1)):.2f}  "
          f"wait_any/wave {pr('SQ_WAIT_ANY', m.get('SQ_WAVE_CYCLES', 1)):.2f}  wait_inst_any/wave {pr('SQ_WAIT_INST_ANY', m.get('SQ_WAVE_CYCLES', 1)):.2f}  "
          f"waves/CU {pr('SQ_WAVE_CYCLES', g * 256):.1f}  LDS/MFMA insts {pr('SQ_INSTS_LDS', m.get('SQ_INSTS_MFMA', 1)):.2f}  "
          f"VMEM lvl {pr('SQ_INST_LEVEL_VMEM', m.get('SQ_WAVE_CYCLES', 1)):.2f}")
