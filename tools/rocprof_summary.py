"""Turn rocprofv3 CSVs (tools/archive/profile.sh output) into the committed summaries.

    python tools/rocprof_summary.py gpurun_out/prof profiles/r01

writes
  <prefix>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <prefix>_kernels.md         per-kernel calls / mean duration / share
  <prefix>_traffic.json       per-kernel mean HBM bytes per dispatch from the
                              FETCH_SIZE and WRITE_SIZE passes (separate runs)
  <prefix>_pmc.json           per-kernel / per-stage SQ counters (pmc1, pmc2
                              passes of tools/archive/profile_r03.sh): MFMA busy
                              fraction, wave-state split, LDS bank conflicts

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles),
kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM_GUI_ACTIVE over the
8 XCDs, MI355X_MICROARCH.md "DVFS give-back").  SQ_VALU_MFMA_BUSY_CYCLES
counts MFMA cycles (32 per 32x32x16 bf16 MFMA, 16 per 16x16x32), i.e.
1024 FLOP per busy cycle at 16-bit: `mfma_tflop_from_busy` cross-checks the
unit against the executed MFMA work.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane, incl.
global_load_lds) streaming read, so it is doubled; WRITE_SIZE is exact for
16 B/lane stores.  Kernels whose loads are narrower (stem224's 1-byte pixel
loads are ~15% of its reads) are only approximately corrected by this rule.
"""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    return name.replace("void ", "").split("(")[0]


def per_kernel(csv_path: Path, counter: str):
    acc = defaultdict(list)
    for r in csv.DictReader(open(csv_path)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def per_stage_all(csv_path: Path):
    """{stage: {counter: mean}} for every counter of a multi-counter pass."""
    rows = list(csv.DictReader(open(csv_path)))
    out = defaultdict(dict)
    for c in sorted({r["Counter_Name"] for r in rows}):
        for st, v in per_stage(csv_path, c).items():
            out[st][c] = v
    return out


def per_kernel_all(csv_path: Path):
    rows = list(csv.DictReader(open(csv_path)))
    out = defaultdict(dict)
    for c in sorted({r["Counter_Name"] for r in rows}):
        for k, v in per_kernel(csv_path, c).items():
            out[k][c] = v
    return out


def derive(m: dict, dur_ns=None) -> dict:
    d = {}
    g = m.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        d["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8), 4)
        d["mfma_tflop_from_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] * 1024 / 1e12, 4)
    if g and dur_ns:
        d["clock_ghz"] = round(g / 8 / dur_ns, 3)
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in m:
                d[k.lower().replace("sq_", "") + "_frac"] = round(m[k] / wc, 4)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_bank_conflict_per_active"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_LDS_IDX_ACTIVE"], 4)
    if m.get("SQ_INSTS_MFMA"):
        d["lds_insts_per_mfma"] = round(m.get("SQ_INSTS_LDS", 0) / m["SQ_INSTS_MFMA"], 3)
        d["valu_insts_per_mfma"] = round(m.get("SQ_INSTS_VALU", 0) / m["SQ_INSTS_MFMA"], 3)
    return d


def stage_durations(trace_csv: Path):
    """Mean duration (ns) per forward stage from the kernel trace (same
    dispatch-order mapping as per_stage)."""
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    acc = defaultdict(list)
    k = None
    for r in rows:
        name = short(r["Kernel_Name"])
        dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        if "stem224_fused" in name:
            acc["conv1"].append(dur)
            k = 0
        elif ("conv3x3_bn_relu" in name or "conv3x3_db" in name or "conv3x3_wino" in name) and k is not None:
            acc[f"conv{k + 4}"].append(dur)
            k += 1
        elif "gemm_nt" in name:
            k = None
    return {s: sum(v) / len(v) for s, v in acc.items()}


def per_stage(csv_path: Path, counter: str):
    """Mean counter per forward stage: the fused stem is conv1, the k-th conv
    kernel dispatched after it is conv(k+3) (dispatch order is fixed)."""
    rows = [r for r in csv.DictReader(open(csv_path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    acc = defaultdict(list)
    k = None
    for r in rows:
        name = short(r["Kernel_Name"])
        if "stem224_fused" in name:
            acc["conv1"].append(float(r["Counter_Value"]))
            k = 0
        elif ("conv3x3_bn_relu" in name or "conv3x3_db" in name or "conv3x3_wino" in name) and k is not None:
            acc[f"conv{k + 4}"].append(float(r["Counter_Value"]))
            k += 1
        elif "gemm_nt" in name:
            k = None
    return {s: sum(v) / len(v) for s, v in acc.items()}


def main(src: str, prefix: str):
    src, prefix = Path(src), Path(prefix)
    prefix.parent.mkdir(parents=True, exist_ok=True)
    stats = src / "trace" / "run_kernel_stats.csv"
    shutil.copy(stats, f"{prefix}_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    lines = ["| kernel | calls | mean us | share % |", "|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['Percentage']):.2f} |")
    Path(f"{prefix}_kernels.md").write_text("\n".join(lines) + "\n")
    traffic = {"by_kernel": {}, "by_stage": {}}
    fetch = src / "fetch" / "run_counter_collection.csv"
    write = src / "write" / "run_counter_collection.csv"
    if fetch.exists() and write.exists():
        for key, fn in (("by_kernel", per_kernel), ("by_stage", per_stage)):
            f, w = fn(fetch, "FETCH_SIZE"), fn(write, "WRITE_SIZE")
            for k in set(f) | set(w):
                traffic[key][k] = {"fetch_kib_raw": f.get(k), "write_kib": w.get(k),
                                   "hbm_bytes": (2 * f.get(k, 0.0) + w.get(k, 0.0)) * 1024.0}
    Path(f"{prefix}_traffic.json").write_text(json.dumps(traffic, indent=1, sort_keys=True))
    passes = [src / p / "run_counter_collection.csv" for p in ("pmc1", "pmc2")]
    if any(p.exists() for p in passes):
        durs = {}
        tr = src / "trace" / "run_kernel_trace.csv"
        if tr.exists():
            durs = stage_durations(tr)
        pmc = {"by_stage": defaultdict(dict), "by_kernel": defaultdict(dict),
               "method": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8); one rocprofv3 run per pass "
                         "(tools/archive/profile_r03.sh); per-stage = mean over that stage's dispatches"}
        for p in passes:
            if not p.exists():
                continue
            for st, m in per_stage_all(p).items():
                pmc["by_stage"][st].update(m)
            for k, m in per_kernel_all(p).items():
                pmc["by_kernel"][k].update(m)
        for key in ("by_stage", "by_kernel"):
            for k, m in pmc[key].items():
                m.update(derive(m, durs.get(k) if key == "by_stage" else None))
                if key == "by_stage" and k in durs:
                    m["duration_us"] = round(durs[k] / 1e3, 3)
        Path(f"{prefix}_pmc.json").write_text(json.dumps(pmc, indent=1, sort_keys=True))
        print(f"wrote {prefix}_pmc.json ({len(pmc['by_stage'])} stages)")
    print(f"wrote {prefix}_kernel_stats.csv, _kernels.md, _traffic.json ({len(traffic['by_kernel'])} kernels)")


if __name__ == "__main__":
    main(*sys.argv[1:3])
