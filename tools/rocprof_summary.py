"""Turn rocprofv3 CSVs (tools/profile.sh output) into the committed summaries.

    python tools/rocprof_summary.py gpurun_out/prof profiles/r01

writes
  <prefix>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <prefix>_kernels.md         per-kernel calls / mean duration / share
  <prefix>_traffic.json       per-kernel mean HBM bytes per dispatch from the
                              FETCH_SIZE and WRITE_SIZE passes (separate runs)

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
        elif "conv3x3_bn_relu" in name and k is not None:
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
    print(f"wrote {prefix}_kernel_stats.csv, _kernels.md, _traffic.json ({len(traffic['by_kernel'])} kernels)")


if __name__ == "__main__":
    main(*sys.argv[1:3])
