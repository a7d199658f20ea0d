"""Summarise tools/pmc_cfg45.sh's passes into one JSON per model.

    python tools/pmc_cfg45_summary.py gpurun_out/pmc_cfg45h profiles/r03h

writes <prefix>_{s3d,resvitkan}_pmc.json: per kernel (template instantiation)
the dispatch count, mean counters per dispatch, MFMA busy fraction, LDS and
wave-state ratios and HBM bytes per dispatch (2 x FETCH_SIZE + WRITE_SIZE,
KiB, the gfx950 correction of tools/rocprof_summary.py); and for the whole
eager forward the cycle-weighted MFMA busy fraction (sum of MFMA busy cycles
over sum of 1024 x GRBM_GUI_ACTIVE / 8) and the HBM bytes per forward, over
the fac:: kernels only (the runtime's copyBuffer dispatches are the one-time
weight uploads of the first forward).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from rocprof_summary import derive, short  # noqa: E402


def load(p: Path):
    """{kernel: {counter: [values per dispatch]}}"""
    out = defaultdict(lambda: defaultdict(list))
    f = p / "run_counter_collection.csv"
    if not f.exists():
        return out
    for r in csv.DictReader(open(f)):
        out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def summarise(src: Path, model: str, forwards: int) -> dict:
    passes = [load(src / f"{model}_p{i}") for i in (1, 2, 3)]
    kernels = sorted(set().union(*[set(p) for p in passes]))
    res = {"by_kernel": {}, "forward": {}}
    tot = defaultdict(float)
    setup = defaultdict(float)  # non-fac dispatches (one-time workspace memset, input copies): kept out of the totals
    for k in kernels:
        vals = {}
        n = 0
        for p in passes:
            for c, v in p.get(k, {}).items():
                vals[c] = sum(v) / len(v)
                if k.startswith("fac::"):  # runtime copies / torch fills: one-time setup, not the forward
                    tot[c] += sum(v)
                else:
                    setup[c] += sum(v)
                n = max(n, len(v))
        m = {"dispatches": n, **{c: round(v, 1) for c, v in vals.items()}, **derive(vals)}
        if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
            m["hbm_bytes"] = round((2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0)
        if "SQ_INSTS_LDS" in vals and vals.get("SQ_INSTS_LDS"):
            m["lds_bank_conflict_per_inst"] = round(vals.get("SQ_LDS_BANK_CONFLICT", 0.0) / vals["SQ_INSTS_LDS"], 4)
        res["by_kernel"][k] = m
    if tot.get("GRBM_GUI_ACTIVE"):
        res["forward"]["mfma_busy_cycle_weighted"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * tot["GRBM_GUI_ACTIVE"] / 8), 4)
        res["forward"]["kernel_cycles_per_forward"] = round(tot["GRBM_GUI_ACTIVE"] / 8 / forwards)
    if tot.get("FETCH_SIZE"):
        res["forward"]["hbm_bytes_per_forward"] = round((2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0 / forwards)
        res["forward"]["hbm_bytes_per_forward_counts"] = "fac:: kernels only"
        res["forward"]["excluded_setup_hbm_bytes_total"] = round((2 * setup.get("FETCH_SIZE", 0.0) +
                                                                  setup.get("WRITE_SIZE", 0.0)) * 1024.0)
        res["forward"]["excluded_setup_kernels"] = sorted(k for k in kernels if not k.startswith("fac::"))
    res["forwards_profiled"] = forwards
    res["method"] = ("rocprofv3 --pmc, one run per pass (tools/pmc_cfg45.sh) over the eager forwards of "
                     "tools/rvk_layers.py; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8)")
    return res


def main(src: str, prefix: str):
    src = Path(src)
    for model, tag, B in (("s3d", "s3d", 256), ("rvk", "resvitkan", 512)):
        r = summarise(src, model, forwards=2)  # warm-up forward + --reps 1
        r["batch"] = B
        Path(f"{prefix}_{tag}_pmc.json").write_text(json.dumps(r, indent=1, sort_keys=True))
        top = sorted(r["by_kernel"].items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0) * kv[1]["dispatches"])[:6]
        print(tag, r["forward"])
        for k, m in top:
            print(f"  {k[:70]:70s} n={m['dispatches']:4d} busy={m.get('mfma_busy')} hbm={m.get('hbm_bytes')}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
