"""One forward's kernel sequence from a rocprofv3 rocpd database (kernel
trace of tools/small_b_trace.py): per kernel launch the duration and the gap
to the previous kernel's end, averaged over the last N forwards (a forward
starts at each `first` kernel).
    python tools/trace_forward.py gpurun_out/prof_small/small_results.db [first-kernel-substring]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    db = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "stem224_fused"
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if first in r[0]]
    fwds = [rows[a:b] for a, b in zip(starts, starts[1:])][-20:]
    n = min(len(f) for f in fwds)
    acc = defaultdict(lambda: [0.0, 0.0])
    names = [r[0] for r in fwds[-1][:n]]
    for f in fwds:
        for i in range(n):
            acc[i][0] += (f[i][2] - f[i][1]) / 1e3
            acc[i][1] += ((f[i][1] - f[i - 1][2]) / 1e3) if i else 0.0
    k = len(fwds)
    tot_d = sum(v[0] for v in acc.values()) / k
    tot_g = sum(v[1] for v in acc.values()) / k
    span = sum((f[n - 1][2] - f[0][1]) / 1e3 for f in fwds) / k
    for i in range(n):
        nm = names[i].split("(")[0]
        print(f"{i:3d} {acc[i][0] / k:8.2f} us  gap {acc[i][1] / k:6.2f}  {nm[:100]}")
    print(f"{k} forwards x {n} kernels: busy {tot_d:.1f} us + gaps {tot_g:.1f} us = span {span:.1f} us")


if __name__ == "__main__":
    main()
