"""Per-kernel resource table (VGPRs, spills, LDS, occupancy) of one csrc file,
from hipcc -Rpass-analysis=kernel-resource-usage.  CPU-only build helper.

    python tools/kres.py conv.hip [substring]
"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "fac_fake_amd" / "csrc"


def main():
    src = CSRC / sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{CSRC}",
                        f"-I{CSRC.parents[1] / 'include'}", "-c", str(src), "-o", "/tmp/kres.o",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    cur, rows = None, []
    for ln in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", ln)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for c in rows:
        if pat in c["name"]:
            dm = subprocess.run(["c++filt", c["name"]], capture_output=True,
                                text=True).stdout.strip()
            print(f"V{c.get('VGPRs'):>4} A{c.get('AGPRs'):>3} spillV{c.get('VGPRs Spill'):>4} "
                  f"LDS{c.get('LDS Size [bytes/block]'):>7} occ{c.get('Occupancy [waves/SIMD]'):>2}  {dm[:150]}")


if __name__ == "__main__":
    main()
