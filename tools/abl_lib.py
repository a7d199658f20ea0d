"""Ablation builds of conv3x3_bn_relu (timing only, WRONG results): each arm
is a text patch of csrc/conv.hip compiled into ab/libfac_abl_<arm>.so with
the other in-tree objects, for tools/conv_sweep.py under FAC_CVIT_LIB.  The
product file is never modified.  CPU-only build helper.

    python tools/abl_lib.py w0 now nomfma nobar noA
"""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
CSRC = REPO / "fac_fake_amd" / "csrc"
OBJ = REPO / "fac_fake_amd" / "_build"
AB = REPO / "ab"

W_NOPB = "issue_w((t + 2) % 3, (c * 9 + t + 2 < nsteps) ? wnext + t * WSL : wsrc);"
MFMA = "for (int ct = 0; ct < CTW; ++ct) acc[rt][ct] = T::mfma(fa[rt], bfr[ct], acc[rt][ct]);"
AREAD = "if (HB == 2 || t < 8) fa[rt] = *(const u16x8*)(hnx + abase[rt] + ntoff);"
BAR = 'asm volatile("s_waitcnt vmcnt(%0)\\n\\ts_waitcnt lgkmcnt(%1)\\n\\ts_barrier" ::"n"(N), "n"(L) : "memory");'
ARMS = {
    "w0": [(W_NOPB, "issue_w((t + 2) % 3, wsrc);")],                       # every slice = slice 0 (L2-hot)
    "now": [(W_NOPB, "")],                                                   # no per-step weight glds
    "nomfma": [(MFMA, 'for (int ct = 0; ct < CTW; ++ct) asm volatile("" ::"v"(fa[rt]), "v"(bfr[ct]));')],
    "nobar": [(BAR, 'asm volatile("s_waitcnt vmcnt(%0)\\n\\ts_waitcnt lgkmcnt(%1)" ::"n"(N), "n"(L) : "memory");')],
    "noA": [(AREAD, "")],
}


def main():
    for arm in sys.argv[1:]:
        src = (CSRC / "conv.hip").read_text()
        for old, new in ARMS[arm]:
            assert old in src, (arm, old)
            src = src.replace(old, new)
        tmp = Path(f"/tmp/conv_abl_{arm}.hip")
        tmp.write_text(src)
        o = Path(f"/tmp/conv_abl_{arm}.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-I{CSRC}",
                        f"-I{REPO / 'include'}", "-c", str(tmp), "-o", str(o)], check=True)
        objs = [str(p) for p in sorted(OBJ.glob("*.o")) if p.name != "conv.o"] + [str(o)]
        AB.mkdir(exist_ok=True)
        out = AB / f"libfac_abl_{arm}.so"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(out), *objs],
                       check=True)
        print(out)


if __name__ == "__main__":
    main()
