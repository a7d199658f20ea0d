"""Build libfac_cvit.so (HIP kernels + C ABI) in-tree for gfx950.

Plain ``hipcc`` invocations, no CMake: each ``csrc/*.hip`` compiles to an
object under ``fac_fake_amd/_build/`` (rebuilt when it or a header is newer)
and the objects link into ``fac_fake_amd/libfac_cvit.so``.  The library only
depends on ``libamdhip64.so.7``; loaded after ``import torch`` it binds to
the HIP runtime torch already mapped (same SONAME).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
OBJDIR = PKG / "_build"
LIB = PKG / "libfac_cvit.so"
ARCH = os.environ.get("FAC_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the fac_cvit HIP library cannot be built")


def _flags():
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
            f"-I{CSRC}", f"-I{INCLUDE}"]


# Per-file extra flags.  stem224.hip: no wave-level atomic aggregation, whose
# prefix-sum code needs the box-claim atomic's return value at once (an
# s_waitcnt vmcnt(0) at every box start); plain, its wait sits at the use.
FILE_FLAGS: dict = {"stem224.hip": ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]}


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.hpp")) + list(INCLUDE.glob("*.h"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _check_conv_waits(compile_fn, verbose: bool) -> None:
    """The conv kernels' relaxed per-tap LDS waits are sound only for the
    issue order the compiler chose (isa_check.py).  Verify it on the fresh
    object; if any wait fails, rebuild conv.hip with every wait strict."""
    from . import isa_check
    obj = OBJDIR / "conv.o"
    rep = isa_check.check_objects([obj], arch=ARCH)
    if verbose:
        print(f"isa_check: {rep.kernels} conv kernels, {rep.waits} relaxed LDS waits, "
              f"{len(rep.problems)} problems", file=sys.stderr)
    if rep.ok and rep.kernels > 0:
        return
    if rep.kernels == 0:
        # nothing disassembled (bundle name mismatch, no llvm-objdump): the
        # relaxed waits cannot be verified, so build the strict variant
        rep.problems.append("no conv3x3 kernels found in the disassembly; relaxed waits unverified")
    print("isa_check: relaxed LDS waits unsound in this build, rebuilding conv.hip with "
          "FAC_CONV_STRICT_LGKM:\n  " + "\n  ".join(rep.problems[:8]), file=sys.stderr)
    FILE_FLAGS["conv.hip"] = FILE_FLAGS.get("conv.hip", []) + ["-DFAC_CONV_STRICT_LGKM"]
    compile_fn((CSRC / "conv.hip", obj))
    rep = isa_check.check_objects([obj], arch=ARCH)
    if not rep.ok:  # (zero kernels found is fine here: every wait is strict)
        raise RuntimeError("isa_check failed even with strict LDS waits:\n" + "\n".join(rep.problems[:8]))


def build(verbose: bool = False, force: bool = False) -> Path:
    """Compile every csrc/*.hip for gfx950 and link libfac_cvit.so."""
    hipcc = _hipcc()
    OBJDIR.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    hdr_t = _headers_mtime()
    jobs = []
    for s in srcs:
        o = OBJDIR / (s.stem + ".o")
        if force or not o.exists() or o.stat().st_mtime < max(s.stat().st_mtime, hdr_t):
            jobs.append((s, o))

    def _compile(so):
        s, o = so
        cmd = [hipcc, *_flags(), *FILE_FLAGS.get(s.name, []), "-c", str(s), "-o", str(o)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s.name}:\n{r.stderr}")
        return o

    with ThreadPoolExecutor(max_workers=min(8, max(1, len(jobs)))) as ex:
        list(ex.map(_compile, jobs))
    if any(s.name == "conv.hip" for s, _ in jobs):
        _check_conv_waits(_compile, verbose)
    objs = [OBJDIR / (s.stem + ".o") for s in srcs]
    if force or jobs or not LIB.exists() or LIB.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
