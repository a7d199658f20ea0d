"""Build-time check of the conv kernels' relaxed per-tap LDS waits.

``conv3x3_bn_relu`` (csrc/conv.hip) ends every tap step with
``s_waitcnt lgkmcnt(L); s_barrier``, L > 0: it retires this step's reads of
the weight-ring slot the next step refills and leaves the L youngest LDS ops
-- the A-fragment prefetches of the next tap, which read the halo buffers --
in flight across the barrier.  That is only sound if the compiler kept that
issue order, which ``sched_group_barrier`` requests but does not guarantee:

* a scalar-memory op (``s_load*``, ``s_memtime`` ...) in the step would make
  the LGKM counter retire out of order;
* a weight-ring read (or any other LDS op) among the L youngest would still
  be in flight when another wave refills its slot after the barrier.

This module disassembles the built code objects and checks every such wait:
no scalar-memory op since the previous barrier, and each of the L youngest
LGKM ops is a ``ds_read_b128`` whose destination registers are next used as
the A operand (the pixel fragment, src0) of an MFMA.  ``build.py`` runs it
after linking and, if a wait fails, rebuilds ``conv.hip`` with
``-DFAC_CONV_STRICT_LGKM`` (L = 0, every wait retires all LDS ops).
"""
from __future__ import annotations

import re
import shutil
import subprocess
import tempfile
from dataclasses import dataclass, field
from pathlib import Path

LLVM_BIN = Path("/opt/rocm/lib/llvm/bin")
ARCH_TAG = "hipv4-amdgcn-amd-amdhsa--"

_SMEM = ("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_sendmsg", "s_atomic", "s_buffer_atomic",
         "s_scratch_load", "s_dcache")
_LINE = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):")
_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_TARGET = re.compile(r"<(.+)\+0x([0-9a-f]+)>")
_VREG = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)(?!\d))")


@dataclass
class Insn:
    addr: int
    op: str
    args: str
    target: int | None = None


@dataclass
class Report:
    kernels: int = 0
    waits: int = 0
    problems: list = field(default_factory=list)

    @property
    def ok(self) -> bool:
        return not self.problems


def _tool(name: str) -> str:
    p = LLVM_BIN / name
    if p.exists():
        return str(p)
    q = shutil.which(name)
    if not q:
        raise RuntimeError(f"{name} not found (needed for the ISA check)")
    return q


def disassemble(obj: Path, arch: str = "gfx950") -> str:
    """Device disassembly of a hipcc -c object (its offload bundle)."""
    with tempfile.TemporaryDirectory() as td:
        cp = Path(td) / obj.name
        shutil.copy(obj, cp)
        subprocess.run([_tool("llvm-objdump"), "--offloading", str(cp)], check=True, capture_output=True)
        dev = [p for p in Path(td).iterdir() if p.name.endswith(ARCH_TAG + arch)]
        if not dev:
            return ""  # host-only object
        r = subprocess.run([_tool("llvm-objdump"), "-d", f"--mcpu={arch}", str(dev[0])], check=True,
                           capture_output=True, text=True)
        return r.stdout


def parse_functions(text: str) -> dict:
    funcs, cur, base = {}, None, 0
    for line in text.splitlines():
        m = _FUNC.match(line)
        if m:
            base, cur = int(m.group(1), 16), m.group(2)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        m = _LINE.match(line)
        if not m:
            continue
        ins = Insn(int(m.group(3), 16), m.group(1), m.group(2))
        if ins.op.startswith(("s_branch", "s_cbranch")):
            t = _TARGET.search(line)
            if t and t.group(1) == cur:
                ins.target = base + int(t.group(2), 16)
        funcs[cur].append(ins)
    return funcs


def _vregs(operand: str) -> frozenset:
    out = set()
    for a, b, c in _VREG.findall(operand):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return frozenset(out)


def _operands(args: str) -> list:
    return [a.strip().split(" ")[0] for a in args.split(",")] if args else []


def _is_lgkm(op: str) -> bool:
    return op.startswith("ds_") or op.startswith(_SMEM)


def _lgkm_wait(ins: Insn):
    if ins.op != "s_waitcnt":
        return None
    m = re.search(r"lgkmcnt\((\d+)\)", ins.args)
    return int(m.group(1)) if m else None


def _first_use(code: list, start: int, regs: frozenset, limit: int = 4000):
    """First instruction at or after `start` that touches `regs`, following
    unconditional branches and (once each) backward conditional branches --
    the loop's next iteration, where the prefetched fragments are consumed."""
    index = {ins.addr: i for i, ins in enumerate(code)}
    i, taken = start, set()
    for _ in range(limit):
        if i >= len(code):
            return None
        ins = code[i]
        ops = _operands(ins.args)
        if any(_vregs(o) & regs for o in ops):
            return ins
        if ins.target is not None and ins.target in index:
            if ins.op == "s_branch" or (ins.target <= ins.addr and i not in taken):
                taken.add(i)
                i = index[ins.target]
                continue
        if ins.op == "s_endpgm":
            return None
        i += 1
    return None


def check_function(name: str, code: list, rep: Report) -> None:
    prev_barrier = -1
    for i, ins in enumerate(code):
        if ins.op == "s_barrier":
            L = _lgkm_wait(code[i - 1]) if i > 0 else None
            if L:
                rep.waits += 1
                seg = code[prev_barrier + 1:i - 1]
                smem = [s for s in seg if s.op.startswith(_SMEM)]
                if smem:
                    rep.problems.append(f"{name} @0x{ins.addr:x}: scalar-memory op {smem[0].op} in a step ending "
                                        f"with lgkmcnt({L})")
                lg = [s for s in seg if _is_lgkm(s.op)]
                if len(lg) < L:
                    rep.problems.append(f"{name} @0x{ins.addr:x}: only {len(lg)} LGKM ops since the previous "
                                        f"barrier, lgkmcnt({L})")
                # the LGKM ops still in flight at the barrier: replay the
                # step's own lgkmcnt waits (each leaves only its k youngest
                # outstanding), then the barrier's lgkmcnt(L)
                pend = []
                for s in seg:
                    if _is_lgkm(s.op):
                        pend.append(s)
                    else:
                        k = _lgkm_wait(s)
                        if k is not None:
                            pend = pend[len(pend) - k:] if k else []
                for r in pend[max(0, len(pend) - L):]:
                    if r.op != "ds_read_b128":
                        rep.problems.append(f"{name} @0x{r.addr:x}: {r.op} among the {L} LDS ops left in flight")
                        continue
                    dst = _vregs(_operands(r.args)[0])
                    use = _first_use(code, i + 1, dst)
                    ok = use is not None and use.op.startswith("v_mfma") and \
                        _vregs(_operands(use.args)[1]) == dst
                    if not ok:
                        what = f"{use.op} {use.args}" if use else "nothing"
                        rep.problems.append(f"{name} @0x{r.addr:x}: ds_read_b128 left in flight feeds {what}, "
                                            f"not an MFMA A operand")
            prev_barrier = i


def check_objects(objs, pattern: str = "conv3x3_bn_relu", arch: str = "gfx950") -> Report:
    rep = Report()
    for obj in objs:
        funcs = parse_functions(disassemble(Path(obj), arch))
        for name, code in funcs.items():
            if pattern in name:
                rep.kernels += 1
                check_function(name, code, rep)
    return rep
