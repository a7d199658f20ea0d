"""The build-time check of the conv kernels' relaxed per-tap LDS waits
(fac_fake_amd/isa_check.py): synthetic disassembly with a sound and two
unsound schedules, and the real code object of this build."""
from pathlib import Path

import pytest

from fac_fake_amd import isa_check

HEAD = "0000000000001000 <_ZN3fac15conv3x3_bn_reluX>:\n"


def _asm(lines):
    out, addr = [HEAD], 0x1000
    for ln in lines:
        out.append(f"\t{ln} // {addr:012X}: 00000000\n")
        addr += 8
    return "".join(out)


def _check(lines):
    rep = isa_check.Report()
    for name, code in isa_check.parse_functions(_asm(lines)).items():
        isa_check.check_function(name, code, rep)
    return rep


STEP = ["ds_read_b128 v[50:53], v90 offset:59392",     # B fragment (ring slot)
        "s_waitcnt lgkmcnt(0)",
        "v_mfma_f32_16x16x32_bf16 v[2:5], v[46:49], v[50:53], v[2:5]",
        "ds_read_b128 v[46:49], v72 offset:16",         # A prefetch for the next tap
        "v_mfma_f32_16x16x32_bf16 v[6:9], v[42:45], v[50:53], v[6:9]",
        "ds_read_b128 v[42:45], v96 offset:16"]
NEXT = ["s_barrier",
        "ds_read_b128 v[50:53], v90 offset:59648",
        "s_waitcnt lgkmcnt(0)",
        "v_mfma_f32_16x16x32_bf16 v[2:5], v[46:49], v[50:53], v[2:5]",
        "v_mfma_f32_16x16x32_bf16 v[6:9], v[42:45], v[50:53], v[6:9]",
        "s_endpgm"]


def test_sound_schedule_passes():
    rep = _check(["s_barrier"] + STEP + ["s_waitcnt lgkmcnt(2)"] + NEXT)
    assert rep.waits == 1 and rep.ok, rep.problems


def test_ring_read_left_in_flight_is_caught():
    # the B read issued last: lgkmcnt(2) leaves it in flight across the barrier
    step = STEP[:-1] + ["ds_read_b128 v[42:45], v96 offset:16", "ds_read_b128 v[54:57], v90 offset:59648"]
    nxt = ["s_barrier", "v_mfma_f32_16x16x32_bf16 v[2:5], v[46:49], v[54:57], v[2:5]", "s_endpgm"]
    rep = _check(["s_barrier"] + step + ["s_waitcnt lgkmcnt(2)"] + nxt)
    assert not rep.ok and any("not an MFMA A operand" in p for p in rep.problems)


def test_ring_read_retired_by_a_step_wait_passes():
    # the B read sits among the last reads in program order, but a
    # lgkmcnt(0) inside the step retires it: only the A prefetch behind that
    # wait is in flight at the barrier (the compiler's order in the round-5
    # chunk-planar 112^2 tiles)
    step = ["ds_read_b128 v[46:49], v72 offset:16", "ds_read_b128 v[50:53], v90 offset:59392",
            "s_waitcnt lgkmcnt(0)",
            "v_mfma_f32_16x16x32_bf16 v[2:5], v[46:49], v[50:53], v[2:5]",
            "ds_read_b128 v[42:45], v96 offset:16"]
    rep = _check(["s_barrier"] + step + ["s_waitcnt lgkmcnt(2)"] + NEXT)
    assert rep.waits == 1 and rep.ok, rep.problems


def test_scalar_load_in_step_is_caught():
    rep = _check(["s_barrier", "s_load_dwordx4 s[4:7], s[0:1], 0x10"] + STEP + ["s_waitcnt lgkmcnt(2)"] + NEXT)
    assert not rep.ok and any("scalar-memory" in p for p in rep.problems)


def test_built_conv_object_passes():
    obj = Path(__file__).resolve().parents[1] / "fac_fake_amd" / "_build" / "conv.o"
    if not obj.exists() or not (isa_check.LLVM_BIN / "llvm-objdump").exists():
        pytest.skip("conv.o not built here")
    rep = isa_check.check_objects([obj])
    assert rep.kernels >= 20 and rep.ok, rep.problems[:5]
