"""The shipped gfx950 code object has no VALU-write -> DPP-read hazard (the fused kernel's
x-neighbour sums are inline asm without hazard wait states, csrc/hip/fused.hpp).  Runs on the
CPU: objcopy + clang-offload-bundler + llvm-objdump on the built libgs_hip.so."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import check_dpp_hazards as chk  # noqa: E402

_DPP = ("\tv_add_f32_dpp v85, v10, v56 wave_shl:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        " // 000000001010: 02AA70FA FF09300A\n")


def _line(text, addr):
    return f"\t{text} // {addr:012X}: 00000000\n"


def test_checker_flags_a_hazard():
    dis = _line("v_add_f32_e32 v10, v1, v2", 0x1008) + _DPP
    n, problems = chk.check(dis)
    assert n == 1 and problems and "written by v_add_f32_e32" in problems[0]


def test_checker_accepts_wait_states_and_loads():
    ok_nop = _line("v_add_f32_e32 v10, v1, v2", 0x1004) + _line("s_nop 1", 0x100C) + _DPP
    ok_far = (_line("v_add_f32_e32 v10, v1, v2", 0x1000) + _line("v_mul_f32_e32 v3, v1, v2", 0x1004)
              + _line("s_add_i32 s4, s4, 1", 0x100C) + _DPP)
    ok_load = _line("buffer_load_dwordx2 v[10:11], v1, s[4:7], 0 offen", 0x1008) + _DPP
    for dis in (ok_nop, ok_far, ok_load):
        n, problems = chk.check(dis)
        assert n == 1 and not problems, problems


def test_checker_flags_exec_write():
    dis = _line("s_mov_b64 exec, s[4:5]", 0x1008) + _DPP
    assert chk.check(dis)[1]


@pytest.mark.skipif(not shutil.which("objcopy") or not os.path.exists(chk.LLVM),
                    reason="binutils / ROCm LLVM tools not available")
def test_built_library_has_no_dpp_hazard():
    lib = os.path.join(ROOT, "grayscott_amd", "_lib", "libgs_hip.so")
    if not os.path.exists(lib):
        pytest.skip("libgs_hip.so not built")
    n, problems = chk.check_all(chk.disassemble(lib))
    assert n > 1000, n
    assert not problems, problems[:5]
