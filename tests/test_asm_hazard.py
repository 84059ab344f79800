"""No kernel issues a load into registers from inline asm (round 3's policy-head counter load did,
and a register-pressure change let the compiler reuse its destination before the hand-placed
wait: tools/asm_hazard.py states the hazard).  The only asm loads left are the LDS-DMA operand
steps of the dW kernels (global_load_lds_*: no register destination).  CPU only: compiles
kernels.hip for gfx950 to assembly."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_asm_register_loads_in_the_compiled_kernels(tmp_path):
    import asm_hazard
    out = tmp_path / "kernels.s"
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
           "-mllvm", "-amdgpu-kernarg-preload-count=6", "-S", "--offload-device-only",
           os.path.join(ROOT, "td3_amd", "csrc", "kernels.hip"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    asm = out.read_text()
    assert "row_kernel" in asm and ";;#ASMSTART" in asm
    assert asm_hazard.scan(asm) == []
    assert asm_hazard.asm_vgpr_loads(asm) == []
    assert "global_load_lds_dwordx4" in asm          # the checker sees the DMA form and passes it


def test_no_register_load_in_inline_asm_source():
    import re
    src = open(os.path.join(ROOT, "td3_amd", "csrc", "kernels.hip")).read()
    for m in re.finditer(r"asm\s+volatile\s*\(\s*\"([^\"]*)\"", src):
        body = m.group(1)
        assert not re.search(r"(global|buffer|flat)_load_(?!lds)", body), body


def test_checker_flags_an_asm_register_load():
    import asm_hazard
    asm = "\n".join(["_ZN3td3k:", ";;#ASMSTART", "global_load_dwordx2 v[2:3], v[4:5], off", ";;#ASMEND"])
    assert len(asm_hazard.asm_vgpr_loads(asm)) == 1
    dma = asm.replace("global_load_dwordx2 v[2:3], v[4:5], off", "global_load_lds_dwordx4 v[4:5], off")
    assert asm_hazard.asm_vgpr_loads(dma) == []


def test_checker_flags_a_moved_destination():
    import asm_hazard
    asm = "\n".join([
        "_ZN3td3k:",
        ";;#ASMSTART",
        "global_load_dwordx2 v[2:3], v[4:5], off",
        ";;#ASMEND",
        "v_accvgpr_write_b32 a0, v2",
        "s_waitcnt vmcnt(0)",
        ".Lfunc_end0:",
    ])
    assert len(asm_hazard.scan(asm)) == 1
    ok = asm.replace("v_accvgpr_write_b32 a0, v2", "v_mov_b32 v7, v8")
    assert asm_hazard.scan(ok) == []
