"""The hand-placed asynchronous counter load of the policy head (kernels.hip row_policy_head) must not
have its destination registers copied or reused before its wait in any compiled row kernel
(tools/asm_hazard.py states the hazard).  CPU only: compiles kernels.hip for gfx950 to assembly."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_policy_head_counter_load_is_not_moved_before_its_wait(tmp_path):
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
