"""CPU checks of the product library's device code (no GPU): the gfx950 code objects
are extracted from libplantos_hip.so and

- no function loads through a null scalar base (the kernarg-segment pointer read in
  a noinline callee is 0 on gfx950 / ROCm 7.2: the fault round 4 hit in the
  pipelined kernel; tools/diag/isa_nullbase.py);
- no step kernel spills more than 8 VGPRs (the product instantiates none of the
  spilling A/B shapes, e.g. 8 waves x 64 envs).
"""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools", "diag"))

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                                reason="ROCm LLVM tools absent")


@pytest.fixture(scope="module")
def checked():
    from plantos_amd import _capi
    if not os.path.exists(_capi.LIB_PATH):
        subprocess.run([sys.executable, os.path.join(REPO, "rl-env_amd", "build.py")], check=True)
    import isa_nullbase
    return isa_nullbase.check_library(_capi.LIB_PATH, pattern="pe_step")


def test_no_null_base_scalar_loads(checked):
    bad, _ = checked
    assert not bad, f"null-base scalar loads in {bad}"


def test_step_kernels_spill_at_most_8_vgprs(checked):
    _, meta = checked
    assert meta, "no step kernels found in the library"
    filt = shutil.which("c++filt")
    over = {k: v["vgpr_spill_count"] for k, v in meta.items() if (v["vgpr_spill_count"] or 0) > 8}
    if filt and over:
        names = subprocess.run([filt], input="\n".join(over), capture_output=True, text=True).stdout.split("\n")
        over = dict(zip(names, over.values()))
    assert not over, f"step kernels spilling > 8 VGPRs: {over}"


def test_guard_detects_a_null_base_load():
    """the guard itself: a synthetic disassembly with the faulting form is flagged, the
    kernel-body form (pointer taken from the kernarg SGPRs) is not"""
    import isa_nullbase
    bad = ("0000000000001000 <_Z3foov>:\n"
           "\ts_mov_b64 s[4:5], 0                        // 000000001000: BE840180\n"
           "\ts_load_dwordx2 s[6:7], s[4:5], 0x10       // 000000001004: C0060182 00000010\n"
           "\ts_setpc_b64 s[30:31]                       // 000000001008: BE801D1E\n")
    good = bad.replace("s_mov_b64 s[4:5], 0 ", "s_mov_b64 s[4:5], s[0:1] ")
    assert isa_nullbase.null_base_loads(bad) == ["_Z3foov"]
    assert isa_nullbase.null_base_loads(good) == []
