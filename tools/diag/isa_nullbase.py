#!/usr/bin/env python3
"""ISA guards on the product library's device code (run by tests/test_kernel_isa.py
on the CPU, and by hand on an A/B build):

* null-base scalar loads: a scalar load through an SGPR pair just set to 0 -- e.g.
  __builtin_amdgcn_kernarg_segment_ptr() read inside a called (noinline) function,
  where it is 0 on gfx950 / ROCm 7.2: an illegal address at run time (round 4's
  pipelined-kernel fault).  Works on `hipcc -S --cuda-device-only` output and on
  `llvm-objdump -d` of the extracted code objects.
* register spills of the step kernels (the code objects' metadata notes).

  python tools/diag/isa_nullbase.py file.s            # assembly
  python tools/diag/isa_nullbase.py lib.so [pattern]  # a built library: both checks
"""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def null_base_loads(text):
    """Functions of the assembly/disassembly `text` with a null-base scalar load."""
    # objdump form -> assembler form: '<_Zname>:' labels, no '// ...' comments
    text = re.sub(r"^[0-9a-f]+ <(\w+)>:", r"\1:", text, flags=re.M)
    text = re.sub(r"[ \t]*//[^\n]*", "", text)
    text = re.sub(r"^\s+", "\t", text, flags=re.M)
    bad = []
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\s*s_(?:setpc_b64|endpgm)", text, re.S | re.M):
        body = m.group(2)
        for z in re.finditer(r"s_mov_b64 (s\[\d+:\d+\]), 0\n", body):
            if re.search(r"s_load_\w+ s[\[\d:\]]+, " + re.escape(z.group(1)), body[z.end():z.end() + 400]):
                bad.append(m.group(1))
                break
    return bad


def code_objects(lib, tmp):
    """Extract the gfx950 code objects of a built library into tmp; their paths."""
    shutil.copy(lib, os.path.join(tmp, "lib.so"))
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", "lib.so"], cwd=tmp, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return sorted(glob.glob(os.path.join(tmp, "*gfx950*")))


def kernel_meta(co):
    """{kernel symbol: {vgpr_count, sgpr_count, vgpr_spill_count, sgpr_spill_count,
    private_segment_fixed_size}} from a code object's notes."""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                           check=True).stdout
    out = {}
    for blk in notes.split("  - .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name:
            continue
        vals = {}
        for k in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size"):
            v = re.search(r"\." + k + r":\s+(\d+)", blk)
            vals[k] = int(v.group(1)) if v else None
        out[name.group(1)] = vals
    return out


def disassemble(co):
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True, text=True, check=True).stdout


def check_library(lib, pattern="pe_step"):
    """(null-base functions, {kernel: meta} of the kernels whose name holds `pattern`)"""
    tmp = tempfile.mkdtemp()
    try:
        bad, meta = [], {}
        for co in code_objects(os.path.abspath(lib), tmp):
            bad += null_base_loads(disassemble(co))
            meta.update({k: v for k, v in kernel_meta(co).items() if pattern in k})
        return bad, meta
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    path = sys.argv[1]
    if path.endswith(".s"):
        bad = null_base_loads(open(path).read())
        meta = {}
    else:
        bad, meta = check_library(path, sys.argv[2] if len(sys.argv) > 2 else "pe_step")
    for b in bad:
        print("null-base scalar load in", b)
    for k, v in sorted(meta.items()):
        print(f"vgpr {v['vgpr_count']:>4} spill {v['vgpr_spill_count']:>3} sspill {v['sgpr_spill_count']:>3} "
              f"priv {v['private_segment_fixed_size']:>4}  {k[:100]}")
    sys.exit(1 if bad else 0)
