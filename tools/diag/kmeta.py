#!/usr/bin/env python3
"""Register / spill / LDS metadata of the step kernels in a built library.

  python tools/diag/kmeta.py build/ab/lib_X.so [substring]

Extracts the gfx950 code objects (llvm-objdump --offloading, into a temp dir) and
prints .vgpr_count, .sgpr_count, spills and the static LDS size from their notes."""
import glob
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = os.path.abspath(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "pe_step"
tmp = tempfile.mkdtemp()
try:
    shutil.copy(lib, os.path.join(tmp, "lib.so"))
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", "lib.so"], cwd=tmp, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for co in sorted(glob.glob(os.path.join(tmp, "*gfx950*"))):
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
        for blk in notes.split("  - .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk)
            if not name or pat not in name.group(1):
                continue
            f = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
            dn = subprocess.run(["c++filt"], input=name.group(1), capture_output=True, text=True).stdout.strip()
            print(f"vgpr {f('vgpr_count'):>4} sgpr {f('sgpr_count'):>4} vspill {f('vgpr_spill_count'):>3} "
                  f"sspill {f('sgpr_spill_count'):>3} lds {f('group_segment_fixed_size'):>6} priv {f('private_segment_fixed_size'):>4}  {dn[:110]}")
finally:
    shutil.rmtree(tmp)
