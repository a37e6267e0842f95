#!/usr/bin/env python3
"""Guard: a scalar load through an SGPR pair just set to 0 in the device assembly
(`hipcc -S --cuda-device-only`) -- e.g. __builtin_amdgcn_kernarg_segment_ptr() read
inside a called (noinline) function, where it is 0 on gfx950 / ROCm 7.2: an illegal
address at run time.   usage: python tools/diag/isa_nullbase.py file.s"""
import re
import sys

s = open(sys.argv[1]).read()
bad = 0
for m in re.finditer(r'^(_Z\w+):[^\n]*\n(.*?)^\s*s_(?:setpc|endpgm)', s, re.S | re.M):
    body = m.group(2)
    for z in re.finditer(r's_mov_b64 (s\[\d+:\d+\]), 0\n', body):
        if re.search(r's_load_\w+ s[\[\d:\]]+, ' + re.escape(z.group(1)), body[z.end():z.end() + 400]):
            print("null-base scalar load in", m.group(1))
            bad += 1
            break
sys.exit(1 if bad else 0)
