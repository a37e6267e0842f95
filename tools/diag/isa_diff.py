#!/usr/bin/env python3
"""Compare the step kernels' instruction streams of two `hipcc -S --cuda-device-only`
outputs (comments, directives and labels dropped): which kernels changed.
  python tools/diag/isa_diff.py base.s new.s [substring]"""
import re
import sys


def kernels(path, sub):
    s = open(path).read()
    out = {}
    for m in re.finditer(r'^(_Z\w+):[^\n]*\n(.*?)^\s*s_endpgm', s, re.S | re.M):
        if sub in m.group(1):
            out[m.group(1)] = [re.sub(r'\.L(BB|tmp)\d+_', r'.L\1_', l.strip()) for l in m.group(2).split('\n')
                               if l.strip() and not l.strip().startswith((';', '.')) and not l.rstrip().endswith(':')]
    return out


if __name__ == "__main__":
    sub = sys.argv[3] if len(sys.argv) > 3 else "pe_step"
    a, b = kernels(sys.argv[1], sub), kernels(sys.argv[2], sub)
    same = 0
    for k in sorted(a):
        if k not in b:
            print("only in first:", k)
        elif a[k] != b[k]:
            print(f"DIFF {k}: {len(a[k])} -> {len(b[k])} instructions")
        else:
            same += 1
    for k in sorted(set(b) - set(a)):
        print("only in second:", k)
    print(f"{len(a)} kernels, {same} identical")
