#!/usr/bin/env python3
"""ISA excerpt of the round-5 register-reuse hazard: in the C64 byte-tile step kernel,
a `v_mov_b64 v[a:b], s[..]` (a hoisted uniform value, e.g. r_invalid) whose VGPR pair a
later `ds_read_b64 v[a:b]` (the target's window row) overwrites within a short distance.
Prints every such pair with its surrounding lines; used on build/ab/lib_gridc.so (the
miscompiled build) and on the product library (where the pattern is expected absent or
benign: the value is dead before the load).
  python tools/diag/regreuse/isa_excerpt.py LIB [kernel-substring]"""
import os
import re
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import isa_nullbase  # noqa: E402


def library_text(lib):
    tmp = tempfile.mkdtemp()
    return "".join(isa_nullbase.disassemble(co) for co in isa_nullbase.code_objects(os.path.abspath(lib), tmp))


def kernels(text, want):
    """[(symbol, body)] of the functions whose symbol holds `want`"""
    return re.findall(r"^[0-9a-f]+ <(_Z\w*" + want + r"\w*)>:\n(.*?)(?=^[0-9a-f]+ <_Z|\Z)", text, re.S | re.M)


def scan(sym, body, quiet=False):
    class M:  # (the match object shape the loop below reads)
        def __init__(self, a, b):
            self.g = (a, b)

        def group(self, k):
            return self.g[k - 1]
    m = M(sym, body)
    lines = [ln.split("//")[0].rstrip() for ln in m.group(2).split("\n")]
    hits = 0
    for i, ln in enumerate(lines):
        mv = re.match(r"\s*v_mov_b64(?:_e32)? (v\[\d+:\d+\]), s\[\d+:\d+\]", ln)
        if not mv:
            continue
        for j in range(i + 1, min(i + 200, len(lines))):
            if re.match(r"\s*ds_read_b64 " + re.escape(mv.group(1)) + r",", lines[j]):
                # a read of the parked pair in between (as a source operand): the value was used
                lo, hi = (int(x) for x in re.findall(r"\d+", mv.group(1)))
                srcs = " ".join(ln2.split(",", 1)[1] for ln2 in lines[i + 1:j] if "," in ln2)
                used = re.search(r"v\[%d:%d\]|\bv%d\b|\bv%d\b" % (lo, hi, lo, hi), srcs)
                if used:
                    break
                hits += 1
                if not quiet:
                    print(f"--- {m.group(1)[:60]} lines {i}..{j}")
                    print("\n".join(lines[max(0, i - 3):j + 4]))
                break
            if re.match(r"\s*s_(setpc|endpgm)", lines[j]) or re.match(r"\s*\w+ " + re.escape(mv.group(1)) + r",", lines[j]):
                break  # (the pair written again before any ds_read_b64 into it)
    return hits


def main():
    lib = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else "pe_step_quadILi64ELi6ELb0ELi4ELb1ELi64E"
    total = 0
    for sym, body in kernels(library_text(lib), want):
        h = scan(sym, body)
        total += h
        print(f"{sym[:70]}: {h} v_mov_b64-from-SGPR pairs overwritten by a ds_read_b64 before any read of them")
    return total


if __name__ == "__main__":
    main()
