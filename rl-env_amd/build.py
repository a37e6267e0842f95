#!/usr/bin/env python3
"""Build libplantos_hip.so (HIP, gfx950) in-tree with hipcc.

  python rl-env_amd/build.py            # build if sources changed
  python rl-env_amd/build.py --force

The three translation units are compiled in parallel (hipcc -c) and linked into
one shared library; the result is byte-identical from run to run (bench.py keys
its committed PMC profiles by the library's hash).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "plantos_batch.hip")
SRC_HOST = os.path.join(HERE, "csrc", "pe_pystream.cpp")
SRC_MCTS = os.path.join(HERE, "csrc", "pe_mcts.hip")
SOURCES = [SRC, SRC_MCTS, SRC_HOST]
DEPS = SOURCES + [os.path.join(HERE, "csrc", f) for f in
                  ("pe_device.hpp", "pe_fast.hpp", "pe_quad.hpp", "pe_coop.hpp", "pe_handle.hpp", "pe_wave.hpp")] + [
    os.path.join(REPO, "include", "plantos_batch.h"), os.path.join(HERE, "tools_gen_lidar.py")]
OUT = os.path.join(HERE, "plantos_amd", "libplantos_hip.so")
OBJ_DIR = os.path.join(REPO, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable"]


def build(force=False, verbose=False, out=OUT, extra_flags=(), obj_dir=OBJ_DIR):
    subprocess.run([sys.executable, os.path.join(HERE, "tools_gen_lidar.py")], check=True)
    deps = [d for d in DEPS if os.path.exists(d)] + [os.path.join(HERE, "csrc", "lidar_tables.inc")]
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    os.makedirs(obj_dir, exist_ok=True)
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        cmd = [HIPCC] + CFLAGS + list(extra_flags) + ["-c", "-o", obj, src]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    failed = [cmd for p, cmd in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs
    if verbose:
        print(" ".join(link))
    subprocess.run(link, check=True)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
