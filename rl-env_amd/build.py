#!/usr/bin/env python3
"""Build libplantos_hip.so (HIP, gfx950) in-tree with hipcc.

  python rl-env_amd/build.py            # build if sources changed
  python rl-env_amd/build.py --force

The three translation units are compiled in parallel (hipcc -c) and linked into
one shared library; the result is byte-identical from run to run (bench.py keys
its committed PMC profiles by the library's hash).
"""
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "plantos_batch.hip")
SRC_HOST = os.path.join(HERE, "csrc", "pe_pystream.cpp")
SRC_MCTS = os.path.join(HERE, "csrc", "pe_mcts.hip")
SOURCES = [SRC, SRC_MCTS, SRC_HOST]
DEPS = SOURCES + [os.path.join(HERE, "csrc", f) for f in
                  ("pe_device.hpp", "pe_fast.hpp", "pe_quad.hpp", "pe_coop.hpp", "pe_handle.hpp", "pe_far.hpp")] + [
    os.path.join(REPO, "include", "plantos_batch.h"), os.path.join(HERE, "tools_gen_lidar.py")]
OUT = os.path.join(HERE, "plantos_amd", "libplantos_hip.so")
OBJ_DIR = os.path.join(REPO, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall",
          "-Wno-unused-function", "-Wno-unused-variable"]


def build(force=False, verbose=False, out=OUT, extra_flags=(), obj_dir=None):
    """Compile + link into `out`.  Objects go to a directory keyed by (flags, out), so
    a flagged A/B variant never links the product's objects; the library is linked
    under a temporary name and renamed into place (a concurrent build or a loader
    never sees a half-written file)."""
    subprocess.run([sys.executable, os.path.join(HERE, "tools_gen_lidar.py")], check=True)
    missing = [d for d in DEPS if not os.path.exists(d)]
    if missing:
        raise FileNotFoundError(f"build dependencies missing: {missing}")
    deps = DEPS + [os.path.join(HERE, "csrc", "lidar_tables.inc")]
    if not force and os.path.exists(out) and os.path.getmtime(out) >= max(os.path.getmtime(d) for d in deps):
        return out
    if obj_dir is None:
        key = hashlib.sha256(repr((sorted(extra_flags), os.path.abspath(out))).encode()).hexdigest()[:12]
        obj_dir = OBJ_DIR if not extra_flags and os.path.abspath(out) == OUT else f"{OBJ_DIR}_{key}"
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
    fd, tmp = tempfile.mkstemp(prefix=".lib", suffix=".so", dir=os.path.dirname(os.path.abspath(out)))
    os.close(fd)
    try:
        link = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp] + objs
        if verbose:
            print(" ".join(link))
        subprocess.run(link, check=True)
        os.chmod(tmp, 0o755)
        shutil.move(tmp, out)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
