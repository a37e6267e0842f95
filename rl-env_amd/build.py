#!/usr/bin/env python3
"""Build libplantos_hip.so (HIP, gfx950) in-tree with hipcc.

  python rl-env_amd/build.py            # build if sources changed
  python rl-env_amd/build.py --force
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "plantos_batch.hip")
SRC_HOST = os.path.join(HERE, "csrc", "pe_pystream.cpp")
SRC_MCTS = os.path.join(HERE, "csrc", "pe_mcts.hip")
DEPS = [SRC, SRC_HOST, SRC_MCTS] + [os.path.join(HERE, "csrc", f) for f in
                                    ("pe_device.hpp", "pe_fast.hpp", "pe_quad.hpp", "pe_coop.hpp", "pe_handle.hpp")] + [
    os.path.join(REPO, "include", "plantos_batch.h"), os.path.join(HERE, "tools_gen_lidar.py")]
OUT = os.path.join(HERE, "plantos_amd", "libplantos_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
         "-Wno-unused-function", "-Wno-unused-variable"]


def build(force=False, verbose=False):
    subprocess.run([sys.executable, os.path.join(HERE, "tools_gen_lidar.py")], check=True)
    deps = DEPS + [os.path.join(HERE, "csrc", "lidar_tables.inc")]
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps):
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT, SRC, SRC_MCTS, SRC_HOST]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
