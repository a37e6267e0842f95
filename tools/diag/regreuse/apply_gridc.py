#!/usr/bin/env python3
"""PATCH_PY for tools/ab_build.sh: apply the round-5 compact grid mirror (gridc) to the
source copy (kernel sources only; its test changes are not needed to reproduce)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
subprocess.run(["git", "apply", "--exclude=tests/*", os.path.join(HERE, "gridc_compact_mirror.diff")], check=True)
