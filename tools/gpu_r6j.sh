#!/usr/bin/env bash
# round-6 session j: the mixed register-window / LDS-table sweep geometries on the tree library;
# phase stamps of the desynchronized steady state with the per-done-count block ends
set -euo pipefail
T=r6j
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_geometry_sweep.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "R14C5 or R13C9 or R14C10" > gpurun_out/tests_mixed_$T.log 2>&1
tail -n 1 gpurun_out/tests_mixed_$T.log
st() { local nm=$1; shift; timeout -k 10 120 python tools/stamps.py run "$@" > gpurun_out/stamps_${nm}_$T.json 2> gpurun_out/stamps_${nm}_$T.err; }
st headd --desync
st g25d --grid 25 --desync
st g64d --grid 64 --rays 64 --range 6 --desync
st codesd --codes --desync
echo all-j done
