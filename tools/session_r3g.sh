#!/usr/bin/env bash
# round-3 GPU session g: early records for up to 4 predicted envs per block (knobs8)
# vs one (knobs7); the short window's first graph replay; desync stamps; tests
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs7.so; B=build/ab/lib_knobs8.so
timeout -k 10 120 python tools/diag/window_overhead3.py > $OUT/window3_r3g.json 2> $OUT/window3_r3g.err
bash tools/ab_bench.sh r3g_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3g_sync 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
timeout -k 10 180 python tools/stamps.py run --desync > $OUT/stampsd_r3g.json 2> $OUT/stampsd_r3g.err
echo stamps done
bash tools/gpu_session.sh r3g tests
