#!/usr/bin/env bash
# round-3 GPU session h: tracked wait for the early record (knobs9) vs knobs7;
# graph upload before the short window; desync stamps; tests; driver-shaped bench
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
A=build/ab/lib_knobs7.so; B=build/ab/lib_knobs9.so
timeout -k 10 120 python tools/diag/window_overhead3.py > $OUT/window3_r3h.json 2> $OUT/window3_r3h.err
bash tools/ab_bench.sh r3h_desync 3 $A $B -- --desync --steps 20480 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3h_sync 3 $A $B -- --steps 4096 --warmup 200 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
timeout -k 10 180 python tools/stamps.py run --desync > $OUT/stampsd_r3h.json 2> $OUT/stampsd_r3h.err
echo stamps done
bash tools/gpu_session.sh r3h tests benchx:drv:--steps_20_--warmup_5 benchx:drv2:--steps_20_--warmup_5
