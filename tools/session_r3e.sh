#!/usr/bin/env bash
# round-3 GPU session e: stamps (desync 65536 / 4096) of the early-record kernel;
# 8 waves x 16 envs vs 4 waves at 2048 / 8192 envs; rocprof of the desync step
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
C=build/ab/lib_knobs6.so
timeout -k 10 180 python tools/stamps.py run --desync > $OUT/stampsd_r3e.json 2> $OUT/stampsd_r3e.err
timeout -k 10 180 python tools/stamps.py run > $OUT/stamps_r3e.json 2> $OUT/stamps_r3e.err
echo stamps done
for n in 2048 8192; do
  bash tools/ab_bench.sh r3e_nw8_$n 3 $C "$C,PE_QUAD_WAVES=8 PE_QUAD_EPB=16" -- --envs $n --steps 20000 --warmup 1000 --desync-steps 20000 --gather-steps 0 > /dev/null
done
echo ab done
bash tools/gpu_session.sh r3e statsd
