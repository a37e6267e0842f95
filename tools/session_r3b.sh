#!/usr/bin/env bash
# round-3 GPU session b: small-batch shapes (A/B over envs per workgroup), stamps at
# 4096 / 65536 envs, the timed window's fixed cost, the driver-shaped bench, tests
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
K=build/ab/lib_knobs2.so
timeout -k 10 120 python tools/diag/window_overhead.py > $OUT/window_r3b.json 2> $OUT/window_r3b.err
echo window done
timeout -k 10 180 python tools/stamps.py run --envs 4096 > $OUT/stamps4096_r3b.json 2> $OUT/stamps4096_r3b.err
timeout -k 10 180 python tools/stamps.py run --envs 4096 --desync > $OUT/stamps4096d_r3b.json 2> $OUT/stamps4096d_r3b.err
timeout -k 10 180 python tools/stamps.py run --desync > $OUT/stampsd_r3b.json 2> $OUT/stampsd_r3b.err
echo stamps done
bash tools/ab_bench.sh epb4096_r3b 3 $K,PE_QUAD_EPB=16 $K,PE_QUAD_EPB=32 $K,PE_QUAD_EPB=64 $K,PE_QUAD_WAVES=8 \
  -- --envs 4096 --steps 20000 --warmup 1000 --desync-steps 20000 --gather-steps 0 > /dev/null
for n in 8192 16384 32768; do
  bash tools/ab_bench.sh epb${n}_r3b 2 $K,PE_QUAD_EPB=16 $K,PE_QUAD_EPB=32 $K,PE_QUAD_EPB=64 \
    -- --envs $n --steps 20000 --warmup 1000 --desync-steps 20000 --gather-steps 0 > /dev/null
done
echo ab done
bash tools/gpu_session.sh r3b benchx:drv:--steps_20_--warmup_5 benchx:n4096:--envs_4096_--steps_20000_--warmup_1000_--desync-steps_20000_--no-cpu-baseline tests
