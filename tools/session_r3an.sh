#!/usr/bin/env bash
# round-3 GPU session an: SQ instruction counters of the final library's one-wave-per-env
# kernel at 64x64/R32 (per-env VALU / SALU / LDS after this round's changes)
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
CTR="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace -f csv -d $OUT/sqn_g64r32_r3an -o run -- \
  python3 bench.py --grid 64 --rays 64 --range 32 --steps 20 --warmup 5 --desync-steps 0 --gather-steps 0 --no-cpu-baseline \
  > $OUT/sqn_g64r32_r3an.json 2> $OUT/sqn_g64r32_r3an.err
echo sq done
