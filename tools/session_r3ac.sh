#!/usr/bin/env bash
# round-3 GPU session ac: the measurement pass of the product library (lib 31af7a2b:
# session ab's with the aligned-window table in the ldxy slot: the headline kernel's code
# is HEAD's again) -- the GPU suite, a same-box A/B against HEAD's library, then bench lines, rocprof kernel
# stats and FETCH / WRITE PMC passes as in session l
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_session.sh r3ac tests
tail -n 1 $OUT/tests_r3ac.log
A=build/ab/lib_base.so; B=tree
bash tools/ab_bench.sh r3ac_g8r20 2 $A $B -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3ac_head 2 $A $B -- --steps 4096 --warmup 200 --desync-steps 4096 --gather-steps 0 > /dev/null
T=r3ac
bash tools/gpu_session.sh $T smoke bench benchx:drv:--steps_20_--warmup_5 bench64 \
  benchx:n4096:--envs_4096_--steps_20000_--warmup_1000_--desync-steps_20000_--cpu-seconds_5 \
  benchx:g25:--grid_25_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g21:--grid_21_--rays_10_--range_2_--plants_8_--obstacles_50_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g15:--grid_15_--rays_16_--range_4_--plants_6_--obstacles_8_--steps_20000_--warmup_1000_--cpu-seconds_5 \
  benchx:g32:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_4000_--warmup_200_--desync-steps_4000_--cpu-seconds_5 \
  benchx:g64r32:--grid_64_--rays_64_--range_32_--steps_2000_--warmup_100_--desync-steps_2000_--cpu-seconds_5 \
  benchx:g40c48:--grid_40_--rays_48_--range_8_--steps_2000_--warmup_100_--desync-steps_2000_--cpu-seconds_5 \
  stats statsd stats64 \
  statsx:n4096:--envs_4096_--steps_4096_--warmup_200_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g25:--grid_25_--steps_4096_--warmup_200_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g32:--grid_32_--rays_24_--range_9_--plants_20_--obstacles_30_--steps_2000_--warmup_100_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  statsx:g64r32:--grid_64_--rays_64_--range_32_--steps_1000_--warmup_50_--desync-steps_0_--gather-steps_0_--no-cpu-baseline \
  pmcf pmcw pmcf64 pmcw64 pmcx:g25:FETCH_SIZE:--grid_25 pmcx:g25:WRITE_SIZE:--grid_25 \
  pmcx:n4096:FETCH_SIZE:--envs_4096 pmcx:n4096:WRITE_SIZE:--envs_4096 \
  pmcx:g64r32:FETCH_SIZE:--grid_64_--rays_64_--range_32 pmcx:g64r32:WRITE_SIZE:--grid_64_--rays_64_--range_32
CTR2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $CTR2 --kernel-trace -f csv -d $OUT/sqn_g64r32_r3ac -o run -- \
  python3 bench.py --grid 64 --rays 64 --range 32 --steps 20 --warmup 5 --desync-steps 0 --gather-steps 0 --no-cpu-baseline > $OUT/sqn_g64r32_r3ac.json 2> $OUT/sqn_g64r32_r3ac.err
echo sq done
