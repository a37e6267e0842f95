#!/usr/bin/env bash
# round-3 GPU session w: issue-side SQ counters of the one-wave-per-env kernel
# (64x64 / C64 / R32) and of the headline sector kernel: which instruction class
# holds the SIMDs (cycles per class, not instruction counts)
set -euo pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace -f csv -d $OUT/sqi_g64r32 -o run -- \
  python3 bench.py --grid 64 --rays 64 --range 32 --steps 20 --warmup 5 --desync-steps 0 --gather-steps 0 --no-cpu-baseline > $OUT/sqi_g64r32.json 2> $OUT/sqi_g64r32.err
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-trace -f csv -d $OUT/sqi_head -o run -- \
  python3 bench.py --steps 50 --warmup 10 --desync-steps 0 --gather-steps 0 --no-cpu-baseline > $OUT/sqi_head.json 2> $OUT/sqi_head.err
CTR2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $CTR2 --kernel-trace -f csv -d $OUT/sqn_g64r32 -o run -- \
  python3 bench.py --grid 64 --rays 64 --range 32 --steps 20 --warmup 5 --desync-steps 0 --gather-steps 0 --no-cpu-baseline > $OUT/sqn_g64r32.json 2> $OUT/sqn_g64r32.err
echo sq done
# the one-wave-per-env kernel with its aligned-window offsets from pe_create and 16-B
# obs row stores (wv1) vs HEAD (base): wave parity first
A=build/ab/lib_base.so; B=build/ab/lib_wv1.so
PLANTOS_HIP_LIB=$B timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_geometry_sweep.py tests/test_gpu_parity.py tests/test_gpu_coop_reset.py tests/test_gpu_curriculum_autoreset.py > $OUT/r3w_tests.log 2>&1
tail -2 $OUT/r3w_tests.log
bash tools/ab_bench.sh r3w_g64r32 3 $A $B -- --grid 64 --rays 64 --range 32 --steps 1000 --warmup 50 --desync-steps 0 --gather-steps 0 > /dev/null
bash tools/ab_bench.sh r3w_g8r20 2 $A $B -- --grid 8 --rays 16 --range 20 --plants 4 --obstacles 3 --steps 2000 --warmup 100 --desync-steps 0 --gather-steps 0 > /dev/null
echo ab done
