set -e
export TMPDIR=/tmp
for L in nop tree; do
  if [ $L = tree ]; then unset PLANTOS_HIP_LIB; else export PLANTOS_HIP_LIB=build/ab/lib_$L.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-trace -f csv -d gpurun_out/sqab_$L -o run -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/sqab_$L.json 2> gpurun_out/sqab_$L.err
done
