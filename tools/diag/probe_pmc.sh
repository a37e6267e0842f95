#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE passes (separate rocprofv3 runs, MI355X_MICROARCH.md) of the
# headline bench over several libraries (timing / traffic probes built by
# tools/ab_build.sh).   usage: bash tools/diag/probe_pmc.sh TAG lib1 lib2 ... [-- bench args]
set -euo pipefail
TAG=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
ARGS=${*:---steps 50 --warmup 10 --desync-steps 0 --gather-steps 0 --no-cpu-baseline}
export TMPDIR=/tmp
for L in "${LIBS[@]}"; do
  n=$(basename "$L" .so)
  export PLANTOS_HIP_LIB=$L
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -f csv -d gpurun_out/pp_${TAG}_${n}_$c -o run -- \
      python3 bench.py $ARGS > gpurun_out/pp_${TAG}_${n}_$c.json 2> gpurun_out/pp_${TAG}_${n}_$c.err
  done
  echo "$n done"
done
unset PLANTOS_HIP_LIB
