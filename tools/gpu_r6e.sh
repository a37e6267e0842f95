#!/usr/bin/env bash
# round-6 session e: the suite on lib_w5 (w4 + the far kernel's info-wave staging), the
# far kernel A/B, phase stamps of the desynchronized multi-word / small-batch / runtime
# kernels with and without the register-staged record
set -euo pipefail
T=r6e
mkdir -p gpurun_out
PLANTOS_HIP_LIB=build/ab/lib_w5.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_w5_$T.log 2>&1
echo "w5 tests done"; tail -n 1 gpurun_out/tests_w5_$T.log
H=build/ab/lib_head.so
W=build/ab/lib_w5.so
GF="--grid_64_--rays_64_--range_32_--steps_1000_--warmup_100_--desync-steps_1000_--gather-steps_0"
bash tools/gpu_session.sh $T "ab:far:2:$H,$W,$W+PE_STAGGER=8:$GF"
S=build/stamps/libplantos_hip_stamps.so
N=build/ab/lib_stamps_nors.so
st() {  # name, lib, args...
  local nm=$1 lib=$2; shift 2
  timeout -k 10 120 python tools/stamps.py run --lib $lib "$@" > gpurun_out/stamps_${nm}_$T.json 2> gpurun_out/stamps_${nm}_$T.err
}
st g25d_rs $S --grid 25 --desync
st g25d_nors $N --grid 25 --desync
st g25s_rs $S --grid 25
st g25s_nors $N --grid 25
st n4096d $S --envs 4096 --epb 16 --waves 8 --desync
st n4096s $S --envs 4096 --epb 16 --waves 8
st g32s $S --grid 32 --rays 24 --range 9
st g64d $S --grid 64 --rays 64 --range 6 --desync
echo all-e done
