#!/usr/bin/env bash
# The hipcc register-reuse hazard of round 5 ("A compiler hazard"):
# with the compact grid mirror's fields added to State / Geo, the C64 byte-tile kernel put
# the hoisted `h = r_invalid` (a move into an obstacle) in the VGPRs it then loaded the
# target's window row into, so the reward came out -0.1 instead of -5.1.
#   CPU:  bash tools/diag/regreuse/repro.sh build   -> build/ab/lib_gridc.so + its C64 ISA excerpt
#   GPU:  bash tools/diag/regreuse/repro.sh run     -> tools/diag/g64_diag.py against the oracle
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../../.." && pwd)
case ${1:-build} in
  build)
    # the diff applies at HEAD too, but reproduces only on the source it was written against
    # (round 6: HEAD + the diff compiles correctly -- the hazard is a property of the exact
    # register allocation, not of the mirror's source)
    PATCH_PY=$ROOT/tools/diag/regreuse/apply_gridc.py bash "$ROOT/tools/ab_build.sh" gridc ${2:-ba3974a}
    python3 "$ROOT/tools/diag/regreuse/isa_excerpt.py" "$ROOT/build/ab/lib_gridc.so" ;;
  run)
    PLANTOS_HIP_LIB=$ROOT/build/ab/lib_gridc.so timeout -k 10 120 python3 "$ROOT/tools/diag/g64_diag.py" ;;
esac
