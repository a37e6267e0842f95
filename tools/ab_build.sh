#!/usr/bin/env bash
# Build libplantos_hip.so of a git revision (default HEAD) into build/ab/lib_<name>.so
# for same-box A/B timing (PLANTOS_HIP_LIB=... python bench.py).
#   usage: [EXTRA_FLAGS=-D...] [PATCH_PY=script run in the source copy] bash tools/ab_build.sh NAME [REV|WORKTREE]
set -euo pipefail
NAME=$1
REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$ROOT/build/ab/src_$NAME
rm -rf "$SRC" && mkdir -p "$SRC"
if [ "$REV" = WORKTREE ]; then
  mkdir -p "$SRC/rl-env_amd" "$SRC/tools/diag" && cp -r "$ROOT/rl-env_amd/csrc" "$SRC/rl-env_amd/" && cp -r "$ROOT/include" "$SRC/"
  cp "$ROOT/tools/diag/pe_pipe.hpp" "$SRC/tools/diag/"  # (the debug-only pipelined kernel)
else
  git -C "$ROOT" archive "$REV" rl-env_amd/csrc include | tar -x -C "$SRC"
  git -C "$ROOT" archive "$REV" tools/diag 2>/dev/null | tar -x -C "$SRC" || true
fi
if [ -n "${PATCH_PY:-}" ]; then (cd "$SRC" && python3 "$PATCH_PY"); fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -w -DPE_DEBUG_KNOBS ${EXTRA_FLAGS:-} \
  -o "$ROOT/build/ab/lib_$NAME.so" "$SRC/rl-env_amd/csrc/plantos_batch.hip" \
  "$SRC/rl-env_amd/csrc/pe_mcts.hip" "$SRC/rl-env_amd/csrc/pe_pystream.cpp"
echo "$ROOT/build/ab/lib_$NAME.so"
