#!/usr/bin/env bash
# round-6 final pass y, call 3: rocprof kernel stats of the desynchronized steady state of every
# geometry (tools/measure_desync.sh)
set -euo pipefail
bash tools/measure_desync.sh r6y
echo y3 done
