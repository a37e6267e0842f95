#!/usr/bin/env bash
# round-6 final pass y, call 2: rocprof kernel stats of every geometry and the FETCH / WRITE PMC
# passes (tools/measure_pass2.sh)
set -euo pipefail
bash tools/measure_pass2.sh r6y
echo y2 done
