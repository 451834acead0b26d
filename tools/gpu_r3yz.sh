#!/bin/bash
# Sessions Y + Z in one call (the pool was busy): bench line after the per-call timing
# change, then the k29/m4 decode knob A/B.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_r3y.sh r3y && bash tools/gpu_r3z.sh r3z
