#!/bin/bash
# Round-3 session O: decode access-pattern floor with the slot map in registers
# (tools/ubench_decode.hip), then session N's chained phase-B comparison.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench_decode > "$OUT/ubench_decode.txt" 2>&1 || { echo "ubench failed"; cat "$OUT/ubench_decode.txt"; exit 1; }
cat "$OUT/ubench_decode.txt"
bash tools/gpu_r3n.sh "$(basename "$OUT")"
