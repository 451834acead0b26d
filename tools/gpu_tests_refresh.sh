#!/bin/bash
# GPU parity suite, then the large-m refresh (bench, kernel stats, PMC, SQ) for $CONFIGS.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-tr}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
bash tools/gpu_large_refresh.sh "$1"
