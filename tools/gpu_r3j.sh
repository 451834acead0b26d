#!/bin/bash
# Round-3 session J: parity of the new phase-B default (selection boundaries, variants),
# then the remaining profiling (k29m4 PMC / SQ, scalar SQ pass, PCIe timeline).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
bash tools/gpu_r3f2.sh "${1:-r3j}" b
