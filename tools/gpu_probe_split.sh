#!/bin/bash
# Split large-m decode (phase-A kernel + lh_inverse_kernel): GPU parity tests, then
# decode timings of its variants on k128m32 and k200m56 (tools/tune.py checks the bytes).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-split}
mkdir -p "$OUT"
export TMPDIR=/tmp
V="${VARIANTS:-pair=LONGHAIR_AMD_INV_PAIR:1|opw8=LONGHAIR_AMD_INV_OPW:8|opw8pair=LONGHAIR_AMD_INV_OPW:8;LONGHAIR_AMD_INV_PAIR:1}"
if [ "$2" != "skip-tests" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
fi
TUNE_VARIANTS="$V" timeout -k 10 300 python tools/tune.py 128 32 8192 8192 > "$OUT/tune_k128.txt" 2>&1 || { tail -20 "$OUT/tune_k128.txt"; exit 1; }
cat "$OUT/tune_k128.txt"
TUNE_VARIANTS="$V" timeout -k 10 300 python tools/tune.py 200 56 65536 64 > "$OUT/tune_k200.txt" 2>&1 || { tail -20 "$OUT/tune_k200.txt"; exit 1; }
cat "$OUT/tune_k200.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_k128m32" -o run --output-format csv -- python3 bench.py --config k128m32 --steps 5 --warmup 2 --cpu-baseline off --dropin-calls 0 > "$OUT/prof_k128m32.log" 2>&1 || { tail -20 "$OUT/prof_k128m32.log"; exit 1; }
find "$OUT/prof_k128m32" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-150
