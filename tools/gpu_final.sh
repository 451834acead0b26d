#!/bin/bash
# Round-end style session: GPU parity suite, smoke, the driver's default bench line (k29m4),
# its rocprofv3 kernel stats, and the k29m4 HBM PMC + SQ passes the bench line cites.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
cut -c1-1200 "$OUT/bench_k29m4.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_k29m4" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --dropin-calls 0 > "$OUT/prof_k29m4.log" 2>&1 || { tail -20 "$OUT/prof_k29m4.log"; exit 1; }
find "$OUT/prof_k29m4" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-150
CONFIGS=k29m4 bash tools/gpu_large_refresh_pmc.sh "$1" || exit 1
