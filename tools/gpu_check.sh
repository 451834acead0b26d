#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.  Each GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -3 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \;
