#!/bin/bash
# Round-3 session A: GPU parity suite (new selection-boundary tests, sweep), smoke, the
# default bench line (k29m4, with the PCIe, drop-in and CPU-baseline legs).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
cut -c1-600 "$OUT/bench_k29m4.json"
