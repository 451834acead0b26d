#!/bin/bash
# Round-3: timeline of the pinned-host decode pipeline (kernel + memory-copy trace, no
# counters) to find where the decode leaves the PCIe link idle against the encode.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3pcie}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/pcie_bench.py k29m4 > "$OUT/pcie.json" 2> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
cat "$OUT/pcie.json" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/prof" -o run --output-format csv -- python3 tools/pcie_bench.py k29m4 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*.csv" | head
