#!/bin/bash
# Round-3 session S: pipelined host batches with the next chunk's copy enqueued before the
# current chunk's kernels (parity + PCIe rates + copy timeline); decode store-policy
# variants of the access-pattern benchmark.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/ubench_decode > "$OUT/ubench_decode.txt" 2>&1 || { echo "ubench failed"; cat "$OUT/ubench_decode.txt"; exit 1; }
cat "$OUT/ubench_decode.txt"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "host" > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2; do
  for c in k29m4 k200m56; do
    timeout -k 10 200 python tools/pcie_bench.py $c >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
  done
done
cut -c1-300 "$OUT/pcie.json"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/pcie_prof" -o run --output-format csv -- python3 tools/pcie_bench.py k29m4 > "$OUT/pcie_prof.log" 2>&1 || { tail -20 "$OUT/pcie_prof.log"; exit 1; }
