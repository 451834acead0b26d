#!/bin/bash
# Round-3 session V: write-back kernel split over block segments for chunks of few large
# stripes; host-batch parity and PCIe-inclusive rates.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "host or config4" > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for rep in 1 2; do
  for c in k200m56 k29m4; do
    timeout -k 10 200 python tools/pcie_bench.py $c >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
  done
done
cut -c1-300 "$OUT/pcie.json"
# Partial-round tail of the k29/m4 kernels: time per stripe at stripe counts that fill
# whole rounds of waves (decode: 3 072 slots x 3 stripes; encode: 4 096 slots x 3) or not.
for s in 55296 64512 65536 73728; do
  TUNE_VARIANTS="b2=" timeout -k 10 300 python -u tools/tune.py 29 4 1296 $s > "$OUT/tune_$s.txt" 2> "$OUT/tune_$s.err" || { tail -20 "$OUT/tune_$s.err"; exit 1; }
  grep -E "^base|^b2" "$OUT/tune_$s.txt" | sed "s/^/$s /"
done
