#!/bin/bash
# GPU parity suite, k29m4 decode load-policy A/B, pinned-host pipeline rates.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r2c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
TUNE_VARIANTS="${VARIANTS:-nt2=LONGHAIR_AMD_JIT_DEFINES:LH_NT_DEC=2}" timeout -k 10 300 python tools/tune.py > "$OUT/tune_k29m4.txt" 2>&1 || { tail -20 "$OUT/tune_k29m4.txt"; exit 1; }
cat "$OUT/tune_k29m4.txt"
for sh in 1 0; do
  PCIE_SHUFFLE=$sh timeout -k 10 300 python tools/pcie_bench.py k29m4 k200m56 >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
cut -c1-300 "$OUT/pcie.json"
