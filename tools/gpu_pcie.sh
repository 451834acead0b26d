#!/bin/bash
# Pinned-host pipeline: parity tests of the host batches, then PCIe-inclusive rates
# (auto chunk) with the write-back kernel and with the range copy, recovery blocks last
# and shuffled.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-pcie}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "host_batch or configs" > "$OUT/pytest_host.txt" 2>&1 || { tail -30 "$OUT/pytest_host.txt"; exit 1; }
tail -2 "$OUT/pytest_host.txt"
for sh in 1 0; do
  for wb in ${WRITEBACKS:-kernel range}; do
    PCIE_SHUFFLE=$sh LONGHAIR_AMD_PIPE_WRITEBACK=$wb timeout -k 10 300 python tools/pcie_bench.py k29m4 k200m56 >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
  done
done
cut -c1-300 "$OUT/pcie.json"
