#!/bin/bash
# Round-3 session L: GPR-indexing readlane probe; host-batch pipeline chunk sweep now that
# the decode pipeline no longer serialises on its status copies.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 tools/probes/gpr_idx_readlane > "$OUT/probe.txt" 2>&1; echo "probe rc=$?" >> "$OUT/probe.txt"
cat "$OUT/probe.txt"
for c in 0 1024 2048 4096; do
  PCIE_CHUNK=$c timeout -k 10 300 python tools/pcie_bench.py k29m4 >> "$OUT/pcie_sweep.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
for c in 0 4 8; do
  PCIE_CHUNK=$c timeout -k 10 300 python tools/pcie_bench.py k200m56 >> "$OUT/pcie_sweep.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/pcie_sweep.json'):
    d=json.loads(l); print(d['config'], d.get('chunk_stripes'), d['encode_GBps_pcie_inclusive'], d['decode_GBps_pcie_inclusive'])"
