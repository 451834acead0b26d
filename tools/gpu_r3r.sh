#!/bin/bash
# Round-3 session R: profile refresh after the fused-decode and phase-B default changes
# (kernel stats, HBM PMC and SQ passes of the three configs, scalar SQ pass, PCIe timeline:
# tools/gpu_r3f2.sh), then the GPU drop-in call under the kernel + copy tracer.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3r}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/dropin" -o run --output-format csv -- python3 tools/dropin_probe.py 300 > "$OUT/dropin.txt" 2>&1 || { tail -20 "$OUT/dropin.txt"; exit 1; }
tail -2 "$OUT/dropin.txt"
bash tools/gpu_r3f2.sh "$(basename "$OUT")"
