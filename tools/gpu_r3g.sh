#!/bin/bash
# Round-3 session G: k29m4 with the decode buffer's recovery slots 128-byte aligned (padded
# stripe stride) against the contiguous layout, alternating on one box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3g}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for al in 0 128 64 32; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --align $al --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_$al.json" 2> "$OUT/b_$al.err" || { tail -20 "$OUT/b_$al.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/b_$al.json')); print('align $al stride', d['config']['decode_buffer_stripe_stride'], d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'])" | tee -a "$OUT/summary.txt"
  done
done
