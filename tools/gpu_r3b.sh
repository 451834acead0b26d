#!/bin/bash
# Round-3 session B: the phase-B kernel variants against the oracle (selection boundaries
# first), then the large-m bench lines with each phase-B kernel on one box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py -m gpu -x -v --timeout 300 --timeout-method thread -k "phase_b or selection" > "$OUT/pytest_pb.txt" 2>&1 || { tail -40 "$OUT/pytest_pb.txt"; exit 1; }
tail -1 "$OUT/pytest_pb.txt"
for cfg in k128m32 k200m56; do
  for jp in 4 5 9 4 5 9; do
    LONGHAIR_AMD_INV_JUMP=$jp timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$jp.json" 2> "$OUT/b_${cfg}_$jp.err" || { tail -20 "$OUT/b_${cfg}_$jp.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b_${cfg}_$jp.json')); print('$cfg jp=$jp', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['kernels']['decode']['kernel'])" | tee -a "$OUT/summary.txt"
  done
done
