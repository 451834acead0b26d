#!/bin/bash
# Round-3 session D: phase-B kernels (next-tile prefetch, indexed single table, 16-row
# tiles above e_max 32) and phase A / encode at 8 rows per wave, large-m bench lines.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py -m gpu -x -v --timeout 300 --timeout-method thread -k "phase_b or selection or chunks" > "$OUT/pytest_pb.txt" 2>&1 || { tail -40 "$OUT/pytest_pb.txt"; exit 1; }
tail -1 "$OUT/pytest_pb.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['kernels']['decode']['kernel'].split('+')[-1])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  run jt_pf0 k128m32 LONGHAIR_AMD_INV_PF=0
  run jt_pf2 k128m32 LONGHAIR_AMD_INV_PF=2
  run ji4_pf2 k128m32 LONGHAIR_AMD_INV_JUMP=5
  run ji8_pf2 k128m32 LONGHAIR_AMD_INV_JUMP=9
  run ji8_pf0 k128m32 LONGHAIR_AMD_INV_JUMP=9 LONGHAIR_AMD_INV_PF=0
  run rows8 k128m32 LONGHAIR_AMD_WIN_ROWS=8
  run jt_all k200m56
  run jt_b16 k200m56 LONGHAIR_AMD_INV_BLK=16
  run ji8_all k200m56 LONGHAIR_AMD_INV_JUMP=9
  run ji8_b16 k200m56 LONGHAIR_AMD_INV_JUMP=9 LONGHAIR_AMD_INV_BLK=16
  run ji4_b16 k200m56 LONGHAIR_AMD_INV_JUMP=5 LONGHAIR_AMD_INV_BLK=16
  run rows8 k200m56 LONGHAIR_AMD_WIN_ROWS=8
done
