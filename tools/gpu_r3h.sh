#!/bin/bash
# Round-3 session H: rows per wave of the windowed large-m ENCODE (LONGHAIR_AMD_WIN_ROWS_ENC),
# the decode's phase A unchanged; one box, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3h}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  run enc16 k128m32
  run enc8 k128m32 LONGHAIR_AMD_WIN_ROWS_ENC=8
  run enc11 k128m32 LONGHAIR_AMD_WIN_ROWS_ENC=11
  run enc14 k200m56
  run enc11 k200m56 LONGHAIR_AMD_WIN_ROWS_ENC=11
  run enc19 k200m56 LONGHAIR_AMD_WIN_ROWS_ENC=19
done
