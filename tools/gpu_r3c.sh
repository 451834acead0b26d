#!/bin/bash
# Round-3 session C: chunked split decode (Infinity Cache reuse of V) and the two-stream
# overlap of phase A / phase B, large-m bench lines on one box.  $2 = phase-B knob.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3c}
mkdir -p "$OUT"
export TMPDIR=/tmp
export LONGHAIR_AMD_INV_JUMP=${2:-4}
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  run whole k128m32 LONGHAIR_AMD_WIDE_CHUNK=0
  for c in 128 256 512 1024; do run c$c k128m32 LONGHAIR_AMD_WIDE_CHUNK=$c; done
  for c in 256 512 1024; do run c${c}ov k128m32 LONGHAIR_AMD_WIDE_CHUNK=$c LONGHAIR_AMD_WIDE_OVERLAP=1; done
  run whole k200m56 LONGHAIR_AMD_WIDE_CHUNK=0
  for c in 8 16 32; do run c$c k200m56 LONGHAIR_AMD_WIDE_CHUNK=$c; done
  for c in 8 16; do run c${c}ov k200m56 LONGHAIR_AMD_WIDE_CHUNK=$c LONGHAIR_AMD_WIDE_OVERLAP=1; done
done
