#!/bin/bash
# Round-3 session AC: phase B with 4 outputs per wave (LONGHAIR_AMD_INV_GTW=4, knob):
# parity of the phase-B variants plus the full suite, then large-m bench lines against the
# 8-output default (more waves per SIMD: AB showed phase B short of latency hiding).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3ac}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['kernels']['decode']['kernel'].split('+')[-1])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for cfg in k128m32 k200m56; do
    run base $cfg
    run gtq4 $cfg LONGHAIR_AMD_INV_GTW=4
  done
done
