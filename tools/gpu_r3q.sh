#!/bin/bash
# Round-3 session Q: full GPU suite; phase-B default = lh_inverse_gt_kernel (packed for
# e_max <= 32) against the previous default (LONGHAIR_AMD_INV_JUMP=9); the pipelined host
# batches with halving tail chunks; k29/m4 pin styles again (more rounds).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3q}
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
    run dma9 $cfg LONGHAIR_AMD_INV_JUMP=9
  done
done
for c in k29m4 k200m56; do
  timeout -k 10 200 python tools/pcie_bench.py $c >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
cut -c1-300 "$OUT/pcie.json"
TUNE_VARIANTS="pw0=LONGHAIR_AMD_JIT_DEFINES:LH_PIN_WORDS=0|b2=|pw0b=LONGHAIR_AMD_JIT_DEFINES:LH_PIN_WORDS=0" \
  timeout -k 10 400 python -u tools/tune.py > "$OUT/tune.txt" 2> "$OUT/tune.err" || { tail -20 "$OUT/tune.err"; exit 1; }
cat "$OUT/tune.txt"
