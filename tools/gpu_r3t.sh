#!/bin/bash
# Round-3 session T: windowed kernels with a private LDS ring per wave (no workgroup barrier
# per column, LONGHAIR_AMD_WIN_LDS=2): parity at configs[2] / configs[4], then large-m bench
# lines against the shared ring.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3t}
mkdir -p "$OUT"
export TMPDIR=/tmp
LONGHAIR_AMD_WIN_LDS=2 LONGHAIR_AMD_JIT_COMPILE=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config4 or config2" > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for cfg in k128m32 k200m56; do
    run base $cfg
    run priv $cfg LONGHAIR_AMD_WIN_LDS=2
  done
done
