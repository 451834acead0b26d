#!/bin/bash
# Round-3 session AA: split-decode phase A reading R_r with the default cache policy before
# storing V_r over it (LH_NT_R=0; the in-place access-pattern benchmark favours default-
# policy loads with non-temporal stores), against the non-temporal default; parity first.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
LONGHAIR_AMD_JIT_DEFINES=LH_NT_R=0 LONGHAIR_AMD_JIT_COMPILE=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config4 or config2" > "$OUT/pytest_ntr.txt" 2>&1 || { tail -40 "$OUT/pytest_ntr.txt"; exit 1; }
tail -1 "$OUT/pytest_ntr.txt"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for cfg in k128m32 k200m56; do
    run base $cfg
    run ntr0 $cfg LONGHAIR_AMD_JIT_DEFINES=LH_NT_R=0
  done
done
