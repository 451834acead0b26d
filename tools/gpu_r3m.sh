#!/bin/bash
# Round-3 session M: phase B through one table per code object (lh_inverse_gt_kernel):
# parity of every phase-B variant, then large-m bench lines against the default.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py -m gpu -x -q --timeout 300 --timeout-method thread -k "phase_b" > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['kernels']['decode']['kernel'].split('+')[-1])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  for cfg in k128m32 k200m56; do
    run base $cfg
    run gt $cfg LONGHAIR_AMD_INV_JUMP=10
    run gtpack $cfg LONGHAIR_AMD_INV_JUMP=10 LONGHAIR_AMD_INV_PACK=1
  done
done
LONGHAIR_AMD_INV_JUMP=10 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_LDS SQ_WAVES --kernel-trace -d "$OUT/sq_gt" -o run --output-format csv -- python3 tools/prof_kernels.py k128m32 > "$OUT/sq.log" 2>&1 || { tail -20 "$OUT/sq.log"; exit 1; }
python3 tools/sq_summary.py "$(find "$OUT/sq_gt" -name '*counter_collection.csv' | head -1)" k128m32_gt > "$OUT/sq_gt.json" || exit 1
