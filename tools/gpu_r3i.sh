#!/bin/bash
# Round-3 session I: phase B with V staged by LDS-DMA (double-buffered tiles) -- parity of
# every phase-B variant, then the large-m bench lines against the register-staged kernels.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3i}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py -m gpu -x -v --timeout 300 --timeout-method thread -k "phase_b or jump or wide" > "$OUT/pytest_pb.txt" 2>&1 || { tail -40 "$OUT/pytest_pb.txt"; exit 1; }
tail -1 "$OUT/pytest_pb.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['kernels']['decode']['kernel'].split('+')[-1])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  run base k128m32
  run dma8 k128m32 LONGHAIR_AMD_INV_DMA=8
  run dma16 k128m32 LONGHAIR_AMD_INV_DMA=16
  run base k200m56
  run dma8 k200m56 LONGHAIR_AMD_INV_DMA=8
  run dma16 k200m56 LONGHAIR_AMD_INV_DMA=16
  run dma8ji k200m56 LONGHAIR_AMD_INV_DMA=8 LONGHAIR_AMD_INV_JUMP=9
done
