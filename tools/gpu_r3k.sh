#!/bin/bash
# Round-3 session K: leaner indexed jump (s_swappc, GPR index kept on across outputs) and the
# pinned staging of the decode pipeline's rows / status: parity (phase B, boundaries,
# host-batch pipeline), large-m bench lines, scalar counters, PCIe-inclusive rates.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_boundaries.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "phase_b or selection or wide or host_batch or chunks" > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
run() {  # name cfg env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/b_${cfg}_$name.json" 2> "$OUT/b_${cfg}_$name.err" || { tail -20 "$OUT/b_${cfg}_$name.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/b_${cfg}_$name.json')); print('$cfg $name', d['value'], d['kernels']['encode']['ms'], d['kernels']['decode']['ms'], d['kernels']['decode']['kernel'].split('+')[-1])" | tee -a "$OUT/summary.txt"
}
for rep in 1 2; do
  run dma8 k128m32
  run dma8 k200m56
done
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_LDS SQ_WAVES --kernel-trace -d "$OUT/sq3_k128m32" -o run --output-format csv -- python3 tools/prof_kernels.py k128m32 > "$OUT/sq3.log" 2>&1 || { tail -20 "$OUT/sq3.log"; exit 1; }
python3 tools/sq_summary.py "$(find "$OUT/sq3_k128m32" -name '*counter_collection.csv' | head -1)" k128m32_r3k > "$OUT/sq3_k128m32.json" || exit 1
for sh in 0 1; do
  PCIE_SHUFFLE=$sh timeout -k 10 300 python tools/pcie_bench.py k29m4 k200m56 >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
cut -c1-200 "$OUT/pcie.json"
