#!/bin/bash
# Round-2 closing session: GPU parity suite, smoke, the three bench lines (driver defaults
# for k29m4), kernel stats of each bench, PCIe-inclusive rates.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r2final}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
for cfg in k29m4 k128m32 k200m56; do
  timeout -k 10 600 python bench.py --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  cut -c1-400 "$OUT/bench_$cfg.json"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 > "$OUT/prof_$cfg.log" 2>&1 || { tail -20 "$OUT/prof_$cfg.log"; exit 1; }
  find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-120
done
for sh in 1 0; do
  PCIE_SHUFFLE=$sh timeout -k 10 300 python tools/pcie_bench.py k29m4 k200m56 >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
cut -c1-200 "$OUT/pcie.json"
