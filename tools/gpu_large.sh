#!/bin/bash
# Large-m session: parity tests, windowed-kernel tune, kernel-trace profiles and HBM PMC
# passes (FETCH_SIZE / WRITE_SIZE, separate runs) for the k128m32 and k200m56 configs.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-large}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -2 "$OUT/pytest_gpu.txt"
fi
timeout -k 10 400 python tools/tune.py 128 32 8192 8192 > "$OUT/tune_k128m32.txt" 2> "$OUT/tune_k128m32.err" || { tail -20 "$OUT/tune_k128m32.err"; exit 1; }
cat "$OUT/tune_k128m32.txt"
for cfg in k128m32 k200m56; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline off > "$OUT/prof_$cfg.log" 2>&1 || { tail -20 "$OUT/prof_$cfg.log"; exit 1; }
  find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-120
  mkdir -p "$OUT/pmc_$cfg"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/fetch.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/fetch.log"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/write.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/write.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$cfg" $cfg > "$OUT/pmc_$cfg/summary.json" && grep -A4 '"encode": {\|"decode": {' "$OUT/pmc_$cfg/summary.json" | head -14
done
