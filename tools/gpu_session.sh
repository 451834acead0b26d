#!/bin/bash
# One GPU session: parity tests, smoke, the BASELINE benches, a kernel-trace profile of
# every bench config and the PCIe-inclusive rate.  Every GPU step has its own time limit;
# the chain stops at the first failure.  Usage: tools/gpu_session.sh OUT_NAME [skip-tests]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -3 "$OUT/pytest_gpu.txt"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
  cat "$OUT/smoke.txt"
fi
timeout -k 10 300 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
cat "$OUT/bench_k29m4.json"
for cfg in ${CONFIGS:-k128m32 k200m56}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  cat "$OUT/bench_$cfg.json"
done
for cfg in k29m4 ${CONFIGS:-k128m32 k200m56}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline off > "$OUT/prof_$cfg.log" 2>&1 || { tail -20 "$OUT/prof_$cfg.log"; exit 1; }
  find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-160
done
for cfg in k29m4 ${CONFIGS:-k128m32 k200m56}; do
  mkdir -p "$OUT/pmc_$cfg"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/fetch.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/fetch.log"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/write.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/write.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$cfg" $cfg > "$OUT/pmc_$cfg/summary.json" || exit 1
  grep -E '"(kernel|ratio_to_algorithmic)"' "$OUT/pmc_$cfg/summary.json"
done
timeout -k 10 600 python tools/pcie_bench.py k29m4 k200m56 > "$OUT/pcie.json" 2> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
cat "$OUT/pcie.json"
