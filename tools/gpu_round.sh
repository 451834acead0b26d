#!/bin/bash
# Full GPU session: parity tests, smoke, headline bench + profiles, other configs, PCIe rate.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-round}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1500 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
for cfg in ${CONFIGS:-k128m32 k200m56}; do
  timeout -k 10 600 python bench.py --config $cfg --steps 5 --warmup 2 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  cat "$OUT/bench_$cfg.json"
done
timeout -k 10 600 python tools/pcie_bench.py k29m4 k200m56 > "$OUT/pcie.json" 2> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
cat "$OUT/pcie.json"
