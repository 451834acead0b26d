#!/bin/bash
# Round-3 session W: fused decode split into whole rounds of resident waves + a tail kernel
# with 3 columns in flight; full GPU suite, interleaved A/B (tail split on / off) at several
# stripe counts, bench line; write-back kernel split over block segments (PCIe rates).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for s in 65536 64512 55296; do
  TUNE_VARIANTS="tail=LONGHAIR_AMD_DEC_TAIL:1|b2=|tail2=LONGHAIR_AMD_DEC_TAIL:1" timeout -k 10 300 python -u tools/tune.py 29 4 1296 $s > "$OUT/tune_$s.txt" 2> "$OUT/tune_$s.err" || { tail -20 "$OUT/tune_$s.err"; exit 1; }
  grep -E "^base|^b2|^tail" "$OUT/tune_$s.txt" | sed "s/^/$s /"
done
LONGHAIR_AMD_DEC_TAIL=1 timeout -k 10 400 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
cut -c1-400 "$OUT/bench_k29m4.json"
for rep in 1 2; do
  for c in k200m56 k29m4; do
    timeout -k 10 200 python tools/pcie_bench.py $c >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
  done
done
cut -c1-300 "$OUT/pcie.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec grep -E '"lh_' {} \; | cut -c1-120
