#!/bin/bash
# Round-3 session P: fused k29/m4 decode with per-word phase-A pins (162 -> 157 VGPRs, 3
# waves/SIMD again) and recovery rows read first (tools/ubench_decode.hip); full GPU suite,
# interleaved A/B against the previous column order / pin style, bench line + kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
TUNE_VARIANTS="rf0=LONGHAIR_AMD_JIT_DEFINES:LH_REC_FIRST=0|old=LONGHAIR_AMD_JIT_DEFINES:LH_REC_FIRST=0,LH_PIN_WORDS=0|pw0=LONGHAIR_AMD_JIT_DEFINES:LH_PIN_WORDS=0" \
  timeout -k 10 400 python -u tools/tune.py > "$OUT/tune.txt" 2> "$OUT/tune.err" || { tail -20 "$OUT/tune.err"; exit 1; }
cat "$OUT/tune.txt"
timeout -k 10 300 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
cat "$OUT/bench_k29m4.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/k29m4_kernel_stats.csv" \;
head -8 "$OUT/k29m4_kernel_stats.csv"
# PCIe-inclusive decode with the rows / status moved once per call: chunk sweep
for c in 0 2048 4096; do
  PCIE_CHUNK=$c timeout -k 10 200 python tools/pcie_bench.py k29m4 >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
for c in 0 8 16; do
  PCIE_CHUNK=$c timeout -k 10 200 python tools/pcie_bench.py k200m56 >> "$OUT/pcie.json" 2>> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
done
cut -c1-300 "$OUT/pcie.json"
