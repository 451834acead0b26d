#!/bin/bash
# Round-3 session F2: per-kernel times (rocprofv3 kernel trace + stats) of the three bench
# configs, HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) and SQ passes (issue /
# wait breakdown; a second pass with the scalar / LDS instruction counts), the available
# counter list.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3f2}
PART=${2:-all}   # a: kernel stats + large-m PMC/SQ; b: k29m4 PMC/SQ, scalar SQ pass, PCIe timeline
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PART" != b ]; then
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" "$OUT/avail.txt" | sort -u | tr '\n' ' ' > "$OUT/sq_names.txt"; head -c 3000 "$OUT/sq_names.txt"; echo
for cfg in k29m4 k128m32 k200m56; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/stats_$cfg.log" 2>&1 || { tail -20 "$OUT/stats_$cfg.log"; exit 1; }
  find "$OUT/stats_$cfg" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-160
done
fi
CFGS="k128m32 k200m56 k29m4"; [ "$PART" = a ] && CFGS="k128m32 k200m56"; [ "$PART" = b ] && CFGS="k29m4"
for cfg in $CFGS; do
  mkdir -p "$OUT/pmc_$cfg"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/fetch.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/fetch.log"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/write.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/write.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$cfg" $cfg > "$OUT/pmc_$cfg/summary.json" && grep -A6 '"decode": {' "$OUT/pmc_$cfg/summary.json" | head -8
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d "$OUT/sq_$cfg" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/sq_$cfg.log" 2>&1 || { tail -20 "$OUT/sq_$cfg.log"; exit 1; }
  python3 tools/sq_summary.py "$(find "$OUT/sq_$cfg" -name '*counter_collection.csv' | head -1)" $cfg > "$OUT/sq_$cfg.json" || exit 1
done
[ "$PART" = a ] && exit 0
# scalar / LDS issue of the large-m kernels (names checked against the available list)
[ -f "$OUT/sq_names.txt" ] || { timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true; grep -oE "SQ_[A-Z0-9_]+" "$OUT/avail.txt" | sort -u | tr '\n' ' ' > "$OUT/sq_names.txt"; }
want="SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES"
have=""; for c in $want; do grep -qw "$c" "$OUT/sq_names.txt" && have="$have $c"; done
echo "SQ pass 2:$have"
if [ -n "$have" ]; then
  timeout -s KILL 240 rocprofv3 --pmc $have --kernel-trace -d "$OUT/sq2_k128m32" -o run --output-format csv -- python3 tools/prof_kernels.py k128m32 > "$OUT/sq2_k128m32.log" 2>&1 || { tail -20 "$OUT/sq2_k128m32.log"; exit 1; }
  python3 tools/sq_summary.py "$(find "$OUT/sq2_k128m32" -name '*counter_collection.csv' | head -1)" k128m32_scalar > "$OUT/sq2_k128m32.json" || exit 1
fi
# pinned-host pipeline timeline (kernel + memory-copy trace, no counters)
timeout -k 10 300 python tools/pcie_bench.py k29m4 > "$OUT/pcie.json" 2> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
cut -c1-300 "$OUT/pcie.json"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/pcie_prof" -o run --output-format csv -- python3 tools/pcie_bench.py k29m4 > "$OUT/pcie_prof.log" 2>&1 || { tail -20 "$OUT/pcie_prof.log"; exit 1; }
find "$OUT/pcie_prof" -name "*.csv" | head
