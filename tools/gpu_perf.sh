#!/bin/bash
# Perf session: microbenchmarks, bench, kernel-trace profile and PMC traffic passes.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-perf}
CFG=${2:-k29m4}
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/ub tools/ubench_loads.hip 2>/dev/null && timeout -k 10 120 /tmp/ub > "$OUT/ubench.txt" 2>&1 || { cat "$OUT/ubench.txt"; exit 1; }
cat "$OUT/ubench.txt"
timeout -k 10 300 python bench.py --config $CFG > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --config $CFG --steps 10 --warmup 2 --cpu-baseline off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py $CFG > "$OUT/pmc_fetch.log" 2>&1 || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py $CFG > "$OUT/pmc_write.log" 2>&1 || { tail -20 "$OUT/pmc_write.log"; exit 1; }
python3 tools/pmc_summary.py "$OUT" $CFG > "$OUT/pmc_summary.json" && cat "$OUT/pmc_summary.json"
find "$OUT/prof" -name "*kernel_stats.csv" -exec grep -E "lh_|Name" {} \;
