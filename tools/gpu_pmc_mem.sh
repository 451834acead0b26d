#!/bin/bash
# Memory-pipeline counter passes (one rocprofv3 --pmc run per block group) for the bench
# kernels of a config: L2 hits / misses / HBM requests, L1 accesses and L1->L2 requests,
# TA busy, plus the wave wait/issue breakdown.  Usage: tools/gpu_pmc_mem.sh OUT [config]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-pmc_mem}; CFG=${2:-k29m4}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
i=0
while read -r counters; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --kernel-trace -d "$OUT/p$i" -o run --output-format csv -- python3 tools/prof_kernels.py $CFG > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($counters) failed"; tail -5 "$OUT/p$i.log"; continue; }
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, statistics
vals = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0]
    if n.startswith("lh_"):
        vals.setdefault((n, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
for (n, c), v in sorted(vals.items()):
    print(f"{n:28s} {c:32s} {statistics.median(v):.4g}")
PY
done <<'LIST'
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_TA_BUSY_sum TA_BUSY_avr
SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS
LIST
