#!/bin/bash
# FETCH_SIZE calibration for 4-, 8- and 16-byte lanes (aligned stream reads of a known
# byte count), plus the stripe-pattern microbenchmark timings.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-calib}
mkdir -p "$OUT"; export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/ub tools/ubench_loads.hip > "$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 1; }
timeout -k 10 120 /tmp/ub > "$OUT/ubench.txt" 2>&1 || { cat "$OUT/ubench.txt"; exit 1; }
cat "$OUT/ubench.txt"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_fetch" -o run --output-format csv -- /tmp/ub > "$OUT/pmc_fetch.log" 2>&1 || { tail -20 "$OUT/pmc_fetch.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, statistics, sys, os
rows = list(csv.DictReader(open(os.path.join(sys.argv[1], "pmc_fetch", "run_counter_collection.csv"))))
vals = {}
for r in rows:
    if r["Counter_Name"] == "FETCH_SIZE":
        vals.setdefault(r["Kernel_Name"][:60], []).append(float(r["Counter_Value"]) * 1024)
for k, v in vals.items():
    print(f"{k:60s} FETCH_SIZE bytes median {statistics.median(v):.4g}  (n={len(v)})")
PY
