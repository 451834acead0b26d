#!/bin/bash
# SQ counter pass (wave occupancy / wait / issue breakdown) for the bench kernels of a config.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-sq}; CFG=${2:-k29m4}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d "$OUT/pmc_sq" -o run --output-format csv -- python3 tools/prof_kernels.py $CFG > "$OUT/pmc_sq.log" 2>&1 || { tail -20 "$OUT/pmc_sq.log"; exit 1; }
find "$OUT/pmc_sq" -name "*counter_collection.csv" | head -1 | xargs -I{} sh -c "head -1 {}; grep -E 'lh_jit' {} | head -40"
