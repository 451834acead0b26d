#!/bin/bash
# HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) and the SQ pass for $CONFIGS.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CONFIGS:-k29m4}; do
  mkdir -p "$OUT/pmc_$cfg"
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/fetch.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/fetch.log"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/write.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/write.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$cfg" $cfg > "$OUT/pmc_$cfg/summary.json" && grep -A6 '"decode": {' "$OUT/pmc_$cfg/summary.json" | head -8
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d "$OUT/sq_$cfg" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/sq_$cfg.log" 2>&1 || { tail -20 "$OUT/sq_$cfg.log"; exit 1; }
  python3 tools/sq_summary.py "$(find "$OUT/sq_$cfg" -name '*counter_collection.csv' | head -1)" $cfg > "$OUT/sq_$cfg.json" || exit 1
done
