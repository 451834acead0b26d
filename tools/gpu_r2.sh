#!/bin/bash
# Round-2 GPU session: parity tests (all of them; test failures are reported, a crash or
# time-out stops the session), smoke, the k29m4 bench, the ceiling microbenchmark, a
# kernel-trace profile of the bench and SQ counter passes of the large-m configs.
# Every GPU step has its own time limit.  Usage: tools/gpu_r2.sh OUT_NAME [steps...]
# steps: tests smoke bench large ubench tune prof profall sq pmc pcie (default: tests smoke bench ubench prof sq)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r2}; shift
STEPS=${*:-tests smoke bench ubench prof sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }   # 1 = test failures: keep going
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.txt" 2>&1
  rc=$?; tail -15 "$OUT/pytest_gpu.txt"; ok $rc || exit $rc
fi
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
  cat "$OUT/smoke.txt"
fi
if has bench; then
  timeout -k 10 400 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
  cat "$OUT/bench_k29m4.json"
fi
if has large; then
  for cfg in k128m32 k200m56; do
    timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
    cat "$OUT/bench_$cfg.json"
  done
fi
if has tune; then
  timeout -k 10 600 python tools/tune.py ${TUNE_SHAPE:-} > "$OUT/tune.txt" 2>&1 || { tail -20 "$OUT/tune.txt"; exit 1; }
  tail -8 "$OUT/tune.txt"
fi
if has ubench; then
  timeout -k 10 120 tools/ubench_ceiling > "$OUT/ubench_ceiling.txt" 2>&1 || { tail -20 "$OUT/ubench_ceiling.txt"; exit 1; }
  cat "$OUT/ubench_ceiling.txt"
fi
if has prof; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_k29m4" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 > "$OUT/prof_k29m4.log" 2>&1 || { tail -20 "$OUT/prof_k29m4.log"; exit 1; }
  find "$OUT/prof_k29m4" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-160
fi
if has sq; then
  for cfg in k128m32 k200m56 k29m4; do
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d "$OUT/sq_$cfg" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/sq_$cfg.log" 2>&1 || { tail -20 "$OUT/sq_$cfg.log"; exit 1; }
    f=$(find "$OUT/sq_$cfg" -name "*counter_collection.csv" | head -1)
    python3 tools/sq_summary.py "$f" $cfg > "$OUT/sq_$cfg.json" && cp profiles/sq_$cfg.json "$OUT/" || exit 1
    grep -E '"lh_|SQ_INSTS_VALU|wait_any' "$OUT/sq_$cfg.json"
  done
fi
if has pmc; then
  for cfg in k29m4 k128m32 k200m56; do
    mkdir -p "$OUT/pmc_$cfg"
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/fetch.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/fetch.log"; exit 1; }
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py $cfg > "$OUT/pmc_$cfg/write.log" 2>&1 || { tail -20 "$OUT/pmc_$cfg/write.log"; exit 1; }
    python3 tools/pmc_summary.py "$OUT/pmc_$cfg" $cfg > "$OUT/pmc_$cfg/summary.json" && cp profiles/pmc_$cfg.json "$OUT/pmc_$cfg/" || exit 1
    grep -E '"(kernel|ratio_to_algorithmic)"' "$OUT/pmc_$cfg/summary.json"
  done
fi
if has profall; then
  for cfg in k128m32 k200m56; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config $cfg --steps 5 --warmup 2 --cpu-baseline off --dropin-calls 0 > "$OUT/prof_$cfg.log" 2>&1 || { tail -20 "$OUT/prof_$cfg.log"; exit 1; }
    find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec grep -E "lh_" {} \; | cut -c1-160
  done
fi
if has pcie; then
  timeout -k 10 600 python tools/pcie_bench.py k29m4 k200m56 > "$OUT/pcie.json" 2> "$OUT/pcie.err" || { tail -20 "$OUT/pcie.err"; exit 1; }
  cat "$OUT/pcie.json"
fi
echo "session done"
