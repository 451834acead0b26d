#!/bin/bash
# The one GPU session script (run through gpurun).  Every GPU step runs under its own time
# limit and the chain stops at the first failure (no step runs after a fault or a timeout).
#
#   tools/gpu.sh OUT STEP [STEP ...]
#
# OUT names gpurun_out/OUT/.  Steps:
#   tests            pytest -m gpu (every GPU parity test), one process
#   tests:EXPR       pytest -m gpu -k EXPR
#   testscheck[:EXPR] pytest -m gpu -k EXPR (default phase_b) on the phase-B checked build
#   smoke            __graft_entry__.smoke()
#   bench[:CFG]      bench.py (default k29m4; k128m32 / k200m56 with 5 steps)
#   prof[:CFG]       rocprofv3 --kernel-trace --stats of a short bench run
#   pmc[:CFG]        FETCH_SIZE and WRITE_SIZE passes (separate runs) + tools/pmc_summary.py
#   sq[:CFG]         one SQ counter pass (waves, cycles, waits, VALU/VMEM issue)
#   pcie             tools/pcie_bench.py k29m4 k200m56
#   ubench:NAME[:G]  tools/NAME (built here beforehand) with optional group list G (commas)
#   stress[:SECONDS]  tools/stress.py: random shapes, strided and pointer-table calls vs the oracle
#   tune:VARIANTS[@k m bytes stripes]  tools/tune.py with TUNE_VARIANTS=VARIANTS (env TUNE_ROUNDS)
#   bench2           bench.py --gpus 2 --share-gpu (the N>1 control path on one GPU)
#   benchg[:CFG]     bench.py on the generic kernels only (LONGHAIR_AMD_PATH=generic), 5 steps
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:?usage: tools/gpu.sh OUT STEP...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "FAILED: $1"; tail -30 "$2"; exit 1; }
for step in "$@"; do
  kind=${step%%:*}
  arg=""
  [ "$kind" != "$step" ] && arg=${step#*:}
  echo "== $step"
  case $kind in
    tests)
      log="$OUT/pytest_gpu${arg:+_$arg}.txt"
      sel=()
      [ -n "$arg" ] && sel=(-k "$arg")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${sel[@]}" > "$log" 2>&1 || fail "$step" "$log"
      tail -3 "$log" ;;
    testscheck)
      # the phase-B checked build (make -C longhair_amd/csrc LH_DEBUG=1 OUT=... BUILD=...)
      log="$OUT/pytest_gpu_check.txt"
      LONGHAIR_AMD_LIBRARY=liblonghair_amd_check.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${arg:-phase_b}" > "$log" 2>&1 || fail "$step" "$log"
      tail -3 "$log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || fail smoke "$OUT/smoke.txt"
      cat "$OUT/smoke.txt" ;;
    bench)
      cfg=${arg:-k29m4}
      extra=()
      [ "$cfg" != k29m4 ] && extra=(--steps 5 --warmup 2)
      timeout -k 10 400 python bench.py --config "$cfg" "${extra[@]}" > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || fail "$step" "$OUT/bench_$cfg.err"
      cat "$OUT/bench_$cfg.json" ;;
    benchg)
      cfg=${arg:-k29m4}
      LONGHAIR_AMD_PATH=generic timeout -k 10 400 python bench.py --config "$cfg" --steps 5 --warmup 2 --cpu-baseline off --pcie off --dropin-calls 0 > "$OUT/benchg_$cfg.json" 2> "$OUT/benchg_$cfg.err" || fail "$step" "$OUT/benchg_$cfg.err"
      cat "$OUT/benchg_$cfg.json" ;;
    bench2)
      timeout -k 10 600 python bench.py --gpus 2 --share-gpu --steps 10 --warmup 2 > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.err" || fail "$step" "$OUT/bench_gpus2.err"
      cat "$OUT/bench_gpus2.json" ;;
    prof)
      cfg=${arg:-k29m4}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$cfg" -o run --output-format csv -- python3 bench.py --config "$cfg" --steps 5 --warmup 2 --cpu-baseline off --pcie off --dropin-calls 0 > "$OUT/prof_$cfg.log" 2>&1 || fail "$step" "$OUT/prof_$cfg.log"
      find "$OUT/prof_$cfg" -name "*kernel_stats.csv" -exec cp {} "$OUT/${cfg}_kernel_stats.csv" \;
      grep -E "lh_" "$OUT/${cfg}_kernel_stats.csv" | cut -c1-160 ;;
    pmc)
      cfg=${arg:-k29m4}
      mkdir -p "$OUT/pmc_$cfg"
      timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_fetch" -o run --output-format csv -- python3 tools/prof_kernels.py "$cfg" > "$OUT/pmc_$cfg/fetch.log" 2>&1 || fail "$step" "$OUT/pmc_$cfg/fetch.log"
      timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_$cfg/pmc_write" -o run --output-format csv -- python3 tools/prof_kernels.py "$cfg" > "$OUT/pmc_$cfg/write.log" 2>&1 || fail "$step" "$OUT/pmc_$cfg/write.log"
      python3 tools/pmc_summary.py "$OUT/pmc_$cfg" "$cfg" > "$OUT/pmc_$cfg/summary.json" || exit 1
      grep -E '"(kernel|ratio_to_algorithmic)"' "$OUT/pmc_$cfg/summary.json" ;;
    sq)
      cfg=${arg:-k29m4}
      mkdir -p "$OUT/sq_$cfg"
      timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU --kernel-trace -d "$OUT/sq_$cfg/p1" -o run --output-format csv -- python3 tools/prof_kernels.py "$cfg" > "$OUT/sq_$cfg/p1.log" 2>&1 || fail "$step" "$OUT/sq_$cfg/p1.log"
      csvf=$(find "$OUT/sq_$cfg/p1" -name "*counter_collection.csv" | head -1)
      python3 tools/sq_summary.py "$csvf" "$cfg" "$OUT/sq_$cfg/summary.json" > /dev/null || exit 1
      head -c 3000 "$OUT/sq_$cfg/summary.json"; echo ;;
    sqc)
      # instruction-fetch side: waits with an instruction ready vs I-cache misses
      cfg=${arg:-k128m32}
      mkdir -p "$OUT/sqc_$cfg"
      timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU --kernel-trace -d "$OUT/sqc_$cfg/p1" -o run --output-format csv -- python3 tools/prof_kernels.py "$cfg" > "$OUT/sqc_$cfg/p1.log" 2>&1 || fail "$step" "$OUT/sqc_$cfg/p1.log"
      csvf=$(find "$OUT/sqc_$cfg/p1" -name "*counter_collection.csv" | head -1)
      python3 tools/sq_summary.py "$csvf" "$cfg" "$OUT/sqc_$cfg/summary.json" > /dev/null || exit 1
      head -c 4000 "$OUT/sqc_$cfg/summary.json"; echo ;;
    pcie)
      timeout -k 10 600 python tools/pcie_bench.py k29m4 k200m56 > "$OUT/pcie.json" 2> "$OUT/pcie.err" || fail pcie "$OUT/pcie.err"
      cat "$OUT/pcie.json" ;;
    ubench)
      name=${arg%%:*}
      groups=""
      [ "$name" != "$arg" ] && groups=${arg#*:}
      timeout -k 10 300 "tools/$name" ${groups//,/ } > "$OUT/$name.txt" 2>&1 || fail "$step" "$OUT/$name.txt"
      cat "$OUT/$name.txt" ;;
    stress)
      secs=${arg:-120}
      timeout -k 10 $((secs + 120)) python -u tools/stress.py "$secs" > "$OUT/stress.txt" 2>&1 || fail "$step" "$OUT/stress.txt"
      tail -3 "$OUT/stress.txt" ;;
    tune)
      n=$((${n:-0} + 1))
      targs=""
      if [ "${arg#*@}" != "$arg" ]; then targs=${arg#*@}; arg=${arg%%@*}; fi
      TUNE_VARIANTS="$arg" timeout -k 10 600 python -u tools/tune.py $targs > "$OUT/tune$n.txt" 2> "$OUT/tune$n.err" || fail "$step" "$OUT/tune$n.err"
      cat "$OUT/tune$n.txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
