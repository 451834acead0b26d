#!/bin/bash
# Round-3 session Y: the default bench line after the per-call timing change, twice.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3y}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 400 python bench.py > "$OUT/bench_k29m4_$rep.json" 2> "$OUT/bench_k29m4_$rep.err" || { tail -20 "$OUT/bench_k29m4_$rep.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_k29m4_$rep.json')); print(d['value'], d['kernels'], d['dropin_per_call'], d['cpu_baseline']['per_call_us'], d['cpu_baseline']['value'])"
done
