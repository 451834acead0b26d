#!/bin/bash
# Round-3 session Z: k29/m4 decode knobs after the column-order change (data columns
# non-temporal, XCD-aware block order off, per-row pins), interleaved.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3z}
mkdir -p "$OUT"
export TMPDIR=/tmp
TUNE_ROUNDS=4 TUNE_VARIANTS="nt2=LONGHAIR_AMD_JIT_DEFINES:LH_NT_DEC=2|noxcd=LONGHAIR_AMD_JIT_DEFINES:LH_XCD=0|pw0=LONGHAIR_AMD_JIT_DEFINES:LH_PIN_WORDS=0|b2=" \
  timeout -k 10 400 python -u tools/tune.py > "$OUT/tune.txt" 2> "$OUT/tune.err" || { tail -20 "$OUT/tune.err"; exit 1; }
cat "$OUT/tune.txt"
