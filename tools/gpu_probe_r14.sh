set -o pipefail
mkdir -p gpurun_out/r14
TUNE_VARIANTS="rows14=LONGHAIR_AMD_WIN_ROWS:14" timeout -k 10 300 python tools/tune.py 200 56 65536 64 > gpurun_out/r14/tune_k200.txt 2>&1 || { tail -20 gpurun_out/r14/tune_k200.txt; exit 1; }
cat gpurun_out/r14/tune_k200.txt
