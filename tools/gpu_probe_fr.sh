set -o pipefail
mkdir -p gpurun_out/fr1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fr1/pytest_gpu.txt 2>&1 || { tail -30 gpurun_out/fr1/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/fr1/pytest_gpu.txt
TUNE_VARIANTS="fr=LONGHAIR_AMD_JIT_DEFINES:LH_PB_FR=1" timeout -k 10 300 python tools/tune.py 128 32 8192 8192 > gpurun_out/fr1/tune_k128.txt 2>&1 || { tail -20 gpurun_out/fr1/tune_k128.txt; exit 1; }
cat gpurun_out/fr1/tune_k128.txt
TUNE_VARIANTS="fr=LONGHAIR_AMD_JIT_DEFINES:LH_PB_FR=1" timeout -k 10 300 python tools/tune.py 200 56 65536 64 > gpurun_out/fr1/tune_k200.txt 2>&1 || { tail -20 gpurun_out/fr1/tune_k200.txt; exit 1; }
cat gpurun_out/fr1/tune_k200.txt
