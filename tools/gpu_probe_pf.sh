#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pf
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "unaligned or host_batch" > gpurun_out/pf/pytest.txt 2>&1 || { tail -30 gpurun_out/pf/pytest.txt; exit 1; }
tail -1 gpurun_out/pf/pytest.txt
VARIANTS="pf2=LONGHAIR_AMD_WIN_PF:2|pf4=LONGHAIR_AMD_WIN_PF:4" bash tools/gpu_probe_split.sh pf skip-tests
