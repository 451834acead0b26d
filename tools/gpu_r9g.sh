set -o pipefail
export TMPDIR=/tmp
for v in "LH_LDS_REC_FIRST=1" "LH_LDS_NT_DEC=0" "LH_LDS_REC_FIRST=1,LH_LDS_NT_DEC=0"; do
  n=$(echo "$v" | tr ',=' '__')
  LONGHAIR_AMD_JIT_DEFINES="$v" tools/gpu.sh r9g_$n pmc > /dev/null || exit 1
  echo "$v"; grep -E '"(kernel|ratio_to_algorithmic|fetch_bytes|write_bytes)"' gpurun_out/r9g_$n/pmc_k29m4/summary.json | tail -8
done
