set -o pipefail
mkdir -p gpurun_out/pcie2
for c in 1 2 5 10 16; do
  PCIE_SHUFFLE=1 PCIE_CHUNK=$c timeout -k 10 200 python tools/pcie_bench.py k200m56 >> gpurun_out/pcie2/pcie.json 2>> gpurun_out/pcie2/pcie.err || { tail -20 gpurun_out/pcie2/pcie.err; exit 1; }
done
for c in 512 2048 8192; do
  PCIE_SHUFFLE=1 PCIE_CHUNK=$c timeout -k 10 200 python tools/pcie_bench.py k29m4 >> gpurun_out/pcie2/pcie.json 2>> gpurun_out/pcie2/pcie.err || { tail -20 gpurun_out/pcie2/pcie.err; exit 1; }
done
cut -c1-330 gpurun_out/pcie2/pcie.json
