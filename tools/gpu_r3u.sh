#!/bin/bash
# Round-3 session U: round-end rehearsal on the committed defaults -- full GPU suite, smoke(),
# the default bench line (N = 1), the same through torchrun (the multi-rank launcher's code
# path with one rank), rocprofv3 kernel stats of the bench command, k200/m56 PCIe timeline.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-r3u}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 400 python bench.py > "$OUT/bench_k29m4.json" 2> "$OUT/bench_k29m4.err" || { tail -20 "$OUT/bench_k29m4.err"; exit 1; }
cat "$OUT/bench_k29m4.json"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 10 --warmup 2 --cpu-baseline off --dropin-calls 0 > "$OUT/bench_torchrun1.json" 2> "$OUT/bench_torchrun1.err" || { tail -20 "$OUT/bench_torchrun1.err"; exit 1; }
cut -c1-400 "$OUT/bench_torchrun1.json"
for cfg in k128m32 k200m56; do
  timeout -k 10 400 python bench.py --config $cfg > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err" || { tail -20 "$OUT/bench_$cfg.err"; exit 1; }
  cut -c1-300 "$OUT/bench_$cfg.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline off --dropin-calls 0 --pcie off > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name '*kernel_stats.csv' -exec grep -E '"lh_' {} \; | cut -c1-120
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/pcie_prof200" -o run --output-format csv -- python3 tools/pcie_bench.py k200m56 > "$OUT/pcie_prof200.log" 2>&1 || { tail -20 "$OUT/pcie_prof200.log"; exit 1; }
