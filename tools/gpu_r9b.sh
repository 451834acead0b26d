set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r9b
mkdir -p $O
tools/gpu.sh r9b prof pmc sq || exit 1
timeout -k 10 300 python tools/cold_probe.py > $O/cold_probe.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --gpus 8 --share-gpu --stripes 16384 --steps 10 --warmup 2 > $O/bench_gpus8_share.json 2> $O/bench_gpus8_share.err || exit 1
cat $O/bench_gpus8_share.json | head -c 1500
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
echo done
