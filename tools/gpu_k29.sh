set -o pipefail
OUT=gpurun_out/r2b; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "not 128 and not 200" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 python tools/tune.py > $OUT/tune.txt 2> $OUT/tune.err || { tail -20 $OUT/tune.err; exit 1; }
cat $OUT/tune.txt
