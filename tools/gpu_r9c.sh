set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r9c
mkdir -p $O
timeout -k 10 560 python -u tools/stress.py 480 6061 --lds-sample 220 > $O/stress_lds.txt 2>&1 || { tail -5 $O/stress_lds.txt; exit 1; }
tail -2 $O/stress_lds.txt
tools/gpu.sh r9c sqc:k128m32 || exit 1
echo done
