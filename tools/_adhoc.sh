set -u
OUT=gpurun_out/r01n; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python tools/kernel_rates.py > $OUT/kernel_rates.jsonl 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
cat $OUT/kernel_rates.jsonl
timeout -k 10 300 python bench.py --config c1 --steps 100 --warmup 10 > $OUT/c1.log 2>&1 || { tail -20 $OUT/c1.log; exit 1; }
tail -1 $OUT/c1.log
