set -u
OUT=gpurun_out/r01d; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python tools/tune_reduce.py --rotate 3 --grid 2048,4096,8192,65536,1048576 > $OUT/tune_rot3.jsonl 2>$OUT/tune.err || exit 1
head -10 $OUT/tune_rot3.jsonl
timeout -k 10 600 python bench.py --no-cpu-baseline --no-host-staged > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log
