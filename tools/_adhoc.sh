set -u
OUT=gpurun_out/r01k; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "host or golden" > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['host_staged'])"
