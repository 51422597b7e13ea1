# round 6, call m: the SMA batch launch merging contiguous buckets
set -o pipefail
D=gpurun_out/r06m; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 120 tools/explore/sma_batch_probe > $D/sma_batch_probe.jsonl 2> $D/sma_batch_probe.err || { tail $D/sma_batch_probe.err; exit 1; }
cat $D/sma_batch_probe.jsonl
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_exchange.py tests/test_collective_gloo.py tests/test_configs_gpu.py tests/test_gpu_parity.py -k "sma or optimizer or c5" > $D/pytest_sma.txt 2>&1; rc=$?; tail -4 $D/pytest_sma.txt; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- python3 tools/pmc_c5.py run > $D/t.log 2>&1 || exit 1
grep -h "sma_batch" $D/t/*kernel_stats.csv
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --no-c1 --no-cpu-baseline --no-host-staged > $D/bench.json 2> $D/bench.err || exit $?
python3 -c "import json; d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], {k:(v['us'],v['frac'],v['correct']) for k,v in d['kernels'].items()})"
