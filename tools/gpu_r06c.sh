# round 6, call c: SMA r05-vs-r06 A/B, C5 fold probe, B1 floor, C5 kernels
# under rocprof on the r06 library
set -o pipefail
D=gpurun_out/r06c; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ab_sma_pk.py run > $D/ab_sma_pk.jsonl 2> $D/ab_sma_pk.err || { tail -20 $D/ab_sma_pk.err; exit 1; }
cat $D/ab_sma_pk.jsonl
timeout -k 10 120 tools/explore/fold_probe > $D/fold_probe.jsonl 2> $D/fold_probe.err || { tail $D/fold_probe.err; exit 1; }
cat $D/fold_probe.jsonl
timeout -k 10 180 tools/explore/b1_floor > $D/b1_floor.jsonl 2> $D/b1_floor.err || { tail $D/b1_floor.err; exit 1; }
cat $D/b1_floor.jsonl
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- python3 tools/pmc_c5.py run > $D/t.log 2>&1 || exit 1
grep -h "sma_batch\|reduce_batch" $D/t/*kernel_stats.csv
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread --durations 10 -p no:cacheprovider tests/test_bench_gpu.py -k ipc_transport tests/test_session.py::test_lone_session_null_stream_with_torch_noise > $D/pytest_new.txt 2>&1; rc=$?; tail -25 $D/pytest_new.txt; exit $rc
