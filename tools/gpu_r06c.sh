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
