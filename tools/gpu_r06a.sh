# round 6, call a: C5 kernel evidence (sma probe, rocprof durations + PMC of
# the C5 shapes)
set -o pipefail
D=gpurun_out/r06a; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 120 tools/explore/sma_probe > $D/sma_probe.jsonl 2> $D/sma_probe.err &&
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- python3 tools/pmc_c5.py run > $D/t.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $D/f -o pmc --output-format csv -- python3 tools/pmc_c5.py run > $D/f.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $D/w -o pmc --output-format csv -- python3 tools/pmc_c5.py run > $D/w.log 2>&1 &&
python3 tools/pmc_c5.py summarize $D/t $D/f $D/w > $D/pmc_c5.jsonl 2>&1
rc=$?; cat $D/sma_probe.jsonl; cat $D/pmc_c5.jsonl; exit $rc
