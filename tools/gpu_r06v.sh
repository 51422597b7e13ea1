# round 6: the C5 blend batch's layout (segments vs allocations) on one box
set -o pipefail
D=gpurun_out/r06v; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 ./tools/explore/sma_layout_probe > $D/sma_layout_probe.jsonl 2> $D/sma_layout_probe.err; rc=$?
cat $D/sma_layout_probe.jsonl $D/sma_layout_probe.err; exit $rc
