# round 6: stream-distance sweep (one kf_sma_blend, C2) on one box
set -o pipefail
D=gpurun_out/r06w; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 ./tools/explore/offset_probe > $D/offset_probe.jsonl 2> $D/offset_probe.err; rc=$?
cat $D/offset_probe.jsonl $D/offset_probe.err; exit $rc
