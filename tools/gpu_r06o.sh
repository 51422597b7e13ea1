# round 6: the shipped kernels at C2's and C5's sizes on one box
set -o pipefail
D=gpurun_out/r06o; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 ./tools/explore/same_box_probe > $D/same_box_probe.jsonl 2> $D/same_box_probe.err; rc=$?
cat $D/same_box_probe.jsonl $D/same_box_probe.err; exit $rc
