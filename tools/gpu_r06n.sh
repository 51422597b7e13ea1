# round 6: tail-round probe (does a partly filled last round of blocks cost C5?)
set -o pipefail
D=gpurun_out/r06n; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 180 ./tools/explore/tail_probe > $D/tail_probe.jsonl 2> $D/tail_probe.err; rc=$?
cat $D/tail_probe.jsonl; exit $rc
