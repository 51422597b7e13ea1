# round 6: the batched launches' bucket lookup (scan vs count) A/B, then the
# batch / SMA / fold GPU tests on the count build
set -o pipefail
D=gpurun_out/r06q; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/ab_batch_seg.py run > $D/ab_batch_seg.jsonl 2> $D/ab_batch_seg.err || { tail -20 $D/ab_batch_seg.err; exit 1; }
cat $D/ab_batch_seg.jsonl
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "batch or sma or shard or fold" tests > $D/pytest_batch.txt 2>&1; rc=$?
tail -3 $D/pytest_batch.txt; exit $rc
