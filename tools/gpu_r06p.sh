# round 6: the bf16 SMA blend's load schedule (3-wait-5 vs all eight first):
# the probe's restatement, then the product's KF_SMA_SCHED variants A/B
set -o pipefail
D=gpurun_out/r06p; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 ./tools/explore/sma_sched_probe > $D/sma_sched_probe.jsonl 2> $D/sma_sched_probe.err || { cat $D/sma_sched_probe.err; exit 1; }
cat $D/sma_sched_probe.jsonl
timeout -k 10 400 python3 -u tools/ab_sma_sched.py run > $D/ab_sma_sched.jsonl 2> $D/ab_sma_sched.err; rc=$?
cat $D/ab_sma_sched.jsonl; tail -5 $D/ab_sma_sched.err; exit $rc
