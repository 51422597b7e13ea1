# round 6: the compile-time-k reduce's load schedule A/B (KF_REDUCE_SCHED)
set -o pipefail
D=gpurun_out/r06s; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/ab_reduce_sched.py run > $D/ab_reduce_sched.jsonl 2> $D/ab_reduce_sched.err; rc=$?
cat $D/ab_reduce_sched.jsonl; tail -5 $D/ab_reduce_sched.err; exit $rc
