# round 6: the runtime-k fold's load schedule A/B (KF_FOLD_SCHED)
set -o pipefail
D=gpurun_out/r06x; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 500 python3 -u tools/ab_fold_sched.py run > $D/ab_fold_sched.jsonl 2> $D/ab_fold_sched.err; rc=$?
cat $D/ab_fold_sched.jsonl; tail -5 $D/ab_fold_sched.err; exit $rc
