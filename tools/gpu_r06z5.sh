# round 6: KF_REDUCE_PIN A/B (raw words + barrier vs + asm pin)
set -o pipefail
D=gpurun_out/r06z5; mkdir -p $D; export TMPDIR=/tmp
AB_VARIANTS=p0,p1 timeout -k 10 600 python3 -u tools/ab_reduce_sched.py run > $D/ab_reduce_pin.jsonl 2> $D/ab_reduce_pin.err; rc=$?
cat $D/ab_reduce_pin.jsonl; tail -5 $D/ab_reduce_pin.err; exit $rc
