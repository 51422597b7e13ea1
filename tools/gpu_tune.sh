#!/usr/bin/env bash
# Geometry sweep + PMC HBM-traffic passes for the C2 reduce kernel.
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== tune ($(date +%T))"
timeout -k 10 600 python tools/tune_reduce.py > "$OUT/tune.jsonl" 2> "$OUT/tune.err" || { echo "tune failed $?"; tail "$OUT/tune.err"; exit 1; }
head -12 "$OUT/tune.jsonl"
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c ($(date +%T))"
  timeout -k 10 300 rocprofv3 --pmc $c -T -d "$OUT/pmc_$c" -o pmc --output-format csv -- \
      python3 bench.py --profile-only --steps 20 --warmup 2 > "$OUT/pmc_$c.log" 2>&1 || { echo "pmc $c failed"; tail "$OUT/pmc_$c.log"; exit 1; }
done
echo done
