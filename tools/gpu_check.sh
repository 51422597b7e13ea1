#!/usr/bin/env bash
# One guarded GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/timeout (exit >= 2 that is not
# a plain test failure) stops everything after it.
#   usage: bash tools/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>
    local name=$1 t=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc"
    tail -5 "$OUT/$name.log"
    return $rc
}

step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed ($rc): stop"; exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 600 python bench.py || exit $?
cat "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
step rocprof_trace 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o trace \
    --output-format csv -- python3 bench.py --profile-only --steps 200 --warmup 20 || exit $?
echo "done"
