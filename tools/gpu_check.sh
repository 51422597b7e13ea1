#!/usr/bin/env bash
# One guarded GPU session: parity tests, smoke, bench, rocprofv3 kernel trace,
# PMC traffic passes. Each GPU step has its own time limit; a crash/timeout
# (anything but a plain test failure) stops everything after it.
#   usage: bash tools/gpu_check.sh [tag] [extra steps: tune|big|rates|rates_prof]
set -u
TAG=${1:-r01}
shift || true
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
    tail -4 "$OUT/$name.log"
    return $rc
}

step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed ($rc): stop"; exit $rc; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step rocprof_trace 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o trace \
    --output-format csv -- python3 bench.py --profile-only --steps 200 --warmup 20 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 300 rocprofv3 --pmc $c -T -d "$OUT/pmc_$c" -o pmc --output-format csv -- \
      python3 bench.py --profile-only --steps 20 --warmup 2 || exit $?
done
python tools/pmc_traffic.py "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" "$OUT/traffic.json" > /dev/null && \
    mkdir -p profiles && cp "$OUT/traffic.json" profiles/traffic.json
step bench 600 python bench.py || exit $?
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
for extra in "$@"; do
  case $extra in
    tune) step tune 600 python tools/tune_reduce.py || exit $? ;;
    rates) step kernel_rates 600 python tools/kernel_rates.py || exit $? ;;
    rates_prof) step kernel_rates_prof 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof_rates" \
              -o rates --output-format csv -- python3 tools/kernel_rates.py || exit $? ;;
    big)  step tune_big 600 python tools/tune_reduce.py --elems 268435456 --rounds 3 \
              --unroll 1,4 --grid 4096,1048576 --loadnt 0,1 --stplain 0 || exit $? ;;
  esac
done
echo "done"
