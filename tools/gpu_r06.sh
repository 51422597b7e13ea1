#!/usr/bin/env bash
# Round-6 GPU sessions, one stage per call. Every GPU step runs under its own
# time limit; an abort, fault or time limit stops the script there.
#   bash tools/gpu_r06.sh <tag> new       # the tests this round added/changed
#   bash tools/gpu_r06.sh <tag> suite     # the whole -m gpu suite + smoke
#   bash tools/gpu_r06.sh <tag> bench     # bench.py N=1 (default line)
#   bash tools/gpu_r06.sh <tag> bench2    # bench.py --gpus 2 rehearsal (self-launch, gloo)
#   bash tools/gpu_r06.sh <tag> asan      # host-code ASan of the C++ hosts
#   bash tools/gpu_r06.sh <tag> c1trace   # C1 np=2 per-chunk timelines (device, cpu)
#   bash tools/gpu_r06.sh <tag> c1ab      # C1 session settings, interleaved A/B
#   bash tools/gpu_r06.sh <tag> session   # the session / hierarchical / C-host GPU tests
#   bash tools/gpu_r06.sh <tag> prof      # rocprofv3 stats + PMC traffic of the C2 kernel
#   bash tools/gpu_r06.sh <tag> stream    # streamed-chunk session tests + C1 A/B against whole chunks
#   bash tools/gpu_r06.sh <tag> c5        # C5's two kernels: rocprofv3 durations (tools/pmc_c5.py)
#   bash tools/gpu_r06.sh <tag> c5pmc     # their PMC bytes (after c5, which it summarizes)
set -u
TAG=${1:?tag}
shift
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

fatal() {  # a crash, abort or time limit: nothing more on the GPU
    case $1 in 0|1) return 1 ;; *) echo "stopping: status $1"; exit "$1" ;; esac
}

PYT="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu"
for stage in "$@"; do
  case $stage in
  new)
    step new_tests 900 $PYT tests/test_bench_gpu.py tests/test_session.py \
        tests/test_exchange.py tests/test_torch_ops_native.py tests/test_hierarchical.py \
        tests/test_c_consumer.py -k "gpus2 or next_call or any_order_device or pipelined_failure \
or named_all_reduce_any_order or multi_rank_by_name or cross_host or two_hosts or native_hier \
or hier_all_reduce or fake_agent or rehearsal or branch_single_rank"
    fatal $? ;;
  suite)
    step pytest_gpu 1100 $PYT --durations=60 tests
    fatal $?
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
  bench)
    step bench 900 python bench.py --steps 20 --warmup 5 || exit $?
    tail -1 "$OUT/bench.log" > "$OUT/bench.json" ;;
  bench2)
    step bench2 300 python bench.py --gpus 2 --dist-backend gloo --device-index 0 --steps 5 \
        --warmup 2 --elems $((16 << 20)) --extras c4_torch,c5_torch --extras-timeout 200 || exit $?
    tail -1 "$OUT/bench2.log" > "$OUT/bench2.json" ;;
  asan)
    step asan_build 600 bash tools/sanitize_gpu_hosts.sh build || exit $?
    step asan 900 bash tools/sanitize_gpu_hosts.sh run || exit $? ;;
  slow)
    KUNGFU_AMD_GPU_SLOW=1 step pytest_gpu_slow 900 $PYT -m gpu_slow tests
    fatal $? ;;
  session)
    step session_tests 1000 $PYT tests/test_session.py tests/test_session_multihost.py \
        tests/test_hierarchical.py tests/test_c_consumer.py tests/test_torch_ops_native.py
    fatal $? ;;
  c1)
    step c1 600 python bench.py --config c1 --c1-modes device,cpu,cpu_dev --c1-repeats 5 \
        --steps 100 --warmup 10 || exit $?
    tail -1 "$OUT/c1.log" > "$OUT/c1.json" ;;
  prof)
    # the C2 kernel's rocprofv3 summary and PMC traffic for this round
    step rocprof_trace 600 rocprofv3 --kernel-trace --stats -T -d "$OUT/prof" -o trace \
        --output-format csv -- python3 bench.py --profile-only --steps 200 --warmup 20 || exit $?
    for c in FETCH_SIZE WRITE_SIZE; do
      step pmc_$c 300 rocprofv3 --pmc $c -T -d "$OUT/pmc_$c" -o pmc --output-format csv -- \
          python3 bench.py --profile-only --steps 20 --warmup 2 || exit $?
    done
    python tools/pmc_traffic.py "$OUT/pmc_FETCH_SIZE" "$OUT/pmc_WRITE_SIZE" \
        "$OUT/traffic.json" > /dev/null ;;
  c1ab)
    step c1ab 900 python tools/c1_ab.py device device:KUNGFU_AMD_PIECE_KB=512 \
        device:KUNGFU_AMD_TX_AHEAD=4 device:KUNGFU_AMD_MIRROR_SIDE=0 \
        device:KUNGFU_AMD_ROOT_MIRROR=0 cpu cpu_dev --repeats 5 --out "$OUT/c1_ab.json" || exit $? ;;
  stream)
    step stream_tests 600 $PYT tests/test_session.py -k "streamed"
    fatal $?
    step c1ab_stream 900 python tools/c1_ab.py device device:KUNGFU_AMD_STREAM=1 \
        device:KUNGFU_AMD_STREAM=out device:KUNGFU_AMD_STREAM=fold device:KUNGFU_AMD_STREAM=in \
        device:KUNGFU_AMD_STREAM=out+fold cpu --repeats 5 \
        --out "$OUT/c1_ab_stream.json" || exit $? ;;
  c1ab_fold)
    step c1ab_fold 900 python tools/c1_ab.py device device:KUNGFU_AMD_STREAM=0 \
        device:KUNGFU_AMD_STREAM=fold+last device:KUNGFU_AMD_STREAM=fold+idle \
        device:KUNGFU_AMD_STREAM=fold+last+idle cpu --repeats 5 \
        --out "$OUT/c1_ab_fold.json" || exit $? ;;
  c1trace)
    step c1trace 600 python tools/c1_trace.py --modes device,cpu --steps 60 \
        --out "$OUT/c1_trace.json" || exit $? ;;
  c5)
    step c5_trace 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/c5" -o t --output-format csv -- \
        python3 tools/pmc_c5.py run || exit $? ;;
  c5pmc)
    # the same two kernels' HBM bytes, one counter per pass, then the summary
    for c in FETCH_SIZE WRITE_SIZE; do
      step c5_pmc_$c 120 rocprofv3 --pmc $c -T -d "$OUT/c5_$c" -o pmc --output-format csv -- \
          python3 tools/pmc_c5.py run || exit $?
    done
    python3 tools/pmc_c5.py summarize "$OUT/c5" "$OUT/c5_FETCH_SIZE" "$OUT/c5_WRITE_SIZE" \
        > "$OUT/pmc_c5.jsonl" && cat "$OUT/pmc_c5.jsonl" ;;
  *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo "all stages done"
