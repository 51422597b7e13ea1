#!/usr/bin/env bash
# AddressSanitizer on the HOST code of the C++ hosts that drive the GPU: the
# exchange (world 1 on librccl, three loopback ranks incl. the name-keyed
# negotiation), the hierarchical all-reduce (device-mode sessions across
# emulated hosts) and the Peer facade over device-mode sessions (np 2-4).
# Device code is not instrumented (-Xarch_host only; GPU ASan is not
# available on this pool).
#   bash tools/sanitize_gpu_hosts.sh build     # here, on the CPU
#   bash tools/sanitize_gpu_hosts.sh run       # on the GPU box
# SAN=thread selects ThreadSanitizer instead (tools/san_build_thread/).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SAN=${SAN:-address}
D="$ROOT/tools/san_build"
[ "$SAN" = address ] || D="$ROOT/tools/san_build_$SAN"
INC="-I$ROOT/include -I$ROOT/tests/c -I/opt/rocm/include"
HIPL="-L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib"
case "${1:-}" in
build)
    mkdir -p "$D"
    SRC="$ROOT/kungfu_amd/csrc"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off \
        -fvisibility=hidden -Xarch_host -fsanitize=$SAN -Wl,-soname,libkungfu_amd.so \
        -I"$ROOT/include" -o "$D/libkungfu_amd.so" \
        $SRC/kf_capi.hip $SRC/kf_ingest.hip $SRC/kf_session.hip $SRC/kf_p2p.hip $SRC/kf_exchange.hip $SRC/kf_stream.hip -ldl
    CXX="/opt/rocm/lib/llvm/bin/clang++ -std=c++17 -O1 -g -fsanitize=$SAN -D__HIP_PLATFORM_AMD__"
    $CXX -fPIC -shared $INC -o "$D/libkf_testing.so" "$ROOT/tests/c/kf_testing.cpp" \
        -L"$D" -lkungfu_amd -Wl,-rpath,'$ORIGIN' $HIPL -ldl -lpthread
    for t in test_exchange test_hier test_peer; do
        $CXX $INC -o "$D/$t" "$ROOT/tests/c/$t.cpp" -L"$D" -lkungfu_amd -lkf_testing \
            -Wl,-rpath,'$ORIGIN' $HIPL -lpthread
    done
    echo "built $D"
    ;;
run)
    # A host passes when it printed its ok line, exited 0 and the sanitizer
    # reported nothing; any other exit fails the run (an ASan CHECK at exit
    # included: the library no longer calls HIP from a destructor, and the
    # hosts call kf_shutdown() before main returns). The raw log of every
    # failing host is kept under gpurun_out/sanitize_logs/.
    # quarantine_size_mb=0: ASan's quarantine also holds the chunks of its
    # DEVICE allocator (every hipFree of the run); the HIP runtime's own
    # teardown in libamdhip64's __cxa_finalize unloads HSA and then frees host
    # objects, and a device chunk pushed out of the quarantine by such a free
    # trips "CHECK !dev_runtime_unloaded_" with no frame of this project on
    # the stack (raw logs: profiles/r04/asan_check_r04c.log,
    # asan_check_r04d_test_hier.log — the second after the hosts had cycled
    # the quarantine themselves before returning). Without a quarantine every
    # free is final at once, while the runtime is up; freed memory stays
    # poisoned until it is reused.
    export ASAN_OPTIONS="detect_leaks=0 halt_on_error=1 protect_shadow_gap=0 quarantine_size_mb=0 thread_local_quarantine_size_kb=0"
    export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1 suppressions=$ROOT/tools/tsan_rocm.supp"
    KEEP="$ROOT/gpurun_out/sanitize_logs"
    cd "$D"
    check() {  # check <log> <ok-pattern> <status> <name>
        cat "$1"
        echo "   exit status $3"
        local bad=""
        case $3 in
        0) ;;
        124|134|137|139) bad="abort, fault or time limit (status $3)" ;;
        *) bad="exit status $3" ;;
        esac
        if [ -z "$bad" ] && grep -q "ERROR: AddressSanitizer\|WARNING: ThreadSanitizer\|CHECK failed" "$1"; then
            bad="sanitizer report"
        fi
        if [ -z "$bad" ] && ! grep -q "$2" "$1"; then bad="no '$2' line"; fi
        if [ -n "$bad" ]; then
            mkdir -p "$KEEP"
            cp "$1" "$KEEP/$SAN-$4.log"
            echo "FAIL: $bad (raw log: gpurun_out/sanitize_logs/$SAN-$4.log)"
            exit 1
        fi
    }
    L=$(mktemp)
    echo "== test_exchange"
    st=0; timeout -k 10 240 ./test_exchange > "$L" 2>&1 || st=$?
    check "$L" "exchange ok" $st test_exchange
    echo "== test_hier"
    P=$((20000 + RANDOM % 12000))  # below the ephemeral range
    H=$(mktemp -d)
    st=0; timeout -k 10 240 ./test_hier $P "$H" > "$L" 2>&1 || st=$?
    check "$L" "hier ok" $st test_hier
    for np in 2 3 4; do
        echo "== test_peer np=$np dev"
        S=$(mktemp -d)
        pids=""
        for r in $(seq 0 $((np - 1))); do
            timeout -k 10 120 ./test_peer $r $np "$S" dev > "$S/out.$r" 2>&1 &
            pids="$pids $!"
        done
        sts=""
        for p in $pids; do st=0; wait $p || st=$?; sts="$sts $st"; done
        r=0
        for st in $sts; do check "$S/out.$r" "peer ok" $st "test_peer_np${np}_r$r"; r=$((r + 1)); done
    done
    echo "$SAN sanitizer, gpu hosts: no report"
    ;;
*)
    echo "usage: $0 build|run" >&2
    exit 2
    ;;
esac
