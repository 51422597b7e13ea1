#!/usr/bin/env bash
# Host-code sanitizer runs of the session engine (CPU only: host-mode
# sessions make no HIP call). Builds libkungfu_amd.so from the product
# sources with ThreadSanitizer, then AddressSanitizer, on the host side only
# (-Xarch_host), links tests/c/test_session_async.cpp against each and runs it
# at np = 2, 3, 4 (async all-reduces started in a different order per rank,
# two steps back to back, then a blocking one).
#   bash tools/sanitize_session.sh > profiles/r03/sanitize_session.txt 2>&1
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=${TMPDIR:-/tmp}/kf_sanitize
mkdir -p "$W"
SRC="$ROOT/kungfu_amd/csrc"
SRCS="$SRC/kf_capi.hip $SRC/kf_ingest.hip $SRC/kf_session.hip $SRC/kf_p2p.hip $SRC/kf_exchange.hip $SRC/kf_stream.hip"
CLANG=/opt/rocm/lib/llvm/bin/clang++
for san in thread address; do
    D="$W/$san"
    mkdir -p "$D"
    echo "== $san: building (host code instrumented)"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -ffp-contract=off \
        -fvisibility=hidden -Xarch_host -fsanitize=$san -Wl,-soname,libkungfu_amd.so \
        -I"$ROOT/include" -o "$D/libkungfu_amd.so" $SRCS -ldl
    $CLANG -std=c++17 -O1 -g -fsanitize=$san -I"$ROOT/include" \
        "$ROOT/tests/c/test_session_async.cpp" -L"$D" -lkungfu_amd -Wl,-rpath,"$D" \
        -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lpthread -o "$D/test_session_async"
    for np in 2 3 4; do
        S=$(mktemp -d "$W/sock.XXXX")
        echo "-- $san np=$np"
        if [ $san = thread ]; then
            TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
                timeout -k 10 300 "$D/test_session_async" $np 2 "$S"
        else
            ASAN_OPTIONS="detect_leaks=1 halt_on_error=1" \
                timeout -k 10 300 "$D/test_session_async" $np 2 "$S"
        fi
        rm -rf "$S"
        S=$(mktemp -d "$W/sock.XXXX")
        echo "-- $san np=$np, last rank gone"
        if [ $san = thread ]; then
            TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" \
                timeout -k 10 300 "$D/test_session_async" $np 1 "$S" dead
        else
            ASAN_OPTIONS="detect_leaks=1 halt_on_error=1" \
                timeout -k 10 300 "$D/test_session_async" $np 1 "$S" dead
        fi
        rm -rf "$S"
    done
done
echo "sanitizers: clean"
