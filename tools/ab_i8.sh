# A/B of the 8-bit lane change: old.so = build before it, new.so = after (both built here into tools/abso/).
set -o pipefail
mkdir -p gpurun_out/i8
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/i8/pytest_parity.log 2>&1 && \
for dt in i8 u8; do for op in sum max; do timeout -k 10 200 python tools/ab_rates.py tools/abso/old.so tools/abso/new.so --k 2,4,8 --dtype $dt --op $op >> gpurun_out/i8/ab.jsonl || exit $?; done; done && \
timeout -k 10 200 python tools/ab_rates.py tools/abso/old.so tools/abso/new.so --k 2,4 --dtype f32 >> gpurun_out/i8/ab.jsonl
