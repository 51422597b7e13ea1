# bf16 narrow: exhaustive hardware-vs-recipe check, then A/B of three builds
# (bf_old.so: branchy recipe, bf_mid.so: select-free recipe, bf_hw.so:
# v_cvt_pk_bf16_f32; built here into tools/abso/), then the bf16 GPU tests
# against the in-tree build.
set -o pipefail
mkdir -p gpurun_out/bf16
timeout -k 10 120 tools/explore/bf16_cvt_check > gpurun_out/bf16/cvt_check.json && \
for k in 2,4,8; do timeout -k 10 300 python tools/ab_rates.py tools/abso/bf_old.so tools/abso/bf_mid.so tools/abso/bf_hw.so --k $k --dtype bf16 >> gpurun_out/bf16/ab.jsonl || exit $?; done && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "bf16 or sma or SMA" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/bf16/pytest.log 2>&1
