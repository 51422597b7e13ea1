# round 6, call i: partly registered host buffers through the drop-in, then
# the gpu_slow tier (stress matrices + the world-8 ipc branch)
set -o pipefail
D=gpurun_out/r06i; mkdir -p $D; export TMPDIR=/tmp
for c in none whole partial; do timeout -k 10 60 python3 tools/explore/partial_register.py $c > $D/partial_$c.txt 2>&1; echo "$c rc=$?"; tail -3 $D/partial_$c.txt; done
KUNGFU_AMD_GPU_SLOW=1 timeout -k 10 1000 python3 -u -m pytest -v --timeout 600 --timeout-method thread --durations 20 -p no:cacheprovider -m gpu_slow tests > $D/pytest_gpu_slow.txt 2>&1; rc=$?
tail -30 $D/pytest_gpu_slow.txt; exit $rc
