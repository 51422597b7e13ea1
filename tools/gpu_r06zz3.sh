# round 6, last call: both GPU tiers + smoke on the committed final tree
set -o pipefail
D=gpurun_out/r06zz3; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations 30 -p no:cacheprovider > $D/pytest_gpu.txt 2>&1; rc=$?
tail -3 $D/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $D/smoke.txt 2>&1 || exit $?
tail -2 $D/smoke.txt
KUNGFU_AMD_GPU_SLOW=1 timeout -k 10 600 python3 -u -m pytest -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu_slow tests > $D/pytest_gpu_slow.txt 2>&1; rc=$?
tail -3 $D/pytest_gpu_slow.txt; exit $rc
