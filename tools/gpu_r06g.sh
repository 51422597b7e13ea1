# round 6, call g: the whole default GPU tier + smoke on the current tree
set -o pipefail
D=gpurun_out/r06g; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations 40 -p no:cacheprovider > $D/pytest_gpu.txt 2>&1; rc=$?
tail -60 $D/pytest_gpu.txt | grep -v "^$"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $D/smoke.txt 2>&1; rc=$?; tail -3 $D/smoke.txt; exit $rc
