# round 6, call j: the drop-in's mixed-range bounce path
set -o pipefail
D=gpurun_out/r06j; mkdir -p $D; export TMPDIR=/tmp
for c in none whole partial; do timeout -k 10 60 python3 tools/explore/partial_register.py $c > $D/partial_$c.txt 2>&1; echo "$c rc=$?"; grep rc $D/partial_$c.txt; done
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "host or dropin" > $D/pytest_host.txt 2>&1; rc=$?; tail -5 $D/pytest_host.txt; exit $rc
