# round 6: host-range classification (two adjacent registrations, a pinned
# middle) and the host / drop-in GPU tests
set -o pipefail
D=gpurun_out/r06y; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu -k "host or transform or dropin or consumer or chunk" tests > $D/pytest_host.txt 2>&1; rc=$?
tail -3 $D/pytest_host.txt; exit $rc
