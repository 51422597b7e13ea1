# round 3: the phase-2 kernels (batched k = 1 in 64-bucket launches), their
# tests, and a rocprof kernel trace of the same program
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread -m gpu tests/test_exchange.py -k "batch_kernel" > gpurun_out/r03i_tests.log 2>&1
timeout -k 10 200 python -u tools/phase2_rates.py > gpurun_out/r03i_phase2.json 2> gpurun_out/r03i_phase2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d gpurun_out/r03i_prof -o phase2 --output-format csv -- python3 tools/phase2_rates.py > gpurun_out/r03i_prof.log 2>&1
timeout -k 10 60 rocprofv3 -L > gpurun_out/r03i_counters.txt 2>&1 || true
