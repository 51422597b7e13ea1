timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_session.py tests/test_session_multihost.py tests/test_bench_gpu.py > gpurun_out/r03h_tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --no-c1 --no-cpu-baseline --no-host-staged > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err
timeout -k 10 400 python -u bench.py --config c1 --steps 100 --warmup 10 --c1-modes device,device_nomirror,cpu,cpu_dev --c1-repeats 3 > gpurun_out/r03h_c1.json 2> gpurun_out/r03h_c1.err
