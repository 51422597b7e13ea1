# round 6, call h: the ipc branch at world 2 with the DEFAULT extras list
# (every sub-benchmark, p2p children included), and the extended host-path
# parity test
set -o pipefail
D=gpurun_out/r06h; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -k "host_paths or host_zero_copy" > $D/pytest_host.txt 2>&1; rc=$?; tail -5 $D/pytest_host.txt; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29592 \
    bench.py --gpus 2 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras-timeout 300 > $D/ipc_w2_all.json 2> $D/ipc_w2_all.err
rc=$?; grep "\[bench\]" $D/ipc_w2_all.err | tail -30; exit $rc
