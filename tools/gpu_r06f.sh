# round 6, call f: the ipc branch with c4_named in-process (world 4 twice)
set -o pipefail
D=gpurun_out/r06f; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread --durations 10 -p no:cacheprovider tests/test_bench_gpu.py -k "ipc_transport" > $D/pytest_ipc.txt 2>&1; rc=$?; tail -12 $D/pytest_ipc.txt; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29577 \
    bench.py --gpus 4 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4,c5,c5_pipe,c4_pipe,c4_rs_avg,c3_pipe,c4_named --extras-timeout 150 > $D/ipc_w4.json 2> $D/ipc_w4.err
rc=$?; grep "\[bench\]" $D/ipc_w4.err | tail -12; [ $rc -eq 0 ] || exit $rc
# world 8: the driver's BASELINE world size, rehearsed on one GPU
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29588 \
    bench.py --gpus 8 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4,c5,c5_pipe,c4_pipe,c4_rs_avg,c3_pipe,c4_named --extras-timeout 200 > $D/ipc_w8.json 2> $D/ipc_w8.err
rc=$?; grep "\[bench\]" $D/ipc_w8.err | tail -14; exit $rc
