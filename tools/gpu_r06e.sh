# round 6, call e: the ipc transport with 64 MiB standalone staging buffers:
# three world-4 runs of the branch (c4 + c4_named), then the new GPU tests
set -o pipefail
D=gpurun_out/r06e; mkdir -p $D; export TMPDIR=/tmp
for i in 1 2 3; do
  GPU_MAX_HW_QUEUES=2 timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29500+i)) \
    bench.py --gpus 4 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4_named,c4 --extras-timeout 150 > $D/ipc_w4_$i.json 2> $D/ipc_w4_$i.err
  rc=$?; echo "run $i rc=$rc"; python3 -c "import json,sys; L=open('$D/ipc_w4_$i.json').read().strip().splitlines(); d=json.loads(L[-1]) if L else {}; print({k: d.get(k) for k in ('c4','c4_named')})" | cut -c1-400
  grep -h "c4_named (rank\|ipc transport\|primary exchange failed" $D/ipc_w4_$i.err | head -8
  case $rc in 124|134|137|139) exit $rc;; esac
done
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread --durations 10 -p no:cacheprovider tests/test_bench_gpu.py tests/test_session.py -k "ipc_transport or torch_noise" > $D/pytest_new.txt 2>&1; rc=$?; tail -25 $D/pytest_new.txt; exit $rc
