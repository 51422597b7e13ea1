# round 6, call l: the ipc transport with group-agreed staging growth and
# 256 MiB staging from the start: the ipc tests at worlds 2, 4, 8, then the
# world-8 branch twice more
set -o pipefail
D=gpurun_out/r06l; mkdir -p $D; export TMPDIR=/tmp
KUNGFU_AMD_GPU_SLOW=1 timeout -k 10 900 python3 -u -m pytest -v --timeout 600 --timeout-method thread --durations 5 -p no:cacheprovider tests/test_bench_gpu.py -k ipc_transport > $D/pytest_ipc.txt 2>&1; rc=$?; tail -8 $D/pytest_ipc.txt; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29620+i)) \
    bench.py --gpus 8 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4,c5,c5_pipe,c4_pipe,c4_rs_avg,c3_pipe,c4_named --extras-timeout 250 > $D/w8_$i.json 2> $D/w8_$i.err
  rc=$?; echo "run $i rc=$rc"; grep -h "failed\|ipc transport" $D/w8_$i.err | head -12 | cut -c1-400
  case $rc in 124|134|137|139) exit $rc;; esac
done
