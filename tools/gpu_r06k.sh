# round 6, call k: the world-8 ipc branch failed once in r06zz (c4: "group
# failed earlier" on rank 0); three runs with every rank's error printed
set -o pipefail
D=gpurun_out/r06k; mkdir -p $D; export TMPDIR=/tmp
for i in 1 2 3; do
  GPU_MAX_HW_QUEUES=1 timeout -k 10 300 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29610+i)) \
    bench.py --gpus 8 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4,c5,c5_pipe,c4_pipe,c4_rs_avg,c3_pipe,c4_named --extras-timeout 250 > $D/w8_$i.json 2> $D/w8_$i.err
  rc=$?; echo "run $i rc=$rc"; grep -h "failed\|ipc transport" $D/w8_$i.err | head -12 | cut -c1-400
  case $rc in 124|134|137|139) exit $rc;; esac
done
