# round 6, call d: the c4_named failure at world 4 over the ipc transport
# (r06c): three runs of the world-4 branch with c4_named only, then the
# new tests
set -o pipefail
D=gpurun_out/r06d; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 120 tools/explore/sma_batch_probe > $D/sma_batch_probe.jsonl 2> $D/sma_batch_probe.err || { tail $D/sma_batch_probe.err; exit 1; }
cat $D/sma_batch_probe.jsonl
export GPU_MAX_HW_QUEUES=2
for i in 1 2 3; do
  timeout -k 10 200 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $((29500+i)) \
    bench.py --gpus 4 --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4_named,c4 --extras-timeout 150 > $D/ipc_w4_$i.json 2> $D/ipc_w4_$i.err
  rc=$?; echo "run $i rc=$rc"; python3 -c "import json,sys; L=open('$D/ipc_w4_$i.json').read().strip().splitlines(); d=json.loads(L[-1]) if L else {}; print({k: d.get(k) for k in ('c4','c4_named')})" | cut -c1-600
  grep -h "c4_named (rank\|ipc transport\|primary exchange failed" $D/ipc_w4_$i.err | head -8
  case $rc in 124|134|137|139) exit $rc;; esac
done
