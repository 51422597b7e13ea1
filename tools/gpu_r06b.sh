# round 6, call b: packed SMA blend timing (C5 shapes, rocprof) + bench.py's
# native N > 1 branch over the test-only IPC transport at worlds 2 and 4
set -o pipefail
D=gpurun_out/r06b; mkdir -p $D; export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $D/t -o t --output-format csv -- python3 tools/pmc_c5.py run > $D/t.log 2>&1 || exit 1
grep -h "sma_batch\|reduce_batch" $D/t/*kernel_stats.csv
for W in 2 4; do
  timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port $((29400+W)) \
    bench.py --gpus $W --dist-backend gloo --device-index 0 --test-transport ipc --steps 3 --warmup 1 --elems 4194304 \
    --extras c4,c5,c5_pipe,c4_pipe,c4_rs_avg,c3_pipe,c4_named --extras-timeout 300 > $D/ipc_w$W.json 2> $D/ipc_w$W.err
  rc=$?; echo "world $W rc=$rc"; tail -c 3000 $D/ipc_w$W.json; [ $rc -eq 0 ] || { tail -40 $D/ipc_w$W.err; exit $rc; }
done
