set -u
OUT=gpurun_out/r01h; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --dist-backend gloo --device-index 0 --steps 3 --warmup 1 > $OUT/rehearse2.log 2>&1 || { tail -20 $OUT/rehearse2.log; exit 1; }
tail -1 $OUT/rehearse2.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 3 --dist-backend gloo --device-index 0 --steps 2 --warmup 1 > $OUT/rehearse3.log 2>&1 || { tail -20 $OUT/rehearse3.log; exit 1; }
tail -1 $OUT/rehearse3.log
