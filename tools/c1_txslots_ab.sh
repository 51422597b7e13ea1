# A/B of the session sender's D2H lookahead (KUNGFU_AMD_TX_SLOTS) on C1,
# interleaved on one box: 1 = the first version (copy, send, copy, ...)
mkdir -p gpurun_out/c1tx
for np in 2 4; do
  for rep in 1 2 3; do
    for sl in 1 4; do
      KUNGFU_AMD_TX_SLOTS=$sl timeout -k 10 300 python bench.py --config c1 --c1-np $np 2>/dev/null \
        | tail -1 > gpurun_out/c1tx/np${np}_slots${sl}_rep${rep}.json || exit 1
    done
  done
done
