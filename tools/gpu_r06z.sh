# round 6, final evidence on the final tree: the mixed-range drop-in probe,
# the whole default GPU tier + smoke, the default N = 1 bench line, the C2
# kernel's rocprofv3 summary + PMC traffic, C5's kernels under rocprofv3
set -o pipefail
D=gpurun_out/r06z; mkdir -p $D; export TMPDIR=/tmp
for c in none whole partial; do timeout -k 10 60 python3 tools/explore/partial_register.py $c > $D/partial_$c.txt 2>&1 || exit $?; grep rc $D/partial_$c.txt; done
bash tools/gpu_r06.sh r06z suite bench prof c5
