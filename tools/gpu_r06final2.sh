# round 6, last call: the default GPU tier + smoke + the N = 1 line + the C2
# profile on the committed final tree
set -o pipefail
bash tools/gpu_r06.sh r06final2 suite bench prof
