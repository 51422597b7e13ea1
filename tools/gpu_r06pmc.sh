# round 6: every kernel family's HBM bytes on the final tree (two PMC passes)
set -o pipefail
D=gpurun_out/r06pmc; mkdir -p $D; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/f -o pmc --output-format csv -- python3 tools/pmc_kernels.py run > $D/f.log 2>&1 || { tail -5 $D/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/w -o pmc --output-format csv -- python3 tools/pmc_kernels.py run > $D/w.log 2>&1 || { tail -5 $D/w.log; exit 1; }
python3 tools/pmc_kernels.py summarize $D/f $D/w > $D/pmc_kernels.jsonl && cat $D/pmc_kernels.jsonl
