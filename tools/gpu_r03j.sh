# round 3: DRAM-side PMC counters of the fold at k = 2/4/8 and the batch
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r03j_pmcd
mkdir -p $D
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d $D/a -o pmc --output-format csv -- python3 tools/pmc_dram.py run > $D/a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum -d $D/b -o pmc --output-format csv -- python3 tools/pmc_dram.py run > $D/b.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum -d $D/c -o pmc --output-format csv -- python3 tools/pmc_dram.py run > $D/c.log 2>&1
python3 tools/pmc_dram.py summarize $D/a $D/b $D/c > $D/pmc_dram.jsonl 2>&1
