#!/bin/bash
# PMC table of the flash-attention kernels (GPT D=128 causal v3 and BERT D=64 with dropout): MFMA
# busy, waits, VALU / LDS instruction counts, LDS bank conflicts — two passes within the per-block
# counter limits, summarised on the box
mkdir -p gpurun_out/fa_pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=/tmp/fa_pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- python3 tools/fa_pmc_run.py > gpurun_out/fa_pmc/p1.log 2>&1
rc=$?; tail -2 gpurun_out/fa_pmc/p1.log; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 tools/fa_pmc_run.py > gpurun_out/fa_pmc/p2.log 2>&1
rc=$?; tail -2 gpurun_out/fa_pmc/p2.log; [ $rc -ne 0 ] && exit $rc
d1=$(dirname $(find $O/p1 -name "*counter_collection.csv" | head -1))
d2=$(dirname $(find $O/p2 -name "*counter_collection.csv" | head -1))
timeout 120 python tools/pmc_summary.py gpurun_out/fa_pmc/summary.txt $d1 $d2
grep -E "fa_|fa64" gpurun_out/fa_pmc/summary.txt | cut -c1-400
