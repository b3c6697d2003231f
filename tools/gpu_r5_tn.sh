#!/bin/bash
# weight-gradient (TN) GEMMs: sustained own vs library, then SQ counters of the fc1 dW product
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python tools/tn_sustain.py > gpurun_out/r5_tn_sustain.log 2>&1 || { tail -20 gpurun_out/r5_tn_sustain.log; exit 1; }
cat gpurun_out/r5_tn_sustain.log | grep -v amdgpu.ids
SHAPES="fc1 dW" SUSTAIN_SECS=0.3 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d /tmp/pmc_tn -o run -- python tools/tn_sustain.py > gpurun_out/pmc_tn.log 2>&1
rc=$?; tail -2 gpurun_out/pmc_tn.log; [ $rc -ne 0 ] && exit $rc
timeout 120 python tools/pmc_db_dump.py /tmp/pmc_tn/run_results.db > gpurun_out/pmc_tn_summary.txt 2>&1
head -40 gpurun_out/pmc_tn_summary.txt
