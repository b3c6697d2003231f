#!/bin/bash
# clock vs cycles: fc2-fwd-shaped NT GEMM (own LV0 / LV8 vs hipBLASLt) under sustained load with
# GRBM_GUI_ACTIVE + SQ busy / wait counters per dispatch (kernel durations from the trace); the
# database is summarised on the box (too big to copy back) and removed
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SHAPES="fc2 fwd" SUSTAIN_SECS=0.3 timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS -d /tmp/pmc_sustain -o run -- python tools/g4p_sustain.py > gpurun_out/pmc_sustain.log 2>&1
rc=$?; tail -3 gpurun_out/pmc_sustain.log; [ $rc -ne 0 ] && exit $rc
timeout 120 python tools/pmc_db_dump.py /tmp/pmc_sustain/run_results.db > gpurun_out/pmc_sustain_summary.txt 2>&1
head -60 gpurun_out/pmc_sustain_summary.txt
