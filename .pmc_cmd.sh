cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/pmc2 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc2/p1 -o p1 -- python tools/g4p_pmc.py > gpurun_out/pmc2/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc2/p2 -o p2 -- python tools/g4p_pmc.py > gpurun_out/pmc2/p2.log 2>&1; echo rc=$?
