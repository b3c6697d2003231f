#!/bin/bash
# PMC counters per kernel of the ResNet-50 training step (eager, 3 steps): MFMA busy, waits, LDS
# conflicts, L2 hit rate — two passes within the per-block counter limits, summarised on the box
mkdir -p gpurun_out/resnet_pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=/tmp/resnet_pmc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- python3 bench.py --model resnet50 --steps 2 --warmup 1 --graph off > gpurun_out/resnet_pmc/p1.log 2>&1
rc=$?; tail -2 gpurun_out/resnet_pmc/p1.log; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 bench.py --model resnet50 --steps 2 --warmup 1 --graph off > gpurun_out/resnet_pmc/p2.log 2>&1
rc=$?; tail -2 gpurun_out/resnet_pmc/p2.log; [ $rc -ne 0 ] && exit $rc
d1=$(dirname $(find $O/p1 -name "*counter_collection.csv" | head -1))
d2=$(dirname $(find $O/p2 -name "*counter_collection.csv" | head -1))
timeout 120 python tools/pmc_summary.py gpurun_out/resnet_pmc/summary.txt $d1 $d2
head -40 gpurun_out/resnet_pmc/summary.txt | cut -c1-300
