#!/bin/bash
# round 6: NT gemm4p LDS-DMA placement (SPREAD variants vs the shipped LV 8 and hipBLASLt)
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/g4p_spread.py > gpurun_out/g4p_spread_r6.log 2>&1
rc=$?; tail -20 gpurun_out/g4p_spread_r6.log; exit $rc
