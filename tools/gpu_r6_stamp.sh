#!/bin/bash
# round 6: where the NT gemm4p K-loop waits (s_memtime stamps, tools/g4p_stamp.py)
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/g4p_stamp.py > gpurun_out/g4p_stamp_r6.log 2>&1
rc=$?; cat gpurun_out/g4p_stamp_r6.log | tail -30; exit $rc
