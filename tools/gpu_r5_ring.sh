#!/bin/bash
# ring-pipeline NT GEMM: bitwise tests, then sustained A/B against the two-buffer kernel and hipBLASLt
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gemm_ring_gpu.py -m gpu -q -x --timeout 60 --timeout-method thread > gpurun_out/r5_ring_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r5_ring_tests.log; [ $rc -ne 0 ] && exit $rc
LVS=adeep timeout -k 10 300 python tools/g4p_sustain.py > gpurun_out/r5_ring_sustain.log 2>&1
rc=$?; cat gpurun_out/r5_ring_sustain.log; exit $rc
