#!/bin/bash
# embedding-bwd chunking + BERT bench; NT GEMM burst-read variant (LV 6 / 14) sustained A/B
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -gt 128 ]; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "embedding" -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_s5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_s5_tests.log; fatal $rc && exit $rc
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/r5_bert2.log 2>&1
rc=$?; tail -1 gpurun_out/r5_bert2.log | cut -c1-200; fatal $rc && exit $rc
LVS=0,8,6,14 timeout -k 10 400 python tools/g4p_sustain.py > gpurun_out/r5_sustain2.log 2>&1
rc=$?; cat gpurun_out/r5_sustain2.log; exit $rc
