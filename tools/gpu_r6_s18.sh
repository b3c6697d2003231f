#!/bin/bash
# round 6 (session 2): native inference engine — bf16 matrix products on libpha_kernels' MFMA GEMM
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_infer.py -x -v -s --timeout 180 --timeout-method thread > gpurun_out/pytest_native_bf16.log 2>&1
rc=$?; grep -E "passed|failed|Error|native-infer|error" gpurun_out/pytest_native_bf16.log | tail -15; exit $rc
