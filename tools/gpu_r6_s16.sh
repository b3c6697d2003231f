#!/bin/bash
# round 6 (session 2): TN weight-gradient schedule variants (PIN / SPREAD) + the D=64 FA suite
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tn_lv_ab.py > gpurun_out/tn_lv_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/tn_lv_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py tests/test_gemm_ring_gpu.py tests/test_tn_colsum_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s16.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s16.log; exit $rc
