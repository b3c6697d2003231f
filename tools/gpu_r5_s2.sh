#!/bin/bash
# round 5 session 2: GPU suite, FA roofline vs SDPA, bench auto vs own GEMM policy.
# A failing test does not stop the call; a crash / abort / time limit (rc > 128 or 124) does.
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -gt 128 ]; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_gputests.log 2>&1
rc=$?; tail -12 gpurun_out/r5_gputests.log; fatal $rc && exit $rc
timeout -k 10 180 python tools/fa_roofline.py > gpurun_out/r5_fa_roofline.log 2>&1
rc=$?; cat gpurun_out/r5_fa_roofline.log; fatal $rc && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r5_bench_auto.log 2>&1
rc=$?; tail -2 gpurun_out/r5_bench_auto.log; fatal $rc && exit $rc
PHA_GEMM_IMPL=own timeout -k 10 300 python bench.py --steps 10 --warmup 3 --gemm-tuning off > gpurun_out/r5_bench_own.log 2>&1
rc=$?; tail -2 gpurun_out/r5_bench_own.log; exit $rc
