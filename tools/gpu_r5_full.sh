#!/bin/bash
# full GPU suite, smoke and the default bench on the current tree
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -gt 128 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_gpu_full.log 2>&1
rc=$?; tail -8 gpurun_out/r5_gpu_full.log; fatal $rc && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r5_smoke.log; fatal $rc && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r5_bench_default.log 2>&1
rc=$?; tail -1 gpurun_out/r5_bench_default.log | cut -c1-400; exit $rc
