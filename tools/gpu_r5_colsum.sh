#!/bin/bash
# bias-gradient column sums on the HIP two-stage reduction: kernel tests, then the GPT bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gelu or col_sum or linear or mlp or bias or layer_norm" > gpurun_out/r5_colsum_tests.log 2>&1 || { tail -30 gpurun_out/r5_colsum_tests.log; exit 1; }
tail -2 gpurun_out/r5_colsum_tests.log
timeout -k 10 300 python bench.py --no-resnet --steps 10 --warmup 3 > gpurun_out/r5_bench_colsum.log 2>&1 || { tail -20 gpurun_out/r5_bench_colsum.log; exit 1; }
tail -1 gpurun_out/r5_bench_colsum.log | cut -c150-260
