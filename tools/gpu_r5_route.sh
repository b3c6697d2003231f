#!/bin/bash
# downsample-block gradient route: tests, then alternating ResNet-50 bench A/B (PHA_RES_ROUTE_CONV 1 / 0)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "route or addend or resnet" > gpurun_out/r5_route_tests.log 2>&1 || { tail -30 gpurun_out/r5_route_tests.log; exit 1; }
tail -2 gpurun_out/r5_route_tests.log
for i in 1 2; do
  for r in 1 0; do
    PHA_RES_ROUTE_CONV=$r timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_route${r}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_route${r}_$i.log; exit 1; }
    echo "route_conv=$r run $i: $(tail -1 gpurun_out/r5_bench_route${r}_$i.log | cut -c100-230)"
  done
done
