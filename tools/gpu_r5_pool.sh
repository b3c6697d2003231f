#!/bin/bash
# 32-bit index walk in the NHWC max-pool kernels: tests, then the ResNet-50 bench and kernel times
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or dispatch or zoo" > gpurun_out/r5_pool_tests.log 2>&1 || { tail -30 gpurun_out/r5_pool_tests.log; exit 1; }
tail -1 gpurun_out/r5_pool_tests.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_pool_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_pool_$i.log; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/r5_bench_pool_$i.log | cut -c100-200)"
done
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_pool -o run -- python bench.py --model resnet50 --steps 5 --warmup 2 --graph off > gpurun_out/prof_pool.log 2>&1 || { tail -5 gpurun_out/prof_pool.log; exit 1; }
f=$(find /tmp/prof_pool -name "*results.db" | head -1)
timeout 200 python tools/prof_db_summary.py "$f" 7 60 > gpurun_out/resnet50_r5_pool_kernels.txt
grep -i "maxpool\|total GPU" gpurun_out/resnet50_r5_pool_kernels.txt
