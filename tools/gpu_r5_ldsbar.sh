#!/bin/bash
# LDS-only barriers in the conv statistics / BN-backward epilogues: tests, per-conv table, ResNet-50
# bench alternating the dgrad-epilogue BN-backward sums off / on
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or bn or batch_norm or resnet" > gpurun_out/r5_ldsbar_tests.log 2>&1 || { tail -30 gpurun_out/r5_ldsbar_tests.log; exit 1; }
tail -1 gpurun_out/r5_ldsbar_tests.log
timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table_ldsbar.log 2>&1 || { tail -30 gpurun_out/r5_conv_table_ldsbar.log; exit 1; }
head -12 gpurun_out/r5_conv_table_ldsbar.log
for i in 1 2; do
  for b in 0 1; do
    PHA_CONV_BN_BWD=$b timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_ldsbar_bnbwd${b}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_ldsbar_bnbwd${b}_$i.log; exit 1; }
    echo "bn_bwd=$b run $i: $(tail -1 gpurun_out/r5_bench_ldsbar_bnbwd${b}_$i.log | cut -c100-200)"
  done
done
