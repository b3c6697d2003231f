#!/bin/bash
# vectorised BN-statistics epilogue: conv / BN GPU tests, per-conv table with the stats epilogue on
# and off, ResNet-50 bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or bn or batch_norm or resnet" > gpurun_out/r5_stats_tests.log 2>&1 || { tail -30 gpurun_out/r5_stats_tests.log; exit 1; }
tail -2 gpurun_out/r5_stats_tests.log
timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table_stats.log 2>&1 || { tail -30 gpurun_out/r5_conv_table_stats.log; exit 1; }
PHA_CONV_BN_STATS=0 timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table_nostats.log 2>&1 || { tail -30 gpurun_out/r5_conv_table_nostats.log; exit 1; }
head -8 gpurun_out/r5_conv_table_stats.log; head -8 gpurun_out/r5_conv_table_nostats.log
timeout -k 10 300 python -u tools/resnet_aten_ops.py 256 > gpurun_out/r5_resnet_aten.log 2>&1 || { tail -20 gpurun_out/r5_resnet_aten.log; exit 1; }
head -16 gpurun_out/r5_resnet_aten.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_stats_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_stats_$i.log; exit 1; }
  echo "run $i: $(tail -1 gpurun_out/r5_bench_stats_$i.log | cut -c100-200)"
done
# every conv / wgrad launch re-timed on the current kernels, alternating against the committed table
T=paddle_hackathon_amd/tuning/conv256_gfx950.json
cp $T gpurun_out/conv256_cur.json
timeout -k 10 600 python -u tools/tune_conv256.py --batch 256 --formats NHWC --retune-all --out gpurun_out/conv256_all.json > gpurun_out/r5_tune_all.log 2>&1 || { tail -30 gpurun_out/r5_tune_all.log; exit 1; }
tail -1 gpurun_out/r5_tune_all.log
for i in 1 2; do
  for v in cur all; do
    cp gpurun_out/conv256_$v.json $T
    timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_tune_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_tune_${v}_$i.log; exit 1; }
    echo "$v run $i: $(tail -1 gpurun_out/r5_bench_tune_${v}_$i.log | cut -c100-200)"
  done
done
