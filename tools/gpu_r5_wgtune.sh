#!/bin/bash
# stem space-to-depth tests, re-time the ResNet-50 weight-gradient launches over tile x split-K (and
# the new stem shape), then alternate the ResNet-50 bench: base (committed table, padded stem), split
# (re-tuned table, padded stem), s2d (re-tuned table, space-to-depth stem)
mkdir -p gpurun_out
T=paddle_hackathon_amd/tuning/conv256_gfx950.json
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stem or dispatch" > gpurun_out/r5_s2d_tests.log 2>&1 || { tail -30 gpurun_out/r5_s2d_tests.log; exit 1; }
tail -2 gpurun_out/r5_s2d_tests.log
cp $T gpurun_out/conv256_old.json
timeout -k 10 600 python -u tools/tune_conv256.py --batch 256 --formats NHWC --retune-tn --out gpurun_out/conv256_new.json > gpurun_out/r5_wgtune.log 2>&1 || { tail -30 gpurun_out/r5_wgtune.log; exit 1; }
tail -2 gpurun_out/r5_wgtune.log
for i in 1 2; do
  for v in base split s2d; do
    if [ $v = base ]; then cp gpurun_out/conv256_old.json $T; else cp gpurun_out/conv256_new.json $T; fi
    S=0; [ $v = s2d ] && S=1
    PHA_CONV_S2D=$S timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_wg_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_wg_${v}_$i.log; exit 1; }
    echo "$v run $i: $(tail -1 gpurun_out/r5_bench_wg_${v}_$i.log | cut -c100-200)"
  done
done
cp gpurun_out/conv256_new.json $T
timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table_new.log 2>&1 || { tail -30 gpurun_out/r5_conv_table_new.log; exit 1; }
head -3 gpurun_out/r5_conv_table_new.log
