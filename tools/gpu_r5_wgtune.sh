#!/bin/bash
# re-time the ResNet-50 weight-gradient launches over tile x split-K, then alternate the ResNet-50
# bench on the committed table (old) and the re-tuned one (new)
mkdir -p gpurun_out
T=paddle_hackathon_amd/tuning/conv256_gfx950.json
cp $T gpurun_out/conv256_old.json
timeout -k 10 600 python -u tools/tune_conv256.py --batch 256 --formats NHWC --retune-tn --out gpurun_out/conv256_new.json > gpurun_out/r5_wgtune.log 2>&1 || { tail -30 gpurun_out/r5_wgtune.log; exit 1; }
tail -2 gpurun_out/r5_wgtune.log
for i in 1 2; do
  for v in old new; do
    cp gpurun_out/conv256_$v.json $T
    timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_wg_${v}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_wg_${v}_$i.log; exit 1; }
    echo "$v run $i: $(tail -1 gpurun_out/r5_bench_wg_${v}_$i.log | cut -c100-200)"
  done
done
cp gpurun_out/conv256_new.json $T
timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table_new.log 2>&1 || { tail -30 gpurun_out/r5_conv_table_new.log; exit 1; }
head -3 gpurun_out/r5_conv_table_new.log
