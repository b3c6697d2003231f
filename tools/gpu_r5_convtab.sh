#!/bin/bash
# per-convolution efficiency table of a ResNet-50 training step (batch 256)
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/resnet_conv_table.py 256 > gpurun_out/r5_conv_table.log 2>&1 || { tail -30 gpurun_out/r5_conv_table.log; exit 1; }
head -60 gpurun_out/r5_conv_table.log
