#!/bin/bash
# conv weight-gradient tile x split-K sweep on the ResNet-50 shapes
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/wgrad_split_sweep.py 256 > gpurun_out/r5_wgrad_sweep.log 2>&1 || { tail -30 gpurun_out/r5_wgrad_sweep.log; exit 1; }
cat gpurun_out/r5_wgrad_sweep.log
