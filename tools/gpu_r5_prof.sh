#!/bin/bash
# GPT step kernel profiles: default policy vs PHA_GEMM_IMPL=own (which kernels the 13 ms/step go to)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_auto -o run -- python bench.py --steps 3 --warmup 2 --no-resnet > gpurun_out/prof_auto.log 2>&1
rc=$?; tail -1 gpurun_out/prof_auto.log; [ $rc -ne 0 ] && exit $rc
PHA_GEMM_IMPL=own timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_own -o run -- python bench.py --steps 3 --warmup 2 --no-resnet --gemm-tuning off > gpurun_out/prof_own.log 2>&1
rc=$?; tail -1 gpurun_out/prof_own.log; exit $rc
