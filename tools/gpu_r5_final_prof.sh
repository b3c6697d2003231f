#!/bin/bash
# kernel profile of the default GPT step (micro-batch 48) and of the ResNet-50 step on the final tree
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof_final_gpt -o run -- python bench.py --steps 3 --warmup 2 --no-resnet > gpurun_out/prof_final_gpt.log 2>&1 || { tail -5 gpurun_out/prof_final_gpt.log; exit 1; }
f=$(find /tmp/prof_final_gpt -name "*results.db" | head -1)
timeout 200 python tools/prof_db_summary.py "$f" 5 45 > gpurun_out/gpt3_r5_final_kernels_mb48.txt
head -12 gpurun_out/gpt3_r5_final_kernels_mb48.txt
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_final_rn -o run -- python bench.py --model resnet50 --steps 5 --warmup 2 --graph off > gpurun_out/prof_final_rn.log 2>&1 || { tail -5 gpurun_out/prof_final_rn.log; exit 1; }
f=$(find /tmp/prof_final_rn -name "*results.db" | head -1)
timeout 200 python tools/prof_db_summary.py "$f" 7 40 > gpurun_out/resnet50_r5_final_kernels_s2d.txt
head -12 gpurun_out/resnet50_r5_final_kernels_s2d.txt
