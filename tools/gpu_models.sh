#!/bin/bash
# The other bench models on the final tree: BERT-base seq 512, ResNet-50 alone, GPT-3 13B with recompute.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 || { tail -5 gpurun_out/bench_bert.log; exit 1; }
tail -1 gpurun_out/bench_bert.log | cut -c1-300
timeout -k 10 300 python bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/bench_resnet.log 2>&1 || { tail -5 gpurun_out/bench_resnet.log; exit 1; }
tail -1 gpurun_out/bench_resnet.log | cut -c1-300
timeout -k 10 500 python bench.py --model gpt3-13b --recompute --steps 3 --warmup 1 > gpurun_out/bench_13b.log 2>&1 || { tail -5 gpurun_out/bench_13b.log; exit 1; }
tail -1 gpurun_out/bench_13b.log | cut -c1-300
