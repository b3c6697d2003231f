#!/bin/bash
# round 6: BERT-base kernel profile of the current tree + a 20-step BERT bench
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_r6.log 2>&1 || { tail -5 gpurun_out/bench_bert_r6.log; exit 1; }
tail -1 gpurun_out/bench_bert_r6.log
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_bert -o run -- python bench.py --model bert-base --steps 5 --warmup 3 > gpurun_out/prof_bert_r6.log 2>&1 || { tail -5 gpurun_out/prof_bert_r6.log; exit 1; }
f=$(find /tmp/prof_bert -name "*results.db" | head -1)
timeout 200 python tools/prof_db_summary.py "$f" 8 50 > gpurun_out/bert_base_r6_kernels.txt
head -60 gpurun_out/bert_base_r6_kernels.txt
