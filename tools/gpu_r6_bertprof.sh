#!/bin/bash
# round 6: BERT-base kernel breakdown on the current tree (graphed step)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_bert -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert_r6b.log 2>&1 || { tail -5 gpurun_out/prof_bert_r6b.log; exit 1; }
f=$(find /tmp/prof_bert -name "*results.db" | head -1)
timeout 200 python tools/prof_db_summary.py "$f" 8 60 > gpurun_out/bert_base_r6b_kernels.txt
head -70 gpurun_out/bert_base_r6b_kernels.txt
