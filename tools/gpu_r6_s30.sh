#!/bin/bash
# batched weight transposes (PHA_WT_BATCH A/B) + pipelined embedding backward: tests, BERT x2, kernel profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_graph_dropout_gpu.py tests/test_kernels_gpu.py tests/test_fa64_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s30.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s30.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for c in 1 0; do
    PHA_WT_BATCH=$c timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s30_c${c}_$i.log 2>&1
    rc=$?; echo "bert wtbatch=$c $i: $(tail -1 gpurun_out/bench_bert_s30_c${c}_$i.log | cut -c1-80)"; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert10 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert10.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert10.log | cut -c1-100; exit $rc
