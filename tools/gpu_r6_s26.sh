#!/bin/bash
# one-pass LN + dropout backward: GPU tests, then BERT alternating PHA_COLSUM1=1/0, then a kernel profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph_dropout_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s26.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s26.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for c in 1 0; do
    PHA_LN_DROP_FUSED=$c timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s26_c${c}_$i.log 2>&1
    rc=$?; echo "bert lndrop=$c $i: $(tail -1 gpurun_out/bench_bert_s26_c${c}_$i.log | cut -c1-80)"; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert6 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert6.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert6.log | cut -c1-100; exit $rc
