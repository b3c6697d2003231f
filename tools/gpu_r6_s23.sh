#!/bin/bash
# word-major D=64 keep bits: tests, BERT with stored bits vs re-hash alternating, then a kernel profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s23.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s23.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for mb in 1 0; do
    PHA_FA64_MASKBITS=$mb timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s23_mb${mb}_$i.log 2>&1
    rc=$?; echo "bert maskbits=$mb $i: $(tail -1 gpurun_out/bench_bert_s23_mb${mb}_$i.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert4 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert4.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert4.log | cut -c1-200; exit $rc
