#!/bin/bash
# one-launch column sums: full GPU suite, then BERT alternating PHA_COLSUM1=1/0, then a kernel profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s25.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s25.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for c in 1 0; do
    PHA_COLSUM1=$c timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s25_c${c}_$i.log 2>&1
    rc=$?; echo "bert colsum1=$c $i: $(tail -1 gpurun_out/bench_bert_s25_c${c}_$i.log | cut -c1-80)"; [ $rc -ne 0 ] && exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert5 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert5.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert5.log | cut -c1-100; exit $rc
