#!/bin/bash
# round 6 (session 2): modelled split-K pick for few-tile weight gradients + the element-wise CE path
# (BERT's 30522 vocabulary): CE / TN tests, then BERT-base x2 and the default bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "softmax_cross_entropy or flash or bert" tests/test_tn_colsum_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s12.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s12.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s12_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s12_$i.log | cut -c1-330)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
