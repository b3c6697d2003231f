#!/bin/bash
# round 6: TN column sums (debug decode, tests, per-shape A/B), BERT bench x2 (host-overhead check)
mkdir -p gpurun_out
timeout -k 10 120 python tools/colsum_debug.py > gpurun_out/colsum_debug.log 2>&1 || { tail -5 gpurun_out/colsum_debug.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_tn_colsum_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tn_colsum_r6.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_tn_colsum_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/tn_colsum_ab.py > gpurun_out/tn_colsum_ab.log 2>&1
rc=$?; cat gpurun_out/tn_colsum_ab.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_r6s6_$i.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_bert_r6s6_$i.log | cut -c1-330; [ $rc -ne 0 ] && exit $rc
done
exit 0
