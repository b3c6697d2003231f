#!/bin/bash
# round 6: graph-safe dropout seeds (tests), BERT graphed vs eager, GPT step with the split-loop
# TN column sums
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_dropout_gpu.py tests/test_tn_colsum_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_graph_dropout_r6.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_graph_dropout_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kern_r6s8.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_kern_r6s8.log; [ $rc -ne 0 ] && exit $rc
for m in on off on; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 --graph $m > gpurun_out/bench_bert_r6s8_$m.log 2>&1
  rc=$?; echo "graph=$m $(tail -1 gpurun_out/bench_bert_r6s8_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('hip_graph'))")"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python bench.py > gpurun_out/bench_r6_s8.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r6_s8.log | cut -c1-400; exit $rc
