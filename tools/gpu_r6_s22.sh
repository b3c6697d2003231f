#!/bin/bash
# D=64 dK/dV at 4 vs 8 waves per workgroup: equality tests, then BERT alternating
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s22.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s22.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for w in 4 8; do
    PHA_FA64_DKDV_WAVES=$w timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s22_w${w}_$i.log 2>&1
    rc=$?; echo "bert w$w $i: $(tail -1 gpurun_out/bench_bert_s22_w${w}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
