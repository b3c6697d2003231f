#!/bin/bash
# round 6 (session 2): D=64 FA with the forward's keep mask stored as bits for the backward
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fa64c.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_fa64c.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/fa_bert_time.py > gpurun_out/fa_bert_time_fa64c.log 2>&1; grep -v amdgpu.ids gpurun_out/fa_bert_time_fa64c.log | head -4
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s15_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s15_$i.log | cut -c150-260)"; [ $rc -ne 0 ] && exit $rc
done
PHA_FA64_MASKBITS=0 timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s15_hash.log 2>&1
rc=$?; echo "bert hash: $(tail -1 gpurun_out/bench_bert_s15_hash.log | cut -c150-260)"; exit $rc
