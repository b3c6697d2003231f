#!/bin/bash
# forward D=64 dropout: one hash per key pair, keep scale on the output: tests, attention timing, BERT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s24.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s24.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/fa_bert_time.py > gpurun_out/fa_bert_time_s24.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fa_bert_time_s24.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s24_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s24_$i.log | cut -c1-100)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
