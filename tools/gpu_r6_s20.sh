#!/bin/bash
# round 6 (session 2): D=64 attention with the cheaper keep draw and keep multipliers; tests, timing, BERT x2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py tests/test_kernels_gpu.py -k "fa64 or flash or bert or dropout" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s20.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s20.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/fa_bert_time.py > gpurun_out/fa_bert_time_s20.log 2>&1; grep -v amdgpu.ids gpurun_out/fa_bert_time_s20.log | head -4
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s20_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s20_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; [ $rc -ne 0 ] && exit $rc
done
exit 0
