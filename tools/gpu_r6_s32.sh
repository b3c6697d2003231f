#!/bin/bash
# D=64 backward keep multipliers from one signed bitfield extract: attention tests, timing, BERT x2, BERT profile
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s32.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s32.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/fa_bert_time.py > gpurun_out/fa_bert_time_s32.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fa_bert_time_s32.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s32_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s32_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert_s32 -o run -- python bench.py --model bert-base --steps 8 --warmup 3 > gpurun_out/prof_bert_s32.log 2>&1
rc=$?; tail -1 gpurun_out/prof_bert_s32.log | cut -c1-100; exit $rc
