#!/bin/bash
# round 6 (session 2): D=64 attention with additive masks; tests, timing, and an alternating BERT A/B of
# the current D=64 kernels against the previous commit's (PHA_KERNELS_LIB=libpha_kernels_old64.so)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py tests/test_kernels_gpu.py -k "fa64 or flash or bert or dropout or mask" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s21.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_s21.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/fa_bert_time.py > gpurun_out/fa_bert_time_s21.log 2>&1; grep -v amdgpu.ids gpurun_out/fa_bert_time_s21.log | head -4
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PHA_KERNELS_LIB=libpha_kernels_old64.so; else unset PHA_KERNELS_LIB; fi
    timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s21_${v}_$i.log 2>&1
    rc=$?; echo "bert $v $i: $(tail -1 gpurun_out/bench_bert_s21_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
