#!/bin/bash
# round 6 (session 2): head-dim-64 flash attention kernels (flash_attn_d64.hip) — numerics vs fp32 and
# vs the generic kernels, FA timing at the BERT shape, BERT-base x2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fa64_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fa64.log 2>&1
rc=$?; grep -E "passed|failed|Error|error" gpurun_out/pytest_fa64.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/fa_bert_time.py > gpurun_out/fa_bert_time_fa64.log 2>&1; cat gpurun_out/fa_bert_time_fa64.log | grep -v amdgpu.ids
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s13_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s13_$i.log | cut -c1-330)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
