#!/bin/bash
# round 6: two-stage column-sum finish, exact-GELU fused MLP for BERT; BERT x2 + GPT bench
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tn_colsum_gpu.py tests/test_graph_dropout_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_s9.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_s9.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/bench_bert_s9_$i.log 2>&1
  rc=$?; echo "bert $i: $(tail -1 gpurun_out/bench_bert_s9_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['final_loss'])")"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python bench.py > gpurun_out/bench_s9.log 2>&1
rc=$?; tail -1 gpurun_out/bench_s9.log | cut -c1-420; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/fa_bert_time.py > gpurun_out/fa_bert_time.log 2>&1; cat gpurun_out/fa_bert_time.log
