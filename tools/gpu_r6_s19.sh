#!/bin/bash
# round 6 (session 2): library-free GEMM policy (PHA_GEMM_IMPL=own, NT on gemm4p with the SPREAD schedule)
# vs the default auto policy, alternating, GPT-3 1.3B and BERT-base
mkdir -p gpurun_out
for i in 1 2; do
  for v in auto own; do
    PHA_GEMM_IMPL=$v timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-resnet > gpurun_out/own2_gpt_${v}_$i.log 2>&1
    rc=$?; echo "gpt $v $i: $(tail -1 gpurun_out/own2_gpt_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; [ $rc -ne 0 ] && exit $rc
  done
done
for i in 1 2; do
  for v in auto own; do
    PHA_GEMM_IMPL=$v timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/own2_bert_${v}_$i.log 2>&1
    rc=$?; echo "bert $v $i: $(tail -1 gpurun_out/own2_bert_${v}_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
