#!/bin/bash
# BERT-base kernel profile (where 29.7 ms/step goes) and ResNet-50 with / without the conv-dgrad
# epilogue BN-backward sums (PHA_CONV_BN_BWD), alternating on one box
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -gt 128 ]; }
timeout -k 10 300 python -u -m pytest tests/test_bmm_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_s4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r5_s4_tests.log; fatal $rc && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o run -- python bench.py --model bert-base --steps 10 --warmup 3 > gpurun_out/r5_prof_bert.log 2>&1
rc=$?; tail -1 gpurun_out/r5_prof_bert.log | cut -c1-300; fatal $rc && exit $rc
python tools/prof_db_summary.py /tmp/prof_bert/run_results.db 13 40 > gpurun_out/r5_bert_kernels.txt 2>&1; head -30 gpurun_out/r5_bert_kernels.txt
for v in 0 1 0 1; do
  PHA_CONV_BN_BWD=$v timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_resnet_bnbwd$v.log 2>&1
  rc=$?; echo "PHA_CONV_BN_BWD=$v: $(tail -1 gpurun_out/r5_resnet_bnbwd$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("resnet50_eager_samples_per_sec"))')"; fatal $rc && exit $rc
done
exit 0
