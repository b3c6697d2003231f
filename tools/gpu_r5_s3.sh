#!/bin/bash
# round 5 session 3: new GPU tests (fused LAMB, bmm, native inference, split extremes), BERT-base
# 20-step bench, ResNet-50-only kernel profile (summarised on the box)
mkdir -p gpurun_out
fatal() { [ "$1" -eq 124 ] || [ "$1" -gt 128 ]; }
timeout -k 10 300 python -u -m pytest tests/test_distributed_fused_lamb.py tests/test_bmm_gpu.py tests/test_native_infer.py tests/test_fp32_paths_gpu.py tests/test_gemm_quant_gpu.py tests/test_resnet_unit.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5_s3_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r5_s3_tests.log; fatal $rc && exit $rc
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/r5_bert.log 2>&1
rc=$?; tail -3 gpurun_out/r5_bert.log; fatal $rc && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_resnet -o run -- python bench.py --model resnet50 --steps 5 --warmup 2 --graph off > gpurun_out/r5_prof_resnet.log 2>&1
rc=$?; tail -2 gpurun_out/r5_prof_resnet.log; fatal $rc && exit $rc
python tools/prof_db_summary.py /tmp/prof_resnet/run_results.db 7 45 > gpurun_out/r5_resnet_kernels.txt 2>&1; head -50 gpurun_out/r5_resnet_kernels.txt
