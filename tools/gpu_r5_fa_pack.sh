#!/bin/bash
# packed-QKV ext attention gradients + GELU epilogue tests, then the BERT-base bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash or gelu or mlp or bert" > gpurun_out/r5_fa_pack.log 2>&1 || { tail -30 gpurun_out/r5_fa_pack.log; exit 1; }
tail -3 gpurun_out/r5_fa_pack.log
timeout -k 10 300 python bench.py --model bert-base --steps 20 --warmup 5 > gpurun_out/r5_bert3.log 2>&1 || { tail -20 gpurun_out/r5_bert3.log; exit 1; }
tail -1 gpurun_out/r5_bert3.log | cut -c1-300
