#!/bin/bash
# round 6 (session 2): BERT-base weight-gradient TN products, own gemm4p split factors vs gemm256 TN vs library
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bert_tn_ab.py > gpurun_out/bert_tn_ab.log 2>&1
rc=$?; cat gpurun_out/bert_tn_ab.log | grep -v amdgpu.ids; exit $rc
