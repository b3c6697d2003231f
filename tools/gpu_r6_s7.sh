#!/bin/bash
# round 6: split-loop TN column sums (tests + per-shape A/B), BERT host profile
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tn_colsum_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_tn_colsum_r6.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_tn_colsum_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/tn_colsum_ab.py > gpurun_out/tn_colsum_ab_split.log 2>&1
rc=$?; cat gpurun_out/tn_colsum_ab_split.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bert_host_prof.py > gpurun_out/bert_host_prof.log 2>&1
rc=$?; head -50 gpurun_out/bert_host_prof.log; exit $rc
