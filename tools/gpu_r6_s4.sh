#!/bin/bash
# round 6: RNN v2 step kernels (tests + timing, v1 vs v2), BERT NT tile A/B, default GPT+ResNet bench
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_rnn_gpu.py -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_rnn_v2_r6.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_rnn_v2_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u tools/rnn_prof.py > gpurun_out/rnn_v2_time.log 2>&1 && PHA_RNN_V1=1 timeout -k 10 120 python -u tools/rnn_prof.py >> gpurun_out/rnn_v2_time.log 2>&1
rc=$?; cat gpurun_out/rnn_v2_time.log | grep LSTM; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/bert_gemm_ab.py > gpurun_out/bert_gemm_ab_r6.log 2>&1
rc=$?; tail -9 gpurun_out/bert_gemm_ab_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_r6_s4.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r6_s4.log; exit $rc
