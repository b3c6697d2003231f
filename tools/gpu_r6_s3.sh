#!/bin/bash
# round 6: native engine 128-tile GEMM / batched conv (tests + ResNet-50 latency) and an RNN profile
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_native_infer.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_infer_r6b.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_infer_r6b.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rnn_prof -o run -- python tools/rnn_prof.py > gpurun_out/rnn_prof.log 2>&1
rc=$?; tail -3 gpurun_out/rnn_prof.log; exit $rc
