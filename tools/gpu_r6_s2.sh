#!/bin/bash
# round 6: K-start stagger A/B (tools/g4p_stamp.py) + the new RNN / native-inference GPU tests
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/g4p_stamp.py > gpurun_out/g4p_kstag_r6.log 2>&1
rc=$?; tail -25 gpurun_out/g4p_kstag_r6.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_rnn_gpu.py tests/test_native_infer.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_rnn_infer_r6.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_rnn_infer_r6.log; exit $rc
