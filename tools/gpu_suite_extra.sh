#!/bin/bash
# GPU test suite (all failures listed), then — only if it ended without a fault / timeout — the
# fp32 and grouped-conv benchmark tools.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -12 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/bench_fp32.py > gpurun_out/bench_fp32.log 2>&1 || { echo "bench_fp32 failed"; tail -5 gpurun_out/bench_fp32.log; exit 1; }
tail -8 gpurun_out/bench_fp32.log
timeout -k 10 300 python tools/bench_gconv.py > gpurun_out/bench_gconv.log 2>&1
rc3=$?
tail -12 gpurun_out/bench_gconv.log
exit $rc3
