#!/bin/bash
# GPU test suite, then (only if the suite ended without a fault / timeout) the default bench.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc2=$?
tail -4 gpurun_out/bench_default.log
exit $rc2
