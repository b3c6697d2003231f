#!/bin/bash
# End-of-session evidence: smoke, the whole GPU suite, the default bench, and a rocprofv3 kernel
# profile of a short bench (stats only).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_gpu_final.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_gpu_final.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -5 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof_final.log 2>&1 || { tail -5 gpurun_out/prof_final.log; exit 1; }
tail -1 gpurun_out/prof_final.log
