#!/bin/bash
# ResNeXt-50 32x4d (grouped 3x3 convs on the grouped implicit GEMM): rocprofv3 kernel stats.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gconv -o run -- python3 tools/bench_gconv.py 1 hip > gpurun_out/prof_gconv.log 2>&1 || { tail -5 gpurun_out/prof_gconv.log; exit 1; }
grep resnext gpurun_out/prof_gconv.log
