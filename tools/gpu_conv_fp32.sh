cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_fp32_paths_gpu.py -q --timeout 120 --timeout-method thread -rf > gpurun_out/pytest_conv_fp32.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_conv_fp32.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_gconv.py > gpurun_out/bench_gconv.log 2>&1 || { tail -5 gpurun_out/bench_gconv.log; exit 1; }
cat gpurun_out/bench_gconv.log | grep resnext
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp32 -o run -- python tools/bench_fp32.py resnet hip > gpurun_out/prof_fp32.log 2>&1 || { tail -5 gpurun_out/prof_fp32.log; exit 1; }
grep resnet gpurun_out/prof_fp32.log
