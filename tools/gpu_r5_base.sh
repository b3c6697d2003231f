cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/r5_bench0.log 2>&1 || { tail -5 gpurun_out/r5_bench0.log; exit 1; }
tail -1 gpurun_out/r5_bench0.log
timeout -k 10 300 python tools/g4p_early_ab.py > gpurun_out/r5_early_ab0.log 2>&1 || { tail -5 gpurun_out/r5_early_ab0.log; exit 1; }
cat gpurun_out/r5_early_ab0.log
