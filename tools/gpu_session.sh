#!/bin/bash
# One GPU session: gpu tests, bench, rocprofv3 kernel stats. Stops at the first fault/timeout.
# usage: tools/gpu_session.sh [tests|bench|prof ...]   (default: all)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|137|134|139|135|136) return 0;; *) return 1;; esac; }
steps=${@:-tests bench prof}
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest gpu rc=$rc"; tail -5 $OUT/pytest_gpu.log
      if fatal $rc; then echo "FATAL in tests"; exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
      if fatal $rc; then exit $rc; fi ;;
    bench)
      timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup ${BENCH_WARMUP:-3} ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
      echo "bench rc=$rc"; tail -3 $OUT/bench.log
      if fatal $rc; then exit $rc; fi ;;
    prof)
      export TMPDIR=/tmp
      rm -rf $OUT/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1; rc=$?
      echo "prof rc=$rc"; tail -3 $OUT/prof.log
      if fatal $rc; then exit $rc; fi ;;
    *) echo "unknown step $s";;
  esac
done
