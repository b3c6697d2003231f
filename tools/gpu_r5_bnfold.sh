#!/bin/bash
# fused BN fold + finalize: BN / conv / ResNet tests, ResNet-50 bench A/B (PHA_BN_FOLD_FUSED 1 / 0)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or batch_norm or resnet or conv or route" > gpurun_out/r5_bnfold_tests.log 2>&1 || { tail -30 gpurun_out/r5_bnfold_tests.log; exit 1; }
tail -2 gpurun_out/r5_bnfold_tests.log
for i in 1 2; do
  for f in 1 0; do
    PHA_BN_FOLD_FUSED=$f timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r5_bench_bnfold${f}_$i.log 2>&1 || { tail -20 gpurun_out/r5_bench_bnfold${f}_$i.log; exit 1; }
    echo "bnfold=$f run $i: $(tail -1 gpurun_out/r5_bench_bnfold${f}_$i.log | cut -c150-260)"
  done
done
