#!/bin/bash
# NT group_m 8 (K < 4096) vs 4: GEMM tests, the fc1-GELU / NT shapes, full GPT step alternating
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_quant_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or mlp or linear or gpt" > gpurun_out/r5_gm8_tests.log 2>&1 || { tail -30 gpurun_out/r5_gm8_tests.log; exit 1; }
tail -1 gpurun_out/r5_gm8_tests.log
timeout -k 10 300 python -u tools/nt_mb48_ab.py > gpurun_out/r5_nt_mb48_gm8.log 2>&1 || { tail -20 gpurun_out/r5_nt_mb48_gm8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5_nt_mb48_gm8.log
for i in 1 2; do
  for gm in 4 0; do
    if [ $gm = 0 ]; then unset PHA_G4P_GROUP_M; else export PHA_G4P_GROUP_M=$gm; fi
    timeout -k 10 400 python bench.py --no-resnet --steps 6 --warmup 3 > gpurun_out/r5_step_gm${gm}_$i.log 2>&1 || { tail -20 gpurun_out/r5_step_gm${gm}_$i.log; exit 1; }
    echo "gm $gm (0 = new default) run $i: $(tail -1 gpurun_out/r5_step_gm${gm}_$i.log | cut -c150-230)"
  done
done
