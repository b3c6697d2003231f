#!/bin/bash
# One GPU session. Steps run in the order given; stops at the first fault/timeout.
# usage: tools/gpu_session.sh smoke bench prof tests tests_fa ...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
cd $ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONUNBUFFERED=1
fatal() { case $1 in 124|137|134|139|135|136) return 0;; *) return 1;; esac; }
for s in "$@"; do
  echo "=== step $s $(date +%T)"
  case $s in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      tail -3 $OUT/smoke.log ;;
    bench_picks)
      PHA_GEMM_PICK_LOG=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $OUT/bench_picks.log 2>&1; rc=$?
      grep -E "gemm-pick|metric" $OUT/bench_picks.log | tail -40 ;;
    bench)
      timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-10} --warmup ${BENCH_WARMUP:-3} ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
      tail -3 $OUT/bench.log ;;
    bench_ln)
      timeout -k 10 300 python tools/bench_ln.py > $OUT/bench_ln.log 2>&1; rc=$?
      tail -3 $OUT/bench_ln.log ;;
    bench_bert)
      timeout -k 10 400 python bench.py --model bert-base --steps 10 --warmup 3 > $OUT/bench_bert.log 2>&1; rc=$?
      tail -3 $OUT/bench_bert.log ;;
    bench_gpt_hipmm)
      PHA_MATMUL_IMPL=hip timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $OUT/bench_gpt_hipmm.log 2>&1; rc=$?
      tail -3 $OUT/bench_gpt_hipmm.log ;;
    bench_gpt13b)
      timeout -k 10 600 python bench.py --model gpt3-13b --micro-batch 2 --recompute --steps 3 --warmup 1 > $OUT/bench_gpt13b.log 2>&1; rc=$?
      tail -4 $OUT/bench_gpt13b.log ;;
    prof_bert)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_bert
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bert -o run --output-format csv -- python3 $ROOT/bench.py --model bert-base --steps 3 --warmup 2 > $OUT/prof_bert.log 2>&1; rc=$?
      tail -3 $OUT/prof_bert.log ;;
    bench_resnet)
      timeout -k 10 400 python bench.py --model resnet50 --steps 10 --warmup 3 > $OUT/bench_resnet.log 2>&1; rc=$?
      tail -3 $OUT/bench_resnet.log ;;
    bench_resnet_lib)
      PHA_CONV_IMPL=library timeout -k 10 400 python bench.py --model resnet50 --steps 10 --warmup 3 > $OUT/bench_resnet_lib.log 2>&1; rc=$?
      tail -3 $OUT/bench_resnet_lib.log ;;
    bench_g256)
      timeout -k 10 300 python tools/bench_gemm256.py > $OUT/bench_g256.log 2>&1; rc=$?
      cat $OUT/bench_g256.log | tail -20 ;;
    prof_resnet_hip)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_resnet_hip
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_resnet_hip -o run --output-format csv -- python3 $ROOT/bench.py --model resnet50 --steps 3 --warmup 2 > $OUT/prof_resnet_hip.log 2>&1; rc=$?
      tail -2 $OUT/prof_resnet_hip.log ;;
    gpt_gemms)
      timeout -k 10 300 python tools/bench_gpt_gemms.py > $OUT/gpt_gemms.log 2>&1; rc=$?
      cat $OUT/gpt_gemms.log | tail -20 ;;
    bench_g8p)
      timeout -k 10 300 python tools/bench_gemm256.py 8p > $OUT/bench_g8p.log 2>&1; rc=$?
      cat $OUT/bench_g8p.log | tail -24 ;;
    g8p_var)
      rc=0; for v in 0 1 2 4 6; do PHA_G8P_VAR=$v timeout -k 10 120 python tools/bench_gemm256.py 8pvar > $OUT/g8p_var$v.log 2>&1 || break; echo "var $v"; tail -4 $OUT/g8p_var$v.log; done ;;
    bench_g256bwd)
      timeout -k 10 400 python tools/bench_gemm256.py bwd > $OUT/bench_g256bwd.log 2>&1; rc=$?
      cat $OUT/bench_g256bwd.log | tail -20 ;;
    prof_g8p)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_g8p; mkdir -p $OUT/prof_g8p
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/prof_g8p/pmc1 -o run --output-format csv -- python3 $ROOT/tools/g256_prof.py 8p > $OUT/prof_g8p/pmc1.log 2>&1; rc=$?
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/prof_g8p/pmc2 -o run --output-format csv -- python3 $ROOT/tools/g256_prof.py 8p > $OUT/prof_g8p/pmc2.log 2>&1; rc=$?; fi
      tail -2 $OUT/prof_g8p/*.log ;;
    prof_g256)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_g256; mkdir -p $OUT/prof_g256
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/prof_g256/pmc1 -o run --output-format csv -- python3 $ROOT/tools/g256_prof.py > $OUT/prof_g256/pmc1.log 2>&1; rc=$?
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/prof_g256/pmc2 -o run --output-format csv -- python3 $ROOT/tools/g256_prof.py > $OUT/prof_g256/pmc2.log 2>&1; rc=$?; fi
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $OUT/prof_g256/pmc3 -o run --output-format csv -- python3 $ROOT/tools/g256_prof.py > $OUT/prof_g256/pmc3.log 2>&1; rc=$?; fi
      tail -2 $OUT/prof_g256/*.log ;;
    prof)
      export TMPDIR=/tmp
      rm -rf $OUT/prof
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --steps 3 --warmup 2 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1; rc=$?
      tail -3 $OUT/prof.log ;;
    prof_resnet)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_resnet
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_resnet -o run --output-format csv -- python3 $ROOT/bench.py --model resnet50 --steps 3 --warmup 2 > $OUT/prof_resnet.log 2>&1; rc=$?
      tail -3 $OUT/prof_resnet.log ;;
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -v -x --timeout 240 -k "not flash" > $OUT/pytest_gpu.log 2>&1; rc=$?
      tail -5 $OUT/pytest_gpu.log ;;
    bench_fa)
      timeout -k 10 300 python tools/bench_fa.py > $OUT/bench_fa.log 2>&1; rc=$?
      cat $OUT/bench_fa.log | tail -10 ;;
    bench_fa_serial)
      PHA_FA_DKDV_ILP=0 timeout -k 10 300 python tools/bench_fa.py > $OUT/bench_fa_serial.log 2>&1; rc=$?
      cat $OUT/bench_fa_serial.log | tail -10 ;;
    tune_gemm)
      # tune GPT + BERT GEMM shapes into gpurun_out/gemm_tunableop_gfx950.csv (copy into paddle_hackathon_amd/tuning/)
      PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 900 python bench.py --steps 1 --warmup 1 --gemm-tuning tune --gemm-tuning-file $OUT/gemm_tunableop_gfx950.csv > $OUT/tune_gpt.log 2>&1; rc=$?
      tail -2 $OUT/tune_gpt.log
      if [ $rc = 0 ]; then PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 600 python bench.py --model bert-base --steps 1 --warmup 1 --gemm-tuning tune --gemm-tuning-file $OUT/gemm_tunableop_gfx950.csv > $OUT/tune_bert.log 2>&1; rc=$?; tail -2 $OUT/tune_bert.log; fi ;;
    bench_tuned)
      timeout -k 10 400 python bench.py --steps 10 --warmup 3 --gemm-tuning db --gemm-tuning-file $OUT/gemm_tunableop_gfx950.csv > $OUT/bench_tuned.log 2>&1; rc=$?
      tail -3 $OUT/bench_tuned.log ;;
    bench_gemm)
      timeout -k 10 600 python tools/bench_gemm.py > $OUT/bench_gemm.log 2>&1; rc=$?
      cat $OUT/bench_gemm.log | tail -20 ;;
    g4w_fixed)
      timeout -k 10 300 python tools/g4w_fixed.py > $OUT/g4w_fixed.log 2>&1; rc=$?
      tail -12 $OUT/g4w_fixed.log ;;
    g4w_nn)
      timeout -k 10 300 python tools/bench_g4w_nn.py > $OUT/g4w_nn.log 2>&1; rc=$?
      tail -40 $OUT/g4w_nn.log ;;
    g4w)
      timeout -k 10 300 python tools/bench_g4w.py > $OUT/g4w.log 2>&1; rc=$?
      tail -40 $OUT/g4w.log ;;
    g4w_s1)
      PHA_G4W_SCHED=1 timeout -k 10 300 python tools/bench_g4w.py > $OUT/g4w_s1.log 2>&1; rc=$?
      tail -30 $OUT/g4w_s1.log ;;
    g4w_var)
      rc=0; for v in 0 2; do PHA_G4W_SCHED=$v timeout -k 10 200 python tools/bench_g4w.py > $OUT/g4w_var$v.log 2>&1 || { rc=$?; break; }; echo "var $v"; grep -E "TF|per-step" $OUT/g4w_var$v.log | tail -20; done ;;
    prof_g4w)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_g4w; mkdir -p $OUT/prof_g4w
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/prof_g4w/pmc1 -o run --output-format csv -- python3 $ROOT/tools/g4w_prof.py > $OUT/prof_g4w/pmc1.log 2>&1; rc=$?
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/prof_g4w/pmc2 -o run --output-format csv -- python3 $ROOT/tools/g4w_prof.py > $OUT/prof_g4w/pmc2.log 2>&1; rc=$?; fi
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d $OUT/prof_g4w/pmc3 -o run --output-format csv -- python3 $ROOT/tools/g4w_prof.py > $OUT/prof_g4w/pmc3.log 2>&1; rc=$?; fi
      tail -2 $OUT/prof_g4w/*.log ;;
    fa_bwd)
      timeout -k 10 300 python tools/bench_fa_bwd.py > $OUT/fa_bwd.log 2>&1; rc=$?
      cat $OUT/fa_bwd.log | tail -12 ;;
    fa_libcmp)
      PHA_KERNELS_LIB=libpha_kernels.so timeout -k 10 120 python tools/fa_lib_compare.py save $OUT/fa_a.pt && PHA_KERNELS_LIB=${FA_LIB_B} timeout -k 10 120 python tools/fa_lib_compare.py save $OUT/fa_b.pt && python tools/fa_lib_compare.py cmp $OUT/fa_a.pt $OUT/fa_b.pt > $OUT/fa_libcmp.log 2>&1; rc=$?
      rm -f $OUT/fa_a.pt $OUT/fa_b.pt; tail -14 $OUT/fa_libcmp.log ;;
    fa_variants)
      rc=0; for lib in ${FA_LIBS:-libpha_kernels.so}; do echo "--- $lib"; PHA_KERNELS_LIB=$lib FA_QUICK=1 timeout -k 10 120 python tools/bench_fa_bwd.py 2>&1 | grep -E "fwd|bwd" || { rc=1; break; }; done > $OUT/fa_variants.log 2>&1
      cat $OUT/fa_variants.log ;;
    prof_g4p)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_g4p; mkdir -p $OUT/prof_g4p
      timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/prof_g4p/pmc1 -o run --output-format csv -- python3 $ROOT/tools/g4p_pmc.py > $OUT/prof_g4p/pmc1.log 2>&1; rc=$?
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/prof_g4p/pmc2 -o run --output-format csv -- python3 $ROOT/tools/g4p_pmc.py > $OUT/prof_g4p/pmc2.log 2>&1; rc=$?; fi
      tail -2 $OUT/prof_g4p/*.log ;;
    rehearse2)
      # two ranks sharing the one GPU over gloo: the multi-rank DP path of bench.py (GPT + ResNet; the
      # multi-rank ResNet step is timed eagerly)
      PHA_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 2 > $OUT/rehearse2.log 2>&1; rc=$?
      grep -E "metric|capture|Error|error" $OUT/rehearse2.log | cut -c1-300 | tail -6 ;;
    bench_forcedp)
      timeout -k 10 400 python bench.py --model resnet50 --force-dp --steps 5 --warmup 3 > $OUT/bench_forcedp.log 2>&1; rc=$?
      tail -1 $OUT/bench_forcedp.log | cut -c1-300 ;;
    bench_ab)
      # alternating default / variant (BENCH_AB_ENV, e.g. PHA_GEMM_AUTO_NT=1) runs of the GPT bench on one box
      rc=0; for i in 1 2; do for v in default variant; do if [ $v = variant ]; then E="$BENCH_AB_ENV"; else E=""; fi; env $E timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-resnet > $OUT/bench_ab_$v$i.log 2>&1 || { rc=1; break 2; }; echo "$v $i $(tail -1 $OUT/bench_ab_$v$i.log | cut -c100-200)"; done; done ;;
    bench_own)
      PHA_GEMM_IMPL=own timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-10} --warmup ${BENCH_WARMUP:-3} --no-resnet > $OUT/bench_own.log 2>&1; rc=$?
      tail -1 $OUT/bench_own.log | cut -c1-400 ;;
    g4p_libs)
      rc=0; for lib in ${G4P_LIBS:-libpha_kernels.so}; do echo "--- $lib"; PHA_KERNELS_LIB=$lib G4P_QUICK=1 timeout -k 10 200 python tools/g4p_early_ab.py 2>&1 | grep -E "TF|sum" || { rc=1; break; }; done > $OUT/g4p_libs.log 2>&1
      cat $OUT/g4p_libs.log ;;
    g4p_early)
      timeout -k 10 300 python tools/g4p_early_ab.py > $OUT/g4p_early.log 2>&1; rc=$?
      cat $OUT/g4p_early.log | tail -16 ;;
    tests_gemm)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "gemm or linear or mlp" > $OUT/pytest_gemm.log 2>&1; rc=$?
      tail -5 $OUT/pytest_gemm.log ;;
    fa_stagger)
      rc=0; for i in 1 2; do for v in 0 1; do echo "--- stagger=$v"; PHA_FA_FWD_STAGGER=$v FA_QUICK=1 timeout -k 10 120 python tools/bench_fa_bwd.py 2>&1 | grep -E "fwd" || { rc=1; break 2; }; done; done > $OUT/fa_stagger.log 2>&1
      cat $OUT/fa_stagger.log ;;
    tests_flash)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "flash" > $OUT/pytest_flash.log 2>&1; rc=$?
      tail -5 $OUT/pytest_flash.log ;;
    tests_all)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 240 --timeout-method thread > $OUT/pytest_gpu_all.log 2>&1; rc=$?
      tail -5 $OUT/pytest_gpu_all.log ;;
    tests_k)
      timeout -k 10 600 python -m pytest tests -m gpu -v -x --timeout 240 -k "${TESTK}" > $OUT/pytest_k.log 2>&1; rc=$?
      tail -15 $OUT/pytest_k.log ;;
    prof_fa)
      # per-kernel times + PMC passes for the flash-attention backward (PHA_FA_BWD selects the path)
      export TMPDIR=/tmp
      rm -rf $OUT/prof_fa; mkdir -p $OUT/prof_fa
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_fa/trace -o run --output-format csv -- python3 $ROOT/tools/fa_prof.py > $OUT/prof_fa/trace.log 2>&1; rc=$?
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $OUT/prof_fa/pmc1 -o run --output-format csv -- python3 $ROOT/tools/fa_prof.py > $OUT/prof_fa/pmc1.log 2>&1; rc=$?; fi
      if [ $rc = 0 ]; then timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/prof_fa/pmc2 -o run --output-format csv -- python3 $ROOT/tools/fa_prof.py > $OUT/prof_fa/pmc2.log 2>&1; rc=$?; fi
      tail -3 $OUT/prof_fa/*.log ;;
    fa_order)
      for g in 0 1 2 4 8; do echo "--- PHA_FA_ORDER_G=$g"; PHA_FA_ORDER_G=$g PHA_FA_BENCH_FAST=1 timeout -k 10 120 python tools/bench_fa.py 2>&1 | grep -E "v2|fused"; rc=$?; done > $OUT/fa_order.log 2>&1
      cat $OUT/fa_order.log ;;
    tests_fa)
      timeout -k 10 600 python -m pytest tests -m gpu -v -x --timeout 120 -k "flash" > $OUT/pytest_fa.log 2>&1; rc=$?
      tail -5 $OUT/pytest_fa.log ;;
    *) echo "unknown step $s"; rc=0 ;;
  esac
  echo "=== step $s rc=$rc $(date +%T)"
  if fatal $rc; then echo "FATAL rc=$rc in $s; stopping"; exit $rc; fi
done
