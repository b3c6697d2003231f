export PHA_DIST_BACKEND=gloo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --graph off > gpurun_out/rehearse_dp2.log 2>&1
rc=$?
tail -5 gpurun_out/rehearse_dp2.log | cut -c1-600
exit $rc
