set -o pipefail
for i in 1 2; do
  for m in epi pass; do
    PHA_FUSED_MLP=$m timeout -k 10 200 python -u bench.py --no-resnet --steps 12 --warmup 3 > gpurun_out/ab_${m}_$i.log 2>&1 || exit 1
    echo "$m $i $(tail -1 gpurun_out/ab_${m}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
