#!/bin/bash
# Submit one gpurun call; when no box / slot is free (exit 3, nothing ran or was charged) wait
# and submit the same call again, at most 8 times. Any other outcome (success, failure, timeout)
# ends here. usage: tools/gpu_call.sh OUT_FILE TIMEOUT_S 'command'
out=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then exit $rc; fi
  sleep 120
done
exit 3
