#!/bin/bash
# run one gpurun call; if the infrastructure reports no slot/box (nothing ran, nothing charged),
# wait and submit again (at most 8 attempts). Any run that actually started is never resubmitted.
cmd="$1"; to="${2:-1200}"
for a in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > /root/repo/gpurun_out/gpu_try.out 2>&1
  rc=$?
  tail -30 /root/repo/gpurun_out/gpu_try.out
  st=$(python3 -c "import json;d=json.load(open('/root/repo/gpurun_out/.last_call.json'));print(d.get('status'), d.get('run_s') or d.get('run',{}).get('run_s'))" 2>/dev/null)
  echo "[try $a] rc=$rc status=$st"
  if grep -q "status=transient" /root/repo/gpurun_out/gpu_try.out && grep -Eq "run (0.0|None)s" /root/repo/gpurun_out/gpu_try.out; then sleep 200; continue; fi
  exit $rc
done
