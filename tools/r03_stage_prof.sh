#!/bin/bash
# kernel-trace stats of config 3 with and without staged chunk walks; a traced general pipeline call
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03; mkdir -p $O
for v in 0 1; do
  cd /tmp
  SKV_STAGE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sp_$v" -o run -- \
    python3 "$R/bench.py" --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$O/sp_$v.log" 2>&1 || exit 1
  cd "$R"
  f=$(ls $O/sp_$v/*kernel_stats.csv | head -1)
  cp "$f" "$O/sp_stats_$v.csv"; rm -rf "$O/sp_$v"
  echo "STAGE=$v"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$O/sp_stats_$v.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:8]: print('  %-40s %6s calls %9.1f us avg' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
done
SKV_HOST_TRACE=1 timeout -k 10 300 python tools/hp_cfg3.py 8 > gpurun_out/r03/hp_trace.log 2>&1 || exit 1
grep "gpipe" gpurun_out/r03/hp_trace.log | sort | uniq -c | head
