#!/bin/bash
# kernel-trace stats of tools/stage_probe.py under one env variant ($1)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/pp" -o run -- \
  python3 "$R/tools/stage_probe.py" "$@" > "$O/pp.log" 2>&1 || exit 1
cd "$R"
f=$(ls $O/pp/*kernel_stats.csv | head -1)
cp "$f" "$O/pp_stats.csv"; rm -rf "$O/pp"
python3 -c "
import csv
rows=list(csv.DictReader(open('$O/pp_stats.csv')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:14]: print('  %-40s %6s calls %9.1f us avg' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
cat $O/pp.log | grep -v amdgpu.ids
