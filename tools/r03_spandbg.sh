#!/bin/bash
# span parse debug: failing lanes on device-generated config-3 runs, kernel times of a small call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r03; mkdir -p $O
timeout -k 10 200 python -u tools/stage_probe.py --run-mib 2 SKV_SPAN=1,SKV_SPAN_DBG=1 > $O/spandbg_dev.log 2>&1 || { tail -30 $O/spandbg_dev.log; exit 1; }
grep -v "^span \|^check\|^\[span\]" $O/spandbg_dev.log | tail -3; grep "^span \|^check\|^\[span\]" $O/spandbg_dev.log | head -40
export TMPDIR=/tmp; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/spk -o run -- python3 $R/tools/span_dbg.py 64 4000000 noref > $O/spk.log 2>&1 || exit 1
cd $R; f=$(ls $O/spk/*kernel_stats.csv | head -1); python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:12]: print('  %-40s %6s calls %9.1f us avg' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e3))"
rm -rf $O/spk
