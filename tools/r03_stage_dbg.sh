#!/bin/bash
# k_spec time of config 3 with staging variants (SKV_STAGE_DBG: 1 no stores, 2 no fingerprint, 3 both)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r03; mkdir -p $O
for v in "0 0" "1 0" "1 1" "1 2" "1 3" "16 0"; do
  set -- $v
  cd /tmp
  SKV_STAGE=$1 SKV_STAGE_DBG=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/sd" -o run -- \
    python3 "$R/bench.py" --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > "$O/sd.log" 2>&1 || exit 1
  cd "$R"
  f=$(ls $O/sd/*kernel_stats.csv | head -1)
  python3 -c "
import csv
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('$f'))}
print('STAGE=$1 DBG=$2', ' '.join('%s=%.1f' % (k.split('::')[-1], float(r['AverageNs'])/1e3) for k, r in rows.items() if any(x in k for x in ('k_spec','k_emit'))))"
  rm -rf "$O/sd"
done
