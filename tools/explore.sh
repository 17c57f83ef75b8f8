#!/bin/bash
# Ad-hoc exploration: bench each (library, bench args) pair listed in $EXPLORE (";"-separated
# "tag|lib|args|VAR=VAL ..." entries), one short run each under its own time limit; stop at the first fatal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/explore
export TMPDIR=/tmp
IFS=';' read -ra ENTRIES <<< "$EXPLORE"
for e in "${ENTRIES[@]}"; do
  IFS='|' read -r tag lib args envs <<< "$e"
  env ${envs:-} SKV_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu-baseline --no-host-path \
    $args > "gpurun_out/explore/$tag.log" 2>&1
  rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['phases_ms'], d['roofline']['frac'])" "gpurun_out/explore/$tag.log" 2>/dev/null)"
  case $rc in 0) ;; *) echo "stopping"; tail -5 "gpurun_out/explore/$tag.log"; exit $rc;; esac
done
