#!/bin/bash
# Bench each tuning variant under skyvault-rs_amd/skv/variants (plus the default build); one
# short bench per library, each under its own time limit, stop at the first fatal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/variants
export TMPDIR=/tmp
for lib in skyvault-rs_amd/skv/libskv.so skyvault-rs_amd/skv/variants/libskv_*.so; do
  [ -f "$lib" ] || continue
  tag=$(basename "$lib" .so)
  SKV_LIB="$PWD/$lib" timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-path \
    ${BENCH_ARGS:-} > "gpurun_out/variants/$tag.log" 2>&1
  rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['phases_ms'], d['roofline']['frac'])" "gpurun_out/variants/$tag.log" 2>/dev/null)"
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
