#!/bin/bash
# Kernel stats (rocprofv3 --kernel-trace --stats) of config 2A per library variant.
# VARIANTS="base c512 ..." Output: gpurun_out/r05/kstats/<v>/ and a per-kernel summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r05/kstats"; mkdir -p "$O"
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  lib=$R/skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=$R/skyvault-rs_amd/skv/variants/libskv_$v.so
  cd /tmp
  SKV_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v" -o run -- \
    python3 "$R/bench.py" --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline --no-host-path ${BARGS:-} > "$O/$v.log" 2>&1
  rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "kstats $v rc=$rc"; tail -5 "$O/$v.log"; exit $rc; }
  f=$(find "$O/$v" -name "*kernel_stats.csv" | head -1)
  echo "== $v"; python3 tools/kstats_skv.py "$f" $(( ${STEPS:-5} + 2 )) | head -14
done
