#!/bin/bash
# PMC passes over the fused tile kernel for the default build and each variant library, one
# rocprofv3 --pmc run per counter group (kernel-trace only). Output: gpurun_out/pmcfx/<lib>/g<i>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p "$R/gpurun_out/pmcfx"
export TMPDIR=/tmp
GROUPS_DEFAULT="FETCH_SIZE WRITE_SIZE TCC_HIT_sum,TCC_MISS_sum SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_INSTS_SALU"
for lib in skyvault-rs_amd/skv/libskv.so ${LIBS:-}; do
  tag=$(basename "$lib" .so)
  i=0
  for grp in ${PMC_GROUPS:-$GROUPS_DEFAULT}; do
    grp=${grp//,/ }
    i=$((i+1))
    cd /tmp
    SKV_LIB="$R/$lib" timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmcfx/$tag/g$i" -o run -- \
      python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path > "$R/gpurun_out/pmcfx/$tag.g$i.log" 2>&1
    rc=$?; echo "$tag pmc group $i ($grp) rc=$rc"
    cd "$R"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
