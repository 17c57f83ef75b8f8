#!/bin/bash
# Fused-tile variants on config 2A: bench phases (10 steps) + one PMC pass (FETCH/WRITE) per library.
# VARIANTS="base c1024 ..." (skv/variants/libskv_<v>.so). Output: gpurun_out/r05/fxvar/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r05/fxvar"; mkdir -p "$O"
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  lib=$R/skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=$R/skyvault-rs_amd/skv/variants/libskv_$v.so
  SKV_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host-path ${BARGS:-} \
    > "$O/bench_$v.log" 2>&1 || { echo "variant $v failed"; tail -5 "$O/bench_$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/bench_$v.log)"
  if [ "${PMC:-1}" = 1 ]; then
    for ctr in FETCH_SIZE WRITE_SIZE; do
      cd /tmp
      SKV_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$v/$ctr" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path ${BARGS:-} > "$O/pmc_${v}_$ctr.log" 2>&1
      rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "pmc $v $ctr rc=$rc"; exit $rc; }
    done
    python3 tools/r05/pmcsum.py "$O/pmc_$v" ${KERNELS:-skv::k_fx_tile}
  fi
done
