#!/bin/bash
# The register-staged tile probe (tools/ubench/rs_tile.hip): time per TAU, then one PMC pass each
# for FETCH_SIZE and WRITE_SIZE at TAU=384. Output: gpurun_out/r05/rs/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r05/rs"; mkdir -p "$O"
export TMPDIR=/tmp
B=${BIN:-tools/ubench/rs_tile_rb18}
for tau in ${TAUS:-384 256 448}; do
  timeout -k 10 120 $B $tau > "$O/rs_$tau.txt" 2>&1 || { echo "tau $tau failed"; tail -5 "$O/rs_$tau.txt"; exit 1; }
  cat "$O/rs_$tau.txt"
done
if [ "${PMC:-1}" = 1 ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    cd /tmp
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc/$ctr" -o run -- "$R/$B" 384 > "$O/pmc_$ctr.log" 2>&1
    rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "pmc $ctr rc=$rc"; tail -3 "$O/pmc_$ctr.log"; exit $rc; }
  done
  python3 tools/r05/pmcsum.py "$O/pmc" k_rs
fi
