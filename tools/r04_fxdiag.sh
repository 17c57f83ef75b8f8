#!/bin/bash
# Round 4: what the fused tile's key-phase traffic costs. Config 2A, for the default build and the
# diagnostic variants (skv/variants/libskv_<tag>.so): kernel-trace stats (k_fx_tile's duration),
# then FETCH_SIZE / WRITE_SIZE passes. diag4 = keys from a compact array written before the tiles
# (no record-head reads in the tile); diag3 = copy only. Output: gpurun_out/r04/fxdiag/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r04/fxdiag"
mkdir -p "$O"
export TMPDIR=/tmp
for v in ${VARIANTS:-base diag4 diag3}; do
  lib=$R/skyvault-rs_amd/skv/libskv.so
  [ "$v" != base ] && lib=$R/skyvault-rs_amd/skv/variants/libskv_$v.so
  cd /tmp
  SKV_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-host-path --no-check > "$O/bench_$v.log" 2>&1 \
    || { echo "prof $v failed"; tail -5 "$O/bench_$v.log"; exit 1; }
  cd "$R"
  python3 tools/kstats_skv.py "$(ls $O/prof_$v/*kernel_stats.csv | head -1)" 8 "$O/kernel_stats_$v.csv" > /dev/null
  rm -rf "$O/prof_$v"
  echo "$v: $(grep -E 'k_fx_tile|k_fx_keys' $O/kernel_stats_$v.csv | cut -c1-120 | tr '\n' ' ')"
  if [ "${PMC:-1}" = 1 ]; then
    i=0
    for grp in FETCH_SIZE WRITE_SIZE; do
      i=$((i+1))
      cd /tmp
      SKV_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d "$O/pmc_$v/g$i" -o run -- \
        python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-host-path --no-check > "$O/pmc_${v}_g$i.log" 2>&1 \
        || { echo "pmc $v $grp failed"; exit 1; }
      cd "$R"
    done
    python3 tools/traffic.py "$O/pmc_$v" 2A "$O/traffic_$v.json" > "$O/traffic_$v.txt" || { echo "traffic $v failed"; exit 1; }
    grep -E "k_fx_tile|k_fx_keys" "$O/traffic_$v.txt"
    rm -rf "$O/pmc_$v"
  fi
done
exit 0
