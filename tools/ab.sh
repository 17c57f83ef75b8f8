#!/bin/bash
# A/B of library variants on one box (the script behind gpurun_out/ab_<tag><round>.log): the default
# build and each variant (skyvault-rs_amd/skv/variants/libskv_<tag>.so, `make variant`) run the
# config-2A bench ROUNDS times, interleaved base, v1, v2, ..., base, v1, ... so that a drift of the
# box over the session lands on every variant alike. One log per (tag, round); the summary line
# per run gives ms per step, the splitter ("check") phase and the k_fx_tile launch time.
# usage: ROUNDS=2 tools/ab.sh tagA tagB ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 0 $(( ${ROUNDS:-2} - 1 ))); do
  for v in base "$@"; do
    lib=skyvault-rs_amd/skv/libskv.so
    [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
    SKV_LIB=$lib timeout -k 10 120 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-host-path \
      > gpurun_out/ab_$v$r.log 2>&1 || { echo "variant $v failed"; exit 1; }
    echo "$v:$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$v$r.log) $(grep -o '"check": [0-9.]*' gpurun_out/ab_$v$r.log) $(grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/ab_$v$r.log)"
  done
done
