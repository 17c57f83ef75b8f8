#!/bin/bash
# Round 4 measurement call: the fused-tile traffic study (tools/r04_fxdiag.sh: default build,
# compact-key diag4, copy-only diag3, with PMC), an A/B of the occupancy variants (u1, u1w8) on the
# config-2A bench, and config 5 with the host trace (where the call's host time goes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
if [ "${DIAG:-1}" = 1 ]; then
  bash tools/r04_fxdiag.sh || exit 1
fi
if [ "${AB:-1}" = 1 ]; then
  for r in 0 1; do
    for v in base u1 u1w8 cap1024; do
      lib=skyvault-rs_amd/skv/libskv.so
      [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
      SKV_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path \
        > "$O/ab_$v$r.log" 2>&1 || { echo "variant $v failed"; tail -3 "$O/ab_$v$r.log"; exit 1; }
      echo "$v:$r $(grep -o '"ms_per_step": [0-9.]*' $O/ab_$v$r.log) $(grep -o '"check": [0-9.]*' $O/ab_$v$r.log) $(grep -o '"avg_launch_ms": [0-9.]*' $O/ab_$v$r.log)"
    done
  done
fi
if [ "${T2K:-1}" = 1 ]; then  # general merge tiles of 2048 (2 workgroups per CU) vs 4096 (1 per CU)
  for c in 3F 3; do
    for v in base tile2k seg512 seg1024; do
      lib=skyvault-rs_amd/skv/libskv.so
      [ "$v" != base ] && lib=skyvault-rs_amd/skv/variants/libskv_$v.so
      SKV_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline --no-host-path \
        > "$O/t2k_${c}_$v.log" 2>&1 || { echo "tile variant $v $c failed"; tail -3 "$O/t2k_${c}_$v.log"; exit 1; }
      echo "$c $v $(grep -o '"ms_per_step": [0-9.]*' $O/t2k_${c}_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/t2k_${c}_$v.log)"
    done
  done
fi
if [ "${C5:-1}" = 1 ]; then
  SKV_HOST_TRACE=1 timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-host-path \
    > "$O/c5_trace.log" 2>&1 || { echo "config 5 failed"; tail -5 "$O/c5_trace.log"; exit 1; }
  tail -1 "$O/c5_trace.log" | cut -c1-400
  # the PCIe-inclusive figure of config 5 (10^6 tiny WAL runs: the cut search over every run on the
  # host, the kernel ingest), with the host milestones of each call
  SKV_HOST_TRACE=1 timeout -k 10 400 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$O/c5_host.log" 2>&1 || { echo "config 5 host failed"; tail -5 "$O/c5_host.log"; exit 1; }
  tail -1 "$O/c5_host.log" | grep -o '"host_path": {[^}]*' | cut -c1-300
fi
exit 0
