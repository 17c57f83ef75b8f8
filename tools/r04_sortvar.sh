#!/bin/bash
# Record-sort variants (tools/build_variants_r04.sh) on config 5, after the sort's parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_fullsize.py tests/test_gpu_hostpipe.py \
  -k "sort or wal or batch or config5 or fan_in or span" -m gpu -x -q --timeout 300 --timeout-method thread > "$O/sortvar_tests.log" 2>&1
rc=$?
tail -2 "$O/sortvar_tests.log"
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)" "$O/sortvar_tests.log" | head -20; exit $rc; }
for v in ${VARIANTS:-base one}; do
  lib=skyvault-rs_amd/skv/libskv.so two=1 hr=0
  # one: the base library with the one-pass bucket search (SKV_SORT_TWO_PASS=0); hostruns: with the
  # host-built run table (SKV_HOST_RUNS=1)
  case $v in base|base2) ;; one) two=0 ;; hostruns|hostruns2) hr=1 ;; *) lib=skyvault-rs_amd/skv/variants/libskv_$v.so ;; esac
  SKV_HOST_RUNS=$hr SKV_SORT_TWO_PASS=$two SKV_LIB=$lib timeout -k 10 300 python bench.py --config 5 --steps 5 --warmup 1 --no-cpu-baseline --no-host-path \
    > "$O/sortvar_$v.log" 2>&1 || { echo "variant $v failed"; tail -5 "$O/sortvar_$v.log"; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/sortvar_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/sortvar_$v.log)"
done
if [ "${PROF:-0}" = 1 ]; then
  SKV_LIB=skyvault-rs_amd/skv/variants/libskv_sortprof.so SKV_SORT_PROF_PRINT=1 timeout -k 10 300 python bench.py --config 5 \
    --steps 2 --warmup 1 --no-cpu-baseline --no-host-path > "$O/sortprof.log" 2>&1 || { tail -5 "$O/sortprof.log"; exit 1; }
  grep "sort prof" "$O/sortprof.log" | tail -4
fi
