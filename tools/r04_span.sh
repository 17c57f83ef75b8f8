#!/bin/bash
# The one-pass span parse (skv_span.hip, SKV_SPAN=1) on one MI355X: its parity tests, the parity
# file with every general-path call forced through it, then configs 3 and 3F timed with the chunk
# walks (SKV_SPAN=0) and with it, plus its phase ticks (SKV_SPAN_DBG=1). Output: gpurun_out/r04/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O="$PWD/gpurun_out/r04"
mkdir -p "$O"
if [ "${PARITY:-1}" = 1 ]; then
SKV_SPAN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$O/span_parity.log" 2>&1
rc=$?
tail -3 "$O/span_parity.log"
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error" "$O/span_parity.log" | head -20; exit $rc; }
SKV_SPAN=1 SKV_SPAN_DBG=1 timeout -k 10 120 python tools/span_dbg.py 16 4000000 > "$O/span_dbg.log" 2>&1 \
  || { tail -20 "$O/span_dbg.log"; exit 1; }
grep -E "span_parse|\[span\]|equal" "$O/span_dbg.log" | head -8
fi
[ "${BENCH:-1}" = 1 ] || exit 0
for c in 3 3F; do
  for v in 0 1; do
    SKV_SPAN=$v timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline \
      --no-host-path > "$O/span_${c}_$v.log" 2>&1 || { echo "bench $c span $v failed"; tail -5 "$O/span_${c}_$v.log"; exit 1; }
    echo "$c span=$v $(grep -o '"ms_per_step": [0-9.]*' $O/span_${c}_$v.log) $(grep -o '"span_parse": [0-9]*' $O/span_${c}_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/span_${c}_$v.log)"
  done
done
for v in span8k span32k; do  # span sizes (the chunk walks' fallback keeps the same chunking)
  for c in 3 3F; do
    SKV_SPAN=1 SKV_LIB=skyvault-rs_amd/skv/variants/libskv_$v.so timeout -k 10 300 python bench.py --config $c --steps 5 \
      --warmup 1 --no-cpu-baseline --no-host-path > "$O/span_${c}_$v.log" 2>&1 || { echo "bench $c $v failed"; tail -5 "$O/span_${c}_$v.log"; exit 1; }
    echo "$c $v $(grep -o '"ms_per_step": [0-9.]*' $O/span_${c}_$v.log) $(grep -o '"span_parse": [0-9]*' $O/span_${c}_$v.log) $(grep -o '"phases_ms": {[^}]*' $O/span_${c}_$v.log)"
  done
done
SKV_SPAN=1 SKV_SPAN_DBG=1 timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline \
  --no-host-path > "$O/span_3_ticks.log" 2>&1 || { tail -5 "$O/span_3_ticks.log"; exit 1; }
grep "\[span\]" "$O/span_3_ticks.log" | tail -2
exit 0
