#!/bin/bash
# k_tile<true> wave-sort merge: xshfl self-check, the general-path parity tests, config 3 / 3F timings
# under the kernel trace (timed compactions only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/p2"; mkdir -p "$O"
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/xchk tools/ubench/xshfl_check.hip 2>/dev/null
timeout -k 10 60 /tmp/xchk || { echo "xshfl check failed"; exit 1; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m "gpu and not slow" \
  tests/test_gpu_parity.py tests/test_gpu_kat.py tests/test_gpu_split.py tests/test_gpu_scan.py tests/test_gpu_search.py tests/test_gpu_shard_split.py \
  > "$O/pytest.log" 2>&1; rc=$?; tail -5 "$O/pytest.log"; [ $rc -ne 0 ] && exit 1
for c in ${CONFIGS:-3 3F}; do
  extra="--steps 10 --warmup 2"; [ "$c" = 3F ] && extra="--steps 5 --warmup 1"
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$O/trace$c" -o run -- \
    python3 "$R/bench.py" --config $c $extra --no-host-path --no-cpu-baseline > "$O/bench_$c.log" 2>&1
  rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "$c rc=$rc"; tail -5 "$O/bench_$c.log"; exit 1; }
  grep -E '^\{"metric"' "$O/bench_$c.log" | tail -1 | cut -c1-200
  f=$(find "$O/trace$c" -name "*kernel_trace.csv" | head -1)
  W=2; K=10; [ "$c" = 3F ] && { W=1; K=5; }
  python3 tools/r06/dispatch.py "$f" $W $K --out "$O/kstats_$c.csv" > "$O/kstats_$c.txt"
  head -12 "$O/kstats_$c.txt"
  rm -rf "$O/trace$c"
done
