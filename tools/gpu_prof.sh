#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (no PMC here; counters in gpu_pmc.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-host-path ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.log"
find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
exit $rc
