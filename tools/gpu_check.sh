#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench. Each GPU step has its own time
# limit; after a crash / timeout nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = exit code of a GPU step
  case "$1" in 0|1) return 0;; *) echo "FATAL rc=$1 — stopping"; exit "$1";; esac
}
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests.log; stop_if_fatal $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log; stop_if_fatal $rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log; stop_if_fatal $rc
fi
