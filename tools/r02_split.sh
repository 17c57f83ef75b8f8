#!/bin/bash
# Parallel-split check on one MI355X: its parity tests, the 3F plan report and a rocprofv3
# kernel-trace summary of the 3F bench. Output: gpurun_out/split_*.log, gpurun_out/sp3f/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/split_t.log 2>&1 || { echo "split tests failed"; exit 1; }
SKV_SPLIT_DEBUG=1 timeout -k 10 300 python bench.py --config 3F --steps 1 --warmup 0 --no-cpu-baseline \
  --no-host-path > gpurun_out/split_b.log 2>&1 || { echo "3F debug bench failed"; exit 1; }
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/sp3f" -o run -- \
  python3 "$R/bench.py" --config 3F --steps 3 --warmup 1 --no-cpu-baseline --no-host-path \
  > "$R/gpurun_out/sp3f.log" 2>&1 || { echo "3F profile failed"; exit 1; }
exit 0
