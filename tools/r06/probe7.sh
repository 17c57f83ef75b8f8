#!/bin/bash
# fused tile with the LDS-DMA copy: parity (fused, pipelines, splits; 2A/2B/L0/config 4 at full
# size), then the 2A bench line and its timed-dispatch kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/p7"; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_fused.py tests/test_gpu_hostpipe.py tests/test_gpu_shard_split.py tests/test_gpu_kat.py \
  "tests/test_gpu_fullsize.py::test_config2_full_size" "tests/test_gpu_fullsize.py::test_config4_eight_compactions_at_once" \
  > "$O/pytest.log" 2>&1; rc=$?; tail -4 "$O/pytest.log"; [ $rc -ne 0 ] && exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace2A" -o run -- \
  python3 "$R/bench.py" --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > "$O/bench_2A.log" 2>&1
rc=$?; cd "$R"; [ $rc -ne 0 ] && { echo "2A rc=$rc"; tail -5 "$O/bench_2A.log"; exit 1; }
grep -E '^\{"metric"' "$O/bench_2A.log" | tail -1 | cut -c1-300
f=$(find "$O/trace2A" -name "*kernel_trace.csv" | head -1)
python3 tools/r06/dispatch.py "$f" 3 20 --out "$O/kstats_2A.csv" > "$O/kstats_2A.txt"
head -6 "$O/kstats_2A.txt"
rm -rf "$O/trace2A"
