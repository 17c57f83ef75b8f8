#!/bin/bash
# LDS-DMA copy probe (tools/ubench/dma_copy.hip): both copies timed and cross-checked, then the
# FETCH_SIZE / WRITE_SIZE passes of each (kernel trace only, one counter group per pass)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R="$PWD"; O="$R/gpurun_out/r06/dma"; mkdir -p "$O"
export TMPDIR=/tmp
for c in ${CHUNKS:-32 16}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDMA_C=$c -o /tmp/dma_copy_$c tools/ubench/dma_copy.hip 2>/dev/null || exit 1
  echo "== C=$c"
  timeout -k 10 300 /tmp/dma_copy_$c 20 both || { echo "probe rc=$?"; exit 1; }
done
cd /tmp
for k in direct dma; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_${k}_$ctr" -o run -- /tmp/dma_copy_32 3 $k > "$O/pmc_${k}_$ctr.log" 2>&1 || { echo "pmc $k $ctr failed"; exit 1; }
  done
done
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, sys, os
O = sys.argv[1]
for k in ("direct", "dma"):
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(os.path.join(O, f"pmc_{k}_{ctr}", "**", "*counter_collection.csv"), recursive=True)
        rows = [r for r in csv.DictReader(open(f[0])) if ("k_" + k) in r["Kernel_Name"]]
        v = [float(r["Counter_Value"]) for r in rows]
        vals[ctr] = sum(v) / len(v) if v else float("nan")  # per launch (KB)
    rd = vals["FETCH_SIZE"] * 2 * 1024 / 1e9  # gfx950: FETCH_SIZE reads half of a wide streaming read (MI355X_MICROARCH.md)
    wr = vals["WRITE_SIZE"] * 1024 / 1e9
    print(f"{k:7s} per launch: read {rd:.3f} GB (FETCH_SIZE x 2), write {wr:.3f} GB; algorithmic 4.295 + 4.295 GB")
PY
rm -rf "$O"/pmc_*/
