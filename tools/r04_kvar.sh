#!/bin/bash
# Per-kernel A/B of library variants on one config: each variant's bench under rocprofv3
# --kernel-trace --stats, the average duration of the kernels named in KERNELS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R="$PWD"
O="$R/gpurun_out/r04/kvar"
mkdir -p "$O"
export TMPDIR=/tmp
C=${CONFIG:-5}
# a variant is a library tag (skv/variants/libskv_<tag>.so), base / base<N> (the default library), or
# NAME=VALUE (the default library with that environment variable)
for v in ${VARIANTS:-base}; do
  lib="$R/skyvault-rs_amd/skv/libskv.so" ev="SKV_KVAR_NONE=1"
  case $v in base|base[0-9]) ;; *=*) ev="$v" ;; *) lib="$R/skyvault-rs_amd/skv/variants/libskv_${v}.so" ;; esac
  cd /tmp
  env "$ev" SKV_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p_$v" -o run -- \
    python3 "$R/bench.py" --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$O/b_$v.log" 2>&1 \
    || { echo "variant $v failed"; tail -3 "$O/b_$v.log"; exit 1; }
  cd "$R"
  cp "$(ls $O/p_$v/*kernel_stats.csv | head -1)" "$O/stats_$v.csv"
  rm -rf "$O/p_$v"
  python3 - "$O/stats_$v.csv" "$v" "${KERNELS:-k_sort}" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[3].split(",")
out = []
for r in rows:
    n = r["Name"].split("(")[0]
    if any(k in n for k in keys):
        out.append(f"{n.replace('skv::', '')} {float(r['TotalDurationNs']) / 1e6 / 5:.3f}")
print(sys.argv[2], "|", "; ".join(out))
PY
done
