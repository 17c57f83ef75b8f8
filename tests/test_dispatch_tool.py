"""tools/r06/dispatch.py (kernel stats without warm-up launches): a synthetic
rocprofv3 kernel trace of W warm-up calls, K timed calls and one invariant-check call. Only the
timed calls' dispatches enter the per-kernel figures, also when every call launches its first
kernel twice (config 5's k_run_info)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "r06", "dispatch.py")


def _trace(path, calls):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 1000
        for call in calls:
            for name, dur in call:
                w.writerow({"Kernel_Name": f"void skv::{name}(int)", "Start_Timestamp": t, "End_Timestamp": t + dur})
                t += dur + 10


def _run(path, W, K):
    out = subprocess.run([sys.executable, TOOL, path, str(W), str(K)], check=True, capture_output=True, text=True)
    rows = {}
    for line in out.stdout.splitlines():
        parts = line.split()
        if parts and parts[0].startswith("k_"):
            rows[parts[0]] = (int(parts[1]), float(parts[2]))
    return out.stdout, rows


def test_only_timed_calls_counted(tmp_path):
    # warm-up calls are slow (10x), the check call too; timed calls take 100 / 200 ns per kernel
    slow = [("k_run_header", 1000), ("k_tile", 20000)]
    fast = [("k_run_header", 100), ("k_tile", 2000)]
    p = str(tmp_path / "t.csv")
    _trace(p, [slow, slow, fast, fast, fast, slow])
    text, rows = _run(p, 2, 3)
    assert "timed 3" in text
    assert rows["k_tile"] == (3, 2.0)  # avg_us of the timed calls only
    assert rows["k_run_header"] == (3, 0.1)


def test_first_kernel_twice_per_call(tmp_path):
    call = [("k_run_info", 100), ("k_tile", 1000), ("k_run_info", 100), ("k_wal", 3000)]
    warm = [("k_run_info", 100), ("k_tile", 9000), ("k_run_info", 100), ("k_wal", 9000)]
    p = str(tmp_path / "t.csv")
    _trace(p, [warm, call, call, warm])  # W=1, K=2, one check call
    text, rows = _run(p, 1, 2)
    assert "timed 2" in text
    assert rows["k_wal"] == (2, 3.0)
    assert rows["k_tile"] == (2, 1.0)
    assert rows["k_run_info"] == (4, 0.1)
