"""tools/traffic.py's per-call traffic: two --pmc passes (FETCH_SIZE, WRITE_SIZE)
of a 3-call bench run (warm-up, timed, check), synthetic counter CSVs. The timed call's dispatches are
summed over every kernel, with FETCH_SIZE x2 and KiB -> bytes; a kernel launched twice per call (and
a call whose first kernel runs twice) is counted per call, not per last launch."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# one call: k_run_info twice (as config 5 launches it), k_a once, k_b twice
CALL = ["skv::k_run_info", "skv::k_a", "skv::k_run_info", "skv::k_b", "skv::k_b"]


def _pass(d, counter, scale):
    os.makedirs(d)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        disp = 1
        for call in range(3):
            for k in CALL:
                v = scale * (call + 1) * (10 if k == "skv::k_b" else 1)
                w.writerow({"Dispatch_Id": disp, "Kernel_Name": f"void {k}(int)", "Counter_Name": counter,
                            "Counter_Value": v})
                disp += 1


def test_call_traffic_sums_the_timed_call(tmp_path):
    root = tmp_path / "pmc"
    _pass(str(root / "FETCH_SIZE"), "FETCH_SIZE", 1.0)
    _pass(str(root / "WRITE_SIZE"), "WRITE_SIZE", 3.0)
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "traffic.py"), str(root), "X", str(out)],
                   check=True, capture_output=True)
    doc = json.load(open(out))
    call = doc["configs"]["X"]["call"]
    # timed call = the second: per launch FETCH 2 KiB (k_run_info, k_a) / 20 KiB (k_b), WRITE x3
    fetch_kib = 2 * 2 + 2 + 2 * 20
    assert call["read_bytes"] == fetch_kib * 1024 * 2
    assert call["write_bytes"] == 3 * fetch_kib * 1024
    assert call["launches"] == len(CALL)
    assert call["kernels"]["skv::k_b"] == 2 * 20 * 2048 + 2 * 60 * 1024
    # the per-launch table keeps the last dispatch (the check call)
    assert doc["configs"]["X"]["kernels"]["skv::k_a"]["read_bytes"] == 3 * 2048
