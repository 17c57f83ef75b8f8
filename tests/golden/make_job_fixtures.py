"""Regenerates tests/golden/job_quirks.json: the job wrappers' outcomes (skv/jobs.py) with the oracle
as the compactor. The quirks it pins are the reference's (src/jobs/*.rs): 16-run fan-in with ALL
runs marked compacted, L0 at SeqNo 0, "No runs were generated during compaction", the Delete
filter at Level::max(), WAL table split and error kinds. Run from the repo root:
    python tests/golden/make_job_fixtures.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "skyvault-rs_amd")]

from test_jobs import OracleCompactor, _jobs_outcome  # noqa: E402

if __name__ == "__main__":
    out = _jobs_outcome(OracleCompactor())
    with open(os.path.join(HERE, "job_quirks.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", len(out), "cases")
