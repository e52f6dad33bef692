"""Writes tests/golden/tutorial3_10k.json: per-frame line counts and digests of the reference's own server
(tests/cpp/_ref/tutorial3_session_ref: Tutorial3 unchanged on NFKernelPlugin's modules, compiled from
/root/reference) at 10k objects, for tests/test_tutorial3.py.  TEST INFRASTRUCTURE ONLY."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.test_tutorial3 import ARGS_10K, GOLDEN, REF_EXE, digests, run  # noqa: E402

if __name__ == "__main__":
    json.dump({"args": list(ARGS_10K), "frames": digests(run(REF_EXE, ARGS_10K))}, open(GOLDEN, "w"), indent=0,
              sort_keys=True)
    print("wrote", GOLDEN)
