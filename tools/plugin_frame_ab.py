"""The C++ plugin frame (tests/cpp/plugin_bench) at config[1] with the per-call consumer, one run per
environment variant given on the command line (e.g. NFGPU_PLUGIN_THREADS=0 NFGPU_PLUGIN_THREADS=4),
interleaved over rounds; one JSON line per run (the variant, its phases).

    python tools/plugin_frame_ab.py [--rounds R] [--calls 0|1] VAR=VALUE ...
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--calls", type=int, default=0)
    p.add_argument("--consumer", type=int, default=0)
    p.add_argument("variants", nargs="+")
    a = p.parse_args()
    from noahgameframe_amd import nfio, workload
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "plugin_bench")
    w = workload.bench_world(n_ticks=23, seed=2031, ext_frac=0.05, host_ops=True)
    with tempfile.TemporaryDirectory() as d:
        wp = os.path.join(d, "w.nfio")
        nfio.write(wp, w)
        for r in range(a.rounds):
            for v in a.variants:
                k, val = v.split("=", 1)
                out = subprocess.run([exe, wp, "3", "20", str(a.calls), str(a.consumer)], capture_output=True,
                                     text=True, timeout=600, env=dict(os.environ, **{k: val}), check=True)
                res = json.loads(out.stdout.strip().splitlines()[-1])
                print(json.dumps({"round": r, "variant": v, "frame_ms": res["plugin_frame_ms"],
                                  "phases_ms": res["phases_ms"], "received": res["received"]}), flush=True)


if __name__ == "__main__":
    main()
