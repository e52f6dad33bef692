"""Interleaved A/B timing of k_tick / k_fanout variants in ONE process (timing-only
ablations via NFGPU_ABLATE; outputs of ablated variants are not valid).
    python tools/ablate.py [--variants 0,1,2,4] [--rounds 5] [--frames 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--entities", type=int, default=1 << 20)
    ap.add_argument("--config", type=int, default=1, help="1: bench_world, 3: fanout_world, 4: record_world (steady)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from noahgameframe_amd import kernel, workload
    torch.cuda.set_device(0)
    w = (workload.record_world(n_ticks=1, steady=True) if a.config == 4
         else workload.fanout_world(n_ticks=1) if a.config == 3
         else workload.bench_world(n_obj=a.entities, n_ticks=1))
    mods = {}
    for i, v in enumerate(int(x, 0) for x in a.variants.split(",")):
        os.environ["NFGPU_ABLATE"] = str(v)
        # (a variant listed twice gets a world of its own: key "v#i")
        key = v if v not in mods else f"{v}#{i}"
        mods[key] = kernel.world_from_workload(w, slack_per_256=-1)  # as bench.py (no membership changes)
    os.environ.pop("NFGPU_ABLATE", None)
    t0 = int(w["tick_time"][0])
    tick = {v: 0 for v in mods}
    for v, m in mods.items():   # warm up: schedules inserted at the end of frame 0
        for _ in range(5):
            m.Execute(t0 + 100 * tick[v]); tick[v] += 1
        m.summary()
    res = {v: {"k_tick": [], "k_records": [], "k_fanout": []} for v in mods}
    for r in range(a.rounds):
        for v, m in mods.items():
            m.reset_kernel_times()
            m.set_profiling(True)
            for _ in range(a.frames):
                m.Execute(t0 + 100 * tick[v]); tick[v] += 1
            m.set_profiling(False)
            ms, n, b = m.kernel_times()
            res[v]["k_tick"].append(1000 * ms[0] / max(n[0], 1))
            res[v]["k_records"].append(1000 * ms[1] / max(n[1], 1))
            res[v]["k_fanout"].append(1000 * ms[2] / max(n[2], 1))
    out = {v: {k: {"median_us": float(np.median(x)), "min_us": float(np.min(x))} for k, x in d.items()}
           for v, d in res.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
