"""Host-side cost of game logic between frames (bench.py's host_calls variant, config[1] with 5 %
of the entities getting a SetProperty and 1/64 a schedule call every frame), split by phase:
each C-ABI queueing call (GUID lookups; the call arrays are gathered beforehand), and
nfk_execute's own host phases (NFGPU_TRACE_EXEC=1 prints them to stderr).  Needs a GPU.
    python tools/host_calls_profile.py [--frames 20]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import torch
    from noahgameframe_amd import kernel, workload
    frames = args.warmup + args.frames
    w = workload.bench_world(n_obj=1 << 20, groups=4096, players_per_group=8, n_ticks=frames, tick_ms=100,
                             seed=2031, ext_frac=0.05, host_ops=True)
    m = kernel.world_from_workload(w, stream=torch.cuda.current_stream().cuda_stream, slack_per_256=-1)
    gh, gd = w["guid_head"], w["guid_data"]
    xs = np.searchsorted(w["x_tick"], np.arange(frames + 1))
    hs = np.searchsorted(w["h_tick"], np.arange(frames + 1))
    t = {k: 0.0 for k in ("gather", "schedule_calls", "set_props", "execute", "outputs", "gpu_sync")}

    pre = []
    for f in range(frames):
        a, b = hs[f], hs[f + 1]
        a2, b2 = xs[f], xs[f + 1]
        ho, xo = w["h_obj"][a:b], w["x_obj"][a2:b2]
        pre.append((gh[ho], gd[ho], gh[xo], gd[xo]))

    def frame(f, acc):
        c0 = time.perf_counter()
        a, b = hs[f], hs[f + 1]
        a2, b2 = xs[f], xs[f + 1]
        hgh, hgd, xgh, xgd = pre[f]
        c1 = time.perf_counter()
        m.schedule_calls(w["h_op"][a:b], hgh, hgd, w["h_kind"][a:b], w["h_interval"][a:b], w["h_count"][a:b],
                         w["h_time"][a:b])
        c2 = time.perf_counter()
        m.set_props(xgh, xgd, w["x_pid"][a2:b2], w["x_bits"][a2:b2])
        c3 = time.perf_counter()
        m.Execute(int(w["tick_time"][f]))
        c4 = time.perf_counter()
        m.outputs_raw()
        c5 = time.perf_counter()
        if acc:
            t["gather"] += c1 - c0
            t["schedule_calls"] += c2 - c1
            t["set_props"] += c3 - c2
            t["execute"] += c4 - c3
            t["outputs"] += c5 - c4
        return b2 - a2, b - a

    for f in range(args.warmup):
        frame(f, False)
    torch.cuda.synchronize()
    ts = time.perf_counter()
    n_set = n_sched = 0
    for f in range(args.warmup, frames):
        ns, nh = frame(f, True)
        n_set += ns
        n_sched += nh
    c = time.perf_counter()
    torch.cuda.synchronize()
    t["gpu_sync"] = time.perf_counter() - c
    el = time.perf_counter() - ts
    m.close()
    print(json.dumps({"frames": args.frames, "ms_per_frame": 1000 * el / args.frames,
                      "set_calls_per_frame": n_set / args.frames, "schedule_calls_per_frame": n_sched / args.frames,
                      "host_ms_per_frame": {k: round(1000 * v / args.frames, 4) for k, v in t.items()}}))


if __name__ == "__main__":
    main()
