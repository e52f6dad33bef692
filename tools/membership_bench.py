"""apply_membership at config[1] size (1M entities, 4096 scene groups): the host planning time and
the device time of a window's membership changes, for
  seg      SwitchScene of `--movers` entities into existing groups (only those segments rewritten),
  newgrp   the same plus one entity into a new (scene, group): the segment table is rebuilt,
  overflow `--movers` entities into ONE existing group, past its slack: rebuilt as well.
Each window is followed by a frame (nfk_execute), timed end to end with a device sync.
    python tools/membership_bench.py [--entities N] [--movers M] [--rounds R]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--entities", type=int, default=1 << 20)
    ap.add_argument("--groups", type=int, default=4096)
    ap.add_argument("--movers", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    from noahgameframe_amd import kernel, workload
    torch.cuda.set_device(0)
    w = workload.bench_world(n_obj=a.entities, groups=a.groups, n_ticks=1)
    w["init_i"][workload.PID["SceneID"]] = w["scene"]
    m = kernel.world_from_workload(w, slack_per_256=16)
    has_stats = hasattr(m.lib, "nfk_membership_stats")
    rng = np.random.default_rng(1)
    gh, gd = w["guid_head"], w["guid_data"]
    scene, group = np.array(w["scene"]), np.array(w["group"])
    pairs = np.unique(np.stack([scene, group], 1), axis=0)
    t0, tick = int(w["tick_time"][0]), 0

    def frame():
        nonlocal tick
        torch.cuda.synchronize()
        t = time.perf_counter()
        m.Execute(t0 + 100 * tick)
        torch.cuda.synchronize()
        tick += 1
        return 1000 * (time.perf_counter() - t)

    for _ in range(3):
        frame()
    base = [frame() for _ in range(3)]
    new_group = int(group.max()) + 1
    res = {"entities": a.entities, "groups": len(pairs), "movers": a.movers, "plain_frame_ms": float(np.median(base))}
    for kind in ("seg", "newgrp", "overflow"):
        walls, dev, host = [], [], []
        for r in range(a.rounds):
            movers = rng.choice(a.entities, a.movers, replace=False)
            if kind == "overflow":
                tgt = pairs[rng.integers(len(pairs))]
                dst = np.repeat(tgt[None, :], a.movers, 0)
            else:
                dst = pairs[rng.integers(0, len(pairs), a.movers)]
            if kind == "newgrp":
                dst[0] = (dst[0][0], new_group)
                new_group += 1
            for o, (sc, gr) in zip(movers, dst):
                m.SwitchScene((int(gh[o]), int(gd[o])), int(sc), int(gr), 0.0, 0.0, 0.0)
                scene[o], group[o] = sc, gr
            pairs = np.unique(np.stack([scene, group], 1), axis=0)
            st0 = m.membership_stats() if has_stats else None
            m.reset_kernel_times()
            m.set_profiling(True)
            walls.append(frame())
            m.set_profiling(False)
            ms, n, _ = m.kernel_times()
            dev.append(float(ms[5]) if len(ms) > 5 else float("nan"))
            if has_stats:
                st1 = m.membership_stats()
                host.append((st1["host_ms_full"] - st0["host_ms_full"]) + (st1["host_ms_seg"] - st0["host_ms_seg"]))
                res.setdefault(kind + "_path", "full" if st1["n_full"] > st0["n_full"] else "seg")
        res[kind] = {"frame_ms": float(np.median(walls)), "membership_device_ms": float(np.median(dev)),
                     "membership_host_ms": float(np.median(host)) if host else None}
    m.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
