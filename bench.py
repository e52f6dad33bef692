"""bench.py — entity-ticks/s of the MI355X NoahGameFrame frame path (BASELINE.json metric).

One "step" = one server frame over this GPU's 1M-entity scene shard: heartbeat scan +
effect programs (property mutation) + dirty diff + scene-group fan-out
(NFCScheduleModule::Execute + NFCKernelModule::Execute + NFCSceneAOIModule fan-out).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Scenes shard naturally: rank r owns scene r+1 with its own 1M entities (weak scaling, no
data-path collective).  Timing: barrier + device sync on both sides of exactly K frames,
max over ranks.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "entity-ticks/sec (update+dirty-diff+fanout) at 1M entities/GPU, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
KNAMES = ["k_tick", "k_records", "k_fanout", "aux", "k_scan_tiles"]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--entities", type=int, default=1 << 20)
    p.add_argument("--groups", type=int, default=4096)
    p.add_argument("--players-per-group", type=int, default=8)
    p.add_argument("--tick-ms", type=int, default=100)
    p.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    p.add_argument("--cpu-sample", type=int, default=65536, help="entities in the CPU baseline sample")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return p.parse_args()


def cpu_baseline(args, w_full):
    """The reference's own classes (oracle/_ref) on a bounded slice of the same workload."""
    from noahgameframe_amd import nfio, workload
    exe = os.path.join(ROOT, "oracle", "_ref", "nf_ref_harness")
    if not os.path.exists(exe):
        return None
    n = min(args.cpu_sample, args.entities)
    groups = max(1, n * args.groups // args.entities)
    ticks = 400
    w = workload.bench_world(n_obj=n, groups=groups, players_per_group=args.players_per_group, n_ticks=ticks,
                             tick_ms=args.tick_ms, seed=2026)
    with tempfile.TemporaryDirectory() as d:
        wp = os.path.join(d, "w.nfio")
        nfio.write(wp, w)
        # calibrate: a short run, then a run sized to ~cpu_seconds of frame work
        r = json.loads(subprocess.run([exe, "--bench", wp, "20"], check=True, capture_output=True,
                                      text=True).stdout)
        per_tick = r["seconds"] / max(r["ticks"], 1)
        t = int(min(ticks, max(20, args.cpu_seconds / max(per_tick, 1e-6))))
        r = json.loads(subprocess.run([exe, "--bench", wp, str(t)], check=True, capture_output=True,
                                      text=True).stdout)
    return {"value": r["entity_ticks_per_s"], "unit": "entity-ticks/s", "cores": 1, "kind": "reference",
            "sample": f"{n} entities ({groups} groups x {n // groups}, {args.players_per_group} players/group), "
                      f"{r['ticks']} frames of the same heartbeat workload through the reference's "
                      f"NFCPropertyManager/NFCProperty + NFCScheduleModule + per-Set GetBroadCastObject "
                      f"lists, single thread, {r['seconds']:.1f} s"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    def barrier():
        if world > 1:
            dist.barrier()

    from noahgameframe_amd import kernel, workload

    # this rank's scene shard: 1M entities in scene rank+1
    w = workload.bench_world(n_obj=args.entities, groups=args.groups, players_per_group=args.players_per_group,
                             n_ticks=1, tick_ms=args.tick_ms, seed=2026 + rank)
    w["scene"][:] = rank + 1
    stream = torch.cuda.current_stream()
    m = kernel.world_from_workload(w, stream=stream.cuda_stream)
    t0 = int(w["tick_time"][0])
    tick = 0

    def frame():
        nonlocal tick
        m.Execute(t0 + tick * args.tick_ms)
        tick += 1

    for _ in range(args.warmup):
        frame()
    s = m.summary()  # also surfaces any device error from warmup
    m.reset_kernel_times()
    m.set_profiling(True)
    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(args.steps):
        frame()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - ts
    m.set_profiling(False)
    s = m.summary()
    ms, nl, byts = m.kernel_times()
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    # per-kernel averages over the timed region (HIP events on the world's stream)
    kern = {}
    for i, name in enumerate(KNAMES):
        if nl[i]:
            kern[name] = {"avg_us": 1000.0 * ms[i] / nl[i], "launches": int(nl[i]),
                          "alg_bytes_per_launch": (float(byts[i]) / nl[i]) if i < 3 else None}
    dom = max((k for k in kern if kern[k]["alg_bytes_per_launch"]), key=lambda k: kern[k]["avg_us"])
    d = kern[dom]
    achieved = d["alg_bytes_per_launch"] / (d["avg_us"] * 1e-6) / 1e9
    traffic = None
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            traffic = pm.get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    total_alg = sum(v["alg_bytes_per_launch"] or 0 for v in kern.values())
    value = world * args.entities * args.steps / elapsed

    out = {
        "metric": METRIC, "value": value, "unit": "entity-ticks/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64/f64", "data": "synthetic",
        "config": {"workload": "BASELINE config[1]: 1M NPC/Player entities per GPU in one scene, "
                               f"{args.groups} groups x {args.entities // args.groups}, "
                               f"{args.players_per_group} players/group, heartbeats HPRegen 1s/MPRegen 2s/"
                               f"Move 0.1s/Patrol 3s/Poison 0.5s, {args.tick_ms} ms frames",
                   "entities_per_gpu": args.entities, "groups": args.groups,
                   "players_per_group": args.players_per_group, "parallelism": f"scene-shard x{world}"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic},
        "kernels": kern,
        "per_frame": {"prop_events": s["n_prop_events"], "rec_events": s["n_rec_events"], "fired": s["n_fired"],
                      "msgs": s["n_msgs"], "alg_bytes_all_kernels": total_alg,
                      "frame_GBps_alg": total_alg / (elapsed / args.steps) / 1e9},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline(args, w)
    if rank == 0:
        print(json.dumps(out), flush=True)
    m.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
