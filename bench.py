"""bench.py — entity-ticks/s of the MI355X NoahGameFrame frame path (BASELINE.json metric).

One "step" = one server frame over this GPU's 1M-entity scene shard: heartbeat scan +
effect programs (property mutation) + dirty diff + scene-group fan-out
(NFCScheduleModule::Execute + NFCKernelModule::Execute + NFCSceneAOIModule fan-out), and the
consumer's nfk_outputs_get (the frame's dense event / message ranks) every frame.

The default line (config[1]) also carries "host_calls": the same world with game logic between
frames (5 % of the entities get a SetProperty, 1/64 an AddSchedule / RemoveSchedule call, every
frame), timed the same way, with the host milliseconds per frame of queueing the calls and of
nfk_execute's host preparation.

    python bench.py [--gpus N] [--steps K] [--warmup W]      (N > 1: bench.py starts the N ranks itself)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Scenes shard naturally: rank r owns scene r+1 with its own 1M entities (weak scaling, no
data-path collective).  Timing: barrier + device sync on both sides of exactly K frames,
max over ranks.  Rank 0 prints one JSON line.
"""
import argparse
import collections
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
HBM_CEILING_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "hbm_ceiling.json")
KNAMES = ["k_tick", "k_records", "k_fanout", "aux", "k_scan_tiles", "membership", "k_chain"]
CONFIG_NAMES = {
    0: "BASELINE config[0]: Tutorial3 (HelloWorld3Module.cpp) scaled to 10k NPC objects in scene 1 group 0: "
       "AddSchedule(self, \"OnHeartBeat\", 5.0, 10) per object (the tutorial's functor-only heartbeat: no "
       "device effect, the fired list goes to the host functor), OnEvent SetPropertyInt(World) on 1 % of the "
       "objects per frame (World's per-object callback), 100 ms frames",
    3: "BASELINE config[3]: 256 scenes x 64 groups, 2M entities per GPU, 32 players per group "
       "(scene-group sync-list fan-out dominated), heartbeats as config[1], 100 ms frames",
    4: "BASELINE config[4]: 500k players per GPU, 64-row skill record each (int cooldown + f64 charge "
       "columns updated by a 100 ms SkillCD heartbeat; steady state: cooldowns of hours, so every frame "
       "updates the same share of cells), groups of 16 players, 100 ms frames",
}


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
    p.add_argument("--cpu-sample", type=int, default=4096, help="entities in the CPU baseline sample (whole groups)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--migrate", type=int, default=256,
                   help="N>1: entities per rank that SwitchScene into the next rank's scene every "
                        "--migrate-every frames (state rows over RCCL all_to_all; BASELINE config[2])")
    p.add_argument("--migrate-every", type=int, default=8,
                   help="frames between migration batches (8 = 256 entities per GPU every 0.8 s)")
    p.add_argument("--slack", type=int, default=None, help="free slots per 256 scene-group members")
    p.add_argument("--self-migrate", action="store_true",
                   help="1 GPU: run config[2]'s migration path with one rank sending its rows to itself "
                        "(host-cost rehearsal; the migration phases are traced with NFGPU_BENCH_TRACE)")
    p.add_argument("--host-calls", choices=["auto", "off"], default="auto",
                   help="config[1], 1 GPU: also time frames with game-logic SetProperty / schedule calls")
    p.add_argument("--plugin-frame", choices=["auto", "off"], default="auto",
                   help="config[1], 1 GPU: also time the C++ plugin's frame (tests/cpp/plugin_bench)")
    p.add_argument("--adapter-frame", choices=["auto", "off"], default="auto",
                   help="config[1], 1 GPU: also time the drop-in path — the reference-side plugin "
                        "(integration/NFGPUKernelPlugin.cpp) inside the reference's own kernel / AOI / schedule "
                        "modules (tests/cpp/_ref/adapter_bench) — at config[1] and at config[0]")
    p.add_argument("--config", type=int, default=1, choices=[0, 1, 3, 4],
                   help="BASELINE config: 0 = Tutorial3 at 10k NPCs (the reference's CPU case), "
                        "1 = 1M entities/GPU (the metric's configuration; with --gpus > 1 "
                        "it becomes config[2]: scene shards + migration), 3 = 256 scenes x 64 groups, 2M "
                        "entities, 32 players/group (fan-out dominated), 4 = 500k players x 64-row records")
    p.add_argument("--other-configs", choices=["auto", "off"], default="auto",
                   help="config[1], 1 GPU: also run short legs of config[0], config[3] and config[4] (each its own "
                        "process, same --steps / --warmup) and report them under 'configs'")
    p.add_argument("--backend", default="nccl", help="process group backend (nccl = RCCL; gloo only to rehearse "
                                                     "several ranks on one GPU)")
    p.add_argument("--shard", choices=["auto", "cpp", "py"], default="auto",
                   help="config[2]'s exchange: cpp = the C++ SceneShard over its own RCCL communicators (the "
                        "plugin's production path, include/nfgpu_shard.h); py = noahgameframe_amd/shard.py over "
                        "the process group; auto = cpp with --backend nccl, py with gloo (RCCL refuses two ranks "
                        "on one GPU)")
    return p.parse_args()


def cpu_baseline(args):
    """The reference's own frame on one host core: oracle/_ref/nf_ref_session runs the reference's
    NFCKernelModule, NFCScheduleModule, NFCSceneAOIModule, NFCEventModule and NFCClassModule
    (compiled from the reference sources where they lie) with the workload's heartbeat programs as
    functors calling NFIKernelModule::Get/SetProperty*, the window's Set / schedule calls, and a
    property-event consumer on the AOI module's recipient lists — on a bounded sample of the same
    workload: whole scene groups of the config's shape, fewer of them."""
    from noahgameframe_amd import nfio, workload
    exe = os.path.join(ROOT, "oracle", "_ref", "nf_ref_session")
    if not os.path.exists(exe):
        return None
    ticks = 400
    if args.config == 0:
        # (the reference's CreateObject of n objects into one group costs O(n^2) in the AOI module's
        # enter broadcasts: 10k objects take minutes to set up, so a smaller group)
        n = 4000
        w = workload.tutorial3_world(n_obj=n, n_ticks=ticks * 2, tick_ms=args.tick_ms)
        what = f"config[0]'s workload at {n} NPC objects (one group)"
    elif args.config == 3:
        n = 4096  # 1 scene x 32 groups of 128, 32 players per group (config[3]'s group shape)
        w = workload.fanout_world(n_ticks=ticks, n_obj=n, scenes=1, groups=32, players_per_group=32)
        what = f"{n} entities (1 scene x 32 groups x 128, 32 players/group: config[3]'s groups)"
    elif args.config == 4:
        n = 1024  # 64-row skill records; the int cooldown column only (see below)
        w = workload.record_world(n_ticks=ticks, n_obj=n, groups=64, steady=True, rec_float_op=False)
        what = (f"{n} players (groups of 16) x 64-row records, the int cooldown column op only: the reference's "
                "NFCRecord::SetFloat stores an int64 variant and cannot run the f64 charge op "
                "(tests/test_oracle.py::test_reference_record_setfloat_bug)")
    else:
        per_group = max(1, args.entities // max(args.groups, 1))
        groups = max(1, min(args.cpu_sample, args.entities) // per_group)
        n = groups * per_group
        w = workload.bench_world(n_obj=n, groups=groups, players_per_group=args.players_per_group, n_ticks=ticks,
                                 tick_ms=args.tick_ms, seed=2026)
        what = f"{n} entities ({groups} groups x {per_group}, {args.players_per_group} players/group: config[1]'s groups)"
    with tempfile.TemporaryDirectory() as d:
        wp = os.path.join(d, "w.nfio")
        nfio.write(wp, w)
        # calibrate: one untimed and one timed frame, then a run sized to ~cpu_seconds of frame work
        r = json.loads(subprocess.run([exe, wp, "2", "1"], check=True, capture_output=True,
                                      text=True).stdout.strip().splitlines()[-1])
        per_tick = r["seconds"] / max(r["frames"], 1)
        t = int(min(int(w["cfg"][7]) - 1, max(2, args.cpu_seconds / max(per_tick, 1e-6))))
        r = json.loads(subprocess.run([exe, wp, str(t + 1), "1"], check=True, capture_output=True,
                                      text=True).stdout.strip().splitlines()[-1])
    return {"value": r["entity_ticks_per_s"], "unit": "entity-ticks/s", "cores": 1, "kind": "reference",
            "sample": f"{what}; {r['frames']} frames after one untimed frame through the reference's own "
                      f"NFCKernelModule + NFCScheduleModule + NFCSceneAOIModule (heartbeat functors calling "
                      f"NFIKernelModule::Get/SetProperty*, the window's SetProperty and schedule calls, a "
                      f"property-event consumer on the AOI module's GetBroadCastObject lists: {r['msgs']} "
                      f"recipients), single thread, {r['seconds']:.1f} s"}


class RowQueue:
    """FIFO of int64 rows kept as a queue of chunks: `append` adds a chunk, `take(n)` removes the
    oldest n rows, so neither copies the rows that stay (a migrating frame of the bench moves a
    few hundred of a rank's million entities)."""

    def __init__(self, rows):
        self.chunks = collections.deque([rows] if len(rows) else [])
        self.head = 0   # rows of chunks[0] already taken

    def __len__(self):
        return sum(len(c) for c in self.chunks) - self.head

    def append(self, rows):
        if len(rows):
            self.chunks.append(rows)

    def take(self, n):
        parts, got = [], 0
        while self.chunks and got < n:
            c = self.chunks[0]
            k = min(n - got, len(c) - self.head)
            parts.append(c[self.head:self.head + k])
            got += k
            self.head += k
            if self.head == len(c):
                self.chunks.popleft()
                self.head = 0
        return np.concatenate(parts) if parts else None


class Migration:
    """BASELINE config[2]: every `every`-th frame each rank's game logic sends `per_frame` of its
    entities into the next rank's scene (SwitchScene across shards, same group id, new position).
    The tickets (one int64 array, shard.TICKET_COLS) are decided after a frame's launch and
    all-gathered over a gloo group asynchronously (gloo's own thread), while this rank waits for
    and launches the next frame; the frame after that starts by moving the state rows GPU-to-GPU
    with one RCCL all_to_all.  Frames without migrations make no collective call at all."""

    def __init__(self, m, w, rank, world, per_frame, every, dev, impl="py"):
        import torch.distributed as dist
        from noahgameframe_amd.shard import CppSceneShard, SceneShard
        self.dist = dist
        self.meta = dist.new_group(backend="gloo") if world > 1 else None
        self.impl = impl
        if impl == "cpp":
            # scene r + 1 belongs to rank r; tickets gathered on every `every`-th frame (the frames
            # this harness queues them on), so the other frames make no transport call
            self.cshard = CppSceneShard(m, rank, world, [-1] + list(range(world)), w["scene_props"],
                                        meta_group=self.meta, exchange_every=max(1, every))
            self.shard = None
        else:
            own = lambda scene: int(scene) - 1
            self.shard = SceneShard(m, rank, world, own, w["scene_props"], group=dist.group.WORLD if world > 1 else None,
                                    meta_group=self.meta, device=dev)
        self.rank, self.world, self.per_frame, self.every = rank, world, per_frame, max(1, every)
        # entities this rank owns (guid head, guid data, group, cls, is_player), oldest first
        self.owned = RowQueue(np.stack([w["guid_head"], w["guid_data"], w["group"], w["cls"], w["is_player"]],
                                       axis=1).astype(np.int64))
        self.rng = np.random.default_rng(77 + rank)
        self.frames = 0
        self.pending = collections.deque()   # (frame count when started, ticket exchange in flight)
        self.after_frame()

    def before_frame(self):
        from noahgameframe_amd.shard import T_GH, T_GD, T_GROUP, T_CLS, T_PL
        if self.impl == "cpp":  # SceneShard::BeginFrame: the rows of the gather the last frame started
            gh, gd, cl, pl, _, gr = self.cshard.begin_frame_cols()
            if len(gh):
                self.owned.append(np.stack([gh, gd, gr.astype(np.int64), cl.astype(np.int64), pl.astype(np.int64)], axis=1))
            return
        # exchanges started at least one frame ago (the same frames on every rank)
        while self.pending and self.pending[0][0] < self.frames:
            recv = self.shard.migrate_array(self.pending.popleft()[1].wait())
            if len(recv):
                self.owned.append(recv[:, [T_GH, T_GD, T_GROUP, T_CLS, T_PL]])

    def finish(self):
        """Waits for the exchanges still in flight (their tickets are not carried out)."""
        if self.impl == "cpp":
            self.cshard.close()   # (its destructor takes the gather in flight, on every rank)
            return
        while self.pending:
            self.pending.popleft()[1].wait()

    def moved(self):
        if self.impl == "cpp":
            return self.cshard.stats()[:2]
        return self.shard.migrated_out, self.shard.migrated_in

    def after_frame(self):
        """The next frame's tickets (only on every `every`-th frame, the same frames on every rank)."""
        from noahgameframe_amd.shard import T_GH, T_GD, T_CLS, T_PL, T_SCENE, T_GROUP, T_X, T_Y, T_Z, T_SRC, T_DST
        self.frames += 1
        if self.frames % self.every:
            if self.impl == "cpp":
                self.cshard.end_frame()   # (not an exchange frame: no transport call)
            return
        dst = (self.rank + 1) % self.world
        o = self.owned.take(self.per_frame)
        if o is None:
            o = np.zeros((0, 5), np.int64)
        n = len(o)
        if self.impl == "cpp":
            # (the columns nfs_queue_switch takes, built directly: the harness's own numpy work is inside
            # the timed frame)
            xy = self.rng.uniform(-500, 500, (2, n)).astype(np.float32)
            self.cshard.queue_cols(np.ascontiguousarray(o[:, 0]), np.ascontiguousarray(o[:, 1]),
                                   o[:, 3].astype(np.int32), o[:, 4].astype(np.int32),
                                   np.full(n, dst + 1, np.int32), o[:, 2].astype(np.int32), xy[0], xy[1],
                                   np.zeros(n, np.float32))
            self.cshard.end_frame()   # the gather starts on the C++ shard's worker thread
            return
        out = np.zeros((n, 11), np.int64)
        out[:, T_GH], out[:, T_GD], out[:, T_GROUP], out[:, T_CLS], out[:, T_PL] = o[:, 0], o[:, 1], o[:, 2], o[:, 3], o[:, 4]
        out[:, T_SCENE] = dst + 1
        xy = self.rng.uniform(-500, 500, (n, 2)).astype(np.float32).astype(np.float64)
        out[:, T_X], out[:, T_Y] = xy[:, 0].view(np.int64), xy[:, 1].view(np.int64)
        out[:, T_Z] = np.zeros(n, np.float64).view(np.int64)
        out[:, T_SRC], out[:, T_DST] = self.rank, dst
        if self.impl == "cpp":
            self.cshard.queue(out)
            self.cshard.end_frame()   # the gather starts on the C++ shard's worker thread
            return
        self.pending.append((self.frames, self.shard.exchange_ticket_array_async(out, max_rows=self.per_frame)))


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(n, i, port, base=None):
    """The environment of rank i of n started by bench.py itself (what torch.distributed.run sets)."""
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(i), "LOCAL_RANK": str(i), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    return env


def spawn_ranks(n, argv, script=None):
    """`bench.py --gpus N` with N > 1 and no launcher: start N rank processes (one per GPU, RANK /
    LOCAL_RANK / WORLD_SIZE set, rendezvous on 127.0.0.1) and wait for them.  This process has not
    touched the GPU (it runs before any torch import) and does not afterwards.  If a rank fails,
    the others are stopped (by their own PIDs) and its exit code is returned; rank 0 prints the
    one JSON line."""
    import signal
    port = free_port()
    script = script or os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=rank_env(n, i, port))
             for i in range(n)]
    rc = 0
    try:
        live = set(range(n))
        while live:
            for i in sorted(live):
                r = procs[i].poll()
                if r is None:
                    continue
                live.discard(i)
                if r != 0 and rc == 0:
                    rc = r
                    print(f"bench.py: rank {i} exited with {r}; stopping the other ranks", file=sys.stderr, flush=True)
                    for j in live:
                        procs[j].send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def world_from_env(gpus):
    """(world size, rank, local rank) from the launcher's environment, checked against --gpus."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: start one rank per GPU "
                         f"(--nproc-per-node {gpus}) or run bench.py --gpus {gpus} without a launcher")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main():
    t_start = time.perf_counter()
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world, rank, local = world_from_env(args.gpus)
    # the drop-in path's config[1] leg builds its 1M host objects through the reference's CreateObject
    # (minutes of single-threaded host work) while this process runs its GPU legs; it touches the GPU
    # only when told to go, after them
    adapter = None
    if world == 1 and args.config == 1 and args.adapter_frame == "auto" and not args.self_migrate:
        adapter = AdapterLeg(args)
    import torch
    import torch.distributed as dist

    if world > 1:
        local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    def barrier():
        if world > 1:
            dist.barrier()

    from noahgameframe_amd import kernel, workload

    # this rank's scene shard: 1M entities in scene rank+1 (GUID heads differ per rank)
    if args.config == 0:
        w = workload.tutorial3_world(n_ticks=1, tick_ms=args.tick_ms, seed=3 + rank, guid_head=rank)
        w["scene"][:] = rank + 1
        w["init_i"][workload.T3_PID["SceneID"]] = w["scene"]
    elif args.config == 3:
        w = workload.fanout_world(n_ticks=1, tick_ms=args.tick_ms, seed=2027 + rank,
                                  guid_heads=(7 + 16 * rank, 9 + 16 * rank))
        w["scene"] += 256 * rank
    elif args.config == 4:
        w = workload.record_world(n_ticks=1, tick_ms=args.tick_ms, seed=2028 + rank, steady=True,
                                  guid_heads=(7 + 16 * rank, 9 + 16 * rank))
        w["scene"][:] = rank + 1
    else:
        w = workload.bench_world(n_obj=args.entities, groups=args.groups, players_per_group=args.players_per_group,
                                 n_ticks=1, tick_ms=args.tick_ms, seed=2026 + rank,
                                 guid_heads=(7 + 16 * rank, 9 + 16 * rank))
        w["scene"][:] = rank + 1
    if args.config != 0:
        w["init_i"][workload.PID["SceneID"]] = w["scene"]
    args.entities = len(w["guid_head"])
    cells = np.unique(w["scene"].astype(np.int64) * (1 << 32) + w["group"], return_counts=True)[1]
    args.groups = len(cells)
    args.players_per_group = int(w["is_player"].sum()) // max(len(cells), 1)
    stream = torch.cuda.current_stream()
    # (--self-migrate: the migration path on one rank, its rows sent to itself — a host-cost
    # rehearsal of config[2] on one GPU; never the headline line)
    migrating = (world > 1 or args.self_migrate) and args.migrate > 0 and args.config == 1
    # config[1] has no membership changes: no slack slots; config[2] keeps 8 per 256 for arrivals (its
    # arrivals land in random groups, ~0.06 per group and exchange; a segment out of slack rebuilds the
    # table with fresh slack.  32 per 256 cost k_tick 7 us of dead slots: profiles/r17e_selfmig_slack.txt)
    slack = args.slack if args.slack is not None else (8 if migrating else -1)
    m = kernel.world_from_workload(w, stream=stream.cuda_stream, slack_per_256=slack)
    t0 = int(w["tick_time"][0])
    tick = 0
    mig = None
    shard_impl = args.shard if args.shard != "auto" else ("cpp" if args.backend == "nccl" else "py")
    if migrating:
        mig = Migration(m, w, rank, world, args.migrate, args.migrate_every, dev, impl=shard_impl)

    trace = {} if os.environ.get("NFGPU_BENCH_TRACE") else None  # host seconds per phase (stderr)
    if mig and trace is not None and mig.shard is not None:
        mig.shard.phase_s = trace   # (migrate_array's own phases: "export", "all_to_all", ...)

    def timed(name, fn):
        if trace is None:
            return fn()
        t = time.perf_counter()
        r = fn()
        trace[name] = trace.get(name, 0.0) + time.perf_counter() - t
        return r

    def frame():
        nonlocal tick
        if mig:
            timed("migrate", mig.before_frame)
        # the C++ shard: this window's departures are queued (the game logic's SwitchScene calls) and their
        # ticket gather started before the frame runs, so it proceeds while this frame is launched
        # (a server's game logic between frames hides it the same way); the Python shard keeps its order
        early = mig is not None and mig.impl == "cpp"
        if early:
            timed("tickets", mig.after_frame)
        timed("execute", lambda: m.Execute(t0 + tick * args.tick_ms))
        m.outputs_raw()   # the consumer's read of the frame's outputs (dense ranks: k_scan_tiles)
        if mig and not early:
            timed("tickets", mig.after_frame)   # tickets, exchanged while this and the next frame run
        tick += 1

    # with migration the untimed frames cover one whole migration cycle (a plan is carried out one
    # frame after it is made), so the timed frames see its steady state, not the first arrival
    warmup = max(args.warmup, args.migrate_every + 2) if mig else args.warmup
    for _ in range(warmup):
        frame()
    s = m.summary()  # also surfaces any device error from warmup
    # the timed region runs without kernel instrumentation ...
    barrier()
    torch.cuda.synchronize()
    if trace is not None:
        trace.clear()
    ts = time.perf_counter()
    for _ in range(args.steps):
        frame()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - ts
    if trace is not None:
        print(json.dumps({"rank": rank, "host_ms_per_frame": {k: 1000 * v / args.steps for k, v in trace.items()},
                          "frame_ms": 1000 * elapsed / args.steps}), file=sys.stderr, flush=True)
    s = m.summary()
    # ... then the same number of frames again with HIP events around every kernel, for the
    # per-kernel durations and algorithmic bytes of the roofline
    m.reset_kernel_times()
    m.set_profiling(True)
    for _ in range(args.steps):
        frame()
    m.set_profiling(False)
    moved_here = list(mig.moved()) if mig else [0, 0]
    if mig:
        mig.finish()
    ms, nl, byts = m.kernel_times()
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    moved = torch.tensor(moved_here, dtype=torch.int64, device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(moved, op=dist.ReduceOp.SUM)
    elapsed = float(el.item())
    moved = [int(x) for x in moved.tolist()]
    m.close()

    # per-kernel averages over the timed region (HIP events on the world's stream)
    kern = {}
    for i, name in enumerate(KNAMES):
        if nl[i]:
            kern[name] = {"avg_us": 1000.0 * ms[i] / nl[i], "launches": int(nl[i]),
                          "alg_bytes_per_launch": (float(byts[i]) / nl[i]) if i < 3 else None}
    dom = max((k for k in kern if kern[k]["alg_bytes_per_launch"]), key=lambda k: kern[k]["avg_us"])
    d = kern[dom]
    achieved = d["alg_bytes_per_launch"] / (d["avg_us"] * 1e-6) / 1e9
    traffic, traffic_src, traffic_rw = None, None, None
    if os.path.exists(args.pmc_json) and not migrating:
        try:
            pm = json.load(open(args.pmc_json))
            ent = pm.get(f"config{args.config}", {}).get(dom) or (pm.get(dom) if args.config == 1 else None)
            traffic = (ent or {}).get("hbm_bytes_per_launch")
            traffic_src = ((pm.get(f"config{args.config}") or {}).get("source") or pm.get("source")) if traffic else None
            if traffic:
                traffic_rw = {"read": ent.get("read_bytes_per_launch"), "written": ent.get("write_bytes_per_launch")}
        except Exception:
            traffic = None
    # k_tick's algorithmic bytes split into written and read (the tally counts both): in a frame without
    # SetProperty calls every dirty event is its slot's 8-byte write-back + a 24-byte event record
    # (slot, property, old, new), every fired heartbeat its 16-byte schedule record + a 12-byte fired
    # record, every recipient a 4-byte word (fused tiles store no per-event message offsets), and with
    # record programs every slot its 4-byte fired mask; the rest of the tally is reads
    alg_rw = None
    if dom == "k_tick" and args.config in (0, 1, 3):
        wr = 32.0 * s["n_prop_events"] + 28.0 * s["n_fired"] + 4.0 * s["n_msgs"]
        alg_rw = {"written": wr, "read": d["alg_bytes_per_launch"] - wr,
                  "how": "written = 32 B per dirty event + 28 B per fired heartbeat + 4 B per recipient (k_tick's "
                         "byte accounting, nfgpu_tick.hpp); read = the in-kernel tally minus that"}
    # the bandwidth a perfectly coalesced stream mix with this kernel's read:write ratio reaches on
    # an MI355X (tools/hbm_mix.hip), beside the 8 TB/s spec peak
    ceiling = None
    if os.path.exists(HBM_CEILING_JSON):
        try:
            hc = json.load(open(HBM_CEILING_JSON))
            mix = hc["ceiling_for"].get(dom)
            if mix:
                ceiling = {"GBps": hc["kernels"][mix]["GBps"], "probe": mix,
                           "frac_achieved": achieved / hc["kernels"][mix]["GBps"],
                           "frac_traffic": (traffic / (d["avg_us"] * 1e-6) / 1e9 / hc["kernels"][mix]["GBps"])
                           if traffic else None, "source": "profiles/hbm_ceiling.json"}
        except Exception:
            ceiling = None
    total_alg = sum(v["alg_bytes_per_launch"] or 0 for v in kern.values())
    value = world * args.entities * args.steps / elapsed

    if args.config == 1:
        rehearsal = ("one-rank rehearsal of config[2]'s migration path (rows sent to the same rank): "
                     if args.self_migrate and world == 1 else "")
        wl_name = rehearsal + ((f"BASELINE config[2]: {world} scene shards (scene r+1 on GPU r), "
                                f"{args.migrate} SwitchScene migrations per rank every {args.migrate_every} "
                                f"frames into the next shard (state rows over "
                                f"{'RCCL' if args.backend == 'nccl' else 'gloo'} all_to_all); per GPU: ")
                               if migrating else "BASELINE config[1]: ") + (
            f"{args.entities} NPC/Player entities per GPU in one scene, "
            f"{args.groups} groups x {args.entities // args.groups}, "
            f"{args.players_per_group} players/group, heartbeats HPRegen 1s/MPRegen 2s/"
            f"Move 0.1s/Patrol 3s/Poison 0.5s, {args.tick_ms} ms frames")
    else:
        wl_name = CONFIG_NAMES[args.config]
    out = {
        "metric": METRIC, "value": value, "unit": "entity-ticks/s", "n_gpus": world, "steps": args.steps,
        "warmup": warmup, "ms_per_step": 1000.0 * elapsed / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int64/f64", "data": "synthetic",
        "config": {"workload": wl_name,
                   "entities_per_gpu": args.entities, "groups": args.groups,
                   "players_per_group": args.players_per_group, "parallelism": f"scene-shard x{world}",
                   "migrations_per_rank_per_frame": args.migrate / args.migrate_every if migrating else 0},
        "migrations": {"out": moved[0], "in": moved[1], "backend": args.backend,
                       "exchange": "C++ SceneShard (RCCL side communicator for tickets, ncclSend/Recv rows)"
                       if shard_impl == "cpp" else "noahgameframe_amd/shard.py (process group)"}
        if migrating else None,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "traffic_rw": traffic_rw, "alg_bytes_rw": alg_rw,
                     "mix_ceiling": ceiling},
        "kernels": kern,
        "per_frame": {"prop_events": s["n_prop_events"], "rec_events": s["n_rec_events"], "fired": s["n_fired"],
                      "msgs": s["n_msgs"], "alg_bytes_all_kernels": total_alg,
                      "frame_GBps_alg": total_alg / (elapsed / args.steps) / 1e9},
        "cpu_baseline": None,
    }
    # a launch-bound world: the per-kernel HIP events around every launch outlast the frame itself, so
    # that kernel time (and a bandwidth from it) is no evidence
    if d["avg_us"] * 1e-3 > out["ms_per_step"]:
        out["roofline"]["frac"] = None
        out["roofline"]["achieved"] = None
        out["roofline"]["note"] = (f"launch-bound: {dom}'s HIP-event time ({d['avg_us']:.1f} us) exceeds the frame "
                                   f"({out['ms_per_step'] * 1000:.1f} us); no bandwidth claimed")
    # what the timed frame produces for the fan-out: the recipient runs per tile; each event's message
    # offset is counted on the device when a consumer reads the frame (k_counted_moff), not in it
    out["per_frame"]["message_offsets"] = ("produced at read time by k_counted_moff (nfk_outputs_get / nfk_read_*), "
                                           "outside the timed frame; the headline loop's nfk_outputs_get builds "
                                           "the dense ranks")
    def progress(what):  # (a line on stderr per leg: the run is visibly alive between legs)
        if rank == 0:
            print(f"bench.py: {what} ({time.perf_counter() - t_start:.0f} s)", file=sys.stderr, flush=True)
    progress("headline frames timed")
    if rank == 0 and world == 1 and args.config == 1 and args.host_calls == "auto":
        out["host_calls"] = host_calls_run(args, torch, kernel, workload)
        progress("host_calls leg done")
    if rank == 0 and world == 1 and args.config == 1 and args.plugin_frame == "auto":
        out["plugin_frame"] = plugin_frame_run(args, workload)
        progress("plugin_frame leg done")
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        out["cpu_baseline"] = cpu_baseline(args)
        progress("cpu_baseline leg done")
    if rank == 0 and world == 1 and args.config == 1 and args.other_configs == "auto" and not args.self_migrate:
        out["configs"] = other_config_legs(args, progress)
    if adapter is not None:
        out["adapter_frame"] = {"config1": adapter.finish(progress=progress)}
        progress("adapter_frame config[1] leg done")
        out["adapter_frame"]["config0"] = adapter_config0_run(args)
        progress("adapter_frame config[0] leg done")
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def other_config_legs(args, progress=lambda what: None):
    """BASELINE config[0], config[3] and config[4] as short legs of the default line: each runs
    `bench.py --config c` in its own process (same --steps / --warmup, no CPU baseline) and reports its
    throughput, frame time, dominant kernel and roofline fraction."""
    legs = {}
    for c in (0, 3, 4):
        cmd = [sys.executable, os.path.abspath(__file__), "--config", str(c), "--steps", str(args.steps),
               "--warmup", str(args.warmup), "--cpu-baseline", args.cpu_baseline, "--cpu-seconds", "8",
               "--other-configs", "off"]
        env = dict(os.environ)
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
            env.pop(k, None)
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        except subprocess.TimeoutExpired:
            legs[f"config{c}"] = {"error": "timeout"}
            continue
        finally:
            progress(f"config[{c}] leg done")
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            legs[f"config{c}"] = {"error": (r.stderr or r.stdout)[-400:]}
            continue
        d = json.loads(line[-1])
        rf = d["roofline"]
        legs[f"config{c}"] = {
            "value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"], "steps": d["steps"],
            "warmup": d["warmup"], "workload": d["config"]["workload"],
            "entities_per_gpu": d["config"]["entities_per_gpu"],
            "dominant_kernel": {"name": rf["kernel"], "avg_us": d["kernels"][rf["kernel"]]["avg_us"],
                                "alg_bytes_per_launch": d["kernels"][rf["kernel"]]["alg_bytes_per_launch"]},
            "kernels": {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()},
            "roofline": {k_: rf.get(k_) for k_ in ("achieved", "peak", "unit", "frac", "traffic", "traffic_source",
                                                   "traffic_rw", "alg_bytes_rw", "note")},
            "per_frame": d["per_frame"], "cpu_baseline": d.get("cpu_baseline")}
    return legs


ADAPTER_EXE = os.path.join(ROOT, "tests", "cpp", "_ref", "adapter_bench")


class AdapterLeg:
    """The drop-in path at config[1]: tests/cpp/_ref/adapter_bench — a NoahGameFrame server with the
    reference-side plugin (NFGPUKernelAdapter, NFGPUSceneAOIAdapter, NFGPUScheduleAdapter) in
    NFKernelPlugin's place among the reference's own modules — on the plugin_frame leg's world (1M
    entities, a heartbeat functor on every schedule, a common property / record callback, the AOI
    module's recipient-list callbacks); and a second server on the same world whose NPCs register
    NFCNPCRefreshModule's HP callback at creation (NFCNPCRefreshModule.cpp:104: every NPC eager, HP logged
    per Set by k_chain).  Started first: they build their host objects through the reference's
    CreateObject while this process runs the GPU legs, then wait; finish() lets each in turn commit its
    world and time its frames on the idle GPU."""
    MODES = (0, 2)

    def __init__(self, args):
        self.procs, self.err = [], None
        if not os.path.exists(ADAPTER_EXE):
            self.err = "tests/cpp/_ref/adapter_bench not built (needs /root/reference at build time)"
            return
        from noahgameframe_amd import nfio, workload
        self.tmp = tempfile.TemporaryDirectory()
        wp = os.path.join(self.tmp.name, "w.nfio")
        w = workload.bench_world(n_obj=args.entities, groups=args.groups, players_per_group=args.players_per_group,
                                 n_ticks=args.warmup + args.steps, tick_ms=args.tick_ms, seed=2031, ext_frac=0.05,
                                 host_ops=True)
        nfio.write(wp, w)
        self.t0 = time.perf_counter()
        for m in self.MODES:
            errf = open(os.path.join(self.tmp.name, f"err{m}.txt"), "w+")
            p = subprocess.Popen([ADAPTER_EXE, wp, str(args.warmup), str(args.steps), str(m), "0", "1"],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=errf, text=True)
            self.procs.append((m, p, errf))

    def _finish_one(self, p, errf, deadline, progress, what):
        try:
            ready = p.stdout.readline()   # (blocks until its host objects are built)
            progress(f"{what}: host objects built")
            p.stdin.write("go\n")
            p.stdin.flush()
            while True:  # (a line a minute while its frames run)
                try:
                    out, _ = p.communicate(timeout=max(1.0, min(60.0, deadline - time.perf_counter())))
                    break
                except subprocess.TimeoutExpired:
                    if time.perf_counter() >= deadline:
                        raise
                    progress(f"{what}: frames running")
            errf.seek(0)
            err = errf.read()
        except Exception as e:  # (a timeout, or the process died before it was ready)
            p.kill()
            p.communicate()
            return {"error": repr(e)[-300:]}
        finally:
            errf.close()
        line = [x for x in out.splitlines() if x.startswith("{") and "adapter_frame_ms" in x]
        if p.returncode != 0 or not line:
            return {"error": (err or out or ready)[-400:]}
        return json.loads(line[-1])

    def finish(self, timeout=1200, progress=lambda what: None):
        if not self.procs:
            return {"error": self.err}
        deadline = self.t0 + timeout
        res = {m: self._finish_one(p, errf, deadline, progress, f"adapter_frame config[1] mode {m}")
               for m, p, errf in self.procs}
        self.tmp.cleanup()
        out = res[0]
        out["npc_hp"] = res[2]
        return out


def adapter_config0_run(args):
    """The drop-in path at config[0]: Tutorial3 (HelloWorld3Module.cpp) at 10k NPC objects through the
    reference-side plugin — OnHeartBeat (5 s x 10, functor-only: an empty device program, its timers
    scanned on the device, the functor on the host), a per-object callback on every object's World
    property, and OnEvent's SetPropertyInt(self, "World", v) on 1 % of the objects per frame."""
    if not os.path.exists(ADAPTER_EXE):
        return {"error": "tests/cpp/_ref/adapter_bench not built"}
    from noahgameframe_amd import nfio, workload
    w = workload.tutorial3_world(n_ticks=args.warmup + args.steps, tick_ms=args.tick_ms)
    with tempfile.TemporaryDirectory() as d:
        wp = os.path.join(d, "w.nfio")
        nfio.write(wp, w)
        try:
            r = subprocess.run([ADAPTER_EXE, wp, str(args.warmup), str(args.steps), "1"], capture_output=True,
                               text=True, timeout=600)
        except subprocess.TimeoutExpired:
            return {"error": "timeout"}
    line = [x for x in r.stdout.splitlines() if x.startswith("{") and "adapter_frame_ms" in x]
    if r.returncode != 0 or not line:
        return {"error": (r.stderr or r.stdout)[-400:]}
    return json.loads(line[-1])


def plugin_frame_run(args, workload):
    """The C++ plugin's frame (NFGPUKernelModule::Execute, tests/cpp/plugin_bench.cpp, no Python in
    the loop) on the host_calls world: a functor on every schedule, a common property callback and
    an AOI recipient callback registered (the reference's per-call API), once without and once with
    the game logic's calls between frames; then with the calls and one frame batch consumer
    (AddFrameCallBack), and with no host consumer.  Host ms per frame and its phases (device frame,
    functors, event read-back, delivery)."""
    import subprocess
    import tempfile
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "cpp", "_bin", "plugin_bench")
    if not os.path.exists(exe):
        return None
    frames = args.warmup + args.steps
    w = workload.bench_world(n_obj=args.entities, groups=args.groups, players_per_group=args.players_per_group,
                             n_ticks=frames, tick_ms=args.tick_ms, seed=2031, ext_frac=0.05, host_ops=True)
    res = {}
    from noahgameframe_amd import nfio
    with tempfile.TemporaryDirectory() as d:
        wp = os.path.join(d, "w.nfio")
        nfio.write(wp, w)
        # (key, game-logic calls between frames, consumer: 0 per-call API, 1 frame batch, 2 none)
        for key, calls, consumer in (("no_calls", 0, 0), ("with_calls", 1, 0),
                                     ("with_calls_frame_batch", 1, 1), ("with_calls_no_consumer", 1, 2)):
            r = subprocess.run([exe, wp, str(args.warmup), str(args.steps), str(calls), str(consumer)],
                               capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                res[key] = {"error": r.stderr[-400:]}
                continue
            res[key] = json.loads(r.stdout.strip().splitlines()[-1])
    return res


def host_calls_run(args, torch, kernel, workload):
    """config[1] with game logic between frames: every frame 5 % of the entities get a SetProperty
    (HP / Gold / EXP / TargetX, 5 % of them twice) and 1/64 of them an AddSchedule or
    RemoveSchedule call (batched per frame, call order kept).  Timed like the headline (warmup,
    then K frames between device syncs); host ms per frame of queueing the calls through the C-ABI
    (batches of >= 4096 calls: NFGUID lookups on the device mirror of the table, SetProperty calls
    queued on the device) and of nfk_execute (uploads and launches: the (slot, property) and
    (slot, kind) folds run on the device), which overlap the previous frame on the GPU."""
    frames = args.warmup + args.steps
    w = workload.bench_world(n_obj=args.entities, groups=args.groups, players_per_group=args.players_per_group,
                             n_ticks=frames, tick_ms=args.tick_ms, seed=2031, ext_frac=0.05, host_ops=True)
    m = kernel.world_from_workload(w, stream=torch.cuda.current_stream().cuda_stream, slack_per_256=-1)
    gh, gd = w["guid_head"], w["guid_data"]
    xs = np.searchsorted(w["x_tick"], np.arange(frames + 1))
    hs = np.searchsorted(w["h_tick"], np.arange(frames + 1))
    # each frame's calls as the game logic hands them over (GUIDs, ids, values), prepared before
    # the timed frames: the timed host work is the C-ABI calls and nfk_execute
    calls = []
    for t in range(frames):
        a, b = hs[t], hs[t + 1]
        ho = w["h_obj"][a:b]
        hc = (w["h_op"][a:b], gh[ho], gd[ho], w["h_kind"][a:b], w["h_interval"][a:b], w["h_count"][a:b],
              w["h_time"][a:b]) if b > a else None
        a, b = xs[t], xs[t + 1]
        xo = w["x_obj"][a:b]
        xc = (gh[xo], gd[xo], w["x_pid"][a:b], w["x_bits"][a:b]) if b > a else None
        calls.append((hc, xc))
    t_calls = t_exec = 0.0

    def frame(t):
        nonlocal t_calls, t_exec
        c0 = time.perf_counter()
        hc, xc = calls[t]
        if hc is not None:
            m.schedule_calls(*hc)
        if xc is not None:
            m.set_props(*xc)
        c1 = time.perf_counter()
        m.Execute(int(w["tick_time"][t]))
        m.outputs_raw()
        c2 = time.perf_counter()
        t_calls += c1 - c0
        t_exec += c2 - c1

    for t in range(args.warmup):
        frame(t)
    m.summary()
    torch.cuda.synchronize()
    t_calls = t_exec = 0.0
    ts = time.perf_counter()
    for t in range(args.warmup, frames):
        frame(t)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - ts
    s = m.summary()
    m.close()
    n_set = int(np.sum((w["x_tick"] >= args.warmup))) / args.steps
    n_sched = int(np.sum((w["h_tick"] >= args.warmup))) / args.steps
    return {"value": args.entities * args.steps / elapsed, "unit": "entity-ticks/s",
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "host_ms_per_frame": {"queue_calls": 1000.0 * t_calls / args.steps,
                                  "nfk_execute": 1000.0 * t_exec / args.steps},
            "set_calls_per_frame": n_set, "schedule_calls_per_frame": n_sched,
            "last_frame": {"prop_events": s["n_prop_events"], "fired": s["n_fired"], "msgs": s["n_msgs"]}}


if __name__ == "__main__":
    main()
