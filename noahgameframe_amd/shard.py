"""Scene shards across GPUs.

One process per GPU owns a range of scenes and runs its own world (libnfgpu.so) on its own
device; frames need no collective because a scene group never spans two shards.  The only
exchange on the path is a SwitchScene (NFCKernelModule::SwitchScene, KM:901-951) whose target
scene belongs to another shard: the entity's state row leaves the source world
(`nfk_export_objects`), travels GPU-to-GPU with one `all_to_all_single` per frame over the
process group (RCCL over xGMI with the "nccl" backend), and enters the owner's world
(`nfk_import_objects`), after which the owner queues the SwitchScene property writes
(GroupID = 0, SceneID, X, Y, Z, GroupID; KM:930-942).  The events of that frame therefore come
from the entity's new scene group, exactly as on a single world.

Tickets (which entity goes where) are control-plane metadata: they are exchanged with
`all_gather_object` over a CPU (gloo) group, or, when every rank already knows the frame's
global migration plan, derived locally (`migrate(..., plan=...)`) so the frame has no host
round trip at all.
"""
import time
from dataclasses import dataclass

import numpy as np


@dataclass
class Ticket:
    """One cross-shard SwitchScene: the entity, its class, the target cell and position."""
    guid_head: int
    guid_data: int
    cls: int
    is_player: int
    scene: int
    group: int
    x: float
    y: float
    z: float
    src: int = -1   # source rank
    dst: int = -1   # destination rank


# A batch of tickets as one int64 array [n, 11] (x, y, z as float64 bit patterns): the form the
# per-frame exchange moves, so a frame's migration costs a few array operations, not n objects.
TICKET_COLS = ("guid_head", "guid_data", "cls", "is_player", "scene", "group", "x", "y", "z", "src", "dst")
T_GH, T_GD, T_CLS, T_PL, T_SCENE, T_GROUP, T_X, T_Y, T_Z, T_SRC, T_DST = range(11)


def tickets_to_array(tickets):
    a = np.zeros((len(tickets), 11), np.int64)
    for i, t in enumerate(tickets):
        a[i] = (t.guid_head, t.guid_data, t.cls, t.is_player, t.scene, t.group, _f64(t.x).view(np.int64),
                _f64(t.y).view(np.int64), _f64(t.z).view(np.int64), t.src, t.dst)
    return a


def array_to_tickets(a):
    f = a[:, T_X:T_Z + 1].copy().view(np.float64)
    return [Ticket(int(r[T_GH]), int(r[T_GD]), int(r[T_CLS]), int(r[T_PL]), int(r[T_SCENE]), int(r[T_GROUP]),
                   float(f[i, 0]), float(f[i, 1]), float(f[i, 2]), int(r[T_SRC]), int(r[T_DST]))
            for i, r in enumerate(a)]


def scene_ranges(scenes, world_size):
    """Contiguous scene ranges, one per rank: returns owner(scene) -> rank."""
    scenes = sorted(set(int(s) for s in scenes))
    per = -(-len(scenes) // world_size)
    table = {s: min(i // per, world_size - 1) for i, s in enumerate(scenes)}

    def owner(scene):
        scene = int(scene)
        if scene in table:
            return table[scene]
        # a scene created later: by position among the known ones
        return table[max([s for s in scenes if s <= scene], default=scenes[0])]
    return owner


class SceneShard:
    """This rank's scene range.  `m` is the rank's NFKernelModule (kernel.py)."""

    def __init__(self, m, rank, world_size, owner, scene_props, group=None, meta_group=None, device=None):
        import torch
        self.torch = torch
        self.m, self.rank, self.ws, self.owner = m, rank, world_size, owner
        self.pid_scene, self.pid_group, self.pid_x, self.pid_y, self.pid_z = (int(p) for p in scene_props)
        self.pg, self.meta_pg = group, meta_group
        self.device = device if device is not None else torch.device("cpu")
        self.rw = m.row_words()
        self.migrated_out = 0
        self.migrated_in = 0
        self.phase_s = None   # a dict to accumulate host seconds per migrate_array phase into (tracing)

    def _mark(self, name, t):
        if self.phase_s is not None:
            now = time.perf_counter()
            self.phase_s[name] = self.phase_s.get(name, 0.0) + now - t
            return now
        return t

    # ---- the SwitchScene call as game logic makes it ----
    def switch_scene(self, guid, cls, is_player, scene, group, x, y, z, out):
        """Local target: SwitchScene on this world.  Remote target: a ticket appended to `out`
        for the next `migrate` (the entity leaves at the start of the frame)."""
        dst = self.owner(scene)
        if dst == self.rank:
            self.m.SwitchScene(guid, scene, group, x, y, z)
            return None
        t = Ticket(int(guid[0]), int(guid[1]), int(cls), int(is_player), int(scene), int(group), float(x), float(y),
                   float(z), self.rank, dst)
        out.append(t)
        return t

    def _exchange_tickets(self, out):
        import torch.distributed as dist
        allt = [None] * self.ws
        dist.all_gather_object(allt, out, group=self.meta_pg)
        return [t for lst in allt for t in lst]

    def exchange_ticket_array(self, out, max_rows=None):
        """All-gather every rank's outgoing ticket array over the meta group (counts first, then
        the rows padded to the largest count; with `max_rows`, a bound every rank knows, one
        all-gather of [count row | rows padded to max_rows]); returns the global plan in (source
        rank, call) order."""
        torch = self.torch
        import torch.distributed as dist
        out = np.ascontiguousarray(out, np.int64).reshape(-1, 11)
        if self.ws == 1:   # (a one-rank rehearsal: the plan is this rank's own tickets)
            return out.copy()
        if max_rows is not None:
            return self.exchange_ticket_array_async(out, max_rows).wait()
        n = torch.tensor([len(out)], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(self.ws)]
        dist.all_gather(ns, n, group=self.meta_pg)
        ns = [int(x.item()) for x in ns]
        mx = max(ns)
        if mx == 0:
            return np.zeros((0, 11), np.int64)
        pad = torch.zeros((mx, 11), dtype=torch.int64)
        pad[:len(out)] = torch.from_numpy(out)
        allp = [torch.zeros((mx, 11), dtype=torch.int64) for _ in range(self.ws)]
        dist.all_gather(allp, pad, group=self.meta_pg)
        return np.concatenate([a[:c].numpy() for a, c in zip(allp, ns)])

    def exchange_ticket_array_async(self, out, max_rows):
        """The one-all-gather form of exchange_ticket_array, started now and finished by the
        returned handle's wait() (-> the global plan): the gather runs on the meta group's own
        thread while the caller goes on (bench.py starts it after a frame's launch and waits one
        frame later).  Every rank starts its exchanges in the same order."""
        torch = self.torch
        import torch.distributed as dist
        out = np.ascontiguousarray(out, np.int64).reshape(-1, 11)
        if len(out) > max_rows:
            raise ValueError("more tickets than max_rows")
        if self.ws == 1:   # (a one-rank rehearsal: the plan is this rank's own tickets)
            return _Ready(out.copy())
        pad = torch.zeros((max_rows + 1, 11), dtype=torch.int64)
        pad[0, 0] = len(out)
        pad[1:1 + len(out)] = torch.from_numpy(out)
        allp = [torch.zeros((max_rows + 1, 11), dtype=torch.int64) for _ in range(self.ws)]
        return _Gather(dist.all_gather(allp, pad, group=self.meta_pg, async_op=True), allp)

    def migrate(self, out, plan=None):
        """Collective (every rank calls it once per frame, possibly with nothing to send).
        `out`: this rank's outgoing tickets.  `plan`: optionally the frame's global ticket list in
        (source rank, call) order, known to every rank; otherwise tickets are all-gathered over
        the meta group.  Returns the tickets this rank received."""
        tickets = plan if plan is not None else self._exchange_tickets(out)
        return array_to_tickets(self.migrate_array(tickets_to_array(tickets)))

    def migrate_array(self, plan):
        """migrate() on a ticket array (TICKET_COLS) holding the frame's global plan in (source
        rank, call) order; returns this rank's received tickets as an array."""
        torch = self.torch
        plan = np.asarray(plan, np.int64).reshape(-1, 11)
        if len(plan) == 0:   # the same decision on every rank: the collective below is skipped by all
            return plan
        send = plan[plan[:, T_SRC] == self.rank]
        recv = plan[plan[:, T_DST] == self.rank]
        send = send[np.argsort(send[:, T_DST], kind="stable")]   # call order within a destination
        recv = recv[np.argsort(recv[:, T_SRC], kind="stable")]
        scount = np.bincount(send[:, T_DST], minlength=self.ws)
        rcount = np.bincount(recv[:, T_SRC], minlength=self.ws)
        rw = self.rw
        t = time.perf_counter()
        sbuf = torch.empty((len(send), rw), dtype=torch.int64, device=self.device)
        if len(send):
            self.m.export_objects(send[:, T_GH], send[:, T_GD], sbuf.data_ptr())
        if self.device.type == "cuda" and self.m.stream != torch.cuda.current_stream(self.device).cuda_stream:
            self.m.synchronize()   # the rows were packed on the world's own stream
        t = self._mark("export", t)
        rbuf = torch.empty((len(recv), rw), dtype=torch.int64, device=self.device)
        self._all_to_all(rbuf, sbuf, [int(c) * rw for c in rcount], [int(c) * rw for c in scount])
        t = self._mark("all_to_all", t)
        if len(recv):
            other_stream = (self.device.type == "cuda" and
                            self.m.stream != torch.cuda.current_stream(self.device).cuda_stream)
            if other_stream:   # the rows arrived on torch's stream; the import copies on the world's
                torch.cuda.current_stream(self.device).synchronize()
            self.m.import_objects(recv[:, T_GH], recv[:, T_GD], recv[:, T_SCENE], recv[:, T_GROUP], recv[:, T_CLS],
                                  recv[:, T_PL], rbuf.data_ptr())
            if other_stream:   # rbuf returns to torch's allocator: the world's copy out of it is done
                self.m.synchronize()
            t = self._mark("import", t)
            # the SwitchScene property writes (KM:930-942), per entity in this order; the scene
            # always changes here
            cols = [(self.pid_group, np.zeros(len(recv), np.int64)), (self.pid_scene, recv[:, T_SCENE]),
                    (self.pid_x, recv[:, T_X]), (self.pid_y, recv[:, T_Y]), (self.pid_z, recv[:, T_Z]),
                    (self.pid_group, recv[:, T_GROUP])]
            cols = [(p, v) for p, v in cols if p >= 0]
            if cols:
                k = len(cols)
                self.m.set_props(np.repeat(recv[:, T_GH], k), np.repeat(recv[:, T_GD], k),
                                 np.tile(np.array([p for p, _ in cols], np.int32), len(recv)),
                                 np.stack([v for _, v in cols], axis=1).reshape(-1).view(np.uint64))
            self._mark("set_props", t)
        self.migrated_out += len(send)
        self.migrated_in += len(recv)
        return recv

    def _all_to_all(self, rbuf, sbuf, rsplit, ssplit):
        torch = self.torch
        import torch.distributed as dist
        if self.ws == 1:   # (a one-rank rehearsal: the rows come back to this rank)
            rbuf.copy_(sbuf)
            return
        if self.device.type == "cuda" and dist.get_backend(self.pg) == "gloo":
            # gloo moves host tensors: stage the rows through host memory
            torch.cuda.current_stream(self.device).synchronize()
            hs, hr = sbuf.cpu(), torch.empty(rbuf.shape, dtype=rbuf.dtype)
            dist.all_to_all_single(hr.view(-1), hs.view(-1), rsplit, ssplit, group=self.pg)
            rbuf.copy_(hr)
        else:
            dist.all_to_all_single(rbuf.view(-1), sbuf.view(-1), rsplit, ssplit, group=self.pg)


class CppSceneShard:
    """The C++ scene shard (include/NFGPUSceneShard.hpp: SceneShard over RcclTransport, through
    include/nfgpu_shard.h in libnfgpu_plugin.so) for this rank's world `m` (kernel.NFKernelModule):
    the production exchange a C++ game server runs.  Per frame: begin_frame() before the world's
    Execute (rows of the tickets gathered one frame ago; no collective when nobody migrates), then
    queue() the window's departures and end_frame() after it (the ticket all-gather starts on a
    worker thread and RCCL's side communicator).  `owner`: owner[scene] = rank.  The RCCL id is made
    by rank 0 and broadcast over `meta_group` (gloo)."""

    def __init__(self, m, rank, world_size, owner, scene_props, meta_group=None, exchange_every=1):
        import ctypes
        import os
        import torch.distributed as dist
        self.ct = ctypes
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnfgpu_plugin.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is not built (python -c 'import __graft_entry__ as g; g.build()')")
        lib = self.lib = ctypes.CDLL(path)
        P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        lib.nfs_rccl_unique_id.argtypes = [P]
        lib.nfs_create_rccl.argtypes = [P, P, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, ctypes.POINTER(P)]
        lib.nfs_destroy.argtypes = [P]
        lib.nfs_destroy.restype = None
        lib.nfs_queue_switch.argtypes = [P, I32] + [P] * 9
        lib.nfs_begin_frame.argtypes = [P, ctypes.POINTER(I64), ctypes.POINTER(I64)]
        lib.nfs_received.argtypes = [P, I64] + [P] * 6
        lib.nfs_end_frame.argtypes = [P]
        lib.nfs_stats.argtypes = [P, P]
        uid = np.zeros(128, np.uint8)
        if rank == 0 and lib.nfs_rccl_unique_id(uid.ctypes.data):
            raise RuntimeError("nfs_rccl_unique_id failed")
        if world_size > 1:
            box = [uid if rank == 0 else None]
            dist.broadcast_object_list(box, src=0, group=meta_group)
            uid = np.ascontiguousarray(box[0], np.uint8)
        self.owner = np.ascontiguousarray(owner, np.int32)
        ps, pg, px, py, pz = (int(p) for p in scene_props)
        h = ctypes.c_void_p()
        r = lib.nfs_create_rccl(m.h, uid.ctypes.data, rank, world_size, self.owner.ctypes.data,
                                len(self.owner), ps, pg, px, py, pz, int(exchange_every), ctypes.byref(h))
        if r:
            raise RuntimeError(f"nfs_create_rccl failed ({r})")
        self.h = h
        self.m, self.rank, self.ws = m, rank, world_size

    def queue(self, tickets):
        """Departures as a ticket array (TICKET_COLS)."""
        t = np.ascontiguousarray(tickets, np.int64).reshape(-1, 11)
        if not len(t):
            return
        i32 = lambda c: np.ascontiguousarray(t[:, c], np.int32)
        f32 = lambda c: np.ascontiguousarray(t[:, c].view(np.float64), np.float32)
        cols = [np.ascontiguousarray(t[:, T_GH]), np.ascontiguousarray(t[:, T_GD]), i32(T_CLS), i32(T_PL),
                i32(T_SCENE), i32(T_GROUP), f32(T_X), f32(T_Y), f32(T_Z)]
        if self.lib.nfs_queue_switch(self.h, len(t), *[c.ctypes.data for c in cols]):
            raise RuntimeError("nfs_queue_switch failed")

    def begin_frame(self):
        """Collective: the rows of the last gather; returns the arrivals as a ticket array."""
        cols = self.begin_frame_cols()
        n = len(cols[0])
        out = np.zeros((n, 11), np.int64)
        if n:
            gh, gd, cl, pl, sc, gr = cols
            out[:, T_GH], out[:, T_GD], out[:, T_CLS], out[:, T_PL], out[:, T_SCENE], out[:, T_GROUP] = gh, gd, cl, pl, sc, gr
            out[:, T_DST] = self.rank
        return out

    def begin_frame_cols(self):
        """begin_frame's arrivals as columns (guid head, guid data, class, is_player, scene, group), without
        the ticket array (a frame loop that only keeps a few of them)"""
        ns, nr = self.ct.c_int64(), self.ct.c_int64()
        r = self.lib.nfs_begin_frame(self.h, self.ct.byref(ns), self.ct.byref(nr))
        if r:
            raise RuntimeError(f"SceneShard::BeginFrame failed ({r})")
        n = nr.value
        gh, gd = np.empty(n, np.int64), np.empty(n, np.int64)
        cl, pl, sc, gr = (np.empty(n, np.int32) for _ in range(4))
        if n:
            self.lib.nfs_received(self.h, n, *[a.ctypes.data for a in (gh, gd, cl, pl, sc, gr)])
        return gh, gd, cl, pl, sc, gr

    def queue_cols(self, gh, gd, cls, pl, scene, group, x, y, z):
        """Departures as contiguous columns (int64 guid halves, int32 class / is_player / scene / group,
        float32 position): queue without building a ticket array."""
        n = len(gh)
        if n and self.lib.nfs_queue_switch(self.h, n, *[c.ctypes.data for c in (gh, gd, cls, pl, scene, group, x, y, z)]):
            raise RuntimeError("nfs_queue_switch failed")

    def end_frame(self):
        if self.lib.nfs_end_frame(self.h):
            raise RuntimeError("SceneShard::EndFrame failed")

    def stats(self):
        """(migrated out, migrated in, transport calls, frames)"""
        a = np.zeros(4, np.int64)
        self.lib.nfs_stats(self.h, a.ctypes.data)
        return tuple(int(x) for x in a)

    def close(self):
        if self.h:
            self.lib.nfs_destroy(self.h)
            self.h = None


class _Ready:
    def __init__(self, plan):
        self.plan = plan

    def wait(self):
        return self.plan


class _Gather:
    """An all-gather of [count row | rows padded to the bound] per rank, in flight."""

    def __init__(self, work, allp):
        self.work, self.allp, self.plan = work, allp, None

    def wait(self):
        if self.plan is None:
            self.work.wait()
            parts = [a[1:1 + int(a[0, 0])].numpy() for a in self.allp]
            self.plan = np.concatenate(parts) if parts else np.zeros((0, 11), np.int64)
        return self.plan


def _f64(x):
    return np.float64(np.float32(x)).view(np.uint64)



def subset_world(w, objs):
    """The workload restricted to the objects `objs` (global indices, ascending): objects,
    creation-time values, records and the AddSchedule calls made before frame 0.  Between-frame
    calls stay global; ShardedReplay routes them to the rank that owns the object."""
    idx = np.asarray(objs, np.int64)
    local = np.full(len(w["guid_head"]), -1, np.int64)
    local[idx] = np.arange(len(idx))
    sub = dict(w)
    sub["cfg"] = w["cfg"].copy()
    sub["cfg"][0] = len(idx)
    for k in ("guid_head", "guid_data", "scene", "group", "cls", "is_player"):
        sub[k] = w[k][idx]
    sub["init_i"] = w["init_i"][:, idx]
    sub["init_f"] = w["init_f"][:, idx]
    for r in range(int(w["cfg"][5])):
        sub[f"rec{r}_cells"] = w[f"rec{r}_cells"][idx]
        sub[f"rec{r}_used"] = w[f"rec{r}_used"][idx]
    sel = local[w["s_obj"]] >= 0
    sub["s_obj"] = local[w["s_obj"][sel]].astype(np.int32)
    for k in ("s_kind", "s_interval", "s_count", "s_time"):
        sub[k] = w[k][sel]
    sub["cfg"][6] = int(sel.sum())
    return sub


class ShardedReplay:
    """Replays a global workload (workload.make_world) on this rank's scene range: SwitchScene
    calls to foreign scenes migrate, the other between-frame calls go to the rank that owns the
    object at that moment, and every frame's outputs are reported with global object indices
    so they can be compared with a single-world run."""

    def __init__(self, w, rank, world_size, group=None, meta_group=None, device=None, stream=None, slack_per_256=0):
        from . import kernel
        self.w, self.rank, self.ws = w, rank, world_size
        self.owner = scene_ranges(np.unique(w["scene"]), world_size)
        n = len(w["guid_head"])
        mine = [o for o in range(n) if self.owner(w["scene"][o]) == rank]
        self.m = kernel.world_from_workload(subset_world(w, mine), capacity=max(64, 2 * n // world_size),
                                            stream=stream, slack_per_256=slack_per_256)
        self.shard = SceneShard(self.m, rank, world_size, self.owner, w["scene_props"], group, meta_group, device)
        self.glob = list(mine)                       # local object index -> global
        self.local_of = {g: i for i, g in enumerate(mine)}
        self.gidx = {(int(w["guid_head"][o]), int(w["guid_data"][o])): o for o in range(n)}
        self.cur_scene = np.array(w["scene"], np.int32)
        self.cur_group = np.array(w["group"], np.int32)

    def _guid(self, o):
        return int(self.w["guid_head"][o]), int(self.w["guid_data"][o])

    def frame(self, t, collect=True):
        w = self.w
        out = []
        if "sw_tick" in w:
            for i in np.nonzero(w["sw_tick"] == t)[0]:
                o = int(w["sw_obj"][i])
                if o not in self.local_of:
                    continue
                sc, gr = int(w["sw_scene"][i]), int(w["sw_group"][i])
                if sc < 0:
                    sc, gr = int(self.cur_scene[o]), int(self.cur_group[o])
                self.shard.switch_scene(self._guid(o), w["cls"][o], w["is_player"][o], sc, gr, w["sw_x"][i],
                                        w["sw_y"][i], w["sw_z"][i], out)
                self.cur_scene[o], self.cur_group[o] = sc, gr
        recv = self.shard.migrate(out)
        for tk in out:
            del self.local_of[self.gidx[(tk.guid_head, tk.guid_data)]]
        for tk in recv:
            o = self.gidx[(tk.guid_head, tk.guid_data)]
            self.local_of[o] = len(self.glob)
            self.glob.append(o)
            self.cur_scene[o], self.cur_group[o] = tk.scene, tk.group
        gh, gd = w["guid_head"], w["guid_data"]
        for i in np.nonzero(w["h_tick"] == t)[0]:
            o = int(w["h_obj"][i])
            if o not in self.local_of:
                continue
            g = self._guid(o)
            op = int(w["h_op"][i])
            if op == 1:
                self.m.add_schedules([g[0]], [g[1]], [w["h_kind"][i]], [w["h_interval"][i]], [w["h_count"][i]],
                                     [w["h_time"][i]])
            elif op == 2:
                self.m.RemoveSchedule(g, int(w["h_kind"][i]))
            else:
                self.m.RemoveSchedule(g)
        xs = [i for i in np.nonzero(w["x_tick"] == t)[0] if int(w["x_obj"][i]) in self.local_of]
        if xs:
            xo = w["x_obj"][xs]
            self.m.set_props(gh[xo], gd[xo], w["x_pid"][xs], w["x_bits"][xs])
        self.m.Execute(int(w["tick_time"][t]))
        if not collect:
            return None
        r = self.m.read_tick()
        g = np.asarray(self.glob, np.int64)
        for k in ("ev_obj", "re_obj", "fi_obj", "mr_obj"):
            r[k] = g[r[k]].astype(np.int32) if len(r[k]) else r[k]
        return r

    def final_state(self):
        """Final properties / records / schedules of the objects this rank owns: {global: ...}."""
        n_int = int(self.w["cfg"][1])
        n_flt = int(self.w["cfg"][2])
        props = np.stack([self.m.read_prop(p).view(np.uint64) for p in range(n_int + n_flt)])
        nx, rm, st = self.m.read_schedules()
        recs = [self.m.read_record(r) for r in range(int(self.w["cfg"][5]))]
        own = sorted(self.local_of.items())
        return {o: (props[:, li], nx[:, li], rm[:, li], st[:, li] & 1, [x[li] for x in recs]) for o, li in own}


def zrevrange_order(gh, gd, score):
    """Indices ordering entries like Redis ZREVRANGE over members NFGUID::ToString()
    ("head-data", NFGUID.h:93): score descending, equal scores by member descending."""
    items = sorted(range(len(score)), key=lambda i: (float(score[i]), f"{int(gh[i])}-{int(gd[i])}"), reverse=True)
    return np.asarray(items, np.int64)


def rank_top_global(m, prop, k, group=None, device=None):
    """Global leaderboard across scene shards (NFIRankRedisModule::GetRange over every shard's
    entities): each rank's exact top k (nfk_rank_top) is all-gathered over the process group
    (RCCL with device tensors under "nccl") and merged in ZREVRANGE order."""
    import torch
    import torch.distributed as dist
    gh, gd, sc = m.rank_top(prop, k)
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    if ws == 1:
        return gh, gd, sc
    dev = device if device is not None and dist.get_backend(group) == "nccl" else torch.device("cpu")
    buf = torch.zeros((k + 1, 3), dtype=torch.int64)
    buf[0, 0] = len(gh)
    if len(gh):
        buf[1:1 + len(gh), 0] = torch.from_numpy(gh)
        buf[1:1 + len(gh), 1] = torch.from_numpy(gd)
        buf[1:1 + len(gh), 2] = torch.from_numpy(sc.view(np.int64))
    buf = buf.to(dev)
    parts = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(parts, buf, group=group)
    H, D, S = [], [], []
    for p in parts:
        p = p.cpu().numpy()
        n = int(p[0, 0])
        H.append(p[1:1 + n, 0])
        D.append(p[1:1 + n, 1])
        S.append(p[1:1 + n, 2].view(np.float64))
    H, D, S = np.concatenate(H), np.concatenate(D), np.concatenate(S)
    o = zrevrange_order(H, D, S)[:k]
    return H[o], D[o], S[o]
