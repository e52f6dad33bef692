"""Scene shards (noahgameframe_amd/shard.py): the cross-shard SwitchScene exchange.

CPU (gloo, world_size 2, no GPU): the migration protocol over a stub world — tickets, the
all_to_all of state rows, the imports and the SwitchScene property writes on the owner.
GPU (two ranks on one device, gloo): a sharded replay of a workload with SwitchScene across
shards matches the single-world oracle, rank by rank, bit for bit."""
import ctypes
import os
import pickle
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from noahgameframe_amd import nfio, workload
from noahgameframe_amd.shard import SceneShard, Ticket, scene_ranges

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_scene_ranges_are_contiguous():
    own = scene_ranges([3, 1, 2, 4, 5, 6, 7], 3)
    assert [own(s) for s in range(1, 8)] == [0, 0, 0, 1, 1, 1, 2]
    assert own(100) == 2 and own(4) == 1


class StubWorld:
    """Host-memory stand-in for NFKernelModule's membership calls (protocol test only)."""
    RW = 5

    def __init__(self, rank):
        self.rank = rank
        self.rows = {}          # guid -> row
        self.stream = None
        self.props = []
        self.imported = []

    def row_words(self):
        return self.RW

    def export_objects(self, gh, gd, ptr):
        rows = np.stack([self.rows.pop((int(h), int(d))) for h, d in zip(gh, gd)]).astype(np.int64)
        ctypes.memmove(ptr, rows.ctypes.data, rows.nbytes)

    def import_objects(self, gh, gd, scene, group, cls, isp, ptr):
        n = len(gh)
        rows = np.zeros((n, self.RW), np.int64)
        ctypes.memmove(rows.ctypes.data, ptr, rows.nbytes)
        for i in range(n):
            self.rows[(int(gh[i]), int(gd[i]))] = rows[i]
            self.imported.append((int(gh[i]), int(gd[i]), int(scene[i]), int(group[i])))

    def set_props(self, gh, gd, pid, bits):
        self.props += list(zip([int(x) for x in gh], [int(x) for x in pid], [int(b) for b in bits]))

    def SwitchScene(self, *a):
        raise AssertionError("local switch in the protocol test")


def _protocol_worker(rank, ws, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    m = StubWorld(rank)
    for i in range(6):   # entities 100*rank + i with a recognisable row
        m.rows[(7, 100 * rank + i)] = np.arange(StubWorld.RW, dtype=np.int64) + 1000 * (100 * rank + i)
    own = scene_ranges([1, 2, 3, 4], ws)
    sh = SceneShard(m, rank, ws, own, [16, 17, 18, 19, 20])
    out = []
    # rank r sends entities i = 0, 2, 4 to a scene of the other rank
    for i in (0, 2, 4):
        dst_scene = 3 if rank == 0 else 1
        sh.switch_scene((7, 100 * rank + i), 1, 1, dst_scene, 5 + i, 1.5, 2.5, 3.5, out)
    recv = sh.migrate(out)
    q.put((rank, sorted((t.guid_data, t.scene, t.group) for t in recv), sorted(m.rows),
           {k: v.tolist() for k, v in m.rows.items()}, m.props))
    dist.destroy_process_group()


def test_migration_protocol_gloo_cpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_protocol_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((x[0], x[1:]) for x in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        recv, keys, rows, props = res[r]
        other = 1 - r
        assert recv == [(100 * other + i, 3 if other == 0 else 1, 5 + i) for i in (0, 2, 4)]
        # kept its own odd entities, gained the other's even ones, rows intact
        assert keys == sorted([(7, 100 * r + i) for i in (1, 3, 5)] + [(7, 100 * other + i) for i in (0, 2, 4)])
        for (h, d), row in rows.items():
            assert row == list(np.arange(StubWorld.RW) + 1000 * d)
        # SwitchScene writes on arrival: GroupID=0, SceneID, X, Y, Z, GroupID (KM:930-942)
        first = [p for p in props if p[0] == 7][:6]
        assert [p[1] for p in first] == [17, 16, 18, 19, 20, 17]
        assert first[0][2] == 0 and first[5][2] == 5


def _oracle_per_rank(w, ref, ws):
    """Single-world oracle outputs split by the rank owning each object's scene at that frame."""
    own = scene_ranges(np.unique(w["scene"]), ws)
    sc, gr = np.array(w["scene"]), np.array(w["group"])
    per = {r: [] for r in range(ws)}
    for t in range(int(w["cfg"][7])):
        if "sw_tick" in w:
            for i in np.nonzero(w["sw_tick"] == t)[0]:
                if w["sw_scene"][i] >= 0:
                    sc[w["sw_obj"][i]], gr[w["sw_obj"][i]] = w["sw_scene"][i], w["sw_group"][i]
        owner = np.array([own(s) for s in sc])
        ne = len(ref[f"ev_t{t}_obj"])
        off = ref[f"mo_t{t}_off"].astype(np.int64)
        mr = ref[f"mr_t{t}_obj"]
        for r in range(ws):
            f = {}
            for p in ("ev", "re", "fi"):
                o = ref[f"{p}_t{t}_obj"]
                keep = owner[o] == r if len(o) else np.zeros(0, bool)
                for k in ("obj", "pid", "old", "new", "rrc", "kind", "rem"):
                    if f"{p}_t{t}_{k}" in ref:
                        f[f"{p}_{k}"] = ref[f"{p}_t{t}_{k}"][keep]
                if p in ("ev", "re"):
                    idx = np.nonzero(keep)[0] + (0 if p == "ev" else ne)
                    f[f"{p}_rcpt"] = [mr[off[e]:off[e + 1]].tolist() for e in idx]
            per[r].append(f)
    return per, sc


@pytest.mark.gpu
@pytest.mark.parametrize("ws,n_obj,n_scenes,slack", [(2, 4000, 4, 0), (2, 4000, 4, -1), (8, 48000, 16, 0)],
                         ids=["2shards", "2shards-noslack", "8shards-config2-shape"])
def test_sharded_replay_matches_single_world_oracle(gpu_available, tmp_path, ws, n_obj, n_scenes, slack):
    """A sharded replay (one rank per scene range, gloo between ranks on the one GPU) matches the
    single-world oracle rank by rank.  The 8-rank case is BASELINE config[2]'s shape scaled to one
    GPU: 8 scene shards, SwitchScene moving entities into other shards every frame."""
    from tests.parity import run_oracle
    w = workload.make_world(n_obj=n_obj, n_scenes=n_scenes, groups_per_scene=5, players_per_group=3, n_ticks=8,
                            seed=71 + ws, switch_frac=0.03, switch_new_groups=True, ext_frac=0.05, records=True,
                            rec_rows=8)
    ref = run_oracle(w)
    wp = str(tmp_path / "w.nfio")
    nfio.write(wp, w)
    env = dict(os.environ, NFK_SLACK=str(slack))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(ws),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "shard_worker.py"), wp, str(tmp_path)]
    subprocess.run(cmd, check=True, env=env, timeout=240)
    per, final_scene = _oracle_per_rank(w, ref, ws)
    moved = 0
    for r in range(ws):
        got = pickle.load(open(tmp_path / f"rank{r}.pkl", "rb"))
        moved += got["out"]
        for t, (g, e) in enumerate(zip(got["frames"], per[r])):
            for p in ("ev", "re", "fi"):
                for k in ("obj", "pid", "old", "new", "rrc", "kind", "rem"):
                    if f"{p}_{k}" in e:
                        a = g[f"{p}_{k}"] if k != "rem" else g["fi_rem"]
                        np.testing.assert_array_equal(a.view(np.uint8), e[f"{p}_{k}"].view(np.uint8),
                                                      err_msg=f"rank {r} frame {t} {p}_{k}")
            off = g["mo_off"].astype(np.int64)
            lists = [g["mr_obj"][off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
            assert lists == e["ev_rcpt"] + e["re_rcpt"], f"rank {r} frame {t} fan-out"
        n_int = int(w["cfg"][1])
        for o, (props, nx, rm, st, recs) in got["final"].items():
            assert ws_owner(w, final_scene, o, ws) == r
            np.testing.assert_array_equal(props[:n_int].view(np.int64), ref["final_i"][:, o])
            np.testing.assert_array_equal(props[n_int:].view(np.float64).view(np.uint64),
                                          ref["final_f"][:, o].view(np.uint64))
            np.testing.assert_array_equal(nx, ref["final_s_next"][:, o])
            np.testing.assert_array_equal(rm, ref["final_s_remain"][:, o])
            np.testing.assert_array_equal(st, ref["final_s_present"][:, o])
            np.testing.assert_array_equal(recs[0], ref["final_rec0"][o])
    assert moved > 50 * (ws // 2)   # entities did cross shards
    # global leaderboards (rank_top_global over RCCL/gloo) equal ZREVRANGE over the oracle's final state
    from tests.redis_zset import zrevrange_top   # (independent of shard.zrevrange_order, the merge)
    for prop, k in (("Level", 50), ("Gold", 20), ("X", 30)):
        pid = workload.PID[prop]
        vals = ref["final_i"][pid].astype(np.float64) if pid < n_int else ref["final_f"][pid - n_int]
        o = np.asarray(zrevrange_top(w["guid_head"], w["guid_data"], vals, k), np.int64)
        for r in range(ws):
            gh, gd, sc = pickle.load(open(tmp_path / f"rank{r}.pkl", "rb"))["ranks"][prop]
            assert list(zip(gh.tolist(), gd.tolist())) == list(zip(w["guid_head"][o].tolist(), w["guid_data"][o].tolist()))
            np.testing.assert_array_equal(sc, vals[o])


def ws_owner(w, scene_of, o, ws=2):
    return scene_ranges(np.unique(w["scene"]), ws)(scene_of[o])


def _ticket_worker(rank, ws, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    sh = SceneShard(StubWorld(rank), rank, ws, scene_ranges([1, 2], ws), [16, 17, 18, 19, 20],
                    meta_group=dist.group.WORLD)
    out = np.arange((rank + 1) * 3 * 11, dtype=np.int64).reshape(-1, 11) + 1000 * rank  # ragged: 3 and 6 rows
    a = sh.exchange_ticket_array(out)                 # counts, then padded rows
    b = sh.exchange_ticket_array(out, max_rows=8)     # one all-gather under a known bound
    c = sh.exchange_ticket_array(out[:0], max_rows=8)
    h1 = sh.exchange_ticket_array_async(out, max_rows=8)   # two exchanges in flight, waited in order
    h2 = sh.exchange_ticket_array_async(out[:1], max_rows=8)
    d, e = h1.wait(), h2.wait()
    q.put((rank, a.tolist(), b.tolist(), c.shape, d.tolist(), e.tolist()))
    dist.destroy_process_group()


def test_ticket_exchange_single_gather_gloo_cpu():
    """exchange_ticket_array with a known bound (one all-gather) returns the same global plan, in
    (source rank, call) order, as the two-collective form."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ticket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((x[0], x[1:]) for x in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
    want = np.concatenate([np.arange(3 * 11).reshape(-1, 11), np.arange(6 * 11).reshape(-1, 11) + 1000]).tolist()
    first = [np.arange(11).tolist(), (np.arange(11) + 1000).tolist()]   # each rank's first ticket
    for r in (0, 1):
        a, b, c, d, e = res[r]
        assert a == want and b == want and tuple(c) == (0, 11)
        assert d == want and e == first
