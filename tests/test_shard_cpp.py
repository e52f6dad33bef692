"""The C++ scene-shard exchange (include/NFGPUSceneShard.hpp, noahgameframe_amd/host/NFGPUSceneShard.cpp):
tests/cpp/shard_protocol.cpp runs two ranks as threads with the host stand-in transport.

CPU: over the recording C-ABI stub — tickets all-gathered in (source rank, call) order, rows
exported, moved and imported intact, the arrivals' SwitchScene property writes in the reference's
order (GroupID = 0, SceneID, X, Y, Z, GroupID; KM:930-942), departed entities gone.
GPU: the same program over libnfgpu.so, two real worlds on the one GPU, rows device to device."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_bin", "shard_protocol")
STUB = os.path.join(ROOT, "tests", "cpp", "_stub")


def _build():
    if not (os.path.exists(EXE) and os.path.exists(DEFER) and os.path.exists(os.path.join(STUB, "libnfgpu.so"))):
        import __graft_entry__
        __graft_entry__.build_plugin()


def test_shard_protocol_host_stub(tmp_path):
    """Also: the per-frame protocol (SceneShard::BeginFrame / EndFrame) with an exchange every 3rd
    frame makes no transport call on a frame that is not an exchange frame or that follows an empty
    gather, moves the rows one frame after the gather, and a failed export on one rank makes every
    rank fail instead of leaving a peer waiting in the row exchange (tests/cpp/shard_protocol.cpp)."""
    _build()
    log = str(tmp_path / "stub.log")
    env = dict(os.environ, NFGPU_STUB_LOG=log, LD_LIBRARY_PATH=STUB + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([EXE, "host"], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [ln.split() for ln in open(log)]
    exports = [(int(x[1]), int(x[2])) for x in lines if x[0] == "export"]
    # the synchronous Migrate of the first scenario, then the per-frame exchange's one entity per rank,
    # then the failing scenario's rank 1 (its export runs before the status exchange stops both ranks)
    assert sorted(exports[:6]) == sorted([(7, i) for i in (0, 2, 4)] + [(7, 100 + i) for i in (0, 2, 4)])
    assert sorted(exports[6:8]) == [(7, 1), (7, 101)] and exports[8:] == [(7, 101)]
    imports = [x for x in lines if x[0] == "import"]
    assert len(imports) == 8
    # per arrival, its writes in order: GroupID 0, SceneID, X, Y, Z, GroupID (pids 1, 0, 3, 4, 5, 1)
    sets = [x for x in lines if x[0] == "set"]
    by = {}
    for x in sets:
        by.setdefault((int(x[1]), int(x[2])), []).append((int(x[3]), int(x[4])))
    for (h, d), w in by.items():
        assert [p for p, _ in w] == [1, 0, 3, 4, 5, 1], (d, w)
        assert w[0][1] == 0 and w[-1][1] == (9 if d % 100 == 1 else 5 + d % 100)


DEFER = os.path.join(ROOT, "tests", "cpp", "_bin", "shard_defer")


def test_plugin_defers_cross_shard_switch_of_moved_entity(tmp_path):
    """A cross-shard SwitchScene of an entity spawned or switched within its shard in the same window
    is deferred until the frame applied that change (the export would be refused and every rank's
    exchange would fail, losing the entity); a settled entity leaves at once.  Stub worlds, whose
    export refuses such an entity as the library's does (tests/cpp/shard_defer.cpp)."""
    _build()
    env = dict(os.environ, NFGPU_STUB_LOG=str(tmp_path / "stub.log"),
               LD_LIBRARY_PATH=STUB + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([DEFER, "host"], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr + r.stdout
    lines = [ln.split() for ln in open(tmp_path / "stub.log")]
    ev = [(x[0], int(x[2]) if x[0] == "export" else 0) for x in lines
          if x[0] == "execute" or (x[0] == "export" and int(x[1]) == 9)]
    exports = [i for i, x in enumerate(ev) if x[0] == "export"]
    # G at MigrateNow (before the window's frame); E and F only after a frame applied their change
    assert [ev[i][1] for i in exports] == [2, 500, 1]
    assert any(x[0] == "execute" for x in ev[exports[0]:exports[1]])


@pytest.mark.gpu
def test_plugin_defers_cross_shard_switch_device(gpu_available):
    _build()
    r = subprocess.run([DEFER, "device"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ok" in r.stdout


@pytest.mark.gpu
def test_shard_protocol_device(gpu_available):
    _build()
    r = subprocess.run([EXE, "device"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ok" in r.stdout


@pytest.mark.gpu
def test_rccl_transport_world_size_1(gpu_available):
    """The scene shards' RCCL transport (RcclTransport: ncclAllGather of the tickets, grouped
    ncclSend / ncclRecv of the rows on the world's stream) at world size 1 on the GPU: tickets and
    rows come back as sent (tests/cpp/rccl_transport.cpp).  More ranks need more GPUs."""
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "rccl_transport")
    env = dict(os.environ, NCCL_DEBUG="WARN")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout
    assert '"fails": 0' in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 4])
def test_plugin_shard_replay_matches_oracle(gpu_available, tmp_path, ranks):
    """Scene shards through the C++ plugin (NFGPUKernelModule::AttachShard + SceneShard), ranks as
    threads on the one GPU: every rank's callbacks (events, recipient lists, heartbeat functors) and
    final state equal the single-world oracle restricted to the objects that rank holds, while
    SwitchScene moves entities across shards every frame (KM:901-951)."""
    import numpy as np
    from noahgameframe_amd import nfio, workload
    from tests.parity import run_oracle
    from tests.test_shard import _oracle_per_rank
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "plugin_shard_replay")
    _build()
    w = workload.make_world(n_obj=4000, n_scenes=4, groups_per_scene=5, players_per_group=3, n_ticks=8, seed=81 + ranks,
                            switch_frac=0.03, switch_new_groups=True, ext_frac=0.05, records=True, rec_rows=8,
                            rec_float_op=False)
    ref = run_oracle(w)
    wp = str(tmp_path / "w.nfio")
    nfio.write(wp, w)
    r = subprocess.run([exe, wp, str(tmp_path), str(ranks)], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    per, _ = _oracle_per_rank(w, ref, ranks)
    moved = 0
    owned = np.zeros(len(w["guid_head"]), np.int64)
    for k in range(ranks):
        got = nfio.read(str(tmp_path / f"rank{k}.nfio"))
        moved += int(got["migrated"][0])
        for t, e in enumerate(per[k]):
            if len(got[f"ev_t{t}_obj"]) != len(e["ev_obj"]):  # name the events that differ
                rows = lambda d, pf: {(int(o), int(q), int(a), int(b)) for o, q, a, b in zip(
                    d[f"{pf}obj"], d[f"{pf}pid"], d[f"{pf}old"].view(np.int64), d[f"{pf}new"].view(np.int64))}
                g_, e_ = rows(got, f"ev_t{t}_"), rows(e, "ev_")
                raise AssertionError(f"rank {k} frame {t}: events only here {sorted(g_ - e_)[:8]}, "
                                     f"only in the oracle {sorted(e_ - g_)[:8]}")
            for p in ("ev", "re"):
                for f in ("obj", "pid", "old", "new", "rrc"):
                    if f"{p}_{f}" in e:
                        np.testing.assert_array_equal(got[f"{p}_t{t}_{f}"].view(np.uint8), e[f"{p}_{f}"].view(np.uint8),
                                                      err_msg=f"rank {k} frame {t} {p}_{f}")
            # functors in NFGUID order (SM:52-80), the oracle in slot order: compare sorted
            a = np.lexsort((got[f"fi_t{t}_kind"], got[f"fi_t{t}_obj"]))
            b = np.lexsort((e["fi_kind"], e["fi_obj"]))
            for f in ("obj", "kind", "rem"):
                np.testing.assert_array_equal(got[f"fi_t{t}_{f}"][a], e[f"fi_{f}"][b], err_msg=f"rank {k} frame {t} fi_{f}")
            off = got[f"mo_t{t}_off"].astype(np.int64)
            lists = [got[f"mr_t{t}_obj"][off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]
            assert lists == e["ev_rcpt"] + e["re_rcpt"], f"rank {k} frame {t} fan-out"
        own = got["final_own"].astype(bool)
        owned += own
        np.testing.assert_array_equal(got["final_i"][:, own], ref["final_i"][:, own])
        np.testing.assert_array_equal(got["final_f"][:, own].view(np.uint64), ref["final_f"][:, own].view(np.uint64))
        np.testing.assert_array_equal(got["final_s_present"][:, own], ref["final_s_present"][:, own])
    assert np.all(owned == 1)        # every entity on exactly one shard
    assert moved > 40 * ranks // 2   # entities did cross shards


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 4])
def test_plugin_shard_async_exchange_keeps_functors(gpu_available, tmp_path, ranks):
    """The plugin's own asynchronous exchange (no MigrateNow: tickets gathered at the end of an
    Execute, rows moved at the start of the next): an entity whose cross-shard SwitchScene is queued
    ticks on its source shard for one more device frame, and its heartbeat functors fire there with it
    (they were dropped at the SwitchScene and those calls were lost on both shards).  The
    schedules travel with the rows, so per frame the functor calls of all ranks together equal the
    single-world oracle's fired list — none lost, none twice — while entities cross shards."""
    import numpy as np
    from noahgameframe_amd import nfio, workload
    from tests.parity import run_oracle
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "plugin_shard_replay")
    _build()
    w = workload.make_world(n_obj=4000, n_scenes=4, groups_per_scene=5, players_per_group=3, n_ticks=10,
                            seed=91 + ranks, switch_frac=0.04, switch_new_groups=True, ext_frac=0.05, host_ops=False)
    ref = run_oracle(w)
    wp = str(tmp_path / "w.nfio")
    nfio.write(wp, w)
    r = subprocess.run([exe, wp, str(tmp_path), str(ranks), "1"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    outs = [nfio.read(str(tmp_path / f"rank{k}.nfio")) for k in range(ranks)]
    moved = sum(int(o["migrated"][0]) for o in outs)
    for t in range(int(w["cfg"][7])):
        got = sorted((int(o_), int(k_), int(r_)) for out in outs
                     for o_, k_, r_ in zip(out[f"fi_t{t}_obj"], out[f"fi_t{t}_kind"], out[f"fi_t{t}_rem"]))
        exp = sorted((int(o_), int(k_), int(r_)) for o_, k_, r_ in
                     zip(ref[f"fi_t{t}_obj"], ref[f"fi_t{t}_kind"], ref[f"fi_t{t}_rem"]))
        assert got == exp, (t, sorted(set(exp) - set(got))[:8], sorted(set(got) - set(exp))[:8])
    owned = sum(out["final_own"].astype(np.int64) for out in outs)
    assert np.all(owned == 1)
    assert moved > 40 * ranks // 2


@pytest.mark.gpu
def test_plugin_shard_writes_in_transit_travel_with_the_row(gpu_available, tmp_path):
    """Calls on an entity in transit (its cross-shard SwitchScene queued, its row not yet exported) made
    after the Execute that started its ticket gather: they were queued in the source world while k_pack
    copied the device row, and lost.  Now a window with calls while an entity departs applies
    them in a device pass of their own before the rows leave: every entity's ATK_VALUE (no program writes
    it) on its owner at the end equals the last value written while it was in transit."""
    import numpy as np
    from noahgameframe_amd import nfio, workload
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "plugin_shard_replay")
    _build()
    w = workload.make_world(n_obj=4000, n_scenes=4, groups_per_scene=5, players_per_group=3, n_ticks=10,
                            seed=97, switch_frac=0.04, switch_new_groups=True, ext_frac=0.05, host_ops=False)
    wp = str(tmp_path / "w.nfio")
    nfio.write(wp, w)
    r = subprocess.run([exe, wp, str(tmp_path), "2", "2"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    outs = [nfio.read(str(tmp_path / f"rank{k}.nfio")) for k in range(2)]
    exp = nfio.read(str(tmp_path / "atk_expect.nfio"))["atk_expect"]
    atk = workload.PID["ATK_VALUE"]
    final = sum(np.where(out["final_own"] == 1, out["final_i"][atk], 0) for out in outs)
    written = exp >= 0
    assert written.sum() > 40 and (exp >= 8000000).sum() > 20
    np.testing.assert_array_equal(final[written], exp[written])


@pytest.mark.parametrize("ranks", [2, 4])
def test_shard_rank_top_host_stub(tmp_path, ranks):
    """NFIRankRedisModule::GetRange across the C++ scene shards (SceneShard::RankTop, what
    NFGPUKernelModule::GetRange uses with a shard attached; NFCRankRedisModule.cpp:109-118): every
    rank's merged top k equals one world's nfk_rank_top over all the entities — an int and an f64
    property with ties, members whose string order is not numeric, k below / at / above the entity
    count — over the host stand-in transport and the stub C-ABI (tests/cpp/shard_rank.cpp)."""
    _build()
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "shard_rank")
    env = dict(os.environ, NFGPU_STUB_LOG=str(tmp_path / "stub.log"),
               LD_LIBRARY_PATH=STUB + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([exe, str(ranks)], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [2, 4])
def test_shard_rank_top_device(gpu_available, ranks):
    """The same with the ranks' worlds on the GPU (libnfgpu.so: nfk_rank_top's device radix select)."""
    _build()
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "shard_rank")
    r = subprocess.run([exe, str(ranks)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ok" in r.stdout
