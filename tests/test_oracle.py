"""CPU: the oracle restatement against the reference's own outputs."""
import glob
import json
import os
import subprocess

import numpy as np
import pytest

from noahgameframe_amd import nfio, workload
from tests.parity import REF, ROOT, compare_runs, run_oracle, run_ref

GOLDEN = os.path.join(ROOT, "tests", "golden")
have_ref = os.path.exists(REF)


@pytest.mark.parametrize("name", sorted(os.path.basename(p)[:-len(".workload.nfio")]
                                        for p in glob.glob(os.path.join(GOLDEN, "*.workload.nfio"))))
def test_oracle_matches_golden(name):
    """tests/golden/*.expected.nfio were produced by the reference's NFCore + NFCScheduleModule."""
    w = nfio.read(os.path.join(GOLDEN, f"{name}.workload.nfio"))
    expected = nfio.read(os.path.join(GOLDEN, f"{name}.expected.nfio"))
    got = run_oracle(w)
    assert set(got) == set(expected)
    compare_runs(got, expected)


def test_golden_fixtures_are_nontrivial():
    e = nfio.read(os.path.join(GOLDEN, "props.expected.nfio"))
    n_ev = sum(len(v) for k, v in e.items() if k.startswith("ev_") and k.endswith("_obj"))
    n_msg = sum(len(v) for k, v in e.items() if k.startswith("mr_"))
    n_fi = sum(len(v) for k, v in e.items() if k.startswith("fi_") and k.endswith("_obj"))
    assert n_ev > 1000 and n_msg > 1000 and n_fi > 1000
    r = nfio.read(os.path.join(GOLDEN, "records.expected.nfio"))
    assert sum(len(v) for k, v in r.items() if k.startswith("re_") and k.endswith("_obj")) > 100


@pytest.mark.skipif(not have_ref, reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed,kw", [
    (1, dict(n_obj=900, n_scenes=3, groups_per_scene=4, players_per_group=2, ext_frac=0.1)),
    (2, dict(n_obj=257, n_scenes=1, groups_per_scene=1, players_per_group=0, ext_frac=0.0, host_ops=True)),
    (3, dict(n_obj=500, n_scenes=2, groups_per_scene=9, players_per_group=5, records=True, rec_rows=64,
             rec_float_op=False)),
    (4, dict(n_obj=1, n_scenes=1, groups_per_scene=1, players_per_group=1, ext_frac=1.0)),
    (5, dict(n_obj=700, n_scenes=2, groups_per_scene=5, players_per_group=3, sched_edges=True)),
    (6, dict(n_obj=800, n_scenes=3, groups_per_scene=4, players_per_group=3, switch_frac=0.05,
             switch_new_groups=True)),
    # two int column ops in one program, the second on a lower column (event order is (row, col))
    (7, dict(n_obj=400, n_scenes=2, groups_per_scene=3, players_per_group=4, records=True, rec_rows=24,
             rec_float_op=False, rec_skill_op=True)),
    # SetProperty on any property (program operands too) and 24-property bursts per entity
    (8, dict(n_obj=600, n_scenes=2, groups_per_scene=4, players_per_group=3, ext_frac=0.15, ext_props="all",
             burst_frac=0.04, burst_props=24, host_ops=True, switch_frac=0.02)),
    # everything at once: create / destroy between frames, scene switches into new groups,
    # read-modify-write Sets, schedule calls and the rescheduling edge cases
    (9, dict(n_obj=700, n_scenes=3, groups_per_scene=4, players_per_group=3, ext_frac=0.05, host_ops=True,
             sched_edges=True, switch_frac=0.02, switch_new_groups=True, rmw_frac=0.02, spawn_frac=0.03,
             destroy_frac=0.03)),
    # one large scene group (40 players) with Sets and schedule calls
    (10, dict(n_obj=500, n_scenes=1, groups_per_scene=2, players_per_group=40, ext_frac=0.08, host_ops=True)),
    # SetRecordInt between frames (used and unused rows, repeated cells) beside the heartbeat's
    # record ops on the same cells, through the compiled NFCRecord::SetInt (RC:182)
    (11, dict(n_obj=400, n_scenes=2, groups_per_scene=3, players_per_group=4, records=True, rec_rows=32,
              rec_float_op=False, rec_set_frac=0.08, rec_set_float=False, ext_frac=0.05)),
    (12, dict(n_obj=300, n_scenes=1, groups_per_scene=4, players_per_group=5, records=True, rec_rows=64,
              rec_float_op=False, rec_skill_op=True, rec_set_frac=0.2, rec_set_float=False, spawn_frac=0.03,
              destroy_frac=0.03)),
    # object (NFGUID) properties through the compiled NFCProperty::SetObject (PR:377): null GUIDs,
    # unchanged values and head-only changes, beside rmw Sets, switches, create / destroy
    (13, dict(n_obj=500, n_scenes=2, groups_per_scene=4, players_per_group=3, obj_props=True, obj_set_frac=0.12,
              ext_frac=0.05, ext_props="all", rmw_frac=0.02, switch_frac=0.02, spawn_frac=0.03, destroy_frac=0.03)),
    (14, dict(n_obj=300, n_scenes=1, groups_per_scene=2, players_per_group=30, obj_props=True, obj_set_frac=0.3,
              ext_frac=0.0, host_ops=False)),
    # record row operations through the compiled NFCRecord::AddRow / Remove / Clear (RC:111, 1086,
    # 1109), interleaved with SetRecordInt on the same rows and the heartbeat's record ops
    (15, dict(n_obj=400, n_scenes=2, groups_per_scene=3, players_per_group=4, records=True, rec_rows=24,
              rec_float_op=False, rec_set_frac=0.08, rec_set_float=False, rec_row_frac=0.1)),
    (16, dict(n_obj=300, n_scenes=1, groups_per_scene=2, players_per_group=5, records=True, rec_rows=64,
              rec_float_op=False, rec_skill_op=True, rec_set_frac=0.2, rec_set_float=False, rec_row_frac=0.2,
              spawn_frac=0.03, destroy_frac=0.03)),
    # guards against constants other than 0 (NFK_GUARD_K): ATK_VALUE driven through negative values to
    # both ends of the constant's range, with SetProperty calls on the guarded properties
    (17, dict(n_obj=600, n_scenes=2, groups_per_scene=3, players_per_group=3, const_guards=True, tick_ms=500,
              ext_frac=0.1, ext_props="all", host_ops=True)),
])
def test_oracle_matches_reference(seed, kw):
    w = workload.make_world(n_ticks=9, seed=seed, **kw)
    compare_runs(run_oracle(w), run_ref(w))


SESSION = os.path.join(ROOT, "oracle", "_ref", "nf_ref_session")


@pytest.mark.skipif(not os.path.exists(SESSION), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed, kw", [
    (31, dict(n_obj=1500, n_scenes=2, groups_per_scene=4, players_per_group=4, ext_frac=0.05, host_ops=True)),
    (32, dict(n_obj=1200, n_scenes=1, groups_per_scene=3, players_per_group=6, ext_frac=0.1, ext_props="all",
              rmw_frac=0.03, sched_edges=True, host_ops=True)),
    (33, dict(n_obj=800, n_scenes=2, groups_per_scene=2, players_per_group=3, records=True, rec_rows=16,
              rec_float_op=False, ext_frac=0.05)),
    (34, dict(n_obj=1000, n_scenes=2, groups_per_scene=3, players_per_group=4, const_guards=True, tick_ms=500,
              ext_frac=0.05, ext_props="all", rmw_frac=0.02, host_ops=True)),
])
def test_oracle_matches_reference_server_modules(tmp_path, seed, kw):
    """The oracle's final state against the reference's own server modules (oracle/ref_session.cpp:
    NFCKernelModule, NFCScheduleModule, NFCSceneAOIModule, NFCClassModule compiled from the reference
    sources; the heartbeat programs as functors calling NFIKernelModule::Get/SetProperty* and
    SetRecordInt, the window's SetProperty / schedule calls through the interfaces): every int / f64
    property of every object bit-exact after the frames, and the scheduler fired the same number of
    heartbeats."""
    w = workload.make_world(n_ticks=8, seed=seed, **kw)
    wp, fp = str(tmp_path / "w.nfio"), str(tmp_path / "f.nfio")
    nfio.write(wp, w)
    r = subprocess.run([SESSION, wp, "8", "0", fp], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    got = nfio.read(fp)
    ref = run_oracle(w)
    for k in ("final_i", "final_f"):
        a, b = np.asarray(got[k]), np.asarray(ref[k])
        assert a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8)), k
    fired = sum(len(ref[k]) for k in ref if k.startswith("fi_t") and k.endswith("_obj"))
    assert int(np.asarray(got["counts"])[0]) == fired


def _dirty_sync_from_reference(fr, t, n_oprops):
    """The frame's dirty-sync list from what the reference's modules raised (nf_ref_session's
    per-frame mode): property events per (object, property) coalesced to (first old, last new) and
    dropped when the bits are unchanged; per (object, record) the row events (Add / Del / Cover) in
    call order, then the cell Updates coalesced per (row, col) in (row, col) order; events of objects
    that left the world in the window dropped; each event's recipients = the compiled
    GetBroadCastObject list of its (object, property / record) at the frame's end."""
    alive = np.asarray(fr[f"al_t{t}_ive"]).astype(bool)
    bc = {}
    off = np.asarray(fr[f"bc_t{t}_off"])
    rc = np.asarray(fr[f"bc_t{t}_rcpt"])
    for i, (o, k) in enumerate(zip(fr[f"bc_t{t}_obj"], fr[f"bc_t{t}_key"])):
        bc[(int(o), int(k))] = [int(x) for x in rc[off[i]:off[i + 1]]]
    first, last, order = {}, {}, []
    for o, p, a, b, ah, bh in zip(fr[f"pe_t{t}_obj"], fr[f"pe_t{t}_pid"], fr[f"pe_t{t}_old"], fr[f"pe_t{t}_new"],
                                  fr[f"pe_t{t}_oldh"], fr[f"pe_t{t}_newh"]):
        key = (int(o), int(p))
        if key not in first:
            first[key] = (int(a), int(ah))
            order.append(key)
        last[key] = (int(b), int(bh))
    props = {k: (first[k], last[k], bc.get(k, [])) for k in order if alive[k[0]] and first[k] != last[k]}
    rows, upd = {}, {}
    for o, rrc, a, b in zip(fr[f"rr_t{t}_obj"], fr[f"rr_t{t}_rrc"], fr[f"rr_t{t}_old"], fr[f"rr_t{t}_new"]):
        o, rrc = int(o), int(rrc)
        if not alive[o]:
            continue
        rec = (rrc >> 16) & 0xFF
        if rrc >> 24:
            rows.setdefault((o, rec), []).append((rrc, 0, 0))
        else:
            u = upd.setdefault((o, rec), {})
            u[rrc] = (u[rrc][0] if rrc in u else int(a), int(b))
    recs = {}
    for key in set(rows) | set(upd):
        ev = list(rows.get(key, [])) + [(rrc, a, b) for rrc, (a, b) in sorted(upd.get(key, {}).items()) if a != b]
        if ev:
            recs[key] = (ev, bc.get((key[0], 0x10000 | key[1]), []))
    fired = sorted(zip(*(np.asarray(fr[f"fi_t{t}_{k}"]).tolist() for k in ("obj", "kind", "rem"))))
    return props, recs, fired


def _dirty_sync_from_oracle(o, t, n_oprops):
    moff = np.asarray(o[f"mo_t{t}_off"])
    mr = np.asarray(o[f"mr_t{t}_obj"])
    ne = len(o[f"ev_t{t}_obj"])
    oh = o.get(f"ev_t{t}_oldh", np.zeros(ne, np.uint64))
    nh = o.get(f"ev_t{t}_newh", np.zeros(ne, np.uint64))
    props = {}
    for e, (ob, p, a, b) in enumerate(zip(o[f"ev_t{t}_obj"], o[f"ev_t{t}_pid"], o[f"ev_t{t}_old"], o[f"ev_t{t}_new"])):
        props[(int(ob), int(p))] = ((int(a), int(oh[e])), (int(b), int(nh[e])), [int(x) for x in mr[moff[e]:moff[e + 1]]])
    recs = {}
    for e, (ob, rrc, a, b) in enumerate(zip(o[f"re_t{t}_obj"], o[f"re_t{t}_rrc"], o[f"re_t{t}_old"], o[f"re_t{t}_new"])):
        key = (int(ob), (int(rrc) >> 16) & 0xFF)
        ev, lists = recs.setdefault(key, ([], []))
        ev.append((int(rrc), int(a) if not int(rrc) >> 24 else 0, int(b) if not int(rrc) >> 24 else 0))
        lists.append([int(x) for x in mr[moff[ne + e]:moff[ne + e + 1]]])
    fired = sorted(zip(*(np.asarray(o[f"fi_t{t}_{k}"]).tolist() for k in ("obj", "kind", "rem"))))
    return props, recs, fired


@pytest.mark.skipif(not os.path.exists(SESSION), reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", [6, 9, 13, 15])
def test_oracle_matches_reference_modules_per_frame(tmp_path, seed):
    """Frame by frame against the reference's own NFCKernelModule / NFCScheduleModule /
    NFCSceneAOIModule (nf_ref_session per-frame mode, compiled from the reference's sources): the
    worlds of test_oracle_matches_reference with SwitchScene into new groups (KM:901-951), CreateObject
    after start and DestroyObject (KM:101, 273-308), object properties (PR:377) and record row
    operations with SetRecordInt (RC:111, 182, 1086, 1109).  Every frame's dirty-sync list — events,
    their recipient lists IN ORDER (GetBroadCastObject, AOI:531-593, at the frame's end), record
    events — and fired heartbeats equal the oracle's, and so does the final state."""
    kw = {6: dict(n_obj=800, n_scenes=3, groups_per_scene=4, players_per_group=3, switch_frac=0.05,
                  switch_new_groups=True),
          9: dict(n_obj=700, n_scenes=3, groups_per_scene=4, players_per_group=3, ext_frac=0.05, host_ops=True,
                  sched_edges=True, switch_frac=0.02, switch_new_groups=True, rmw_frac=0.02, spawn_frac=0.03,
                  destroy_frac=0.03),
          13: dict(n_obj=500, n_scenes=2, groups_per_scene=4, players_per_group=3, obj_props=True, obj_set_frac=0.12,
                   ext_frac=0.05, ext_props="all", rmw_frac=0.02, switch_frac=0.02, spawn_frac=0.03,
                   destroy_frac=0.03),
          15: dict(n_obj=400, n_scenes=2, groups_per_scene=3, players_per_group=4, records=True, rec_rows=24,
                   rec_float_op=False, rec_set_frac=0.08, rec_set_float=False, rec_row_frac=0.1)}[seed]
    nt = 9
    w = workload.make_world(n_ticks=nt, seed=seed, **kw)
    wp, fp, pp = str(tmp_path / "w.nfio"), str(tmp_path / "f.nfio"), str(tmp_path / "p.nfio")
    nfio.write(wp, w)
    r = subprocess.run([SESSION, wp, str(nt), "0", fp, pp], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    fr = nfio.read(pp)
    fr.update({k: v for k, v in nfio.read(fp).items() if k.startswith("final_")})
    no = len(workload.OBJ_PROPS) if kw.get("obj_props") else 0
    n_ev, n_msg = _compare_dirty_sync(fr, run_oracle(w), nt, no)
    assert n_ev > 300 and n_msg > 300, (n_ev, n_msg)


def _compare_dirty_sync(fr, o, nt, n_oprops):
    n_ev = n_msg = 0
    for t in range(nt):
        rp, rr, rf = _dirty_sync_from_reference(fr, t, n_oprops)
        op, orr, of = _dirty_sync_from_oracle(o, t, n_oprops)
        assert rf == of, f"frame {t}: fired"
        assert rp == op, f"frame {t}: property events / recipients"
        assert set(rr) == set(orr), f"frame {t}: record events"
        for key, (ev, lst) in rr.items():
            assert ev == orr[key][0] and all(x == lst for x in orr[key][1]), f"frame {t}: record events of {key}"
        n_ev += len(rp) + sum(len(v[0]) for v in rr.values())
        n_msg += sum(len(v[2]) for v in rp.values())
    for k in ("final_i", "final_f"):
        a, b = np.asarray(fr[k]), np.asarray(o[k])
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), k
    return n_ev, n_msg


@pytest.mark.parametrize("name", sorted(os.path.basename(p)[:-len(".session.nfio")]
                                        for p in glob.glob(os.path.join(GOLDEN, "*.session.nfio"))))
def test_oracle_matches_session_golden(name):
    """tests/golden/<name>.session.nfio: what the reference's own NFCKernelModule / NFCScheduleModule /
    NFCSceneAOIModule raised in every frame of the fixture's workload (tests/golden/gen_golden.py,
    oracle/_ref/nf_ref_session per-frame mode).  The oracle's every frame — events, ordered recipient
    lists, record row and cell events, fired heartbeats — and final state equal them: the membership
    (switch, lifecycle), object-property and row-operation fixtures are pinned on the compiled modules
    frame by frame, not only on the harness's restatement."""
    w = nfio.read(os.path.join(GOLDEN, f"{name}.workload.nfio"))
    fr = nfio.read(os.path.join(GOLDEN, f"{name}.session.nfio"))
    no = int(np.asarray(w["n_oprops"])[0]) if "n_oprops" in w else 0
    n_ev, n_msg = _compare_dirty_sync(fr, run_oracle(w), int(w["cfg"][7]), no)
    assert n_ev > 300 and n_msg > 300


@pytest.mark.skipif(not have_ref, reason="oracle/_ref not built (needs /root/reference)")
def test_reference_record_setfloat_bug():
    """NFCRecord::SetFloat stores a const double into the int64 alternative of the variant;
    the next GetFloat throws.  Our record f64 ops implement the intended semantics."""
    out = subprocess.run([REF, "--repro-record-float"], check=True, capture_output=True, text=True).stdout
    r = json.loads(out)
    assert r == {"which_before": 1, "which_after": 0, "getfloat_throws": True}


def test_oracle_record_float_threshold():
    """Record f64 cells follow TData::operator== (|d| < 0.001 is 'unchanged')."""
    w = workload.make_world(n_obj=200, n_scenes=1, groups_per_scene=2, players_per_group=200, n_ticks=4,
                            seed=9, records=True, rec_rows=8, ext_frac=0.0, host_ops=False)
    o = run_oracle(w)
    rrc = np.concatenate([o[f"re_t{t}_rrc"] for t in range(4)])
    old = np.concatenate([o[f"re_t{t}_old"] for t in range(4)])
    new = np.concatenate([o[f"re_t{t}_new"] for t in range(4)])
    f = (rrc & 0xFF) == 2
    assert f.any()
    d = new[f].view(np.float64) - old[f].view(np.float64)
    assert np.all(np.abs(d) >= 0.001)


def test_oracle_empty_world():
    w = workload.make_world(n_obj=1, n_scenes=1, groups_per_scene=1, players_per_group=0, n_ticks=2, seed=1,
                            ext_frac=0.0, host_ops=False)
    w["s_obj"] = w["s_obj"][:0]
    for k in ("s_kind", "s_interval", "s_count", "s_time"):
        w[k] = w[k][:0]
    w["cfg"][6] = 0
    o = run_oracle(w)
    assert all(len(o[f"ev_t{t}_obj"]) == 0 and len(o[f"fi_t{t}_obj"]) == 0 for t in range(2))
