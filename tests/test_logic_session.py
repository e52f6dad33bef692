"""Game logic written against the reference's interfaces (tests/cpp/logic_session.cpp) on two servers:
the reference's own NFCKernelModule + NFCScheduleModule (logic_session_ref, CPU) and the reference-side
GPU plugin (integration/NFGPUKernelPlugin.cpp over libnfgpu, logic_session).  The logic registers
per-object callbacks (NFIKernelModule::AddPropertyCallBack / AddRecordCallBack, NFIKernelModule.h:28-45),
writes device state both through NFIKernelModule and straight through the objects
(GetObject(self)->SetProperty*, FindRecord(self, r)->SetInt / AddRow / Remove), and runs Tutorial3's own
sequence (HelloWorld3Module.cpp: class callback, functor-only OnHeartBeat, dynamic Hello / World
properties with per-object callbacks, DoEvent).  Compared frame by frame:

* the heartbeat functors, Tutorial3's callback lines, and every object's properties and rec0 cells read
  through the HOST objects and through NFIKernelModule: equal;
* per-object callbacks of the window's calls (phase 0): the same sequence;
* per-object callbacks fired by Execute (phase 1): per (object, property / cell) the reference's
  chain (one callback per heartbeat functor Set) coalesced to (first old, last new) and dropped when
  they are equal — the device applies a frame's programs and reports each (entity, property) once —
  equal to the GPU plugin's, which fires once per (object, property / cell)."""
import os
import subprocess

import numpy as np
import pytest

from noahgameframe_amd import nfio, workload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GPU_EXE = os.path.join(ROOT, "tests", "cpp", "_ref", "logic_session")
REF_EXE = os.path.join(ROOT, "tests", "cpp", "_ref", "logic_session_ref")


def _world(seed, n_obj=1200, n_ticks=12):
    w = workload.make_world(n_obj=n_obj, n_scenes=2, groups_per_scene=3, players_per_group=4, n_ticks=n_ticks,
                            tick_ms=1000, seed=seed, ext_frac=0.05, host_ops=True, rmw_frac=0.02, spawn_frac=0.02,
                            destroy_frac=0.02, records=True, rec_rows=16, rec_float_op=False, rec_set_frac=0.03,
                            rec_set_float=False, rec_row_frac=0.02)
    # an int-only record (the reference's NFCRecord::SetFloat cannot hold an f64 cell, test_oracle.py):
    # the charge column becomes an int column with the same bits; no program touches it
    w["rec_ctype"] = np.zeros_like(w["rec_ctype"])
    return w


def _run(exe, w, tmp_path, tag):
    wp, op = str(tmp_path / f"{tag}_w.nfio"), str(tmp_path / f"{tag}_o.nfio")
    nfio.write(wp, w)
    subprocess.run([exe, wp, op], check=True, timeout=600)
    return nfio.read(op)


def _chains(out, t, pfx, key):
    """Per-object callbacks of frame t as {phase: [(obj, key, old, new), ...]} in firing order."""
    ph = np.asarray(out[f"{pfx}_t{t}_phase"])
    rows = list(zip(out[f"{pfx}_t{t}_obj"], out[f"{pfx}_t{t}_{key}"], out[f"{pfx}_t{t}_old"], out[f"{pfx}_t{t}_new"]))
    return {p: [tuple(int(x) for x in r) for r, q in zip(rows, ph) if q == p] for p in (0, 1)}


def _coalesce(seq):
    """(obj, key) -> (first old, last new) over the phase's callbacks, dropping net-zero chains; record
    row events (Add / Del / Cover) are kept as they come."""
    first, last, rows = {}, {}, []
    for o, k, a, b in seq:
        if k >> 24:
            rows.append((o, k))
            continue
        first.setdefault((o, k), a)
        last[(o, k)] = b
    return {key: (first[key], last[key]) for key in first if first[key] != last[key]}, sorted(rows)


def _t3(out, t):
    return bytes(np.asarray(out[f"t3_t{t}_log"], np.uint8)).decode()


def test_logic_session_reference_runs_tutorial3(tmp_path):
    """CPU: the logic on the reference's own modules — Tutorial3's sequence (its class callback, the
    per-object callbacks on the dynamic World / Hello properties, DoEvent's handler whose
    SetPropertyInt on the string property is refused) and its functor-only OnHeartBeat firing every
    5 s with the remaining count."""
    if not os.path.exists(REF_EXE):
        pytest.skip("logic_session_ref not built (needs /root/reference at build time)")
    w = _world(71, n_obj=300)
    out = _run(REF_EXE, w, tmp_path, "ref")
    setup = bytes(np.asarray(out["t3_setup"], np.uint8)).decode().splitlines()
    assert any("OnClassCallBackEvent Player 10" in s for s in setup)
    assert "-1 OnPropertyCallBackEvent 10 World 0 1111" in setup
    assert "-1 OnPropertyStrCallBackEvent 10 Hello  hello,World" in setup
    assert "-1 OnEvent sets 01" in setup and "-1 OnPropertyStrCallBackEvent 10 Hello hello,World 200" in setup
    hb = [ln for t in range(int(w["cfg"][7])) for ln in _t3(out, t).splitlines() if "OnHeartBeat 0-10 " in ln]
    # next = start + 5000 * (all - remain) after each fire (SM:71-72): the first fire leaves next
    # where it was, so the schedule fires on frames 5, 6 (start + 5 s) and 10 (start + 10 s)
    assert hb == [f"{t} OnHeartBeat 0-10 OnHeartBeat 5.000000 {c}" for t, c in ((5, 9), (6, 8), (10, 7))]
    assert any("OnEvent 1 10 1003 s3" in ln for ln in _t3(out, 3).splitlines())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [71, 72])
def test_logic_session_gpu_plugin_matches_reference(gpu_available, tmp_path, seed):
    if not (os.path.exists(GPU_EXE) and os.path.exists(REF_EXE)):
        pytest.skip("logic_session not built (needs /root/reference at build time)")
    w = _world(seed)
    got, ref = _run(GPU_EXE, w, tmp_path, "gpu"), _run(REF_EXE, w, tmp_path, "ref")
    nt = int(w["cfg"][7])
    assert bytes(np.asarray(got["t3_setup"], np.uint8)) == bytes(np.asarray(ref["t3_setup"], np.uint8))
    n_obj_cb = n_rec_cb = 0
    for t in range(nt):
        assert _t3(got, t) == _t3(ref, t), t
        fo = lambda o: sorted(zip(o[f"fi_t{t}_obj"], o[f"fi_t{t}_kind"], o[f"fi_t{t}_rem"]))
        assert fo(got) == fo(ref), t
        for k in ("v_t{}_host", "v_t{}_kernel", "r_t{}_cells", "r_t{}_used"):
            np.testing.assert_array_equal(got[k.format(t)], ref[k.format(t)], err_msg=k.format(t))
        # the host objects agree with NFIKernelModule's reads (the device's, on the GPU plugin)
        np.testing.assert_array_equal(got[f"v_t{t}_host"], got[f"v_t{t}_kernel"])
        for pfx, key in (("pc", "pid"), ("rc", "rrc")):
            g, r = _chains(got, t, pfx, key), _chains(ref, t, pfx, key)
            assert g[0] == r[0], (t, pfx)   # the window's calls fire in call order, as in the reference
            assert _coalesce(g[1]) == _coalesce(r[1]), (t, pfx)
            # the GPU plugin fires each (object, property / cell) once per Execute
            assert len({(o, k) for o, k, _, _ in g[1] if not k >> 24}) == sum(1 for _, k, _, _ in g[1] if not k >> 24)
            if pfx == "pc":
                n_obj_cb += len(g[0]) + len(g[1])
            else:
                n_rec_cb += len(g[0]) + len(g[1])
    assert n_obj_cb > 1000 and n_rec_cb > 100, (n_obj_cb, n_rec_cb)
