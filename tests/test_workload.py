"""CPU: synthetic world invariants the parity tests rely on."""
import numpy as np

from noahgameframe_amd import workload as wl


def test_kind_ids_follow_lexical_schedule_names():
    assert wl.KINDS == sorted(wl.KINDS)


def test_world_shapes_and_uniqueness():
    w = wl.make_world(n_obj=1000, n_scenes=2, groups_per_scene=5, players_per_group=3, n_ticks=4, seed=3,
                      records=True, rec_rows=32)
    n = 1000
    guid = set(zip(w["guid_head"].tolist(), w["guid_data"].tolist()))
    assert len(guid) == n
    assert w["init_i"].shape == (wl.N_INT, n) and w["init_f"].shape == (wl.N_FLT, n)
    assert w["rec0_cells"].shape == (n, 3, 32)
    assert np.all(w["rec0_used"] < (1 << 32))
    cells = set(zip(w["scene"].tolist(), w["group"].tolist()))
    assert len(cells) == 10
    for c in cells:
        m = (w["scene"] == c[0]) & (w["group"] == c[1])
        assert w["is_player"][m].sum() == min(3, m.sum())
    assert np.all(np.diff(w["x_tick"]) >= 0) and np.all(np.diff(w["h_tick"]) >= 0)


def test_programs_only_write_declared_columns():
    ops, n = wl.programs(True)
    dst = {int(ops[k, i]["dst"]) for k in range(len(wl.KINDS)) for i in range(n[k])
           if ops[k, i]["code"] in (wl.OP_IADD_CLAMP, wl.OP_FLERP, wl.OP_FAFFINE)}
    assert len(dst) <= 8
