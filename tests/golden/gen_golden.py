"""Regenerate the golden fixtures: synthetic workloads run through the REFERENCE's own
classes (oracle/_ref/nf_ref_harness, built from /root/reference by oracle/build_ref.sh).
Each fixture = <name>.workload.nfio (inputs) + <name>.expected.nfio (reference outputs).

    python tests/golden/gen_golden.py [name ...]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from noahgameframe_amd import nfio, workload  # noqa: E402

FIXTURES = {
    # property path: heartbeats, SetProperty calls (incl. duplicates), Add/RemoveSchedule calls
    "props": dict(n_obj=600, n_scenes=2, groups_per_scene=6, players_per_group=3, n_ticks=10, seed=101,
                  ext_frac=0.08, host_ops=True),
    # record path (int cooldown column; see DESIGN.md for the reference's f64 record bug)
    "records": dict(n_obj=300, n_scenes=1, groups_per_scene=5, players_per_group=4, n_ticks=8, seed=202,
                    records=True, rec_rows=16, rec_float_op=False, ext_frac=0.05),
    # one group, every object a player, no between-frame calls
    "allplayers": dict(n_obj=64, n_scenes=1, groups_per_scene=1, players_per_group=64, n_ticks=12, seed=303,
                       ext_frac=0.0, host_ops=False),
    # SwitchScene between frames (KM:901-951): group/scene changes, own-cell switches, new groups
    "switch": dict(n_obj=400, n_scenes=3, groups_per_scene=4, players_per_group=3, n_ticks=8, seed=404,
                   ext_frac=0.05, switch_frac=0.05, switch_new_groups=True),
    # SetProperty on every property (program operands MAXHP / HPREGEN / TargetX included) and
    # bursts of 20 distinct properties on one entity in one frame (beyond the programs' working set)
    "wide_sets": dict(n_obj=500, n_scenes=2, groups_per_scene=5, players_per_group=4, n_ticks=8, seed=505,
                      ext_frac=0.1, ext_props="all", burst_frac=0.03, burst_props=20, host_ops=True),
    # read-modify-write game logic: SetProperty(p, GetProperty(p) + delta), often twice on one
    # (entity, property) in one window, so the second Get must see the first Set (KM:401 after KM:323)
    "rmw": dict(n_obj=500, n_scenes=2, groups_per_scene=4, players_per_group=3, n_ticks=8, seed=707,
                ext_frac=0.05, ext_props="all", rmw_frac=0.06, host_ops=True, switch_frac=0.02),
    # CreateObject after start (KM:101-271) and DestroyObject (KM:273-308) between frames, with
    # SwitchScene, read-modify-write Sets and schedule calls around them; int record column
    "lifecycle": dict(n_obj=600, n_scenes=2, groups_per_scene=4, players_per_group=3, n_ticks=8, seed=808,
                      ext_frac=0.05, host_ops=True, switch_frac=0.02, rmw_frac=0.02, spawn_frac=0.03,
                      destroy_frac=0.03, records=True, rec_rows=12, rec_float_op=False),
    # SetRecordInt between frames (KM:505 -> NFCRecord::SetInt, RC:182): used and unused rows, cells
    # set twice, cells the heartbeat's record ops also change in the same frame
    "recsets": dict(n_obj=400, n_scenes=2, groups_per_scene=4, players_per_group=4, n_ticks=8, seed=909,
                    records=True, rec_rows=24, rec_float_op=False, rec_set_frac=0.1, rec_set_float=False,
                    ext_frac=0.03),
    # object (NFGUID) properties: SetPropertyObject (KM:362 -> NFCProperty::SetObject, PR:377) among
    # the window's other Sets — other objects' GUIDs, the null GUID, unchanged values, head-only
    # changes — with create / destroy and scene switches around them
    "objects": dict(n_obj=500, n_scenes=2, groups_per_scene=4, players_per_group=3, n_ticks=8, seed=1010,
                    ext_frac=0.05, ext_props="all", obj_props=True, obj_set_frac=0.08, host_ops=True,
                    switch_frac=0.02, spawn_frac=0.03, destroy_frac=0.03),
    # record row operations: AddRow (first unused row / a given row, covering a used one), Remove,
    # ClearRecord (NFCRecord.cpp:111, 1086, 1109; KM:492) interleaved with SetRecordInt calls on the
    # same rows, beside the heartbeat's cooldown op, with create / destroy
    # assignment ops in the heartbeat programs (ISET / FSET: SetPropertyInt / SetPropertyFloat with a
    # constant or another property's value) beside the add / lerp / affine ones, SetProperty calls on
    # their operands, records
    "setops": dict(n_obj=500, n_scenes=2, groups_per_scene=4, players_per_group=3, n_ticks=10, seed=1212,
                   ext_frac=0.05, ext_props="all", host_ops=True, set_ops=True, records=True, rec_rows=16,
                   rec_float_op=False),
    # guards against constants other than 0 (NFK_GUARD_K: a functor's `if (GetPropertyInt(self, g) > 30)`,
    # negative constants, both ends of the range) with SetProperty calls on the guarded properties
    "constguards": dict(n_obj=500, n_scenes=2, groups_per_scene=4, players_per_group=3, n_ticks=12, seed=1313,
                        tick_ms=500, ext_frac=0.05, ext_props="all", host_ops=True, rmw_frac=0.02,
                        const_guards=True),
    "rowops": dict(n_obj=400, n_scenes=2, groups_per_scene=4, players_per_group=4, n_ticks=8, seed=1111,
                   records=True, rec_rows=24, rec_float_op=False, rec_set_frac=0.08, rec_set_float=False,
                   rec_row_frac=0.08, ext_frac=0.03, spawn_frac=0.02, destroy_frac=0.02),
}


# BASELINE config[0]: Tutorial3 (HelloWorld3Module.cpp) heartbeats + property callbacks, scaled down
TUTORIAL3 = {"tutorial3": dict(n_obj=2000, n_ticks=80, seed=606, world_effect=True)}


# fixtures whose frames are also pinned on the reference's own server modules
# (oracle/_ref/nf_ref_session per-frame mode: NFCKernelModule / NFCScheduleModule / NFCSceneAOIModule
# compiled from the reference): <name>.session.nfio holds what those modules raised in every frame
# (property / record events in call order, fired heartbeats, GetBroadCastObject lists at the frame's
# end) and their final state; tests/test_oracle.py derives each frame's dirty-sync list from it
SESSION_FIXTURES = ["switch", "lifecycle", "rowops", "objects", "setops", "constguards"]


def session(name, w, wp):
    exe = os.path.join(ROOT, "oracle", "_ref", "nf_ref_session")
    sp = os.path.join(HERE, f"{name}.session.nfio")
    fp = sp + ".final"
    nt = str(int(w["cfg"][7]))
    subprocess.run([exe, wp, nt, "0", fp, sp], check=True, stdout=subprocess.DEVNULL)
    out = nfio.read(sp)
    for k, v in nfio.read(fp).items():
        if k.startswith("final_"):
            out[k] = v
    os.remove(fp)
    nfio.write(sp, out)
    return sp


def main(names=None):
    exe = os.path.join(ROOT, "oracle", "_ref", "nf_ref_harness")
    for name, kw in {**FIXTURES, **TUTORIAL3}.items():
        if names and name not in names:
            continue
        w = workload.tutorial3_world(**kw) if name in TUTORIAL3 else workload.make_world(**kw)
        wp = os.path.join(HERE, f"{name}.workload.nfio")
        ep = os.path.join(HERE, f"{name}.expected.nfio")
        nfio.write(wp, w)
        subprocess.run([exe, wp, ep], check=True)
        print(name, os.path.getsize(wp), os.path.getsize(ep))
        if name in SESSION_FIXTURES:
            print(name, "session", os.path.getsize(session(name, w, wp)))


if __name__ == "__main__":
    main(sys.argv[1:])
