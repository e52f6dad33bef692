"""Parity helpers (test infrastructure): run the CPU oracle / reference harness and
the HIP path on the same workload and compare every output bit for bit."""
import os
import subprocess
import tempfile

import numpy as np

from noahgameframe_amd import nfio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "_bin", "nf_oracle")
REF = os.path.join(ROOT, "oracle", "_ref", "nf_ref_harness")


def ensure_oracle():
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return ORACLE


def _run_cli(exe, w):
    with tempfile.TemporaryDirectory() as d:
        wp, op = os.path.join(d, "w.nfio"), os.path.join(d, "o.nfio")
        nfio.write(wp, w)
        subprocess.run([exe, wp, op], check=True)
        return nfio.read(op)


def run_oracle(w):
    return _run_cli(ensure_oracle(), w)


def run_ref(w):
    return _run_cli(REF, w)


def run_gpu(w, msg_capacity=0, slack_per_256=0):
    """Replay the workload through libnfgpu.so; returns arrays named like the oracle's."""
    from noahgameframe_amd import kernel

    m = kernel.world_from_workload(w, msg_capacity=msg_capacity, slack_per_256=slack_per_256)
    out = {}
    n_ticks = int(w["cfg"][7])
    for t in range(n_ticks):
        r = kernel.run_workload(m, w, t)
        for k in ("ev_obj", "ev_pid", "ev_old", "ev_new", "re_obj", "re_rrc", "re_old", "re_new",
                  "fi_obj", "fi_kind", "fi_rem"):
            pfx, nm = k.split("_", 1)
            out[f"{pfx}_t{t}_{nm}"] = r[k]
        out[f"mo_t{t}_off"] = r["mo_off"]
        out[f"mr_t{t}_obj"] = r["mr_obj"]
        if "ev_oldh" in r:
            out[f"ev_t{t}_oldh"] = r["ev_oldh"]
            out[f"ev_t{t}_newh"] = r["ev_newh"]
    n_int, n_flt, n_rec = int(w["cfg"][1]), int(w["cfg"][2]), int(w["cfg"][5])
    out["final_i"] = np.stack([m.read_prop(p) for p in range(n_int)])
    out["final_f"] = np.stack([m.read_prop(n_int + p) for p in range(n_flt)])
    for r in range(n_rec):
        out[f"final_rec{r}"] = m.read_record(r)
    if m.n_oprops:
        hd = [m.read_object(n_int + n_flt + p) for p in range(m.n_oprops)]
        out["final_oh"] = np.stack([h for h, _ in hd])
        out["final_od"] = np.stack([d for _, d in hd])
    nx, rm, st = m.read_schedules()
    out["final_s_next"] = nx
    out["final_s_remain"] = rm
    out["final_s_present"] = (st & 1).astype(np.uint8)
    m.close()
    return out


def compare_runs(got, ref, w=None):
    missing = sorted(set(ref) - set(got))
    assert not missing, f"outputs missing from the GPU run: {missing[:8]}"
    bad = []
    for k in sorted(ref):
        a, b = np.asarray(got[k]), np.asarray(ref[k])
        if a.shape != b.shape:
            bad.append(f"{k}: shape {a.shape} != {b.shape}")
            continue
        if not np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8)):
            idx = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
            bad.append(f"{k}: {len(idx)} differing elements, first at {idx[:5]}: "
                       f"{a.reshape(-1)[idx[:3]]} vs {b.reshape(-1)[idx[:3]]}")
    assert not bad, "GPU vs oracle mismatch:\n  " + "\n  ".join(bad[:20])
