"""(debugging aid) run tests/cpp/_ref/logic_session (GPU plugin) and logic_session_ref on one seed / mode
and print the first frame where their fired lists, component logs or cross-object reads differ."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from noahgameframe_amd import nfio  # noqa: E402
from tests.test_logic_session import GPU_EXE, REF_EXE, _lines, _world  # noqa: E402


def main(seed, mode, lethal=True):
    w = _world(seed, lethal=lethal, logic_mode=mode)
    with tempfile.TemporaryDirectory() as d:
        wp = os.path.join(d, "w.nfio")
        nfio.write(wp, w)
        outs = []
        for exe in (GPU_EXE, REF_EXE):
            op = os.path.join(d, os.path.basename(exe) + ".nfio")
            subprocess.run([exe, wp, op], check=True, timeout=300, capture_output=True)
            outs.append(nfio.read(op))
    got, ref = outs
    for t in range(int(w["cfg"][7])):
        fo = lambda o: sorted(zip(*(np.asarray(o[f"fi_t{t}_{c}"]).tolist() for c in ("obj", "kind", "rem"))))
        g, r = fo(got), fo(ref)
        if g != r:
            print(f"seed {seed} mode {mode} frame {t}: fired only gpu {sorted(set(g) - set(r))[:10]} only ref {sorted(set(r) - set(g))[:10]}")
            print("  comp gpu", _lines(got, f"k_t{t}_comp"), "ref", _lines(ref, f"k_t{t}_comp"))
            print("  comp gpu t-1", _lines(got, f"k_t{t-1}_comp") if t else None)
            return
        if _lines(got, f"k_t{t}_comp") != _lines(ref, f"k_t{t}_comp"):
            print(f"seed {seed} mode {mode} frame {t}: comp gpu {_lines(got, f'k_t{t}_comp')} ref {_lines(ref, f'k_t{t}_comp')}")
            return
        for k in ("hp", "x", "mp", "self"):
            a, b = np.asarray(got[f"xr_t{t}_{k}"]), np.asarray(ref[f"xr_t{t}_{k}"])
            if len(a) != len(b) or (a != b).any():
                i = np.nonzero(a != b)[0][:5] if len(a) == len(b) else []
                print(f"seed {seed} mode {mode} frame {t}: xr {k} differs at {i}",
                      [(int(got[f'xr_t{t}_obj'][j]), int(got[f'xr_t{t}_kind'][j]), int(got[f'xr_t{t}_peer'][j]), int(a[j]), int(b[j])) for j in i])
                return
    print(f"seed {seed} mode {mode}: equal")


if __name__ == "__main__":
    for a in sys.argv[1:]:
        s, m = a.split(":")
        main(int(s), int(m))
