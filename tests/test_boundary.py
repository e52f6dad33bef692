"""CPU: the C-ABI library loads, exports every declared entry point, agrees on struct
layouts, and refuses to run without a GPU (no silent CPU fallback)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from noahgameframe_amd import kernel, workload
from tests.parity import ROOT

HDR = os.path.join(ROOT, "include", "nfgpu.h")


def declared_symbols():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(nfk_\w+)\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    lib = kernel.load_library()
    syms = declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_nm_shows_extern_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", kernel.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (nfk_\w+)", out))
    assert set(declared_symbols()) <= exported


def test_struct_layouts_match_header():
    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "nfgpu.h"
int main(void){printf("%zu %zu %zu %zu %zu\n", sizeof(nfk_op), sizeof(nfk_config), sizeof(nfk_summary),
 sizeof(nfk_outputs), offsetof(nfk_config, msg_capacity));return 0;}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "s")
        subprocess.run(["gcc", "-I", os.path.dirname(HDR), c, "-o", exe], check=True)
        sizes = [int(x) for x in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    assert sizes == [workload.OP_DTYPE.itemsize, ctypes.sizeof(kernel.Config), ctypes.sizeof(kernel.Summary),
                     ctypes.sizeof(kernel.Outputs), kernel.Config.msg_capacity.offset]


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(kernel.NFKError) as e:
        kernel.NFKernelModule(16)
    assert "NFK_ERR_HIP" in str(e.value)


def test_missing_library_raises(tmp_path):
    with pytest.raises(ImportError):
        kernel._lib = None
        try:
            kernel.load_library(str(tmp_path / "nope.so"))
        finally:
            kernel._lib = None


REF_TREE = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF_TREE, "NFComm")), reason="reference tree not present")
def test_integration_adapter_compiles_against_reference_headers():
    """integration/NFGPUKernelPlugin.cpp is the reference-side plugin: it
    implements every NFIScheduleModule pure virtual (NFIScheduleModule.h:23-39) and overrides
    NFIKernelModule's frame-path calls (NFIKernelModule.h:103-148) against the reference's own
    headers; REGISTER_MODULE instantiates both adapters, so a missing override fails here."""
    subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-I", REF_TREE, "-I", os.path.join(REF_TREE, "Dependencies"),
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "integration", "NFGPUKernelPlugin.cpp")],
                   check=True)


def _module_script(rng, n_lines=400):
    """a random module-schedule session: adds (sometimes of an existing name, count 0, forever),
    removes (of existing and unknown names), ExistSchedule probes, Execute every ~100 ms"""
    names = ["Alpha", "Beta", "Gamma", "Delta"]
    now, lines = 1_700_000_000_000, []
    for _ in range(n_lines):
        now += int(rng.integers(0, 60))
        r = rng.random()
        nm = names[int(rng.integers(0, len(names)))]
        if r < 0.25:
            ft = float(rng.choice([0.05, 0.1, 0.25, 0.5, -0.05]))
            cnt = int(rng.choice([1, 2, 3, 5, 0, -1]))
            lines.append(f"{now} add {nm} {ft} {cnt}")
        elif r < 0.35:
            lines.append(f"{now} remove {nm}")
        elif r < 0.5:
            lines.append(f"{now} exist {nm}")
        else:
            lines.append(f"{now} exec")
    return "\n".join(lines) + "\n"


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "nf_ref_harness")),
                    reason="oracle/_ref not built (needs /root/reference)")
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_module_schedules_match_reference(tmp_path, seed):
    """NFIScheduleModule module schedules (AddSchedule(name, cb, fTime, nCount) / RemoveSchedule /
    ExistSchedule, SM:123-216): the plugin's host-side ModuleScheduler against the reference's
    compiled NFCScheduleModule on the same script — every functor call and every probe."""
    import numpy as np
    exe = os.path.join(ROOT, "tests", "cpp", "_bin", "module_sched")
    if not os.path.exists(exe):
        import __graft_entry__
        __graft_entry__.build_plugin()
    sp = tmp_path / "s.txt"
    sp.write_text(_module_script(np.random.default_rng(seed)))
    ref = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "nf_ref_harness"), "--module-script", str(sp)],
                         check=True, capture_output=True, text=True).stdout
    got = subprocess.run([exe, str(sp)], check=True, capture_output=True, text=True).stdout
    assert ref.count("fire") > 20 and ref.count("exist") > 20
    assert got == ref


@pytest.mark.parametrize("which", ["config1", "tutorial3", "records", "set_ops", "const_guards"])
def test_jit_preview_compiles_for_gfx950(which):
    """nfk_jit_preview (nfgpu.h): the schema policy nfk_commit generates for a world is valid
    hipRTC input — k_tick<.., JitSchema> builds for gfx950 with no GPU present.  (GPU parity runs
    with the specialisation on by default; NFGPU_JIT=0 selects the library's DynSchema kernels.)"""
    w = {"config1": lambda: workload.make_world(n_obj=512, n_ticks=1),
         "tutorial3": lambda: workload.tutorial3_world(n_obj=512, n_ticks=1),
         "records": lambda: workload.make_world(n_obj=512, n_ticks=1, records=True),
         "set_ops": lambda: workload.make_world(n_obj=512, n_ticks=1, set_ops=True, records=True),
         "const_guards": lambda: workload.make_world(n_obj=512, n_ticks=1, const_guards=True)}[which]()
    src, ok, _ = kernel.jit_preview(w, compile=False)
    assert ok and "struct JitSchema" in src
    assert f"kNK = {int(w['cfg'][4])};" in src
    if which == "const_guards":  # guards against constants are literals of the generated programs
        for k in (30, 1500, -100, workload.GUARD_KMIN, workload.GUARD_KMAX, 2, 61):
            assert f"(int64_t)({k})" in src, k
    _, ok, msg = kernel.jit_preview(w, compile=True)
    assert ok, msg
    assert msg.startswith("_ZN5nfgpu6k_tick") and "JitSchema" in msg
