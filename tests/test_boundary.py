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
