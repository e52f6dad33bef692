"""Register budget of the hipRTC-specialised k_tick for a bench config, without a GPU: the
JitSchema source nfk_jit_preview generates, compiled offline by hipcc with the library's own
device headers, and the compiler's resource-usage remarks (VGPRs, spills, occupancy) printed
next to the library's DynSchema instantiations.
    python tools/jit_resources.py [config]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from noahgameframe_amd import kernel, workload  # noqa: E402

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(ROOT, "noahgameframe_amd", "csrc")


def remarks(src_path, extra=()):
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c", src_path, "-o", os.devnull,
                        "-Rpass-analysis=kernel-resource-usage", *extra], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-4000:])
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("sgpr_spill", r"SGPRs Spill: (\d+)"),
                         ("vgpr_spill", r"VGPRs Spill: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return [k for k in out if "k_tick" in k["name"]]


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    # the bench configs' schemas (bench.py main), at a small entity count
    if cfg == 0:
        w = workload.tutorial3_world(n_obj=1024, n_ticks=1)
    elif cfg == 4:
        w = workload.record_world(n_ticks=1, steady=True)
    else:
        w = workload.make_world(n_obj=1024, n_ticks=1)
    src, _, _ = kernel.jit_preview(w, compile=False)
    _, ok2, msg2 = kernel.jit_preview(w, compile=True)
    low = msg2.split()[0] if ok2 else ""
    m = re.match(r"_ZN5nfgpu6k_tickILi(\d+)ELi(\d+)E", low)
    waves, u = (int(m.group(1)), int(m.group(2))) if m else (7, 12)
    if len(sys.argv) > 2:
        waves = int(sys.argv[2])
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "jit.hip")
        with open(p, "w") as f:
            f.write('#include <hip/hip_runtime.h>\n#include "nfgpu_device.hpp"\n#include "nfgpu_tick.hpp"\n')
            f.write(src)
            f.write(f"\ntemplate __global__ void nfgpu::k_tick<{waves}, {u}, nfgpu::JitSchema>(nfgpu::Dev);\n")
        for k in remarks(p):
            print("jit ", k)
    if len(sys.argv) <= 3:
        for k in remarks(os.path.join(CSRC, "nfgpu_host.hip")):
            print("lib ", k)


if __name__ == "__main__":
    main()
