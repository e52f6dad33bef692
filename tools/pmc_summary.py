"""Summarise rocprofv3 --pmc passes into per-launch HBM traffic for the frame kernels.

    python tools/pmc_summary.py --calib gpurun_out/T/calib_fetch gpurun_out/T/calib_write \
        --bench gpurun_out/T/pmc_fetch gpurun_out/T/pmc_write [--sq gpurun_out/T/pmc_sq] \
        --out profiles/pmc_traffic.json

FETCH_SIZE / WRITE_SIZE (rocprofv3 derived counters, from TCC_EA0_RDREQ / _WRREQ) are converted
to bytes with factors measured by tools/pmc_calib (known-byte streaming kernels at 4, 8 and 16 B
per lane over a 1 GiB buffer, larger than the Infinity Cache): MI355X_MICROARCH.md §HBM says
FETCH_SIZE reads 1/2 of a 16-B/lane stream on gfx950 and that other widths must be calibrated.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

CALIB_BYTES = 1 << 30


def short(name):
    m = re.search(r"(?:nfgpu::)?(k_\w+|calib_\w+<[^>]*>|calib_\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def load_counters(d):
    """{kernel: {counter: [value per dispatch]}} from every *counter_collection.csv under d."""
    out = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise FileNotFoundError(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Kernel_Name"])
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                out[k][row["Counter_Name"]][disp] += float(row["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in out.items()}


def mean(xs):
    return sum(xs) / len(xs) if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib", nargs=2, metavar=("FETCH_DIR", "WRITE_DIR"))
    ap.add_argument("--bench", nargs=2, metavar=("FETCH_DIR", "WRITE_DIR"), required=True)
    ap.add_argument("--sq", default=None)
    ap.add_argument("--alg", default=None, help="bench JSON line (for algorithmic bytes per launch)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    res = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                     "bytes = counter x factor measured by tools/pmc_calib (1 GiB known-byte streams)"}
    rf = wf = None
    if a.calib:
        cf, cw = load_counters(a.calib[0]), load_counters(a.calib[1])
        cal = {}
        for k, cs in cf.items():
            if k.startswith("calib_read") and "FETCH_SIZE" in cs:
                cal[k] = {"raw_per_launch": mean(cs["FETCH_SIZE"]), "factor": CALIB_BYTES / mean(cs["FETCH_SIZE"])}
        for k, cs in cw.items():
            if k.startswith("calib_write") and "WRITE_SIZE" in cs:
                cal[k] = {"raw_per_launch": mean(cs["WRITE_SIZE"]), "factor": CALIB_BYTES / mean(cs["WRITE_SIZE"])}
        res["calibration"] = cal
        reads = [v["factor"] for k, v in cal.items() if k.startswith("calib_read")]
        writes = [v["factor"] for k, v in cal.items() if k.startswith("calib_write")]
        rf = mean(reads)
        wf = mean(writes)
        res["read_factor"], res["write_factor"] = rf, wf
        res["read_factor_spread"] = (max(reads) / min(reads)) if reads else None
        res["write_factor_spread"] = (max(writes) / min(writes)) if writes else None
    bf, bw = load_counters(a.bench[0]), load_counters(a.bench[1])
    alg = {}
    if a.alg and os.path.exists(a.alg):
        for line in open(a.alg):
            line = line.strip()
            if line.startswith("{"):
                alg = json.loads(line).get("kernels", {})
    sq = load_counters(a.sq) if a.sq else {}
    kern = {}
    for k in sorted(set(bf) | set(bw)):
        if not k.startswith("k_"):
            continue
        fr = mean(bf.get(k, {}).get("FETCH_SIZE", []))
        wr = mean(bw.get(k, {}).get("WRITE_SIZE", []))
        e = {"launches": len(bf.get(k, {}).get("FETCH_SIZE", [])), "fetch_raw_per_launch": fr,
             "write_raw_per_launch": wr}
        if rf and wf and fr is not None and wr is not None:
            e["read_bytes_per_launch"] = fr * rf
            e["write_bytes_per_launch"] = wr * wf
            e["hbm_bytes_per_launch"] = fr * rf + wr * wf
            ab = (alg.get(k) or {}).get("alg_bytes_per_launch")
            if ab:
                e["alg_bytes_per_launch"] = ab
                e["traffic_over_alg"] = e["hbm_bytes_per_launch"] / ab
        if k in sq:
            e["sq"] = {c: mean(v) for c, v in sq[k].items()}
        kern[k] = e
    res["kernels"] = kern
    for k, e in kern.items():  # flat view read by bench.py
        res[k] = {"hbm_bytes_per_launch": e.get("hbm_bytes_per_launch")}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
