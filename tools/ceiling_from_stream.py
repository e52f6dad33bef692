"""profiles/hbm_ceiling.json from a tuned streaming-probe run (tools/hbm_stream.hip output, one JSON
object per line): for every read:write mix, the best rate any launch shape reached (one-shot grid,
persistent grid-stride with 4 / 8 / 16 workgroups per CU, non-temporal stores / loads and stores)
over >= 1 GiB per launch.  bench.py prices the dominant kernel against the mix with its read:write
ratio (`ceiling_for`).

    python tools/ceiling_from_stream.py profiles/r06c_hbm_stream.jsonl [--out profiles/hbm_ceiling.json]
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIX_NAMES = {"mix_10_13_ktick": "mix_10_13_ktick_ratio", "mix_4_9_krecords": "mix_4_9_krecords_ratio"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stream_jsonl")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "hbm_ceiling.json"))
    a = ap.parse_args()
    best = {}
    for line in open(a.stream_jsonl):
        d = json.loads(line)
        if "case" not in d:
            continue
        mix, shape = d["case"].split("/", 1)
        name = MIX_NAMES.get(mix, mix)
        gbps = 1000.0 * d["TBps_best"]
        if name not in best or gbps > best[name]["GBps"]:
            best[name] = {"read_arrays": d["read_arrays"], "write_arrays": d["write_arrays"], "GBps": round(gbps, 1),
                          "shape": shape, "bytes_per_launch": d["bytes_per_launch"],
                          "median_GBps": round(1000.0 * d["TBps_median"], 1)}
    out = {
        "source": (f"tools/hbm_stream.hip on one MI355X ({os.path.relpath(a.stream_jsonl, ROOT)}): for each read:write "
                   "mix the best launch shape (one-shot grid or persistent grid-stride at 4/8/16 workgroups per CU, "
                   "with and without non-temporal loads/stores), >= 1 GiB per launch (beyond the 256 MiB Infinity "
                   "Cache), best of 10 launches; tools/ceiling_from_stream.py"),
        "kernels": best,
        "ceiling_for": {"k_tick": "mix_10_13_ktick_ratio", "k_records": "mix_4_9_krecords_ratio"},
    }
    json.dump(out, open(a.out, "w"), indent=1)
    for k, v in best.items():
        print(f"{k:26s} {v['GBps']:8.1f} GB/s  ({v['shape']})")


if __name__ == "__main__":
    main()
