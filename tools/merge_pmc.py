"""Fold one GPU session's PMC summary (tools/pmc_summary.py's pmc_traffic.json) into the committed
profiles/pmc_traffic.json that bench.py reads for `roofline.traffic`: per kernel the HBM bytes per
launch, split into read and written, under the config's key (config1 at the top level, as before).
    python tools/merge_pmc.py <session pmc_traffic.json> <config> "<source text>" """
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def main():
    src, cfg, note = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    s = json.load(open(src))
    d = json.load(open(DST))
    ent = {}
    for name, v in s.get("kernels", {}).items():
        if not isinstance(v, dict) or "hbm_bytes_per_launch" not in v:
            continue
        e = {"hbm_bytes_per_launch": v["hbm_bytes_per_launch"]}
        for k in ("read_bytes_per_launch", "write_bytes_per_launch", "sq"):
            if k in v:
                e[k] = v[k]
        ent[name] = e
    if cfg == 1:
        for name, e in ent.items():
            d[name] = e
        d["source"] = note
        for k in ("calibration", "read_factor", "write_factor"):
            if k in s:
                d[k] = s[k]
    else:
        ent["source"] = note
        d[f"config{cfg}"] = ent
    json.dump(d, open(DST, "w"), indent=1)
    print("merged", len(ent), "kernels into", DST, f"(config{cfg})")


if __name__ == "__main__":
    main()
