#!/bin/bash
# Instruction-mix PMC passes over config[1] under k_tick timing ablations (NFGPU_ABLATE):
# one rocprofv3 --pmc run per (ablation, counter set), each under its own time limit.
#   tools/pmc_mix.sh <tag> [ablations...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-mix}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
B="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES"
for abl in "${@:-0}"; do
  for set in ${SETS:-A B}; do
    eval "C=\$$set"
    echo "=== abl=$abl set=$set"
    NFGPU_ABLATE=$abl timeout -k 5 -s KILL ${PMC_T:-90} rocprofv3 --pmc $C --output-format csv -d "$OUT/a${abl}_$set" -o run -- \
      python bench.py --steps 10 --warmup 2 --cpu-baseline off ${BENCH_ARGS:-} > "$OUT/a${abl}_$set.log" 2>&1
    rc=$?
    echo "rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/a${abl}_$set.log"; exit $rc; }
  done
done
python - "$OUT" "$@" <<'PY'
import sys, os, json
sys.path.insert(0, "tools")
from pmc_summary import load_counters
out, abls = sys.argv[1], sys.argv[2:] or ["0"]
res = {}
for a in abls:
    r = {}
    for s in os.environ.get("SETS", "A B").split():
        c = load_counters(os.path.join(out, f"a{a}_{s}"))
        k = [x for x in c if x.startswith(os.environ.get("KERN", "k_tick"))][0]
        for name, per in c[k].items():
            v = sorted(per.values() if isinstance(per, dict) else per)
            r[name] = v[len(v) // 2]
    res[a] = r
    print(a, json.dumps({k: round(v) for k, v in sorted(r.items())}))
json.dump(res, open(os.path.join(out, "mix.json"), "w"), indent=1)
PY
