#!/bin/bash
# The drop-in adapter's frame at config[1] profiled: OnFrame's parts (NFGPU_ADAPTER_PROF=1, the -O2
# binary) and a gprof of the -pg build (tools/_bin/adapter_bench_pg: adapter_bench built with -pg;
# writes gmon.out in the cwd).  usage: tools/prof_adapter.sh <mode> <tag>   (mode 2: the NPC HP callbacks)
set -eu
ROOT=$(pwd)
MODE=${1:-2}; TAG=${2:-pg}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
python -c "
import sys; sys.path.insert(0,'.')
from noahgameframe_amd import nfio, workload
w = workload.bench_world(n_obj=1<<20, groups=4096, players_per_group=8, n_ticks=12, tick_ms=100, seed=2031, ext_frac=0.05, host_ops=True)
nfio.write('/tmp/aw.nfio', w)"
NFGPU_ADAPTER_PROF=1 timeout -k 10 400 tests/cpp/_ref/adapter_bench /tmp/aw.nfio 2 10 $MODE 0 0 > gpurun_out/$TAG/run.txt 2> gpurun_out/$TAG/onframe.txt
echo "adapter_bench rc=$?"
cd gpurun_out/$TAG
timeout -k 10 400 $ROOT/tools/_bin/adapter_bench_pg /tmp/aw.nfio 2 10 $MODE 0 0 > run_pg.txt 2>&1
echo "adapter_bench_pg rc=$?"
gprof -b $ROOT/tools/_bin/adapter_bench_pg gmon.out > gprof.txt
rm -f /tmp/aw.nfio gmon.out
