#!/bin/bash
# gprof of the drop-in adapter's frame at config[1] (tools/_bin/adapter_bench_pg: adapter_bench
# built with -pg; writes gmon.out in the cwd)
set -e
python -c "
import sys; sys.path.insert(0,'.')
from noahgameframe_amd import nfio, workload
w = workload.bench_world(n_obj=1<<20, groups=4096, players_per_group=8, n_ticks=12, tick_ms=100, seed=2031, ext_frac=0.05, host_ops=True)
nfio.write('gpurun_out/aw.nfio', w)"
mkdir -p gpurun_out/pg && cd gpurun_out/pg
timeout -k 10 400 ../../tools/_bin/adapter_bench_pg ../aw.nfio 2 10 0 0 0 > run.txt 2>&1
gprof -b ../../tools/_bin/adapter_bench_pg gmon.out > gprof.txt
rm -f ../aw.nfio
