#!/bin/bash
# The drop-in adapter's frame at config[0] (Tutorial3, 10k objects) profiled: the device kernels of a
# frame (rocprofv3 --kernel-trace --stats), nfk_execute's host phases (NFGPU_TRACE_EXEC) and a gprof
# of the -pg build over many frames.  usage: tools/prof_config0.sh <tag>
set -eu
ROOT=$(pwd)
TAG=${1:-c0}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
python -c "
import sys; sys.path.insert(0,'.')
from noahgameframe_amd import nfio, workload
nfio.write('/tmp/t3a.nfio', workload.tutorial3_world(n_ticks=60, tick_ms=100))
nfio.write('/tmp/t3b.nfio', workload.tutorial3_world(n_ticks=20010, tick_ms=100))"
timeout -k 10 120 tests/cpp/_ref/adapter_bench /tmp/t3a.nfio 10 50 1 > gpurun_out/$TAG/run.txt
echo "run rc=$?"
NFGPU_TRACE_EXEC=1 timeout -k 10 120 tests/cpp/_ref/adapter_bench /tmp/t3a.nfio 10 50 1 > gpurun_out/$TAG/run_trace.txt 2> gpurun_out/$TAG/trace.txt
echo "trace rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $ROOT/gpurun_out/$TAG/prof -o c0 -- tests/cpp/_ref/adapter_bench /tmp/t3a.nfio 10 50 1 > gpurun_out/$TAG/run_prof.txt 2>&1
echo "rocprof rc=$?"
cd gpurun_out/$TAG
timeout -k 10 300 $ROOT/tools/_bin/adapter_bench_pg /tmp/t3b.nfio 10 20000 1 > run_pg.txt 2>&1
echo "pg rc=$?"
gprof -b $ROOT/tools/_bin/adapter_bench_pg gmon.out > gprof.txt
rm -f /tmp/t3a.nfio /tmp/t3b.nfio gmon.out
