#!/bin/bash
# tools/_bin/adapter_bench_pg: tests/cpp/adapter_bench.cpp built with -pg (gprof) against the reference's
# sources where they lie (tools/prof_adapter.sh, tools/prof_config0.sh run it on the GPU box)
set -eu
REF=${REF:-/root/reference}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/noahgameframe_amd
SRC=""
for f in NFCDataList NFCProperty NFCPropertyManager NFCRecord NFCRecordManager NFCObject NFCComponentManager NFCMemManager NFMemoryCounter; do SRC="$SRC $REF/NFComm/NFCore/$f.cpp"; done
for f in NFCKernelModule NFCSceneAOIModule NFCEventModule NFCScheduleModule; do SRC="$SRC $REF/NFComm/NFKernelPlugin/$f.cpp"; done
SRC="$SRC $REF/NFComm/NFConfigPlugin/NFCClassModule.cpp $REF/NFComm/NFConfigPlugin/NFCElementModule.cpp"
mkdir -p $ROOT/tools/_bin
g++ -std=c++14 -O2 -pg -DADAPTER_BENCH_PG -w -I$REF -I$REF/Dependencies -I$ROOT/include -I$ROOT/oracle \
    -o $ROOT/tools/_bin/adapter_bench_pg $ROOT/tests/cpp/adapter_bench.cpp $SRC \
    -L$PKG -lnfgpu_plugin -lnfgpu -Wl,-rpath,$PKG -lpthread
