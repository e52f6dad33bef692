set -u
T=${1:-r17f}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_logic_session.py tests/test_adapter.py tests/test_tutorial3.py > gpurun_out/$T/tests.log 2>&1
echo "tests rc=$?"
tail -4 gpurun_out/$T/tests.log
python -c "
import sys; sys.path.insert(0,'.')
from noahgameframe_amd import nfio, workload
w = workload.bench_world(n_obj=1<<20, groups=4096, players_per_group=8, n_ticks=12, tick_ms=100, seed=2031, ext_frac=0.05, host_ops=True)
nfio.write('/tmp/aw.nfio', w)"
for V in 1 0; do
  NFGPU_CHAIN_U=$V timeout -k 10 400 tests/cpp/_ref/adapter_bench /tmp/aw.nfio 2 10 2 0 0 > gpurun_out/$T/npc_chainu$V.txt 2>&1
  echo "npc chain_u=$V rc=$?"
  tail -1 gpurun_out/$T/npc_chainu$V.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['adapter_frame_ms'], d['phases_ms']['mirror'], d['device_kernels_ms_per_frame'])"
done
rm -f /tmp/aw.nfio
