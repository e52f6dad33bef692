set -u
T=${1:-r17p}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_adapter.py tests/test_logic_session.py tests/test_tutorial3.py > gpurun_out/$T/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || exit 1
python -c "
import sys; sys.path.insert(0,'.')
from noahgameframe_amd import nfio, workload
nfio.write('/tmp/t3a.nfio', workload.tutorial3_world(n_ticks=160, tick_ms=100))"
for i in 1 2; do
  timeout -k 10 120 tests/cpp/_ref/adapter_bench /tmp/t3a.nfio 10 150 1 > gpurun_out/$T/c0_$i.txt 2>&1
  tail -1 gpurun_out/$T/c0_$i.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('config0 adapter', d['adapter_frame_ms'], d['phases_ms'], d['device_kernels_ms_per_frame'])"
done
SLACKS=8 bash tools/_session_mig.sh $T
