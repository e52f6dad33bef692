set -u
T=${1:-r17y}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/host_calls_profile.py --frames 30 > gpurun_out/$T/hc.log 2> gpurun_out/$T/hc.err
rc=$?
echo "hc rc=$rc"; tail -1 gpurun_out/$T/hc.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 50 --warmup 5 --cpu-baseline off --plugin-frame off --other-configs off --adapter-frame off > gpurun_out/$T/bench.log 2> gpurun_out/$T/bench.err
rc=$?
echo "bench rc=$rc"
python -c "
import json; d=json.loads(open('gpurun_out/$T/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac']); print(d['host_calls'])"
exit $rc
