set -u
T=${1:-r17e}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for S in ${SLACKS:-8}; do
  NFGPU_BENCH_TRACE=1 NFGPU_TRACE_MEMBERSHIP=1 NFGPU_TRACE_SHARD=1 timeout -k 10 300 python bench.py --self-migrate --steps 40 --warmup 10 --cpu-baseline off --host-calls off --plugin-frame off --adapter-frame off --other-configs off --slack $S > gpurun_out/$T/selfmig_s$S.log 2> gpurun_out/$T/selfmig_s$S.err || { echo "selfmig $S failed"; tail -5 gpurun_out/$T/selfmig_s$S.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/$T/selfmig_s$S.log').read().strip().splitlines()[-1])
print('slack $S', round(d['ms_per_step']*1000,1), {k: round(v['avg_us'],1) for k,v in d['kernels'].items()}, d['migrations'])"
  grep "apply_membership\|shard rows" gpurun_out/$T/selfmig_s$S.err | tail -4 | cut -c1-300
  grep host_ms_per_frame gpurun_out/$T/selfmig_s$S.err | tail -1 | cut -c1-600
done
