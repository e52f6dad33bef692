set -e
mkdir -p gpurun_out/sz
for n in 458752 917504 1048576 1376256; do
  g=$((n/256))
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --cpu-baseline off --entities $n --groups $g > gpurun_out/sz/b$n.log 2>&1
  python -c "
import json,sys; d=json.loads(open('gpurun_out/sz/b$n.log').read().strip().splitlines()[-1]); print($n, d['ms_per_step'], d['kernels']['k_tick']['avg_us'], d['roofline']['frac'])"
done
ABL=0,4,512,2048 timeout -k 10 300 python tools/ablate.py --variants 0,4,512,2048 > gpurun_out/sz/abl.log 2>&1
python -c "
import json; t=open('gpurun_out/sz/abl.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d.items(): print(k, v['k_tick']['median_us'])"
