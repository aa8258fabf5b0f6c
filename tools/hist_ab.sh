set -e
for w in c3 c4; do for pw in 0 1; do
ECDNA_HIST_PER_WAVE=$pw timeout -k 10 300 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG:-r05q}_hist_${w}_$pw.json 2>/dev/null
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG:-r05q}_hist_${w}_$pw.json').read().splitlines()[-1]); c=d['config']
print('$w per_wave=$pw', 'hist ms %.3f'%c['hist_kernel_ms_avg'], 'kernel ms %.2f'%c['kernel_ms_avg'], 'step ms %.2f'%d['ms_per_step'], 'events', c['events_per_step'])"
done; done
