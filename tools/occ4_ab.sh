set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rotation.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02j_parity.log 2>&1 || exit 1
for s in 2 0 2 0; do
  ECDNA_SSA_SCHED=$s timeout -k 10 120 python bench.py --workload c4 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/r02j_c4_s$s.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02j_c4_s$s.json'));print('sched',$s,'ms',round(d['config']['kernel_ms_avg'],1),'lanes',d['config']['grid_lanes'],'value',d['value'])" | tee -a gpurun_out/r02j_c4.txt
done
