set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/ks_report.py > gpurun_out/r04_ks_report.json 2> gpurun_out/r04_ks_report.err
echo ks-done
for w in c2 c4 c5; do
  timeout -k 10 300 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r04_bench_$w.json 2> gpurun_out/r04_bench_$w.err
  echo bench-$w-done
done
bash tools/c4_shards.sh
