#!/bin/bash
# One GPU session: bench (N=1), rocprofv3 kernel-trace stats of the same command, PMC passes
# (FETCH_SIZE and WRITE_SIZE in separate passes) of a 1-step bench and of the calibration program.
# Usage: bash tools/gpu_profile.sh <round-tag> [bins|rows]
set -euo pipefail
TAG=${1:-r01}
STORE=${2:-bins}
# (bench.py defaults: bin store with bin_kmax 32 for C3)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof_$TAG
mkdir -p $O
python3 -c "import sys; sys.argv=['x']; import runpy; g=runpy.run_path('bench.py', run_name='bench_digest'); print(g['kernel_sources_digest']())" > $O/kernel_sources_sha256.txt
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --store $STORE > $O/bench.json 2> $O/bench.err
echo "bench done" 
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --store $STORE > $O/kt.log 2>&1
echo "kernel trace done"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --store $STORE > $O/pmc_fetch.log 2>&1
echo "pmc fetch done"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --store $STORE > $O/pmc_write.log 2>&1
echo "pmc write done"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -T --output-format csv -d $O/pmc_sq -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --store $STORE > $O/pmc_sq.log 2>&1
echo "pmc sq done"
if [ -x tools/bin/pmc_calib ]; then  # (the access-shape calibration, profiles/r01*_pmc_calibration.json)
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/calib_fetch -o pmc -- tools/bin/pmc_calib > $O/calib_fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/calib_write -o pmc -- tools/bin/pmc_calib > $O/calib_write.log 2>&1
echo "calib done"
fi
