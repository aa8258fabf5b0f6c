set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/r04_ab.sh base chm
L=$PWD/ecdna-evo_amd/lib_ab/cyc/libecdna_ssa.so
ECDNA_SSA_LIB=$L timeout -k 10 200 python3 tools/cycle_stats.py c5 > gpurun_out/cyc_c5.json
cat gpurun_out/cyc_c5.json
ECDNA_SSA_LIB=$L timeout -k 10 200 python3 tools/cycle_stats.py c2 > gpurun_out/cyc_c2.json
cat gpurun_out/cyc_c2.json
