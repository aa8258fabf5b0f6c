set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python3 -m pytest tests/ -q -m gpu -x --deselect tests/test_gpu_statistics.py::test_c5_shard_full_size_properties > gpurun_out/q_tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 tools/sweep.py ECDNA_SSA_WINDOW=1 > gpurun_out/q_sweep.log 2>&1
timeout -k 10 300 python3 tools/probe_configs.py c2 c5 > gpurun_out/q_probe.log 2>&1
