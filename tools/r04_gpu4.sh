set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_bench_instances.py::test_c4_bench_shard_instance_bit_exact --deselect tests/test_gpu_bench_instances.py::test_c3_bench_instance_bit_exact --deselect tests/test_gpu_bench_instances.py::test_c4_bench_whole_instance_bit_exact > gpurun_out/r04d_gputests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error|assert" gpurun_out/r04d_gputests.log | head -30; tail -3 gpurun_out/r04d_gputests.log; }
tail -2 gpurun_out/r04d_gputests.log
bash tools/r04_sched.sh
