set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g17_torchrun.json 2> gpurun_out/g17_torchrun.err
cat gpurun_out/g17_torchrun.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['config']['parallelism'], d['store'])"
