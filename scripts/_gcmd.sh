set -e
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --L 128 --steps 60 --warmup 6 --transport host > gpurun_out/bench2_host.json 2> gpurun_out/bench2_host.err
cut -c1-400 gpurun_out/bench2_host.json; python -c "import json; d=json.load(open('gpurun_out/bench2_host.json')); print(json.dumps(d['data_path_tuning'], indent=0))"
