set -o pipefail
mkdir -p gpurun_out/r4v
CLRSDP_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/r4v/b2.log 2>&1; echo "rc=$?"; tail -1 gpurun_out/r4v/b2.log | cut -c1-400
