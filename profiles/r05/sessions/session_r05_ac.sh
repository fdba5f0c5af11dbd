# the driver's multi-GPU launch form at N = 1 (torch.distributed.run, RCCL world of one)
mkdir -p gpurun_out/r05_ac
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 5 --warmup 1 > gpurun_out/r05_ac/torchrun_n1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 5 --warmup 1 --check --no-cpu > gpurun_out/r05_ac/check_n1.log 2>&1 || exit $?
