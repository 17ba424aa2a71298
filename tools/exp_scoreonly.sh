set -e
B="python bench.py --no-cpu-baseline"
timeout -k 10 200 $B --L1 1000000 --L2 100000 --outputs '' --steps 2 --warmup 1 > gpurun_out/so_1Mx100k.log 2>&1
timeout -k 10 200 $B --L1 100000 --L2 1000000 --outputs '' --steps 2 --warmup 1 > gpurun_out/so_100kx1M.log 2>&1
timeout -k 10 200 $B --outputs '' --steps 5 --warmup 1 > gpurun_out/so_100k.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --device 0 --pg-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/n2_rehearsal.log 2>&1
