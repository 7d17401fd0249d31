set -u
mkdir -p gpurun_out/r01n
export RXG_BENCH_REHEARSE=1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r01n/bench2.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r01n/bench2.log | tail -5; echo "rc=$rc"
