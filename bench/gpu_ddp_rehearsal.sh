# 2-rank rehearsal of the data-parallel paths on a ONE-GPU box (gloo over GPU tensors)
set -o pipefail
mkdir -p gpurun_out
export PENROZ_BENCH_DEVICE=0 PENROZ_DIST_BACKEND=gloo
timeout -k 10 240 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ddp_test.log 2>&1 || { tail -40 gpurun_out/ddp_test.log; exit 1; }
tail -3 gpurun_out/ddp_test.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 16 > gpurun_out/ddp_bench.log 2>&1 || { tail -40 gpurun_out/ddp_bench.log; exit 1; }
grep metric gpurun_out/ddp_bench.log
