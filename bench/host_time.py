"""Host time per step of the headline executor loop (bench.py's step), with the GPU idle and
with the GPU busy ahead of the host: shows whether the host's enqueue rate can keep up with the
GPU (profiles/notes_r6.md §1: 10-13 ms of host time against a 61 ms GPU step).

    python bench/host_time.py
"""
import os, sys, time, torch
sys.path.insert(0, os.getcwd())
import bench
args = bench.parse_args(["--steps", "10"])
cfg = bench.MODELS["gpt2-124m"]
dev = torch.device("cuda", 0)
model, runner = bench._build(args, cfg, dev, "fused", 1)
g = torch.Generator().manual_seed(0)
pool = [torch.randint(0, 50304, (64, 1025), generator=g).pin_memory() for _ in range(4)]
step = bench._make_step(runner, pool, dev)
for i in range(5): step(i)
torch.cuda.synchronize()
hs = []
t0 = time.perf_counter()
for i in range(20):
    a = time.perf_counter(); step(i); hs.append(time.perf_counter() - a)
torch.cuda.synchronize()
tw = (time.perf_counter() - t0) / 20
print(f"host per step: median {sorted(hs)[10]*1e3:.2f} ms, min {min(hs)*1e3:.2f}, max {max(hs)*1e3:.2f}; wall per step {tw*1e3:.2f} ms")
# host time with the GPU pre-blocked: enqueue 3 steps behind a long sleep kernel
torch.cuda._sleep(int(2e9))
a = time.perf_counter()
for i in range(3): step(i)
h3 = (time.perf_counter() - a) / 3
torch.cuda.synchronize()
print(f"host per step with the GPU busy ahead: {h3*1e3:.2f} ms")
