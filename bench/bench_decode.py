"""KV-cache decode throughput, random weights, one MI355X: GPT-2 124M (reference example layout)
or a Gemma-3 1B shaped model (RoPE, GQA 4:1, head_dim 256, 262k vocab; HF config builder).

python bench/bench_decode.py [--model gpt2|gemma3-1b] [--batch 64] [--prompt 64] [--new 128] [--turbo]
Prints one JSON line: generated tokens/s over all rows (BASELINE config 4: batch 64 /generate).
"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.models import kv_cache as KV
import penroz.models.model as M

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--prompt", type=int, default=64)
ap.add_argument("--new", type=int, default=128)
ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
ap.add_argument("--turbo", action="store_true")
ap.add_argument("--model", default="gpt2", choices=["gpt2", "gemma3-1b"])
# the generation window (block_size): a context longer than it is cropped and re-prefilled every
# token, so long-context rows need --block >= prompt + new
ap.add_argument("--block", type=int, default=1024)
a = ap.parse_args()
if a.turbo:
    M.create_kv_cache = lambda n, cap=None: KV.TurboQuantKVCache(n, cap)
torch.manual_seed(0)
if a.model == "gpt2":
    layers, V = bench.gpt2_layers(), 50304
else:  # google/gemma-3-1b-pt text config (shapes only; no checkpoint)
    from types import SimpleNamespace
    V = 262144
    layers = Mapper.from_hf_config(SimpleNamespace(
        model_type="gemma3_text", vocab_size=V, hidden_size=1152, intermediate_size=6912, num_hidden_layers=26,
        num_attention_heads=4, num_key_value_heads=1, head_dim=256, rms_norm_eps=1e-6, rope_theta=1e6,
        rope_local_base_freq=10000.0, attention_dropout=0.0, hidden_activation="gelu_pytorch_tanh",
        query_pre_attn_scalar=256, sliding_window=512))
m = NeuralNetworkModel("dec", Mapper(layers, {"adamw": {"lr": 6e-4}})).to("cuda")
if a.dtype == "bf16":
    m.to(dtype=torch.bfloat16)
ctx = torch.randint(0, V, (a.batch, a.prompt)).tolist()
m.generate_batch(ctx, a.block, 4, temperature=1.0, top_k=50)  # warmup
torch.cuda.synchronize()
t0 = time.perf_counter()
out = m.generate_batch(ctx, a.block, a.new, temperature=1.0, top_k=50)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"metric": "decode tokens/sec (all rows)", "value": a.batch * a.new / dt, "batch": a.batch,
                  "prompt": a.prompt, "new_tokens": a.new, "block": a.block, "ms_per_step": dt / a.new * 1e3, "dtype": a.dtype,
                  "kv_cache": "int8-turboquant" if a.turbo else a.dtype, "model": "gpt2-124m" if a.model == "gpt2" else "gemma3-1b-shape", "data": "random weights"}))
