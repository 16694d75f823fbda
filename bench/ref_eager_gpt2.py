"""Reference-semantics GPT-2 step on one GPU: stock PyTorch eager + bf16 autocast + AdamW.

This reproduces what the reference's ``train_model`` does per epoch (``neural_net_model.py:
614-681``: autocast forward, CE, backward, ``optimizer.step()``) with the reference's example
layer layout (``main.py:57-83``), using only stock torch modules.  It is the on-device
*baseline* that the native path is compared against.

Usage: python bench/ref_eager_gpt2.py [B] [steps]
"""
import json
import math
import sys
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Attn(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.h = h

    def forward(self, qkv):
        B, T, C3 = qkv.shape
        C = C3 // 3
        q, k, v = qkv.split(C, dim=2)
        q, k, v = (t.view(B, T, self.h, C // self.h).transpose(1, 2) for t in (q, k, v))
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        return o.transpose(1, 2).contiguous().view(B, T, C)


class Res(nn.Sequential):
    def forward(self, x):
        for m in self:
            x = x + m(x)
        return x


class Emb(nn.Module):
    def __init__(self, V, P, C):
        super().__init__()
        self.wte = nn.Embedding(V, C)
        self.wpe = nn.Embedding(P, C)

    def forward(self, idx):
        return self.wte(idx) + self.wpe(torch.arange(idx.shape[1], device=idx.device))


def build(V=50304, C=768, L=12, H=12, P=1024):
    layers = [Emb(V, P, C), nn.Dropout(0.0)]
    for _ in range(L):
        layers.append(Res(nn.Sequential(nn.LayerNorm(C), nn.Linear(C, 3 * C), Attn(H), nn.Linear(C, C),
                                        nn.Dropout(0.0)),
                          nn.Sequential(nn.LayerNorm(C), nn.Linear(C, 4 * C), nn.GELU(), nn.Linear(4 * C, C),
                                        nn.Dropout(0.0))))
    layers += [nn.LayerNorm(C), nn.Linear(C, V, bias=False)]
    m = nn.Sequential(*layers)
    for mod in m.modules():
        if isinstance(mod, (nn.Linear, nn.Embedding)):
            nn.init.normal_(mod.weight, 0.0, 0.02)
    return m


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    T, V = 1024, 50304
    torch.manual_seed(0)
    model = build().cuda()
    opt = torch.optim.AdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), eps=1e-8)
    x = torch.randint(0, V, (B, T), device="cuda")
    y = torch.randint(0, V, (B, T), device="cuda")

    def step():
        opt.zero_grad()
        with torch.amp.autocast("cuda", dtype=torch.bfloat16):
            logits = model(x)
            loss = F.cross_entropy(logits.view(-1, V), y.view(-1))
        loss.backward()
        opt.step()
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"mode": "reference_eager_autocast", "B": B, "T": T, "ms_per_step": dt * 1e3,
                      "tokens_per_sec": B * T / dt, "loss": float(loss),
                      "max_mem_gb": torch.cuda.max_memory_allocated() / 2**30}))


if __name__ == "__main__":
    main()
