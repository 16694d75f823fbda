"""Decode attention (csrc/kernels/decode_attn.hip) at batched-decode shapes: µs per launch in a
replayed graph over 12 per-layer caches (as in a decode step), with the fused K/V append and the
device-side length, against the bytes it must read (K and V of every cached position).

    python bench/decode_attn_bench.py [--B 64] [--H 12] [--Hkv 12] [--D 64] [--S 64,128,192,512]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from penroz.ops import attention as A  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--Hkv", type=int, default=12)
    ap.add_argument("--D", type=int, default=64)
    ap.add_argument("--S", default="64,128,192,512")
    ap.add_argument("--cap", type=int, default=1024)
    a = ap.parse_args()
    L, dev, bf = 12, "cuda", torch.bfloat16
    B, H, Hkv, D = a.B, a.H, a.Hkv, a.D
    kc = [torch.randn(B, Hkv, a.cap, D, device=dev, dtype=bf) for _ in range(L)]
    vc = [torch.randn(B, Hkv, a.cap, D, device=dev, dtype=bf) for _ in range(L)]
    rows = torch.randn(B, 1, (H + 2 * Hkv) * D, device=dev, dtype=bf)
    q = rows[:, :, :H * D].view(B, 1, H, D)
    k = rows[:, :, H * D:(H + Hkv) * D].view(B, 1, Hkv, D)
    v = rows[:, :, (H + Hkv) * D:].view(B, 1, Hkv, D)
    for S in [int(x) for x in a.S.split(",")]:
        sl = torch.tensor([S], device=dev)

        def step():
            for l in range(L):
                A.decode_attention(q, kc[l], vc[l], a.cap, seq_len_dev=sl, k_new=k, v_new=v)

        step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(4):
                step()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / (5 * 4 * L) * 1e6
        gb = 2 * B * Hkv * S * D * 2 / 1e9
        print(json.dumps({"B": B, "H": H, "Hkv": Hkv, "D": D, "S": S, "us": round(us, 2),
                          "kv_GB": round(gb, 4), "TBps": round(gb / us * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
