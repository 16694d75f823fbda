"""Graph-captured decoding (models/graph_decode.py) vs the eager per-token path on MI355X:
greedy generation must produce identical tokens (same kernels, same cache contents), through the
sliding-window re-prefill, with a stop token, streaming, multiple rows and the int8 cache.

The module-forward graph is compared with the eager module path token for token. The GPT decode
program (fp32 residual stream, fused add+LN) is compared with the module step's logits within
bf16 tolerance, and its graph replay with the same program run eagerly, token for token."""
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU runner
    pytest.skip("needs a GPU", allow_module_level=True)

import bench
from penroz.models import graph_decode as gd
from penroz.models import kv_cache as kvc
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel


def _model(dtype):
    torch.manual_seed(11)
    m = NeuralNetworkModel("gd", Mapper(bench.gpt2_layers(V=256, C=128, L=2, H=2, P=64),
                                        {"adamw": {"lr": 1e-3}})).to("cuda")
    if dtype == torch.bfloat16:
        m.to(dtype=torch.bfloat16)
    return m


def _both(monkeypatch, fn):
    monkeypatch.setattr(gd, "DECODE_PROGRAM", False)  # the module-forward graph: same numerics as eager
    monkeypatch.setattr(gd, "GRAPH_DECODE", False)
    eager = fn()
    monkeypatch.setattr(gd, "GRAPH_DECODE", True)
    graphed = fn()
    return eager, graphed


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_greedy_batch_matches_eager_through_sliding_window(monkeypatch, dtype):
    m = _model(dtype)
    ctx = torch.randint(0, 256, (3, 5), generator=torch.Generator().manual_seed(0)).tolist()
    eager, graphed = _both(monkeypatch, lambda: m.generate_batch(ctx, 16, 40, temperature=0.0))
    assert graphed == eager
    assert len(graphed[0]) == 45
    assert any(d.graph is not None for d in m._graph_decoders.values()), "graph path not taken"


def test_stop_token_and_stream_match_eager(monkeypatch):
    m = _model(torch.bfloat16)
    ctx = [[3, 1, 4, 1, 5]]
    full_e, full_g = _both(monkeypatch, lambda: m.generate_tokens(ctx, 32, 30, temperature=0.0))
    assert full_g == full_e
    stop = full_e[5 + 7]  # the 8th generated token
    se, sg = _both(monkeypatch, lambda: m.generate_tokens(ctx, 32, 30, temperature=0.0, stop_token=stop))
    assert sg == se and sg[-1] == stop
    st_e, st_g = _both(monkeypatch, lambda: list(m.generate_tokens_stream(ctx, 32, 12, temperature=0.0)))
    assert st_g == st_e and len(st_g) == 12


def test_sampling_and_int8_cache(monkeypatch):
    m = _model(torch.bfloat16)
    ctx = torch.randint(0, 256, (4, 6), generator=torch.Generator().manual_seed(1)).tolist()
    out = m.generate_batch(ctx, 24, 30, temperature=1.0, top_k=5)
    assert len(out) == 4 and all(len(r) == 36 for r in out)
    assert all(0 <= t < 256 for r in out for t in r)
    monkeypatch.setattr(kvc, "TURBO_QUANT_ENABLED", True)
    eager, graphed = _both(monkeypatch, lambda: m.generate_batch(ctx, 24, 10, temperature=0.0))
    assert graphed[0][:7] == eager[0][:7]  # int8 rounding may differ later (kernel vs torch quantiser)
    assert all(len(r) == 16 for r in graphed)


class _EagerGraph:
    """Stands in for a captured graph: replay() runs the decode step eagerly."""

    def __init__(self, dec):
        self.dec = dec

    def replay(self):
        self.dec._step()


@pytest.mark.parametrize("rows", [1, 3, 6, 40])
def test_decode_program_graph_replay_matches_eager_program(monkeypatch, rows):
    m = _model(torch.bfloat16)
    assert gd.GPTDecodeProgram.build(m) is not None, "GPT pattern must select the decode program"
    ctx = torch.randint(0, 256, (rows, 5), generator=torch.Generator().manual_seed(2)).tolist()
    graphed = m.generate_batch(ctx, 16, 40, temperature=0.0)  # through the sliding window too
    assert all(d.program is not None and isinstance(d.graph, torch.cuda.CUDAGraph) for d in m._graph_decoders.values())
    m.__dict__.pop("_graph_decoders")

    def eager_capture(self, last_tok, cache_len, start=0):
        self._set_state(last_tok, cache_len, start)
        self.graph = _EagerGraph(self)

    monkeypatch.setattr(gd.GraphDecoder, "_capture", eager_capture)
    eager = m.generate_batch(ctx, 16, 40, temperature=0.0)
    assert graphed == eager


@pytest.mark.parametrize("rows", [1, 3, 6, 24, 64])
def test_decode_program_step_matches_module_step(rows):
    """One decode-program step vs the module forward: rows 1 and 3 run the decode GEMV path, 6 the
    fused LN-linear path, 24 and 64 the batched block (decode_ln_gemm / decode_gemm_acc)."""
    m = _model(torch.bfloat16)
    cap = 32
    dec = gd.GraphDecoder(m, rows, cap, 0.0, None)
    assert dec.program is not None
    idx = torch.randint(0, 256, (rows, 7), device="cuda", generator=torch.Generator("cuda").manual_seed(3))
    with torch.inference_mode():
        dec.attach()
        try:
            m(idx[:, :6], skip_softmax=True)  # prefill through the modules
            assert dec.cache.seq_len() == 6
            tok = idx[:, 6:]
            dec._set_state(tok, 6)
            for p in dec.pos_layers:
                p.position_offset_tensor = dec.cache.pos_t
            dec.cache.graph_mode = True
            acts, _ = m(tok, skip_softmax=True)
            ref = acts[-1][:, -1, :].float()
            got = dec.program.forward(tok, dec.cache).float()  # rewrites the same cache slot
        finally:
            dec.cache.graph_mode = False
            dec.detach()
    rel = (got - ref).norm() / ref.norm()
    assert rel < 2e-2, rel


def _gemma_model(head_dim, model_type="gemma3_text", intermediate_size=128):
    """Tiny Gemma style model (RoPE, GQA 4:1, RMSNorm, gated MLP) from the HF config builder."""
    from types import SimpleNamespace
    tc = SimpleNamespace(vocab_size=256, hidden_size=64, num_attention_heads=4, num_key_value_heads=1,
                         head_dim=head_dim, num_hidden_layers=2, intermediate_size=intermediate_size,
                         rms_norm_eps=1e-6,
                         rope_theta=10000.0, attention_dropout=0.0, hidden_activation="gelu_pytorch_tanh",
                         model_type=model_type)
    torch.manual_seed(5)
    m = NeuralNetworkModel("gg", Mapper(Mapper.from_hf_config(tc), {"adamw": {"lr": 1e-3}})).to("cuda")
    return m.to(dtype=torch.bfloat16)


@pytest.mark.parametrize("head_dim", [64, 256])
def test_rope_model_graph_decode_matches_eager(monkeypatch, head_dim):
    """RoPE models replay the module forward with a device-offset cos/sin table: same tokens as
    the eager per-token path, through the sliding-window re-prefill, and with the int8 cache."""
    m = _gemma_model(head_dim)
    assert gd.applicable(m) and gd.GemmaDecodeProgram.build(m) is not None
    ctx = torch.randint(0, 256, (2, 5), generator=torch.Generator().manual_seed(4)).tolist()
    eager, graphed = _both(monkeypatch, lambda: m.generate_batch(ctx, 16, 30, temperature=0.0))
    assert graphed == eager
    assert any(d.graph is not None and d.program is None for d in m._graph_decoders.values()), "graph path not taken"
    monkeypatch.setattr(kvc, "TURBO_QUANT_ENABLED", True)
    eager, graphed = _both(monkeypatch, lambda: m.generate_batch(ctx, 24, 10, temperature=0.0))
    assert graphed[0][:7] == eager[0][:7]


@pytest.mark.parametrize("model_type", ["gemma", "gemma2", "gemma3_text"])  # post-norm modes 2, 1, 0
# 1, 3: decode GEMV path; 8: skinny MFMA kernels; 24, 64: decode_gemm / hipBLASLt, with RoPE applied
# inside the decode attention kernel (the opt-in PENROZ_DECODE_ROPE_IN_ATTN=1) or by the RoPE pass
@pytest.mark.parametrize("rows,rope_in_attn", [(1, "0"), (3, "0"), (8, "0"), (24, "0"), (24, "1"), (64, "1")])
def test_gemma_program_step_matches_module_step(monkeypatch, model_type, rows, rope_in_attn):
    monkeypatch.setenv("PENROZ_DECODE_ROPE_IN_ATTN", rope_in_attn)
    m = _gemma_model(256, model_type)
    cap = 32
    dec = gd.GraphDecoder(m, rows, cap, 0.0, None)
    assert isinstance(dec.program, gd.GemmaDecodeProgram)
    idx = torch.randint(0, 256, (rows, 7), device="cuda", generator=torch.Generator("cuda").manual_seed(3))
    with torch.inference_mode():
        dec.attach()
        try:
            m(idx[:, :6], skip_softmax=True)  # prefill through the modules
            tok = idx[:, 6:]
            dec._set_state(tok, 6)
            dec.cache.graph_mode = True
            dec.cache.begin_step()
            acts, _ = m(tok, skip_softmax=True)
            ref = acts[-1][:, -1, :].float()
            dec.cache.begin_step()
            if rope_in_attn == "1":
                assert dec.cache.rope_attend_ok(rows, 4, 1, 256), "in-kernel RoPE path not taken"
            got = dec.program.forward(tok, dec.cache).float()  # rewrites the same cache slot
        finally:
            dec.cache.graph_mode = False
            dec.detach()
    rel = (got - ref).norm() / ref.norm()
    assert rel < 2e-2, rel


@pytest.mark.parametrize("rows", [1, 3])
def test_gemma_program_wide_mlp_falls_back_from_gemv(rows):
    """An intermediate size above decode_gemv's K <= 8192 (Gemma-4 e2b's double-wide MLPs are
    12288): the program must not take the GEMV path for the down projection."""
    m = _gemma_model(64, intermediate_size=8192 + 256)
    dec = gd.GraphDecoder(m, rows, 32, 0.0, None)
    assert isinstance(dec.program, gd.GemmaDecodeProgram)
    assert not dec.program._gemv_ok(rows, 64)
    idx = torch.randint(0, 256, (rows, 7), device="cuda", generator=torch.Generator("cuda").manual_seed(3))
    with torch.inference_mode():
        dec.attach()
        try:
            m(idx[:, :6], skip_softmax=True)
            tok = idx[:, 6:]
            dec._set_state(tok, 6)
            dec.cache.graph_mode = True
            dec.cache.begin_step()
            acts, _ = m(tok, skip_softmax=True)
            ref = acts[-1][:, -1, :].float()
            dec.cache.begin_step()
            got = dec.program.forward(tok, dec.cache).float()
        finally:
            dec.cache.graph_mode = False
            dec.detach()
    rel = (got - ref).norm() / ref.norm()
    assert rel < 2e-2, rel


def test_gemma_program_graph_replay_matches_eager_program(monkeypatch):
    m = _gemma_model(256)
    ctx = torch.randint(0, 256, (2, 5), generator=torch.Generator().manual_seed(6)).tolist()
    graphed = m.generate_batch(ctx, 16, 30, temperature=0.0)
    assert all(isinstance(d.program, gd.GemmaDecodeProgram) and isinstance(d.graph, torch.cuda.CUDAGraph)
               for d in m._graph_decoders.values())
    m.__dict__.pop("_graph_decoders")

    def eager_capture(self, last_tok, cache_len, start=0):
        self._set_state(last_tok, cache_len, start)
        self.graph = _EagerGraph(self)

    monkeypatch.setattr(gd.GraphDecoder, "_capture", eager_capture)
    assert m.generate_batch(ctx, 16, 30, temperature=0.0) == graphed


@pytest.mark.parametrize("top_k", [None, 5])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_seeded_stream_equals_non_stream_with_sampling(dtype, top_k):
    """Reference test_neural_net_model.py:289-304 at temperature 1.0 on the GPU: under the same
    torch.manual_seed the streamed tokens (graph bursts of 1) equal the non-streamed ones (one long
    burst), through the sliding-window re-prefill, with a freshly captured AND a reused graph."""
    m = _model(dtype)
    ctx = [[7, 3, 9]]
    for _ in range(2):  # 1st: the stream captures the graph; 2nd: both reuse it
        torch.manual_seed(42)
        streamed = list(m.generate_tokens_stream(ctx, 16, 40, temperature=1.0, top_k=top_k))
        torch.manual_seed(42)
        full = m.generate_tokens(ctx, 16, 40, temperature=1.0, top_k=top_k)
        assert len(streamed) == 40
        assert full == ctx[0] + streamed
    assert any(d.graph is not None for d in m._graph_decoders.values()), "graph path not taken"
    torch.manual_seed(43)
    other = m.generate_tokens(ctx, 16, 40, temperature=1.0, top_k=top_k)
    assert other != full  # the seed matters
