"""HIP kernel parity: every kernel vs a plain PyTorch fp32 reference of the same op (MI355X)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover - CPU runner
    pytest.skip("needs a GPU", allow_module_level=True)

from penroz.ops import _ext, attention as A, norms as Nm, activations as Ac, fused as Fu, sampling as Sa, rope as Ro

DEV = "cuda"


def test_extension_is_native():
    assert _ext.available(), "penroz_kernels must be importable on the GPU box"
    import penroz_kernels
    assert penroz_kernels.__file__.endswith(".so")


def _close(a, b, atol, rtol=0.0, msg=""):
    err = (a.float() - b.float()).abs().max().item()
    lim = atol + rtol * b.float().abs().max().item()
    assert err <= lim, f"{msg} max err {err} > {lim}"


@pytest.mark.parametrize("C", [768, 1600, 256, 100])
@pytest.mark.parametrize("xdt", [torch.float32, torch.bfloat16])
def test_layernorm_fwd(C, xdt):
    torch.manual_seed(0)
    x = (torch.randn(300, C, device=DEV) * 3 + 1).to(xdt)
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    y, mean, rstd = Nm.ln_fwd(x, w, b, 1e-5, torch.float32)
    ry, rm, rr = Nm.reference_layer_norm(x, w, b, 1e-5)
    _close(y, ry, 2e-4, 1e-4)
    _close(mean, rm, 1e-4)
    _close(rstd, rr, 1e-3, 1e-4)
    yb, _, _ = Nm.ln_fwd(x, w, b, 1e-5, torch.bfloat16)
    _close(yb, ry, 0.05, 0.01)


@pytest.mark.parametrize("C", [768, 1600])
def test_add_layernorm_fwd(C):
    x = torch.randn(257, C, device=DEV)
    d = torch.randn(257, C, device=DEV).to(torch.bfloat16)
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    out = torch.empty_like(x)
    y, _, _ = Nm.add_ln_fwd(x, d, out, w, b, 1e-5)
    ref = x + d.float()
    _close(out, ref, 1e-6)
    ry, _, _ = Nm.reference_layer_norm(ref, w, b, 1e-5)
    _close(y, ry, 0.06, 0.01)


@pytest.mark.parametrize("C", [768, 4100])  # register-resident and looping kernels
def test_add_layernorm_fwd_delta_bias(C):
    x = torch.randn(33, C, device=DEV)
    d = torch.randn(33, C, device=DEV).to(torch.bfloat16)
    db = torch.randn(C, device=DEV)
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    out = torch.empty_like(x)
    y, _, _ = Nm.add_ln_fwd(x, d, out, w, b, 1e-5, delta_bias=db)
    ref = x + d.float() + db
    _close(out, ref, 1e-5)
    ry, _, _ = Nm.reference_layer_norm(ref, w, b, 1e-5)
    _close(y, ry, 0.06, 0.01)


@pytest.mark.parametrize("C", [768, 1600])
def test_layernorm_bwd(C):
    torch.manual_seed(1)
    N = 1000
    x = torch.randn(N, C, device=DEV) * 2
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    dy = torch.randn(N, C, device=DEV).to(torch.bfloat16)
    _, mean, rstd = Nm.ln_fwd(x, w, b, 1e-5, torch.float32)
    base = torch.randn(N, C, device=DEV)
    dres = base.clone()
    dres_bf = torch.empty(N, C, device=DEV, dtype=torch.bfloat16)
    dw, db, dbp = (torch.ones(C, device=DEV) for _ in range(3))
    Nm.ln_bwd(dy, x, mean, rstd, w, dres, True, dres_bf, dw, db, dbp)
    rdx, rdw, rdb = Nm.reference_layer_norm_bwd(dy, x, mean, rstd, w)
    _close(dres, base + rdx, 2e-3, 1e-4, "dx")
    _close(dres_bf, base + rdx, 0.05, 0.01, "dx bf16")
    _close(dw, 1 + rdw, 1e-2, 1e-4, "dw")
    _close(db, 1 + rdb, 1e-2, 1e-4, "db")
    _close(dbp, 1 + (base + rdx).sum(0), 1e-2, 1e-4, "dbias")


@pytest.mark.parametrize("approx", ["none", "tanh"])
def test_gelu(approx):
    x = (torch.randn(512, 3072, device=DEV) * 3).to(torch.bfloat16)
    y = Ac.gelu_fwd(x, approx)
    _close(y, F.gelu(x.float(), approximate=approx), 0.03, 0.01)
    dy = torch.randn_like(x)
    ref = Ac.reference_gelu_bwd(dy, x, approx)
    dx = Ac.gelu_bwd(dy, x, approx)
    _close(dx, ref, 0.05, 0.01)
    dbias = torch.zeros(3072, device=DEV)
    out = dy.clone()
    Ac.gelu_bwd(out, x, approx, dbias, out=out)  # in place + fused column sum
    _close(out, ref, 0.05, 0.01)
    _close(dbias, ref.sum(0), 0.05, 2e-3, "dbias vs fp32 reference")  # independent fp32 column sum


@pytest.mark.parametrize("rows", [8192, 8191])
def test_gelu_wide_grid_stride_and_row_pairs(rows):
    """Sizes past one trip of the grid: the GELU forward's 4-chunk unrolled trips and its tail, the
    backward + column-sum kernel's two-rows-per-trip loop with odd row counts per wave."""
    torch.manual_seed(rows)
    x = (torch.randn(rows, 3072, device=DEV) * 3).to(torch.bfloat16)
    y = Ac.gelu_fwd(x, "none")
    _close(y, F.gelu(x.float()), 0.03, 0.01)
    dy = torch.randn_like(x)
    ref = Ac.reference_gelu_bwd(dy, x, "none")
    dbias = torch.zeros(3072, device=DEV)
    out = dy.clone()
    Ac.gelu_bwd(out, x, "none", dbias, out=out)
    _close(out, ref, 0.05, 0.01)
    _close(dbias, ref.sum(0), 0.25, 2e-3, "dbias vs fp32 reference")  # independent fp32 column sum


@pytest.mark.parametrize("N,V", [(64, 50304), (37, 262144), (5, 1000)])
def test_fused_cross_entropy_autograd_matches_torch(N, V):
    """fused_ops.cross_entropy (bf16 logits, separate gradient buffer, device-side mean over the
    non-ignored rows) == F.cross_entropy on the fp32 logits; the logits are left intact."""
    torch.manual_seed(0)
    logits = (torch.randn(N, V, device=DEV) * 3).to(torch.bfloat16).requires_grad_()
    tg = torch.randint(0, V, (N,), device=DEV)
    tg[1] = -100  # ignored row
    keep = logits.detach().clone()
    loss = Fu.cross_entropy(logits, tg)
    (loss * 0.5).backward()
    assert torch.equal(logits.detach(), keep)
    ref = logits.detach().float().requires_grad_()
    rl = F.cross_entropy(ref, tg)
    (rl * 0.5).backward()
    assert abs(loss.item() - rl.item()) < 2e-3 * max(1.0, abs(rl.item()))
    rel = ((logits.grad.float() - ref.grad).norm() / ref.grad.norm()).item()
    assert rel < 0.01, rel
    assert logits.grad[1].abs().max().item() == 0.0


def test_fused_cross_entropy_no_grad_and_all_ignored():
    """Under no_grad the fused CE computes the loss only (no gradient buffer, logits untouched);
    every target ignored gives NaN like F.cross_entropy; fp16 logits run torch's CE."""
    logits = (torch.randn(16, 1000, device=DEV) * 3).to(torch.bfloat16)
    tg = torch.randint(0, 1000, (16,), device=DEV)
    keep = logits.clone()
    with torch.no_grad():
        loss = Fu.cross_entropy(logits, tg)
    assert torch.equal(logits, keep)
    assert abs(loss.item() - F.cross_entropy(logits.float(), tg).item()) < 2e-3
    allign = torch.full((16,), -100, device=DEV, dtype=torch.long)
    assert torch.isnan(Fu.cross_entropy(logits, allign)) and torch.isnan(F.cross_entropy(logits.float(), allign))
    h = logits.half().requires_grad_()
    lh = Fu.cross_entropy(h, tg)
    lh.backward()
    assert lh.grad_fn.name() != "_FusedCrossEntropyFnBackward" and torch.isfinite(h.grad).all()


def test_cross_entropy_single_unpadded_row_is_refused():
    """A lone [1, V] row with V % 8 != 0 and no allocated padding: the kernel's last 16-B chunk
    would run past the allocation, so the call is refused instead (pad the buffer)."""
    logits = torch.randn(1, 50257, device=DEV).to(torch.bfloat16)
    with pytest.raises(RuntimeError, match="padding"):
        Fu.cross_entropy_fwd_bwd(logits, torch.tensor([5], device=DEV), 1.0)
    buf = torch.zeros(1, 50264, device=DEV, dtype=torch.bfloat16)
    buf[:, :50257] = logits
    loss = Fu.cross_entropy_fwd_bwd(buf[:, :50257], torch.tensor([5], device=DEV), 0.0)
    assert abs(loss.item() - F.cross_entropy(logits.float(), torch.tensor([5], device=DEV)).item()) < 2e-3


def test_colsum():
    x = torch.randn(4099, 2304, device=DEV).to(torch.bfloat16)
    out = torch.full((2304,), 2.0, device=DEV)
    Fu.colsum(x, out)
    _close(out, 2 + x.float().sum(0), 0.05, 1e-4)


def test_embedding():
    V, P, C, B, T = 1000, 64, 768, 3, 50
    wte, wpe = torch.randn(V, C, device=DEV), torch.randn(P, C, device=DEV)
    idx = torch.randint(0, V, (B, T), device=DEV)
    idx[0, :5] = 7  # repeated tokens exercise the scatter-add
    out = Fu.embedding_fwd(idx, wte, wpe, 3)
    _close(out, Fu.reference_embedding_fwd(idx, wte, wpe, 3), 1e-6)
    dout = torch.randn(B * T, C, device=DEV)
    dwte, dwpe = torch.zeros(V, C, device=DEV), torch.zeros(P, C, device=DEV)
    Fu.embedding_bwd(dout, idx, dwte, dwpe, 3)
    w1, w2 = wte.clone().requires_grad_(), wpe.clone().requires_grad_()
    (Fu.reference_embedding_fwd(idx, w1, w2, 3) * dout).sum().backward()
    _close(dwte, w1.grad, 1e-4)
    _close(dwpe, w2.grad, 1e-4)


@pytest.mark.parametrize("V", [50304, 50257 - 1, 1000])
def test_cross_entropy(V):
    V = V - V % 8
    N = 64
    logits = (torch.randn(N, V, device=DEV) * 3).to(torch.bfloat16)
    tgt = torch.randint(0, V, (N,), device=DEV)
    tgt[3] = -100
    ref_loss = F.cross_entropy(logits.float(), tgt, reduction="none", ignore_index=-100)
    lf = logits.float().requires_grad_()
    F.cross_entropy(lf, tgt, ignore_index=-100, reduction="sum").backward()
    g = logits.clone()
    loss = Fu.cross_entropy_fwd_bwd(g, tgt, 0.5)
    _close(loss, ref_loss, 2e-3, 1e-4, "loss")
    _close(g, 0.5 * lf.grad, 2e-3, 1e-2, "grad")
    g2 = logits.clone()
    Fu.cross_entropy_fwd_bwd(g2, tgt, 0.0)
    assert torch.equal(g2, logits), "eval mode must not modify logits"


@pytest.mark.parametrize("V", [50257, 1001, 9])
def test_cross_entropy_any_vocab_padded_rows(V):
    """HF GPT-2's V = 50257: rows at a padded stride (multiple of 8); pads read as -inf, get 0."""
    N, ld = 40, (V + 7) // 8 * 8
    buf = torch.full((N, ld), 7.0, device=DEV, dtype=torch.bfloat16)  # pads hold junk
    logits = buf[:, :V]
    logits.copy_((torch.randn(N, V, device=DEV) * 3).to(torch.bfloat16))
    tgt = torch.randint(0, V, (N,), device=DEV)
    tgt[0] = V - 1
    ref_loss = F.cross_entropy(logits.float(), tgt, reduction="none")
    lf = logits.float().requires_grad_()
    F.cross_entropy(lf, tgt, reduction="sum").backward()
    loss = Fu.cross_entropy_fwd_bwd(logits, tgt, 0.25)
    _close(loss, ref_loss, 2e-3, 1e-4, "loss")
    _close(logits, 0.25 * lf.grad, 2e-3, 1e-2, "grad")
    assert torch.all(buf[:, V:] == 0), "pad columns must get a zero gradient"
    # the lm_head GEMM writes straight into the strided view (no hidden copy)
    x = torch.randn(N, 64, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(V, 64, device=DEV, dtype=torch.bfloat16)
    ptr = logits.data_ptr()
    torch.mm(x, w.t(), out=logits)
    assert logits.data_ptr() == ptr
    _close(logits, x.float() @ w.float().t(), 0.1, 0.01)


@pytest.mark.parametrize("n", [10007, 10_000_003])  # the second runs the 2-group unrolled trips
def test_adamw_flat_matches_torch(n):
    torch.manual_seed(0)
    p = torch.randn(n, device=DEV)
    ref = p.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    shadow = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    for step in range(1, 6):
        g = torch.randn(n, device=DEV)
        ref.grad = g.clone()
        opt.step()
        Fu.adamw_step(p, g, m, v, shadow, 1e-2, 0.9, 0.95, 1e-8, 0.1, step)
    _close(p, ref.detach(), 1e-5, 1e-5)
    _close(shadow, ref.detach(), 0.02, 0.01)


def test_fused_optimizer_list_mode():
    from penroz.models.optim import FusedAdamW, FusedAdam
    torch.manual_seed(0)
    for cls, tcls in ((FusedAdamW, torch.optim.AdamW), (FusedAdam, torch.optim.Adam)):
        ps = [torch.randn(s, device=DEV, requires_grad=True) for s in ((33, 17), (5,), (70000,))]
        rs = [p.detach().clone().requires_grad_() for p in ps]
        o1, o2 = cls(ps, lr=3e-3, weight_decay=0.05), tcls(rs, lr=3e-3, weight_decay=0.05)
        for _ in range(3):
            for p, r in zip(ps, rs):
                g = torch.randn_like(p)
                p.grad, r.grad = g.clone(), g.clone()
            o1.step()
            o2.step()
        for p, r in zip(ps, rs):
            _close(p, r, 1e-5, 1e-5)
        assert set(o1.state_dict()["state"][0].keys()) == set(o2.state_dict()["state"][0].keys())


def test_fused_optimizer_list_mode_bf16_params():
    """bf16 parameters (HF / Gemma imports on the generic engine): bf16 state like torch keeps, the
    update done in fp32 and rounded once — within bf16 rounding of an fp32 AdamW on the same
    values, and closer to it than torch's own bf16 foreach step."""
    from penroz.models.optim import FusedAdamW
    torch.manual_seed(0)
    shapes = ((33, 17), (5,), (70000,))
    ps = [torch.randn(s, device=DEV).to(torch.bfloat16).requires_grad_() for s in shapes]
    f32 = [p.detach().float().clone().requires_grad_() for p in ps]
    tb = [p.detach().clone().requires_grad_() for p in ps]
    o1 = FusedAdamW(ps, lr=3e-3, weight_decay=0.05)
    o2 = torch.optim.AdamW(f32, lr=3e-3, weight_decay=0.05)
    o3 = torch.optim.AdamW(tb, lr=3e-3, weight_decay=0.05)
    for _ in range(3):
        for p, r, t in zip(ps, f32, tb):
            g = torch.randn(p.shape, device=DEV).to(torch.bfloat16)
            p.grad, r.grad, t.grad = g.clone(), g.float(), g.clone()
        o1.step()
        o2.step()
        o3.step()
    for p, r, t in zip(ps, f32, tb):
        assert p.dtype == torch.bfloat16 and o1.state[p]["exp_avg"].dtype == torch.bfloat16
        err = (p.float() - r).abs().max().item()
        assert err <= 0.02 * r.abs().max().item() + 1e-2, err
        assert err <= (t.float() - r).abs().max().item() + 1e-2


def _qkv(B, T, H, Hkv, D=64, scale=1.0):
    return (torch.randn(B, T, (H + 2 * Hkv) * D, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("variant", [1, 3])
@pytest.mark.parametrize("B,T,H,Hkv", [(2, 1024, 4, 4), (1, 200, 3, 3), (2, 130, 4, 2), (1, 64, 2, 1), (1, 5, 2, 2),
                                       (1, 192, 2, 2), (1, 320, 2, 2)])
def test_flash_fwd(B, T, H, Hkv, variant):
    torch.manual_seed(0)
    qkv = _qkv(B, T, H, Hkv, scale=1.5)
    k = _ext.kernels()
    prev = k.flash_fwd_variant(variant)
    try:
        out, lse = A.flash_fwd(qkv, H, Hkv, 64)
    finally:
        k.flash_fwd_variant(prev)
    ro, rl = A.reference_attention_lse(qkv, H, Hkv, 64)
    _close(out, ro, 0.02, 0.01, "out")
    _close(lse, rl, 2e-3, 1e-4, "lse")


@pytest.mark.parametrize("variant", [1, 3])
@pytest.mark.parametrize("profile", ["grow", "shrink", "spike"])
def test_flash_fwd_running_max_paths(profile, variant):
    """The running-max paths on data built to take them (random data almost never does):
    'grow' — key magnitudes rise along the sequence, so most tiles raise m (fwd4: the tile sum
    exceeds 2^8 and the rare path recomputes the tile); 'shrink' — the first tile holds the
    maximum and later tiles' p underflow towards 0; 'spike' — one very large key per 200 in an
    otherwise flat row (a single p far above the running max). Exercises the deferred-rescale
    branch (kRescaleThr) of both forward kernels."""
    torch.manual_seed(1)
    B, T, H = 2, 640, 3
    qkv = torch.randn(B, T, 3 * H * 64, device=DEV)
    t = torch.arange(T, device=DEV, dtype=torch.float32)
    if profile == "grow":
        f = 0.2 + 3.0 * t / T
    elif profile == "shrink":
        f = 3.2 - 3.0 * t / T
    else:
        f = torch.full((T,), 0.3, device=DEV)
        f[::200] = 6.0
    qkv[:, :, H * 64:2 * H * 64] *= f.view(1, T, 1)
    qkv[:, :, :H * 64] *= 2.0
    qkv = qkv.to(torch.bfloat16)
    k = _ext.kernels()
    prev = k.flash_fwd_variant(variant)
    try:
        out, lse = A.flash_fwd(qkv, H, H, 64)
    finally:
        k.flash_fwd_variant(prev)
    ro, rl = A.reference_attention_lse(qkv, H, H, 64)
    _close(out, ro, 0.03, 0.01, "out")
    _close(lse, rl, 0.02, 1e-3, "lse")


def test_flash_bwd_stamps_diagnostic_is_transparent():
    """The s_memtime phase build of the dK/dV kernel (bench/attn_stamps.py) counts every ring
    iteration and returns the same gradients as the production build."""
    torch.manual_seed(0)
    B, T, H = 2, 384, 4
    qkv = _qkv(B, T, H, H)
    out, lse = A.flash_fwd(qkv, H, H, 64)
    dout = torch.randn_like(out)
    ref = A.flash_bwd(dout, qkv, out, lse, H, H, 64)
    k = _ext.kernels()
    buf = torch.zeros(6, dtype=torch.int64, device=DEV)
    k.flash_bwd_stamps(buf)
    try:
        got = A.flash_bwd(dout, qkv, out, lse, H, H, 64)
    finally:
        k.flash_bwd_stamps(None)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    v = buf.tolist()
    nblk = T // 128
    assert v[5] == B * H * 4 * sum(T // 64 - 2 * kb for kb in range(nblk))  # wave iterations
    assert all(x > 0 for x in v[:5])


@pytest.mark.parametrize("B,T,H,Hkv", [(2, 512, 4, 4), (1, 200, 3, 3), (2, 130, 4, 2), (1, 7, 2, 1), (1, 1024, 2, 2),
                                       (1, 320, 4, 1)])
def test_flash_bwd(B, T, H, Hkv):
    torch.manual_seed(0)
    qkv = _qkv(B, T, H, Hkv)
    out, lse = A.flash_fwd(qkv, H, Hkv, 64)
    dout = torch.randn(B, T, H * 64, device=DEV).to(torch.bfloat16)
    dq = A.flash_bwd(dout, qkv, out, lse, H, Hkv, 64)
    x = qkv.float().requires_grad_()
    ro, _ = A.reference_attention_lse(x, H, Hkv, 64)
    (ro * dout.float()).sum().backward()
    ref = x.grad
    for name, sl in (("dq", slice(0, H * 64)), ("dk", slice(H * 64, (H + Hkv) * 64)), ("dv", slice((H + Hkv) * 64, None))):
        a, r = dq[..., sl].float(), ref[..., sl]
        rel = (a - r).norm() / r.norm()
        assert rel < 0.02, f"{name} relative error {rel}"


@pytest.mark.parametrize("B,T,H,Hkv,p", [(2, 512, 4, 4, 0.0), (1, 200, 3, 3, 0.0), (2, 130, 4, 2, 0.0),
                                         (1, 7, 2, 1, 0.0), (1, 300, 2, 2, 0.1)])
def test_flash_bwd_fused_bias_grad(B, T, H, Hkv, p):
    """dbias (the qkv bias gradient) from the attention-backward epilogues == the column sums of the
    dqkv the same call stored, accumulated onto the existing value (fp32 torch reference)."""
    torch.manual_seed(0)
    qkv = _qkv(B, T, H, Hkv)
    out, lse = A.flash_fwd(qkv, H, Hkv, 64, p, 7)
    dout = torch.randn(B, T, H * 64, device=DEV).to(torch.bfloat16)
    base = torch.randn((H + 2 * Hkv) * 64, device=DEV)
    dbias = base.clone()
    dq = A.flash_bwd(dout, qkv, out, lse, H, Hkv, 64, p, 7, dbias=dbias)
    dq_plain = A.flash_bwd(dout, qkv, out, lse, H, Hkv, 64, p, 7)
    torch.testing.assert_close(dq, dq_plain, rtol=0, atol=0)  # the epilogue does not change dqkv
    ref = base + dq.float().reshape(-1, dq.shape[-1]).sum(0)
    torch.testing.assert_close(dbias, ref, rtol=1e-4, atol=1e-3)


def test_flash_dropout_matches_masked_reference():
    """With one-hot V rows the forward output reveals the dropout mask exactly; the backward
    must reproduce the gradients of softmax -> mask/(1-p) -> @V with that same mask."""
    _dropout_masked_reference()


def _dropout_masked_reference():
    torch.manual_seed(0)
    B, T, H, D, p = 1, 64, 1, 64, 0.3
    qkv = _qkv(B, T, H, H)
    qkv[..., 2 * D:] = torch.eye(T, D, device=DEV).to(torch.bfloat16)  # V[key] = e_key
    out, lse = A.flash_fwd(qkv, H, H, D, p, seed=99)
    out2, _ = A.flash_fwd(qkv, H, H, D, p, seed=99)
    assert torch.equal(out, out2)
    causal = torch.ones(T, T, device=DEV, dtype=torch.bool).tril()
    mask = (out[0].float() != 0) & causal
    frac = mask.sum() / causal.sum()
    assert 0.55 < frac < 0.85, frac
    x = qkv.float().requires_grad_()
    q, k, v = x[0, :, :D], x[0, :, D:2 * D], x[0, :, 2 * D:]
    s = (q @ k.t()) / math.sqrt(D)
    s = s.masked_fill(~causal, float("-inf"))
    pd = torch.softmax(s, -1) * mask / (1 - p)
    ref = pd @ v
    _close(out[0], ref, 0.02, 0.01, "dropout fwd")
    dout = torch.randn(B, T, H * D, device=DEV).to(torch.bfloat16)
    (ref * dout[0].float()).sum().backward()
    g = A.flash_bwd(dout, qkv, out, lse, H, H, D, p, seed=99).float()
    rel = (g - x.grad).norm() / x.grad.norm()
    assert rel < 0.02, rel


# ---- head_dim 128 / 256 / 512 (csrc/kernels/flash_attn_gen.hip): Gemma-3 1B is H=4, Hkv=1, D=256;
# 512 is Gemma-4's global_head_dim (full-attention layers)
@pytest.mark.parametrize("D", [128, 256, 512])
@pytest.mark.parametrize("B,T,H,Hkv", [(2, 512, 4, 1), (1, 200, 3, 3), (2, 130, 4, 2), (1, 5, 2, 2), (1, 1024, 4, 1),
                                       (1, 96, 8, 2)])
def test_flash_gen_fwd_bwd(D, B, T, H, Hkv):
    torch.manual_seed(0)
    assert D in A.SUPPORTED_HEAD_DIMS
    qkv = _qkv(B, T, H, Hkv, D, scale=1.2)
    out, lse = A.flash_fwd(qkv, H, Hkv, D)
    ro, rl = A.reference_attention_lse(qkv, H, Hkv, D)
    _close(out, ro, 0.02, 0.01, "out")
    _close(lse, rl, 2e-3, 1e-4, "lse")
    dout = torch.randn(B, T, H * D, device=DEV).to(torch.bfloat16)
    dq = A.flash_bwd(dout, qkv, out, lse, H, Hkv, D)
    x = qkv.float().requires_grad_()
    ro2, _ = A.reference_attention_lse(x, H, Hkv, D)
    (ro2 * dout.float()).sum().backward()
    ref = x.grad
    for name, sl in (("dq", slice(0, H * D)), ("dk", slice(H * D, (H + Hkv) * D)), ("dv", slice((H + Hkv) * D, None))):
        a, r = dq[..., sl].float(), ref[..., sl]
        rel = (a - r).norm() / r.norm()
        assert rel < 0.02, f"D={D} {name} relative error {rel}"


@pytest.mark.parametrize("D", [128, 256, 512])
@pytest.mark.parametrize("B,T,H,Hkv", [(8, 1024, 4, 1), (1, 300, 3, 3), (2, 130, 4, 2)])
def test_flash_gen_kv_split(monkeypatch, D, B, T, H, Hkv):
    """Work-list split (flash_attn_gen.hip attn_plan): every block but the first swept as two
    key-range halves with fp32 partials merged by fa_gen_combine (PENROZ_ATTN_KV_SPLIT=2) vs no
    split (=0): both match the fp32 reference, and with dropout the two agree (same mask)."""
    torch.manual_seed(3)
    qkv = _qkv(B, T, H, Hkv, D, scale=1.1)
    dout = torch.randn(B, T, H * D, device=DEV).to(torch.bfloat16)
    x = qkv.float().requires_grad_()
    ro, rl = A.reference_attention_lse(x, H, Hkv, D)
    (ro * dout.float()).sum().backward()
    res = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("PENROZ_ATTN_KV_SPLIT", mode)
        out, lse = A.flash_fwd(qkv, H, Hkv, D)
        _close(out, ro.detach(), 0.02, 0.01, f"out mode {mode}")
        _close(lse, rl.detach(), 2e-3, 1e-4, f"lse mode {mode}")
        g = A.flash_bwd(dout, qkv, out, lse, H, Hkv, D).float()
        rel = (g - x.grad).norm() / x.grad.norm()
        assert rel < 0.02, f"mode {mode} grad relative error {rel}"
        od, ld = A.flash_fwd(qkv, H, Hkv, D, 0.1, seed=9)
        res[mode] = (od.float(), A.flash_bwd(dout, qkv, od, ld, H, Hkv, D, 0.1, seed=9).float())
    for a, b in zip(res["0"], res["2"]):
        assert ((a - b).norm() / b.norm()) < 1e-2


@pytest.mark.parametrize("D", [32, 80, 96, 160, 384])
@pytest.mark.parametrize("B,T,H,Hkv,p", [(2, 130, 4, 2, 0.0), (1, 300, 3, 3, 0.0), (2, 64, 4, 1, 0.1)])
def test_flash_padded_head_dims(D, B, T, H, Hkv, p):
    """Head dims without their own kernel run the next wider one on zero-padded heads: forward
    and input gradient vs the fp32 reference (with dropout: finite output and gradient)."""
    torch.manual_seed(D + T)
    qkv = _qkv(B, T, H, Hkv, D, scale=1.1).requires_grad_()
    if p == 0.0:
        out = A.causal_attention_qkv(qkv, H, Hkv, D)
        x = qkv.detach().float().requires_grad_()
        ro, _ = A.reference_attention_lse(x, H, Hkv, D)
        _close(out, ro, 0.02, 0.01, "out")
        dout = torch.randn_like(out)
        out.backward(dout)
        (ro * dout.float()).sum().backward()
        rel = (qkv.grad.float() - x.grad).norm() / x.grad.norm()
        assert rel < 0.02, rel
    else:
        torch.manual_seed(5)
        out = A.causal_attention_qkv(qkv, H, Hkv, D, dropout_p=p)
        assert torch.isfinite(out.float()).all()
        out.float().sum().backward()
        assert torch.isfinite(qkv.grad.float()).all() and qkv.grad.abs().sum() > 0


@pytest.mark.parametrize("D", [128, 256, 512])
def test_flash_gen_rescale_branch(D):
    """One key spiking far above the rest at a late tile forces the online-softmax rescale."""
    torch.manual_seed(1)
    B, T, H, Hkv = 1, 256, 2, 1
    qkv = _qkv(B, T, H, Hkv, D, scale=0.3)
    q = qkv[..., :D].float()
    qkv[0, 200, H * D:(H + 1) * D] = (q[0, 230] * 6).to(torch.bfloat16)  # key 200 aligned with query 230
    out, lse = A.flash_fwd(qkv, H, Hkv, D)
    ro, rl = A.reference_attention_lse(qkv, H, Hkv, D)
    _close(out, ro, 0.03, 0.01, "out")
    _close(lse, rl, 5e-3, 1e-4, "lse")


@pytest.mark.parametrize("D", [128, 256, 512])
def test_flash_gen_dropout_matches_masked_reference(D):
    """One-hot V rows (V[k] = e_k, T <= D) make the forward output reveal each head's dropout mask;
    the backward must reproduce the fp32 gradients of softmax -> mask/(1-p) -> @V with it."""
    torch.manual_seed(2)
    B, T, H, Hkv, p = 1, 96, 2, 1, 0.2
    qkv = _qkv(B, T, H, Hkv, D)
    qkv[..., (H + Hkv) * D:] = torch.eye(T, D, device=DEV).to(torch.bfloat16)
    out, lse = A.flash_fwd(qkv, H, Hkv, D, p, seed=7)
    out2, _ = A.flash_fwd(qkv, H, Hkv, D, p, seed=7)
    assert torch.equal(out, out2)
    causal = torch.ones(T, T, device=DEV, dtype=torch.bool).tril()
    x = qkv.float().requires_grad_()
    k, v = x[0, :, H * D:(H + 1) * D], x[0, :, (H + 1) * D:]
    refs = []
    for h in range(H):
        mask = (out[0, :, h * D:h * D + T].float() != 0) & causal
        frac = mask.sum() / causal.sum()
        assert 0.7 < frac < 0.9, frac
        q = x[0, :, h * D:(h + 1) * D]
        s_ = ((q @ k.t()) / math.sqrt(D)).masked_fill(~causal, float("-inf"))
        refs.append(torch.softmax(s_, -1) * mask / (1 - p) @ v)
    ref = torch.cat(refs, dim=1)
    _close(out[0], ref, 0.02, 0.01, "dropout fwd")
    dout = torch.randn(B, T, H * D, device=DEV).to(torch.bfloat16)
    (ref * dout[0].float()).sum().backward()
    g = A.flash_bwd(dout, qkv, out, lse, H, Hkv, D, p, seed=7).float()
    for name, sl in (("dq", slice(0, H * D)), ("dk", slice(H * D, (H + Hkv) * D)), ("dv", slice((H + Hkv) * D, None))):
        rel = (g[..., sl] - x.grad[..., sl]).norm() / x.grad[..., sl].norm()
        assert rel < 0.03, f"D={D} {name} relative error {rel}"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float16])
@pytest.mark.parametrize("D", [32, 64, 128, 256, 512])
@pytest.mark.parametrize("B,H,Hkv,S,Tq", [(2, 4, 4, 300, 1), (1, 8, 2, 1024, 1), (3, 4, 4, 64, 5), (64, 12, 12, 600, 1),
                                          (2, 16, 1, 777, 1), (1, 12, 12, 1, 1)])
def test_decode_attention(dtype, D, B, H, Hkv, S, Tq):
    """Chunked decode kernel: several 256-key chunks without splits (B=64), G=16 groups, fp32
    rows (64/128-key chunks), S=1; the cache beyond S holds NaN and must never be read."""
    cap = 1100
    q = torch.randn(B, Tq, H, D, device=DEV).to(dtype)
    kc = torch.randn(B, Hkv, cap, D, device=DEV).to(dtype)
    vc = torch.randn(B, Hkv, cap, D, device=DEV).to(dtype)
    kc[:, :, S:] = float("nan")
    vc[:, :, S:] = float("nan")
    out = A.decode_attention(q, kc, vc, S)
    ref = A.reference_cache_attention(q.float(), kc[:, :, :S].float(), vc[:, :, :S].float(), S - Tq)
    _close(out, ref, 0.02, 0.01)
    if Tq == 1:  # q read in place from fused QKV rows (a size-1 dim's stride is arbitrary)
        rows = torch.randn(B, 1, (H + 2 * Hkv) * D, device=DEV).to(dtype)
        rows[:, :, :H * D] = q.reshape(B, 1, H * D)
        qv = rows[:, :, :H * D].view(B, 1, H, D)
        _close(A.decode_attention(qv, kc, vc, S), out, 0.0)


@pytest.mark.parametrize("B,H,Hkv,S,D", [(1, 12, 12, 1000, 64), (2, 8, 2, 3000, 128), (1, 4, 1, 5000, 256),
                                         (3, 4, 4, 257, 64), (16, 8, 4, 8000, 64)])
def test_decode_split_merge_in_launch_matches_combine_kernel(B, H, Hkv, S, D):
    """Split decode attention: the last split workgroup's in-launch merge (arrival counters) matches
    the fp32 reference, leaves every counter at zero, and repeated launches on the same counters
    (a replayed graph) give the same result. Where both rules pick the same split count (64 items:
    8 splits either way at 8000 keys) it is bitwise the combine kernel's output."""
    from penroz.ops import _ext
    k = _ext.kernels()
    cap = S + 64
    q = torch.randn(B, 1, H, D, device=DEV).to(torch.bfloat16)
    kc = torch.randn(B, Hkv, cap, D, device=DEV).to(torch.bfloat16)
    vc = torch.randn(B, Hkv, cap, D, device=DEV).to(torch.bfloat16)
    cnt = torch.zeros(4096, dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(D)
    merged = [k.decode_attn(q, kc, vc, None, None, S, S - 1, scale, None, None, None, cnt) for _ in range(3)]
    combined = k.decode_attn(q, kc, vc, None, None, S, S - 1, scale, None, None, None, None)
    for m in merged:
        assert torch.equal(m, merged[0])
    ref = A.reference_cache_attention(q.float(), kc[:, :, :S].float(), vc[:, :, :S].float(), S - 1)
    _close(merged[0], ref, 0.02, 0.01)
    _close(combined, ref, 0.02, 0.01)
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0
    if B * Hkv == 64:
        assert torch.equal(merged[0], combined)


def test_decode_attention_int8():
    B, H, S, D, cap = 2, 4, 200, 64, 256
    q = torch.randn(B, 1, H, D, device=DEV).to(torch.bfloat16)
    k = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16)
    v = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16)
    kq, vq = torch.empty(B, H, cap, D, dtype=torch.int8, device=DEV), torch.empty(B, H, cap, D, dtype=torch.int8, device=DEV)
    ks, vs = torch.ones(B, H, cap, device=DEV), torch.ones(B, H, cap, device=DEV)
    Sa.kv_quantize_into(k, kq, ks, 0)
    Sa.kv_quantize_into(v, vq, vs, 0)
    rq, rs = Sa.reference_quantize(k.float().transpose(1, 2))
    assert (kq[:, :, :S].int() - rq.int()).abs().max() <= 1
    _close(ks[:, :, :S], rs.squeeze(-1), 1e-6)
    out = A.decode_attention(q, kq, vq, S, ks, vs)
    ref = A.reference_cache_attention(q.float(), k.transpose(1, 2).float(), v.transpose(1, 2).float(), S - 1)
    _close(out, ref, 0.05, 0.02)


def test_sampling():
    torch.manual_seed(0)
    logits = torch.randn(8, 50304, device=DEV).to(torch.bfloat16)
    g = Sa.sample(logits, 0.0, None)
    assert torch.equal(g.view(-1), logits.float().argmax(-1))
    for _ in range(5):
        t = Sa.sample(logits, 1.0, 5)
        # by value: bf16 rows this wide have ties at the 5th largest logit
        fifth = logits.float().topk(5, dim=-1).values[:, -1:]
        assert bool((logits.float().gather(1, t) >= fifth).all())
    # distribution: a peaked 4-way row sampled many times matches its softmax
    row = torch.full((1, 64), -30.0, device=DEV)
    row[0, :4] = torch.tensor([2.0, 1.0, 0.0, -1.0], device=DEV)
    counts = torch.zeros(64)
    for _ in range(4000):
        counts[Sa.sample(row, 1.0, None).item()] += 1
    probs = torch.softmax(row[0, :4].cpu(), -1)
    assert torch.allclose(counts[:4] / 4000, probs, atol=0.03)
    # top-k + temperature: empirical frequencies follow softmax(top-k logits / T)
    row = torch.full((1, 4096), -5.0, device=DEV)
    row[0, [10, 200, 3000, 4000]] = torch.tensor([3.0, 2.5, 2.0, 1.0], device=DEV)
    counts = torch.zeros(4096)
    for _ in range(4000):
        counts[Sa.sample(row, 0.7, 3).item()] += 1
    assert counts[4000] == 0 and counts.sum() == counts[[10, 200, 3000]].sum()
    probs = torch.softmax(torch.tensor([3.0, 2.5, 2.0]) / 0.7, -1)
    assert torch.allclose(counts[[10, 200, 3000]] / 4000, probs, atol=0.03)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32, torch.float16])
@pytest.mark.parametrize("V", [50304, 50257, 24576, 96000])
def test_sampling_wide_rows(dt, V):
    """Full-vocabulary rows: register-resident kernel (V % 8 == 0, bf16 up to 64 Ki / fp32 up to
    32 Ki) and the streaming kernel (other widths, fp16) against fp32 torch references."""
    torch.manual_seed(V)
    B = 64
    logits = (torch.randn(B, V, device=DEV) * 3).to(dt)
    lf = logits.float()
    assert torch.equal(Sa.sample(logits, 0.0, None).view(-1), lf.argmax(-1))
    for k in (1, 50, 1000):  # k > 512 skips the per-thread-maxima prefilter
        top = lf.topk(k, dim=-1).values[:, -1:]
        for _ in range(3):
            t = Sa.sample(logits, 0.8, k)
            assert bool((lf.gather(1, t) >= top).all())
    # one hot row repeated: frequencies of 4 planted logits (spread over the row) follow softmax
    row = torch.full((1, V), -20.0, device=DEV)
    hot = [7, V // 3 + 1, V // 2 + 5, V - 1]
    row[0, hot] = torch.tensor([2.0, 1.5, 1.0, 0.0], device=DEV)
    rows = row.to(dt).expand(4000, V).contiguous()
    draws = Sa.sample(rows, 1.0, 3 if V % 2 else None).view(-1).cpu()
    k = 3 if V % 2 else 4
    assert bool(torch.isin(draws, torch.tensor(hot[:k])).all())
    freq = torch.stack([(draws == h).float().mean() for h in hot[:k]])
    probs = torch.softmax(torch.tensor([2.0, 1.5, 1.0, 0.0])[:k], -1)
    assert torch.allclose(freq, probs, atol=0.03), (freq, probs)


@pytest.mark.parametrize("autocast", [False, True])
@pytest.mark.parametrize("xdt,wdt", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                     (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("C", [640, 2560, 5376, 1100])
def test_rmsnorm(xdt, wdt, autocast, C):
    """HIP RMSNorm (also under bf16 autocast, as the generic engine runs it) vs the reference
    expression; widths past the register kernel (Gemma-3 4B 2560, 27B 5376) and one that is not a
    multiple of 64 take the wide backward kernel / the masked lanes."""
    x = torch.randn(100, C, device=DEV).to(xdt)
    w = torch.randn(C, device=DEV).to(wdt)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        y = Nm.rms_norm(x, w, 1e-6)
    assert y.dtype == torch.promote_types(xdt, wdt)
    _close(y, Nm.reference_rms_norm(x, w, 1e-6), 0.03, 0.01)
    xr, wr = x.detach().float().clone().requires_grad_(), w.detach().float().clone().requires_grad_()
    dy = torch.randn(100, C, device=DEV)
    Nm.reference_rms_norm(xr, wr, 1e-6).backward(dy)
    xg, wg = x.detach().clone().requires_grad_(), w.detach().clone().requires_grad_()
    Nm.rms_norm(xg, wg, 1e-6).backward(dy.to(y.dtype))
    _close(xg.grad, xr.grad, 0.05, 0.02)
    _close(wg.grad, wr.grad, 0.5, 0.02)


@pytest.mark.parametrize("H,Hkv,D,dt", [(4, 2, 64, torch.float32), (4, 1, 256, torch.bfloat16),
                                         (3, 3, 24, torch.float32), (2, 1, 128, torch.bfloat16)])
def test_rope(H, Hkv, D, dt):
    """Vectorised (D % 16 == 0) and scalar RoPE kernels vs the torch reference, fwd + bwd."""
    qkv = torch.randn(2, 33, (H + 2 * Hkv) * D, device=DEV).to(dt).float() if dt == torch.float32 else \
        torch.randn(2, 33, (H + 2 * Hkv) * D, device=DEV).to(dt)
    if dt == torch.bfloat16:
        inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=DEV).float() / D))
        out = Ro.apply_rope_qkv(qkv, H, Hkv, D, inv, 7)
        ref = Ro.reference_apply_rope_qkv(qkv.float(), H, Hkv, D, inv, 7)
        _close(out, ref, 0.02, 0.01)
        return
    inv = 1.0 / (10000 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    out = Ro.apply_rope_qkv(qkv, H, Hkv, D, inv, 7)
    ref = Ro.reference_apply_rope_qkv(qkv, H, Hkv, D, inv, 7)
    _close(out, ref, 1e-4)
    x = qkv.clone().requires_grad_()
    Ro.apply_rope_qkv(x, H, Hkv, D, inv, 7).sum().backward()
    xr = qkv.clone().requires_grad_()
    Ro.reference_apply_rope_qkv(xr, H, Hkv, D, inv, 7).sum().backward()
    _close(x.grad, xr.grad, 1e-4)


def test_tensor_stats():
    x = torch.randn(100000, device=DEV) * 2 + 1
    mean, std, mn, mx, hist, edges = Fu.tensor_stats(x, 100)
    h = torch.histogram(x.cpu(), bins=100, density=True)
    _close(mean, x.mean(), 1e-4)
    _close(std, x.std(), 1e-3)
    _close(edges.cpu(), h.bin_edges, 1e-4)
    _close(hist.cpu(), h.hist, 2e-3, 0.01)


@pytest.mark.parametrize("tile,variant", [(128, 0), (256, 4), (256, 6), (256, 8)])
@pytest.mark.parametrize("K,M,N", [(65536, 2304, 768), (4096, 768, 768), (1000, 200, 136), (8192, 50304, 768), (3000, 1600, 6400),
                                   (4096, 13816, 1144), (1000, 13824, 1152), (512, 1104, 1096)])
def test_wgrad_gemm(K, M, N, tile, variant):
    """(8192, 50304, 768), (4096, 13816, 1144), (1000, 13824, 1152): split-tail plans for the ring16o
    variants (full rounds direct, the last round's tiles split along K into per-tile slabs), with
    ragged tail tiles and a ragged K. Half tiles (<= 128 live columns or rows: the re-laid-out
    4 x 2 / 2 x 4 waves): N = 1144 / 1152 / 1096, M = 1600 / 50304 / 1104 (1104 x 1096: a corner tile
    that is half in both)."""
    from penroz.ops import gemm as G
    torch.manual_seed(0)
    dy = torch.randn(K, M, device=DEV).to(torch.bfloat16)
    x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    grad = torch.randn(M, N, device=DEV)
    ref = grad + dy.float().t() @ x.float()
    _ext.kernels().wgrad_gemm(dy, x, grad, tile, variant)
    rel = (grad - ref).norm() / ref.norm()
    assert rel < 1e-4, rel


@pytest.mark.parametrize("M,K,N", [(64, 768, 2304), (64, 768, 768), (64, 3072, 768), (64, 768, 3072), (1, 768, 50304),
                                   (17, 96, 40), (33, 768, 2304), (64, 768, 50257), (5, 4096, 1024)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_skinny_gemm(M, K, N, with_bias):
    """Decode-shaped GEMM vs fp32 torch: split-K (narrow N), masked rows/columns, repeated calls
    (the split-K arrival counters must come back to zero), strided x rows."""
    from penroz.ops import gemm as Gm
    torch.manual_seed(M + K + N)
    big = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)
    x = big[:, 32:32 + K]  # row stride K + 64, 16-B aligned
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16) if with_bias else None
    ref = x.float() @ w.float().t() + (b.float() if with_bias else 0)
    ws, cnt = Gm.skinny_workspace(x.device)
    for _ in range(3):
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        split = _ext.kernels().skinny_gemm(x, w, b, out, ws, cnt)
        _close(out, ref, 0.03, 0.01, f"split={split}")
    assert int(cnt.abs().sum()) == 0, "split-K counters must be reset by the last arriver"
    assert Gm.skinny_ok(x, w)
    _close(Gm.skinny_linear(x.reshape(1, M, K), w, b).view(M, N), ref, 0.03, 0.01, "module path")


@pytest.mark.parametrize("M,K,I", [(1, 1152, 6912), (64, 1152, 6912), (17, 768, 264), (33, 256, 1000), (5, 96, 8)])
@pytest.mark.parametrize("kind", ["gelu", "gelu_tanh", "silu"])
def test_skinny_gated(M, K, I, kind):
    """Fused gate|up projection + gated activation == the unfused pair (skinny GEMM at split 1,
    then the packed activation kernel) bit for bit, and close to fp32 torch; partial last column
    tile (I % 16 != 0), masked rows, strided x rows."""
    from penroz.ops import activations as Ac
    from penroz.ops import gemm as Gm
    torch.manual_seed(M + K + I)
    big = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)
    x = big[:, 32:32 + K]
    gu = (torch.randn(2 * I, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    ws, cnt = Gm.skinny_workspace(x.device)
    lin = torch.empty(M, 2 * I, device=DEV, dtype=torch.bfloat16)
    _ext.kernels().skinny_gemm(x, gu, None, lin, ws, cnt, 1)
    unfused = _ext.kernels().gated_act_packed(lin, Ac._GATED[kind])
    fused = Gm.skinny_gated(x, gu, Ac._GATED[kind])
    assert fused.shape == (M, I)
    assert torch.equal(fused, unfused)
    h = x.float() @ gu.float().t()
    ref = Ac.reference_gated_act(h[:, :I], h[:, I:], kind)
    _close(fused.float(), ref, 0.03, 0.02)


@pytest.mark.parametrize("M,K,H,Hkv,D", [(1, 1152, 4, 1, 256), (64, 1152, 4, 1, 256), (17, 768, 12, 12, 64),
                                         (33, 256, 8, 2, 32), (5, 96, 2, 1, 128)])
@pytest.mark.parametrize("split", [0, 1, 2])
def test_skinny_qkv_rope(M, K, H, Hkv, D, split):
    """Fused decode QKV projection + RoPE (Q and K heads rotated, V passed through) vs the unfused
    pair (skinny GEMM at the same split-K, then the RoPE kernel) and vs fp32 torch; repeated calls
    leave the split-K counters at zero."""
    from penroz.ops import gemm as Gm
    from penroz.ops import rope as Ro
    torch.manual_seed(M + K + D + split)
    N = (H + 2 * Hkv) * D
    big = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)
    x = big[:, 32:32 + K]
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=DEV, dtype=torch.float32) / D))
    cos, sin = Ro.rope_table(inv, 37, 1, DEV)
    ws, cnt = Gm.skinny_workspace(x.device)
    assert Gm.skinny_qkv_rope_ok(x, w, D)
    for _ in range(2):
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        used = _ext.kernels().skinny_qkv_rope(x, w, cos, sin, D, H + Hkv, out, ws, cnt, split)
        lin = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        _ext.kernels().skinny_gemm(x, w, None, lin, ws, cnt, used)
        unfused = _ext.kernels().rope_qkv(lin.view(M, 1, N), cos, sin, H, Hkv, D, False, None).view(M, N)
        assert torch.allclose(out.float(), unfused.float(), rtol=8e-3, atol=1e-5), (out.float() - unfused.float()).abs().max()
    assert int(cnt.abs().sum()) == 0
    ref = Ro.reference_apply_rope_qkv((x.float() @ w.float().t()).view(M, 1, N), H, Hkv, D, inv, 37).view(M, N)
    _close(out.float(), ref.float(), 0.03, 0.02)
    _close(Gm.skinny_qkv_rope(x, w, cos, sin, D, H + Hkv).float(), ref.float(), 0.03, 0.02, "python entry")


@pytest.mark.parametrize("R,C", [(768, 2304), (3072, 768), (64, 64), (50304, 768)])
def test_transpose_bf16(R, C):
    x = torch.randn(R, C, device=DEV).to(torch.bfloat16)
    out = torch.empty(C, R, device=DEV, dtype=torch.bfloat16)
    _ext.kernels().transpose_bf16(x, out)
    assert torch.equal(out, x.t())


@pytest.mark.parametrize("dtype,int8", [(torch.bfloat16, False), (torch.float32, False), (torch.float16, False),
                                        (torch.bfloat16, True)])
@pytest.mark.parametrize("D,H,Hkv,S", [(64, 12, 12, 100), (128, 8, 2, 300), (64, 4, 1, 1), (128, 4, 4, 257),
                                       (256, 8, 1, 300), (256, 4, 2, 65),  # Gemma head_dim 256
                                       (32, 4, 4, 77), (512, 8, 1, 130), (512, 16, 2, 33)])  # 32; Gemma-4 global 512
def test_decode_attention_fused_append(dtype, int8, D, H, Hkv, S):
    """Decode attention that appends this step's K/V itself (slot S-1, read from the fused QKV
    rows) == kv_append followed by decode attention: same output, same cache contents."""
    torch.manual_seed(S + D)
    B, cap = 3, 320
    rows = torch.randn(B, 1, (H + 2 * Hkv) * D, device=DEV).to(dtype)
    q = rows[:, :, :H * D].view(B, 1, H, D)
    k = rows[:, :, H * D:(H + Hkv) * D].view(B, 1, Hkv, D)
    v = rows[:, :, (H + Hkv) * D:].view(B, 1, Hkv, D)
    sl = torch.tensor([S], device=DEV)
    pos = torch.tensor([S - 1], device=DEV)
    if int8:
        kc = torch.randint(-128, 127, (B, Hkv, cap, D), device=DEV, dtype=torch.int8)
        vc = torch.randint(-128, 127, (B, Hkv, cap, D), device=DEV, dtype=torch.int8)
        ks, vs = torch.rand(B, Hkv, cap, device=DEV) * 0.02, torch.rand(B, Hkv, cap, device=DEV) * 0.02
    else:
        kc = torch.randn(B, Hkv, cap, D, device=DEV).to(dtype)
        vc = torch.randn(B, Hkv, cap, D, device=DEV).to(dtype)
        ks = vs = None
    c1 = [t.clone() if t is not None else None for t in (kc, vc, ks, vs)]
    c2 = [t.clone() if t is not None else None for t in (kc, vc, ks, vs)]
    _ext.kernels().kv_append(k, v, c1[0], c1[1], c1[2], c1[3], pos, 0)
    ref = A.decode_attention(q, c1[0], c1[1], cap, c1[2], c1[3], seq_len_dev=sl)
    out = A.decode_attention(q, c2[0], c2[1], cap, c2[2], c2[3], seq_len_dev=sl, k_new=k, v_new=v)
    for a, b in zip(c1, c2):
        if a is not None:
            assert torch.equal(a, b), "cache contents differ"
    _close(out, ref, 1e-6 if dtype != torch.float16 else 1e-3)


@pytest.mark.parametrize("B,H,Hkv,D,S", [(64, 4, 1, 256, 1), (64, 4, 1, 256, 700), (17, 4, 1, 256, 1024),
                                          (3, 8, 2, 128, 40), (2, 8, 2, 128, 300), (5, 8, 4, 64, 77)])
def test_decode_attention_rope_in_kernel(B, H, Hkv, D, S):
    """decode_attention(rope=) rotates q and the appended key itself == RoPE kernel (rope_vec,
    the eager decode path) on the QKV rows, then the fused-append decode: same cache contents,
    same output (both round the rotated values to bf16 once)."""
    from penroz.ops import rope as R
    torch.manual_seed(S + D + B)
    cap = 1024
    assert A.decode_rope_fusable(B, H, Hkv, D, cap, torch.bfloat16)
    rows = torch.randn(B, 1, (H + 2 * Hkv) * D, device=DEV).bfloat16()
    inv = 1.0 / (10000.0 ** (torch.arange(0, D, 2, device=DEV, dtype=torch.float32) / D))
    pos = torch.tensor([S - 1], device=DEV)
    cos, sin = R.rope_table(inv, 0, 1, DEV, offset_dev=pos)
    rot = R.apply_rope_qkv(rows, H, Hkv, D, inv, 0, table=(cos, sin))
    kc = torch.randn(B, Hkv, cap, D, device=DEV).bfloat16()
    vc = torch.randn(B, Hkv, cap, D, device=DEV).bfloat16()
    c1, c2 = (kc.clone(), vc.clone()), (kc.clone(), vc.clone())
    sl = torch.tensor([S], device=DEV)

    def split(r):
        return (r[:, :, :H * D].view(B, 1, H, D), r[:, :, H * D:(H + Hkv) * D].view(B, 1, Hkv, D),
                r[:, :, (H + Hkv) * D:].view(B, 1, Hkv, D))
    q1, k1, v1 = split(rot)
    ref = A.decode_attention(q1, c1[0], c1[1], cap, seq_len_dev=sl, k_new=k1, v_new=v1)
    q2, k2, v2 = split(rows)
    out = A.decode_attention(q2, c2[0], c2[1], cap, seq_len_dev=sl, k_new=k2, v_new=v2,
                             rope=(cos.view(-1), sin.view(-1)))
    torch.cuda.synchronize()
    assert torch.equal(c1[1], c2[1])
    kd = (c1[0].float() - c2[0].float()).abs()
    # the appended key: at most one bf16 ulp apart (fma contraction may differ between the kernels)
    assert kd.max().item() <= 2 ** -7 * c1[0].float().abs().max().item(), kd.max().item()
    assert torch.equal(c1[0][:, :, :S - 1], c2[0][:, :, :S - 1]) and torch.equal(c1[0][:, :, S:], c2[0][:, :, S:])
    _close(out, ref, 2e-2)


@pytest.mark.parametrize("V,dt", [(50304, torch.bfloat16), (50257, torch.bfloat16), (4096, torch.float32)])
def test_sample_step_and_advance(V, dt):
    """Graph-decode sampler: token -> idx_out[r] and out_buf[r, *step]; device-hashed uniforms
    give valid top-k draws that follow the softmax; decode_advance bumps three counters."""
    K = _ext.kernels()
    B, n = 64, 8
    torch.manual_seed(V)
    logits = (torch.randn(B, V, device=DEV) * 2).to(dt)
    seed, step = torch.tensor([1234], device=DEV), torch.tensor([3], device=DEV)
    idx = torch.zeros(B, 1, dtype=torch.long, device=DEV)
    out = torch.full((B, n), -1, dtype=torch.long, device=DEV)
    K.sample_step(logits, 0.0, 0, seed, step, idx, out)
    assert torch.equal(idx.view(-1), logits.float().argmax(-1)) and torch.equal(out[:, 3], idx.view(-1))
    assert bool((out[:, [0, 1, 2, 4, 5, 6, 7]] == -1).all())
    fifth = logits.float().topk(5, dim=-1).values[:, -1:]
    K.sample_step(logits, 1.0, 5, seed, step, idx, out)
    assert bool((logits.float().gather(1, idx) >= fifth).all()) and torch.equal(out[:, 3], idx.view(-1))
    a, b, c = (torch.tensor([x], device=DEV) for x in (5, 6, 7))
    K.decode_advance(a, b, c)
    assert (a.item(), b.item(), c.item()) == (6, 7, 8)
    # distribution over many (seed, step) pairs of one 3-way row
    row = torch.full((1, V), -30.0, device=DEV)
    row[0, :3] = torch.tensor([1.0, 0.5, 0.0], device=DEV)
    rows = row.to(dt).expand(B, V).contiguous()
    counts = torch.zeros(3)
    for s in range(40):
        seed.fill_(s * 7919)
        K.sample_step(rows, 1.0, 0, seed, step, idx, out)
        counts += torch.bincount(idx.view(-1).cpu(), minlength=3)[:3].float()
    assert torch.allclose(counts / counts.sum(), torch.softmax(torch.tensor([1.0, 0.5, 0.0]), -1), atol=0.03)


@pytest.mark.parametrize("B", [1, 3, 64])
@pytest.mark.parametrize("topk", [0, 50])
def test_sample_step_fused_advance(B, topk):
    """sample_step with the counters: same tokens as without, out_buf written at the OLD step, and
    the last row's writer bumps (pos, len, step) by one and re-arms the arrival counter, over
    repeated calls (graph replay)."""
    K = _ext.kernels()
    V, n = 50304, 6
    torch.manual_seed(B + topk)
    logits = (torch.randn(B, V, device=DEV) * 2).to(torch.bfloat16)
    seed = torch.tensor([99], device=DEV)
    temp = 0.0 if topk == 0 else 1.0
    ref_idx = torch.zeros(B, 1, dtype=torch.long, device=DEV)
    ref_out = torch.full((B, n), -1, dtype=torch.long, device=DEV)
    idx = torch.zeros_like(ref_idx)
    out = torch.full_like(ref_out, -1)
    pos, ln, step = (torch.tensor([v], device=DEV) for v in (10, 11, 0))
    done = torch.zeros(1, dtype=torch.int32, device=DEV)
    for s in range(4):
        K.sample_step(logits, temp, topk, seed, torch.tensor([s], device=DEV), ref_idx, ref_out)
        K.sample_step(logits, temp, topk, seed, step, idx, out, pos, ln, done)
        torch.cuda.synchronize()
        assert torch.equal(idx, ref_idx), s
        assert (pos.item(), ln.item(), step.item(), done.item()) == (11 + s, 12 + s, 1 + s, 0)
    assert torch.equal(out[:, :4], ref_out[:, :4]) and bool((out[:, 4:] == -1).all())


@pytest.mark.parametrize("C", [64, 1152, 2304, 5376])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("with_y", [True, False])
def test_rms_residual(C, mode, with_y):
    """Fused residual add + post norm + next norm (Gemma decode program) == the module sequence
    of torch bf16 adds and reference RMSNorms."""
    from penroz.ops import norms as Nm
    torch.manual_seed(C + mode)
    N = 5
    x, a = (torch.randn(N, C, device=DEV) * 3).to(torch.bfloat16), torch.randn(N, C, device=DEV).to(torch.bfloat16)
    w1, w2 = (1 + torch.rand(C, device=DEV)).to(torch.bfloat16), (1 + torch.rand(C, device=DEV)).to(torch.bfloat16)
    if mode == 0:
        h = Nm.reference_rms_norm(x + a, w1, 1e-6)
    elif mode == 1:
        h = x + Nm.reference_rms_norm(a, w1, 1e-6)
    else:
        h = x + a
    gh, gy = _ext.kernels().rms_residual(x, a, w1 if mode != 2 else None, w2 if with_y else None, mode, 1e-6, 1e-5)
    _close(gh.float(), h.float(), 0.02, 0.02)
    assert (gh.float() - h.float()).abs().gt(0.05 * h.float().abs() + 0.05).float().mean() < 1e-3
    if with_y:
        _close(gy.float(), Nm.reference_rms_norm(gh, w2, 1e-5).float(), 0.02, 0.02)
    else:
        assert gy is None  # an undefined tensor crosses pybind as None


@pytest.mark.parametrize("kind", ["gelu", "gelu_tanh", "silu"])
def test_gated_act_packed(kind):
    from penroz.ops import activations as Ac
    gu = torch.randn(7, 2 * 6912, device=DEV).to(torch.bfloat16)
    out = _ext.kernels().gated_act_packed(gu, Ac._GATED[kind])
    ref = Ac.reference_gated_act(gu[:, :6912].float(), gu[:, 6912:].float(), kind)
    _close(out.float(), ref, 0.02, 0.02)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_sampling_two_stage_wide_vocab(dt):
    """V = 262 144 (Gemma): the two-stage sampler (4096-logit parts, candidate merge) for greedy
    and top-k <= 64 — argmax exact, draws inside the top-k (ties included), the kept set in index
    order equals the torch reference's kept set, and planted logits in different parts are drawn
    with softmax(v / T) frequencies."""
    torch.manual_seed(1)
    B, V = 16, 262144
    logits = (torch.randn(B, V, device=DEV) * 3).to(dt)
    lf = logits.float()
    assert torch.equal(Sa.sample(logits, 0.0, None).view(-1), lf.argmax(-1))
    K = _ext.kernels()
    for k in (1, 50, 64, 100):  # 100: the one-stage streaming kernel
        top = lf.topk(k, dim=-1).values[:, -1:]
        for u in (0.0, 0.37, 0.999):
            t = K.sample_tokens(logits, torch.full((B,), u, device=DEV), 0.8, k)
            assert bool((lf.gather(1, t) >= top).all())  # k = 1 with a tied maximum: either one
    # u -> token is the inverse CDF over the kept set in index order: u = 0 draws the lowest index
    u0 = K.sample_tokens(logits, torch.zeros(B, device=DEV), 0.8, 50).view(-1)
    kept = lf >= lf.topk(50, dim=-1).values[:, -1:]
    first = torch.argmax(kept.int(), dim=-1)
    assert torch.equal(u0, first)
    row = torch.full((1, V), -20.0, device=DEV)
    hot = [7, 70000, 150001, V - 1]
    row[0, hot] = torch.tensor([2.0, 1.5, 1.0, 0.0], device=DEV)
    rows = row.to(dt).expand(2000, V).contiguous()
    draws = Sa.sample(rows, 1.0, 3).view(-1).cpu()
    assert bool(torch.isin(draws, torch.tensor(hot[:3])).all())
    freq = torch.stack([(draws == h).float().mean() for h in hot[:3]])
    probs = torch.softmax(torch.tensor([2.0, 1.5, 1.0]), -1)
    assert torch.allclose(freq, probs, atol=0.04), (freq, probs)


# ---- residual / embedding dropout (HF GPT-2 resid_pdrop / embd_pdrop in the fused executor) ----
def _mask_of(C, N, p, seed):
    """The kernels' mask/(1-p) for element (row, col), read back through add_ln_fwd with
    resid_in = 0 and delta = 1."""
    zeros = torch.zeros(N, C, device=DEV)
    ones = torch.ones(N, C, device=DEV, dtype=torch.bfloat16)
    w, b = torch.ones(C, device=DEV), torch.zeros(C, device=DEV)
    m = torch.empty(N, C, device=DEV)
    Nm.add_ln_fwd(zeros, ones, m, w, b, 1e-5, dropout_p=p, dropout_seed=seed)
    return m


@pytest.mark.parametrize("C", [768, 4100])
def test_add_layernorm_fwd_dropout(C):
    torch.manual_seed(2)
    N, p, seed = 129, 0.1, 1234
    m = _mask_of(C, N, p, seed)
    kept = (m != 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.02, kept
    assert torch.allclose(m[m != 0], torch.full_like(m[m != 0], 1 / (1 - p)))
    assert not torch.equal(m, _mask_of(C, N, p, seed + 1))  # the seed selects the mask
    x = torch.randn(N, C, device=DEV)
    d = torch.randn(N, C, device=DEV).to(torch.bfloat16)
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    out = torch.empty_like(x)
    y, _, _ = Nm.add_ln_fwd(x, d, out, w, b, 1e-5, dropout_p=p, dropout_seed=seed)
    ref = x + d.float() * m
    _close(out, ref, 1e-5)
    ry, _, _ = Nm.reference_layer_norm(ref, w, b, 1e-5)
    _close(y, ry, 0.06, 0.01)


def test_layernorm_bwd_dropout():
    """The fp32 residual gradient is unmasked; the branch gradient (bf16 copy) and the producing
    linear's bias gradient carry the forward's mask."""
    torch.manual_seed(3)
    N, C, p, seed = 512, 768, 0.1, 99
    m = _mask_of(C, N, p, seed)
    x = torch.randn(N, C, device=DEV) * 2
    w, b = torch.randn(C, device=DEV), torch.randn(C, device=DEV)
    dy = torch.randn(N, C, device=DEV).to(torch.bfloat16)
    _, mean, rstd = Nm.ln_fwd(x, w, b, 1e-5, torch.float32)
    base = torch.randn(N, C, device=DEV)
    dres = base.clone()
    dres_bf = torch.empty(N, C, device=DEV, dtype=torch.bfloat16)
    dw, db, dbp = (torch.zeros(C, device=DEV) for _ in range(3))
    Nm.ln_bwd(dy, x, mean, rstd, w, dres, True, dres_bf, dw, db, dbp, dropout_p=p, dropout_seed=seed)
    rdx, rdw, rdb = Nm.reference_layer_norm_bwd(dy, x, mean, rstd, w)
    full = base + rdx
    _close(dres, full, 2e-3, 1e-4, "dx")
    _close(dres_bf, full * m, 0.06, 0.01, "branch grad")
    _close(dbp, (full * m).sum(0), 2e-2, 1e-4, "dbias")
    _close(dw, rdw, 1e-2, 1e-4, "dw")


def test_embedding_dropout():
    V, P, C, B, T, p, seed = 1000, 64, 768, 3, 50, 0.1, 7
    wte, wpe = torch.randn(V, C, device=DEV), torch.randn(P, C, device=DEV)
    idx = torch.randint(0, V, (B, T), device=DEV)
    m = _mask_of(C, B * T, p, seed)
    out = Fu.embedding_fwd(idx, wte, wpe, 3, dropout_p=p, dropout_seed=seed)
    _close(out, Fu.reference_embedding_fwd(idx, wte, wpe, 3) * m, 1e-5)
    dout = torch.randn(B * T, C, device=DEV)
    dwte, dwpe = torch.zeros(V, C, device=DEV), torch.zeros(P, C, device=DEV)
    Fu.embedding_bwd(dout, idx, dwte, dwpe, 3, dropout_p=p, dropout_seed=seed)
    w1, w2 = wte.clone().requires_grad_(), wpe.clone().requires_grad_()
    (Fu.reference_embedding_fwd(idx, w1, w2, 3) * m * dout).sum().backward()
    _close(dwte, w1.grad, 1e-4)
    _close(dwpe, w2.grad, 1e-4)


@pytest.mark.parametrize("tile,variant", [(128, 0), (256, 4), (256, 6), (256, 8)])
@pytest.mark.parametrize("M", [50257, 1001])
def test_wgrad_gemm_padded_rows(M, tile, variant):
    """HF GPT-2 vocab (V = 50257): dlogits rows padded to a multiple of 8 (zero pad columns, as the
    CE kernel leaves them); only the first M gradient rows are touched."""
    torch.manual_seed(0)
    K, N = 2048, 768
    Mp = (M + 7) // 8 * 8
    buf = torch.zeros(K, Mp, device=DEV, dtype=torch.bfloat16)
    dy = buf[:, :M]
    dy.copy_(torch.randn(K, M, device=DEV).to(torch.bfloat16))
    x = torch.randn(K, N, device=DEV).to(torch.bfloat16)
    flat = torch.randn(M * N + 4096, device=DEV)
    grad = flat[:M * N].view(M, N)
    tail = flat[M * N:].clone()
    ref = grad + dy.float().t() @ x.float()
    _ext.kernels().wgrad_gemm(dy, x, grad, tile, variant)
    assert (grad - ref).norm() / ref.norm() < 1e-4
    assert torch.equal(flat[M * N:], tail), "wrote past the gradient's M rows"


@pytest.mark.parametrize("M,K,N", [(64, 768, 2304), (3, 128, 200), (17, 256, 1000), (33, 1024, 64)])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("with_delta", [True, False])
def test_decode_ln_linear(M, K, N, act, with_delta):
    """Fused decode kernel: out = act(LN(resid + delta + dbias)·Wᵀ + b) vs fp32 torch (+ the
    residual sum it writes)."""
    torch.manual_seed(0)
    rin = torch.randn(M, K, device=DEV)
    delta = torch.randn(M, K, device=DEV).to(torch.bfloat16) if with_delta else None
    dbias = torch.randn(K, device=DEV) if with_delta else None
    rout = torch.empty(M, K, device=DEV) if with_delta else None
    gamma, beta = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    _ext.kernels().decode_ln_linear(rin, delta, dbias, rout, gamma, beta, 1e-5, w, b, out, act)
    s = rin + (delta.float() + dbias) if with_delta else rin
    y = F.layer_norm(s, (K,), gamma, beta, 1e-5).to(torch.bfloat16).float()
    ref = y @ w.float().t() + b.float()
    if act:
        ref = F.gelu(ref.to(torch.bfloat16).float(), approximate="tanh" if act == 2 else "none")
    _close(out, ref, 2e-2, 2e-2, "out")
    if with_delta:
        _close(rout, s, 1e-6, 1e-6, "resid_out")


@pytest.mark.parametrize("M,K,N", [(1, 768, 2304), (2, 768, 3072), (4, 1024, 75), (3, 96, 50), (1, 1152, 1024)])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("with_delta", [True, False])
@pytest.mark.parametrize("rpw", [0, 2, 8])
def test_decode_gemv_ln(M, K, N, act, with_delta, rpw):
    """Decode GEMV, LN mode: out = act(LN(resid + delta + dbias)·Wᵀ + b) vs fp32 torch (+ the
    residual sum); partial last waves (N % rows-per-wave != 0) and chunk tails (K % 256 != 0)."""
    if K > 1024:
        pytest.skip("LN mode is K <= 1024")
    torch.manual_seed(0)
    rin = torch.randn(M, K, device=DEV) * 2 + 0.5
    delta = torch.randn(M, K, device=DEV).to(torch.bfloat16) if with_delta else None
    dbias = torch.randn(K, device=DEV) if with_delta else None
    rout = torch.full((M, K), 7.0, device=DEV) if with_delta else None
    gamma, beta = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    full = torch.full((M, N + 3), 5.0, device=DEV, dtype=torch.bfloat16)
    out = full[:, :N]
    _ext.kernels().decode_gemv(None, rin, delta, dbias, rout, gamma, beta, 1e-5, w, b, out, act, rpw)
    s = rin + (delta.float() + dbias) if with_delta else rin
    y = F.layer_norm(s, (K,), gamma, beta, 1e-5).to(torch.bfloat16).float()
    ref = y @ w.float().t() + b.float()
    if act:
        ref = F.gelu(ref.to(torch.bfloat16).float(), approximate="tanh" if act == 2 else "none")
    _close(out, ref, 2e-2, 2e-2, "out")
    assert torch.all(full[:, N:] == 5.0), "wrote past N"
    if with_delta:
        _close(rout, s, 1e-6, 1e-6, "resid_out")


@pytest.mark.parametrize("M,K,N", [(1, 768, 768), (1, 3072, 768), (4, 768, 50304), (2, 6912, 1152), (3, 40, 33),
                                   (1, 8192, 16)])
@pytest.mark.parametrize("rpw", [0, 2, 4, 8])
def test_decode_gemv_plain(M, K, N, rpw):
    """Decode GEMV on a bf16 x (strided rows) vs fp32 torch, with and without bias."""
    torch.manual_seed(1)
    xb = torch.randn(M, K + 16, device=DEV).to(torch.bfloat16)
    x = xb[:, :K]
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    for bias in (None, b):
        out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        _ext.kernels().decode_gemv(x, None, None, None, None, None, None, 0.0, w, bias, out, 0, rpw)
        ref = x.float() @ w.float().t() + (0 if bias is None else b.float())
        _close(out, ref, 2e-2, 2e-2, "out")


@pytest.mark.parametrize("M,K,I", [(1, 1152, 6912), (3, 64, 128), (4, 1536, 1000), (2, 1792, 33)])
@pytest.mark.parametrize("kind", [0, 1, 2])
@pytest.mark.parametrize("ppw", [0, 1, 4])
def test_decode_gemv_gated(M, K, I, kind, ppw):
    """Paired-row GEMV, gated mode: act(x·Wgᵀ) ⊙ (x·Wuᵀ) on the packed [gate; up] weight, with
    gate and up rounded to bf16 first (the unfused GEMM's output), vs fp32 torch."""
    torch.manual_seed(2)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    gu = (torch.randn(2 * I, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = torch.empty(M, I, device=DEV, dtype=torch.bfloat16)
    _ext.kernels().decode_gemv_pair(x, gu, out, 1, kind, pairs_per_wave=ppw)
    y = (x.float() @ gu.float().t()).to(torch.bfloat16).float()
    g, u = y[:, :I], y[:, I:]
    a = {0: F.gelu(g), 1: F.gelu(g, approximate="tanh"), 2: F.silu(g)}[kind]
    _close(out, a * u, 3e-2, 2e-2, "gated")


@pytest.mark.parametrize("M,K,H,Hkv,D", [(1, 1152, 4, 1, 256), (3, 64, 2, 2, 64), (4, 1536, 8, 1, 512), (2, 96, 3, 1, 32)])
@pytest.mark.parametrize("ppw", [0, 2])
def test_decode_gemv_rope(M, K, H, Hkv, D, ppw):
    """Paired-row GEMV, RoPE mode: rotate-half RoPE on the first H + Hkv heads of the QKV
    projection (V passed through), both halves rounded to bf16 before the rotation."""
    torch.manual_seed(3)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    N = (H + 2 * Hkv) * D
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    ang = torch.rand(D // 2, device=DEV) * 6.0
    cos, sin = torch.cos(ang).view(1, -1).contiguous(), torch.sin(ang).view(1, -1).contiguous()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    _ext.kernels().decode_gemv_pair(x, w, out, 2, 0, D, H + Hkv, cos, sin, ppw)
    y = (x.float() @ w.float().t()).to(torch.bfloat16).float().view(M, H + 2 * Hkv, D)
    x1, x2 = y[..., :D // 2], y[..., D // 2:]
    rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
    ref = torch.cat([rot[:, :H + Hkv], y[:, H + Hkv:]], dim=1).view(M, N)
    _close(out, ref, 3e-2, 2e-2, "rope")


@pytest.mark.parametrize("M,K,N", [(64, 768, 2304), (64, 768, 3072), (37, 1024, 320), (16, 256, 64), (9, 96, 1040)])
@pytest.mark.parametrize("act", [0, 2])
def test_decode_ln_gemm(M, K, N, act):
    """Batched decode LN-GEMM: out = act(LN(resid)·Wᵀ + b) vs fp32 torch; rows past M and the
    partial last column tile (N % 64 != 0) are never written."""
    torch.manual_seed(0)
    rin = torch.randn(M, K, device=DEV) * 3 + 1
    gamma, beta = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16)
    big = torch.full((M + 1, N + 16), 7.0, device=DEV, dtype=torch.bfloat16)
    out = big[:M, :N]  # strided rows; the guard column / row must stay untouched
    _ext.kernels().decode_ln_gemm(rin, gamma, beta, 1e-5, w, b, out, act)
    y = F.layer_norm(rin, (K,), gamma, beta, 1e-5).to(torch.bfloat16).float()
    ref = y @ w.float().t() + b.float()
    if act:
        ref = F.gelu(ref.to(torch.bfloat16).float(), approximate="tanh")
    _close(out, ref, 2e-2, 2e-2, "out")
    assert (big[M] == 7).all() and (big[:, N:] == 7).all()


@pytest.mark.parametrize("M,K,N", [(64, 768, 768), (64, 3072, 768), (23, 160, 48), (1, 32, 16), (50, 4096, 1600)])
@pytest.mark.parametrize("with_bias", [True, False])
def test_decode_gemm_acc(M, K, N, with_bias):
    """Batched decode accumulate-GEMM: resid += x·Wᵀ + b in place (fp32) vs torch; repeated calls
    accumulate (one owner per element: deterministic)."""
    torch.manual_seed(1)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV).to(torch.bfloat16) if with_bias else None
    r0 = torch.randn(M, N, device=DEV)
    r = r0.clone()
    kk = _ext.kernels()
    kk.decode_gemm_acc(x, w, b, r)
    step = x.float() @ w.float().t() + (b.float() if with_bias else 0)
    _close(r, r0 + step, 1e-3, 1e-4, "resid")
    r1 = r.clone()
    kk.decode_gemm_acc(x, w, b, r)
    kk.decode_gemm_acc(x, w, b, r1)
    assert torch.equal(r, r1), "not deterministic"
    _close(r, r0 + 2 * step, 2e-3, 1e-4, "resid x2")


@pytest.mark.parametrize("M,K,N", [(64, 1152, 1536), (64, 6912, 1152), (17, 1024, 1152), (40, 1152, 13824), (64, 1152, 4096), (50, 6912, 6912),
                                   (33, 160, 48)])
@pytest.mark.parametrize("kind", [-1, 0, 1, 2])
def test_decode_gemm_plain_and_gated(M, K, N, kind):
    """Batched decode GEMM (17-64 rows, 1 or 4 row blocks per workgroup): out = x·Wᵀ vs fp32 torch;
    gated (kind >= 0, packed [gate; up] weight [2N, K]): the same GEMM followed by gated_act_packed
    up to the last bf16 bit of a few elements (measured: ≤ 16 of 552 960 differ), and close to
    act(x·Wgᵀ)·(x·Wuᵀ) in fp32. Rows past M and the rest of a wider out stay untouched."""
    torch.manual_seed(M + N)
    kk = _ext.kernels()
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * N if kind >= 0 else N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    big = torch.full((M + 2, N + 16), 7.0, device=DEV).to(torch.bfloat16)
    out = big[:M, :N]
    kk.decode_gemm(x, w, out, kind)
    ref = x.float() @ w.float().t()
    if kind < 0:
        _close(out, ref, 1e-2, 1e-2, "plain")
    else:
        plain = torch.empty(M, 2 * N, device=DEV, dtype=torch.bfloat16)
        kk.decode_gemm(x, w, plain, -1)
        pair = kk.gated_act_packed(plain, kind)
        assert (out != pair).float().mean() < 1e-3, "gated epilogue != GEMM + gated_act_packed"
        torch.testing.assert_close(out.float(), pair.float(), rtol=1e-2, atol=1e-2)
        g, u = ref[:, :N], ref[:, N:]
        act = {0: lambda t: F.gelu(t), 1: lambda t: F.gelu(t, approximate="tanh"), 2: F.silu}[kind]
        _close(out, act(g) * u, 3e-2, 3e-2, "gated")
    assert (big[M:] == 7).all() and (big[:, N:] == 7).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_update_moments_matches_torch_std(dtype):
    """Per-epoch weight-update diagnostics: the chunked fp64 moments kernel == torch's per-tensor
    std(w - prev) and std(w) (unbiased), over sizes below, at and across the 8192-element chunk."""
    from penroz.ops import _ext
    from penroz.utils import diagnostics
    g = torch.Generator(device="cuda").manual_seed(11)
    shapes = [(3, 5), (64, 128), (8192, 1), (257, 769), (1024, 3072)]
    ws = [torch.randn(s, device="cuda", generator=g).to(dtype) for s in shapes]
    ps = [(w.float() + 1e-3 * torch.randn(w.shape, device="cuda", generator=g)).to(dtype) for w in ws]
    got = _ext.kernels().update_moments(ws, ps).cpu()
    for i, (w, p) in enumerate(zip(ws, ps)):
        ref = torch.stack([(w - p).float().std(), w.float().std()]).cpu()
        assert torch.allclose(got[i], ref, rtol=2e-3, atol=1e-7), (shapes[i], got[i], ref)
    started = diagnostics.start_update_ratios([ps[0], None, ps[2]], [ws[0], ws[1], ws[2]])
    torch.cuda.synchronize()  # the pinned copy is asynchronous: finish only after it has landed
    r = diagnostics.finish_update_ratios(started)
    old = diagnostics.weight_update_ratios([ps[0], None, ps[2]], [ws[0], ws[1], ws[2]])
    assert r[1] is None and old[1] is None
    assert abs(r[0] - old[0]) <= 2e-3 * abs(old[0]) and abs(r[2] - old[2]) <= 2e-3 * abs(old[2])
