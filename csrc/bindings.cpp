// Python bindings for the penroz CDNA4 kernels (module ``penroz_kernels``).
#include <torch/extension.h>
#include <hip/hip_runtime.h>
#include <vector>

// layernorm.hip
void layernorm_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps, torch::Tensor y, torch::Tensor mean,
                   torch::Tensor rstd);
void add_layernorm_fwd(torch::Tensor resid_in, torch::Tensor delta, torch::Tensor resid_out, torch::Tensor w,
                       torch::Tensor b, double eps, torch::Tensor y, torch::Tensor mean, torch::Tensor rstd,
                       c10::optional<torch::Tensor> delta_bias, double dropout_p, int64_t dropout_seed);
void layernorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor mean, torch::Tensor rstd, torch::Tensor w,
                   torch::Tensor dresid, bool accumulate, c10::optional<torch::Tensor> dresid_bf, torch::Tensor dw,
                   torch::Tensor db, c10::optional<torch::Tensor> dbias_prev, double dropout_p, int64_t dropout_seed);
// rmsnorm.hip
std::vector<torch::Tensor> rmsnorm_fwd(torch::Tensor x, torch::Tensor w, double eps);
std::vector<torch::Tensor> rmsnorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor rstd);
std::vector<torch::Tensor> rms_residual(torch::Tensor x, torch::Tensor a, c10::optional<torch::Tensor> w1,
                                        c10::optional<torch::Tensor> w2, int64_t mode, double eps1, double eps2);
// elementwise.hip
void gelu_fwd(torch::Tensor x, int64_t approx, torch::Tensor y);
void gelu_bwd(torch::Tensor dy, torch::Tensor x, int64_t approx, c10::optional<torch::Tensor> dbias, torch::Tensor out);
void colsum(torch::Tensor x, torch::Tensor out);
torch::Tensor gated_act_fwd(torch::Tensor g, torch::Tensor u, int64_t kind);
torch::Tensor gated_act_packed(torch::Tensor gu, int64_t kind, c10::optional<torch::Tensor> out);
std::vector<torch::Tensor> gated_act_bwd(torch::Tensor dy, torch::Tensor g, torch::Tensor u, int64_t kind);
void gated_act_bwd_packed(torch::Tensor dy, torch::Tensor gu, torch::Tensor dgu, int64_t kind);
// gemma_train.hip
void gemma_combine_fwd(int64_t mode, torch::Tensor x, c10::optional<torch::Tensor> a, c10::optional<torch::Tensor> w1,
                       torch::Tensor w2, double eps1, double eps2, c10::optional<torch::Tensor> h_out, torch::Tensor y_out,
                       c10::optional<torch::Tensor> s_save, c10::optional<torch::Tensor> r1, torch::Tensor r2);
void gemma_combine_bwd(int64_t mode, torch::Tensor dy, c10::optional<torch::Tensor> dh_in, torch::Tensor h,
                       c10::optional<torch::Tensor> s_save, c10::optional<torch::Tensor> a_save,
                       c10::optional<torch::Tensor> r1, torch::Tensor r2, c10::optional<torch::Tensor> w1,
                       torch::Tensor w2, torch::Tensor dx, c10::optional<torch::Tensor> da,
                       c10::optional<torch::Tensor> dw1, torch::Tensor dw2, c10::optional<torch::Tensor> dh_save);
void transpose_bf16(torch::Tensor in, torch::Tensor out);
void embedding_fwd(torch::Tensor idx, torch::Tensor wte, torch::Tensor wpe, int64_t off, torch::Tensor out,
                   c10::optional<torch::Tensor> off_dev, double dropout_p, int64_t dropout_seed);
void embedding_bwd(torch::Tensor dout, torch::Tensor idx, torch::Tensor dwte, torch::Tensor dwpe, int64_t off,
                   double dropout_p, int64_t dropout_seed);
torch::Tensor rope_qkv(torch::Tensor qkv, torch::Tensor cosv, torch::Tensor sinv, int64_t H, int64_t Hkv, int64_t D,
                       bool inverse, c10::optional<torch::Tensor> out);
void kv_quantize(torch::Tensor x, torch::Tensor q, torch::Tensor scale, int64_t pos);
std::vector<torch::Tensor> tensor_stats(torch::Tensor x, int64_t bins);
// cross_entropy.hip
torch::Tensor cross_entropy_fwd_bwd(torch::Tensor logits, torch::Tensor targets, double scale, int64_t ignore_index,
                                    c10::optional<torch::Tensor> grad_out);
// adamw.hip
void adamw_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
                double lr, double b1, double b2, double eps, double wd, int64_t step, double grad_scale, bool maximize);
void adam_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
               double lr, double b1, double b2, double eps, double wd, int64_t step, double grad_scale, bool maximize);
void multi_tensor_adam(std::vector<torch::Tensor> ps, std::vector<torch::Tensor> gs, std::vector<torch::Tensor> ms,
                       std::vector<torch::Tensor> vs, double lr, double b1, double b2, double eps, double wd,
                       int64_t step, double grad_scale, bool maximize, bool decoupled);
void adam_rows_step(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> shadow,
                    int64_t C, torch::Tensor mask, c10::optional<torch::Tensor> rows, int64_t mode, double lr, double b1,
                    double b2, double eps, double wd, int64_t step, double grad_scale, bool maximize, bool decoupled);
// sampling.hip
torch::Tensor sample_tokens(torch::Tensor logits, c10::optional<torch::Tensor> uniform, double temperature,
                            int64_t top_k);
void sample_step(torch::Tensor logits, double temperature, int64_t top_k, torch::Tensor seed, torch::Tensor step,
                 torch::Tensor idx_out, torch::Tensor out_buf, c10::optional<torch::Tensor> adv_a,
                 c10::optional<torch::Tensor> adv_b, c10::optional<torch::Tensor> done);
void decode_advance(torch::Tensor a, torch::Tensor b, torch::Tensor c);
// decode_attn.hip
torch::Tensor decode_attn(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, c10::optional<torch::Tensor> k_scale,
                          c10::optional<torch::Tensor> v_scale, int64_t S, int64_t q_offset, double scale,
                          c10::optional<torch::Tensor> seq_len_dev,
                          c10::optional<torch::Tensor> k_new, c10::optional<torch::Tensor> v_new,
                          c10::optional<torch::Tensor> counters, c10::optional<torch::Tensor> rope_cos,
                          c10::optional<torch::Tensor> rope_sin);
bool decode_small_applies(int64_t B, int64_t Tq, int64_t H, int64_t Hkv, int64_t D, int64_t S);
// elementwise.hip (deferred.h)
void set_deferred_reduce_stream(int64_t stream, int64_t device);
// decode_attn.hip
void kv_append(torch::Tensor k, torch::Tensor v, torch::Tensor kc, torch::Tensor vc, c10::optional<torch::Tensor> ks,
               c10::optional<torch::Tensor> vs, c10::optional<torch::Tensor> pos_dev, int64_t pos);
// skinny_gemm.hip
int64_t skinny_gemm(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor out,
                    torch::Tensor ws, torch::Tensor cnt, int64_t splitk);
void skinny_gated(torch::Tensor x, torch::Tensor gu, torch::Tensor out, int64_t kind);
std::vector<int64_t> skinny_qkv_rope_plan(int64_t M, int64_t N, int64_t K);
std::vector<int64_t> attn_work_plan(int64_t nblk, int64_t nvh, int64_t slots, int64_t BM, int64_t BN, int64_t T,
                                    int64_t D, double tile_us);
int64_t skinny_qkv_rope(torch::Tensor x, torch::Tensor w, torch::Tensor cosv, torch::Tensor sinv, int64_t D,
                        int64_t nrot, torch::Tensor out, torch::Tensor ws, torch::Tensor cnt, int64_t splitk);
void decode_ln_linear(torch::Tensor rin, c10::optional<torch::Tensor> delta, c10::optional<torch::Tensor> dbias,
                      c10::optional<torch::Tensor> rout, torch::Tensor gamma, torch::Tensor beta, double eps,
                      torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor out, int64_t act);
// decode_linear.hip
void decode_ln_gemm(torch::Tensor resid, torch::Tensor gamma, torch::Tensor beta, double eps, torch::Tensor w,
                    c10::optional<torch::Tensor> bias, torch::Tensor out, int64_t act, int64_t flags);
void decode_gemv(c10::optional<torch::Tensor> x, c10::optional<torch::Tensor> rin, c10::optional<torch::Tensor> delta,
                 c10::optional<torch::Tensor> dbias, c10::optional<torch::Tensor> rout,
                 c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta, double eps, torch::Tensor w,
                 c10::optional<torch::Tensor> bias, torch::Tensor out, int64_t act, int64_t rows_per_wave,
                 c10::optional<torch::Tensor> emb_idx, c10::optional<torch::Tensor> emb_wte,
                 c10::optional<torch::Tensor> emb_wpe, c10::optional<torch::Tensor> emb_pos);
void decode_gemv_pair(torch::Tensor x, torch::Tensor w, torch::Tensor out, int64_t mode, int64_t kind, int64_t D,
                      int64_t nrot, c10::optional<torch::Tensor> cosv, c10::optional<torch::Tensor> sinv,
                      int64_t pairs_per_wave);
void decode_gemm_acc(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, torch::Tensor resid,
                     int64_t flags);
void decode_gemm(torch::Tensor x, torch::Tensor w, torch::Tensor out, int64_t kind);
torch::Tensor update_moments(std::vector<torch::Tensor> ws, std::vector<torch::Tensor> ps);
// gemm_nt.hip
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K);
void gemm_nt(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias, torch::Tensor out,
             c10::optional<torch::Tensor> act, int64_t approx, int64_t group_m, int64_t grid, int64_t ablate);
// gemm_wgrad.hip
void wgrad_gemm(torch::Tensor dy, torch::Tensor x, torch::Tensor grad, int64_t tile, int64_t variant, bool accumulate);
// flash_attn.hip
void flash_attn_fwd(torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, int64_t H, int64_t Hkv, int64_t D,
                    double scale, double p_drop, int64_t seed);
int64_t flash_fwd_variant(int64_t v);
void flash_bwd_stamps(c10::optional<torch::Tensor> buf);
void flash_attn_bwd(torch::Tensor dout, torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, torch::Tensor dqkv,
                    int64_t H, int64_t Hkv, int64_t D, double scale, double p_drop, int64_t seed,
                    c10::optional<torch::Tensor> dbias);
// flash_attn_gen.hip (head_dim 128 / 256)
void flash_attn_gen_fwd(torch::Tensor qkv, torch::Tensor out, torch::Tensor lse, int64_t H, int64_t Hkv, int64_t D,
                        double scale, double p_drop, int64_t seed);
void flash_attn_gen_bwd(torch::Tensor dout, torch::Tensor qkv, torch::Tensor out, torch::Tensor lse,
                        torch::Tensor dqkv, int64_t H, int64_t Hkv, int64_t D, double scale, double p_drop,
                        int64_t seed);

// A stream whose kernels may only run on the CUs set in `mask` (32-bit words, CU i = bit i % 32
// of word i / 32): the executor's side stream can be confined to a CU subset so the critical-path
// GEMMs keep the rest (A/B switch PENROZ_SIDE_CUS). Returned as the raw hipStream_t for
// torch.cuda.ExternalStream; the stream lives for the process.
static int64_t cu_masked_stream(int64_t device, std::vector<int64_t> mask) {
  std::vector<uint32_t> m(mask.begin(), mask.end());
  int prev = 0;
  TORCH_CHECK(hipGetDevice(&prev) == hipSuccess, "hipGetDevice failed");
  TORCH_CHECK(hipSetDevice((int)device) == hipSuccess, "hipSetDevice failed");
  hipStream_t st = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data());
  (void)hipSetDevice(prev);
  TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(st);
}

static int64_t cu_count(int64_t device) {
  int n = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, (int)device) == hipSuccess,
              "hipDeviceGetAttribute failed");
  return n;
}

PYBIND11_MODULE(penroz_kernels, m) {
  m.doc() = "penroz hand-written HIP kernels for MI355X (gfx950)";
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("add_layernorm_fwd", &add_layernorm_fwd, pybind11::arg("resid_in"), pybind11::arg("delta"),
        pybind11::arg("resid_out"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("eps"), pybind11::arg("y"),
        pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("delta_bias") = pybind11::none(),
        pybind11::arg("dropout_p") = 0.0, pybind11::arg("dropout_seed") = 0);
  m.def("layernorm_bwd", &layernorm_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("mean"),
        pybind11::arg("rstd"), pybind11::arg("w"), pybind11::arg("dresid"), pybind11::arg("accumulate"),
        pybind11::arg("dresid_bf"), pybind11::arg("dw"), pybind11::arg("db"), pybind11::arg("dbias_prev"),
        pybind11::arg("dropout_p") = 0.0, pybind11::arg("dropout_seed") = 0);
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("rmsnorm_bwd", &rmsnorm_bwd);
  m.def("rms_residual", &rms_residual);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("colsum", &colsum);
  m.def("gated_act_fwd", &gated_act_fwd);
  m.def("gated_act_packed", &gated_act_packed, pybind11::arg("gu"), pybind11::arg("kind"),
        pybind11::arg("out") = pybind11::none());
  m.def("gated_act_bwd", &gated_act_bwd);
  m.def("gated_act_bwd_packed", &gated_act_bwd_packed, "dgu [N, 2I] from dy [N, I] and the packed gu [N, 2I]");
  m.def("gemma_combine_fwd", &gemma_combine_fwd, pybind11::arg("mode"), pybind11::arg("x"), pybind11::arg("a"),
        pybind11::arg("w1"), pybind11::arg("w2"), pybind11::arg("eps1"), pybind11::arg("eps2"), pybind11::arg("h_out"),
        pybind11::arg("y_out"), pybind11::arg("s_save"), pybind11::arg("r1"), pybind11::arg("r2"),
        "Gemma residual combine + post-norm + next RMSNorm (modes 0: Gemma3+, 1: Gemma2, 2: Gemma1, 3: norm only)");
  m.def("gemma_combine_bwd", &gemma_combine_bwd, pybind11::arg("mode"), pybind11::arg("dy"), pybind11::arg("dh_in"),
        pybind11::arg("h"), pybind11::arg("s_save"), pybind11::arg("a_save"), pybind11::arg("r1"), pybind11::arg("r2"),
        pybind11::arg("w1"), pybind11::arg("w2"), pybind11::arg("dx"), pybind11::arg("da"), pybind11::arg("dw1"),
        pybind11::arg("dw2"), pybind11::arg("dh_save") = pybind11::none(),
        "backward of gemma_combine_fwd (dw1 / dw2 accumulated; dh_save: dL/dh for diagnostics)");
  m.def("transpose_bf16", &transpose_bf16, "out [C, R] = in [R, C]^T (bf16, dims % 64 == 0)");
  m.def("embedding_fwd", &embedding_fwd, pybind11::arg("idx"), pybind11::arg("wte"), pybind11::arg("wpe"),
        pybind11::arg("off"), pybind11::arg("out"), pybind11::arg("off_dev") = pybind11::none(),
        pybind11::arg("dropout_p") = 0.0, pybind11::arg("dropout_seed") = 0);
  m.def("embedding_bwd", &embedding_bwd, pybind11::arg("dout"), pybind11::arg("idx"), pybind11::arg("dwte"),
        pybind11::arg("dwpe"), pybind11::arg("off"), pybind11::arg("dropout_p") = 0.0,
        pybind11::arg("dropout_seed") = 0);
  m.def("rope_qkv", &rope_qkv, pybind11::arg("qkv"), pybind11::arg("cosv"), pybind11::arg("sinv"), pybind11::arg("H"),
        pybind11::arg("Hkv"), pybind11::arg("D"), pybind11::arg("inverse"), pybind11::arg("out") = pybind11::none());
  m.def("kv_quantize", &kv_quantize);
  m.def("tensor_stats", &tensor_stats);
  m.def("cross_entropy_fwd_bwd", &cross_entropy_fwd_bwd, pybind11::arg("logits"), pybind11::arg("targets"),
        pybind11::arg("scale"), pybind11::arg("ignore_index"), pybind11::arg("grad_out") = pybind11::none());
  m.def("adamw_step", &adamw_step);
  m.def("adam_step", &adam_step);
  m.def("adam_rows_step", &adam_rows_step, "row-split Adam/AdamW step of an embedding table (mode 0: untouched rows, 1: touched rows)");
  m.def("multi_tensor_adam", &multi_tensor_adam);
  m.def("sample_tokens", &sample_tokens);
  m.def("sample_step", &sample_step, "decode-step sampler: device-hashed uniforms, writes idx_out and out_buf[:, *step]; "
        "with adv_a / adv_b / done the last row's writer also advances the counters",
        pybind11::arg("logits"), pybind11::arg("temperature"), pybind11::arg("top_k"), pybind11::arg("seed"),
        pybind11::arg("step"), pybind11::arg("idx_out"), pybind11::arg("out_buf"), pybind11::arg("adv_a") = pybind11::none(),
        pybind11::arg("adv_b") = pybind11::none(), pybind11::arg("done") = pybind11::none());
  m.def("decode_advance", &decode_advance, "+1 on three device int64 scalars");
  m.def("decode_attn", &decode_attn, pybind11::arg("q"), pybind11::arg("kc"), pybind11::arg("vc"), pybind11::arg("k_scale"),
        pybind11::arg("v_scale"), pybind11::arg("S"), pybind11::arg("q_offset"), pybind11::arg("scale"),
        pybind11::arg("seq_len_dev") = pybind11::none(), pybind11::arg("k_new") = pybind11::none(),
        pybind11::arg("v_new") = pybind11::none(), pybind11::arg("counters") = pybind11::none(),
        pybind11::arg("rope_cos") = pybind11::none(), pybind11::arg("rope_sin") = pybind11::none());
  m.def("decode_small_applies", &decode_small_applies, "decode_attn takes the one-workgroup-per-item kernel");
  m.def("set_deferred_reduce_stream", &set_deferred_reduce_stream);
  m.def("kv_append", &kv_append, pybind11::arg("k"), pybind11::arg("v"), pybind11::arg("kc"), pybind11::arg("vc"),
        pybind11::arg("ks") = pybind11::none(), pybind11::arg("vs") = pybind11::none(),
        pybind11::arg("pos_dev") = pybind11::none(), pybind11::arg("pos") = 0);
  m.def("skinny_gemm", &skinny_gemm, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bias"),
        pybind11::arg("out"), pybind11::arg("ws"), pybind11::arg("cnt"), pybind11::arg("splitk") = 0,
        "decode-shaped out[M<=64, N] = x·wᵀ (+bias), bf16; returns the split-K factor used");
  m.def("skinny_gated", &skinny_gated, pybind11::arg("x"), pybind11::arg("gu"), pybind11::arg("out"),
        pybind11::arg("kind"),
        "decode gated MLP projection: out[M<=64, I] = act(x·gu[:I]ᵀ)·(x·gu[I:]ᵀ), bf16, one launch");
  m.def("attn_work_plan", &attn_work_plan, pybind11::arg("nblk"), pybind11::arg("nvh"), pybind11::arg("slots"),
        pybind11::arg("BM"), pybind11::arg("BN"), pybind11::arg("T"), pybind11::arg("D"), pybind11::arg("tile_us"),
        "causal attention work list (flash_attn_gen.hip attn_plan): [items, split0, block | part << 16 ...]");
  m.def("skinny_qkv_rope_plan", &skinny_qkv_rope_plan, pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"),
        "(split-K, fp32 workspace floats, counters) skinny_qkv_rope uses at this shape (host only)");
  m.def("skinny_qkv_rope", &skinny_qkv_rope, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("cos"),
        pybind11::arg("sin"), pybind11::arg("D"), pybind11::arg("nrot"), pybind11::arg("out"), pybind11::arg("ws"),
        pybind11::arg("cnt"), pybind11::arg("splitk") = 0,
        "decode QKV projection with RoPE on the first nrot heads in the epilogue, M <= 64; returns the split");
  m.def("decode_ln_linear", &decode_ln_linear, pybind11::arg("resid_in"), pybind11::arg("delta"),
        pybind11::arg("dbias"), pybind11::arg("resid_out"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("eps"), pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("out"), pybind11::arg("act") = 0,
        "decode step: out = act(LN(resid_in + delta + dbias)·wᵀ + bias) for M <= 64 rows, K <= 1024; "
        "resid_out receives the residual sum");
  m.def("decode_ln_gemm", &decode_ln_gemm, pybind11::arg("resid"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("eps"), pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("out"), pybind11::arg("act") = 0,
        pybind11::arg("flags") = 0, "batched decode: out = act(LayerNorm(resid)·wᵀ + bias), fp32 resid [M, K <= 1024]");
  m.def("decode_gemv", &decode_gemv, pybind11::arg("x"), pybind11::arg("resid_in"), pybind11::arg("delta"),
        pybind11::arg("dbias"), pybind11::arg("resid_out"), pybind11::arg("gamma"), pybind11::arg("beta"),
        pybind11::arg("eps"), pybind11::arg("w"), pybind11::arg("bias"), pybind11::arg("out"), pybind11::arg("act") = 0,
        pybind11::arg("rows_per_wave") = 0, pybind11::arg("emb_idx") = pybind11::none(),
        pybind11::arg("emb_wte") = pybind11::none(), pybind11::arg("emb_wpe") = pybind11::none(),
        pybind11::arg("emb_pos") = pybind11::none(),
        "decode GEMV for 1..4 rows: act(x · Wᵀ + bias), or act(LN(resid_in + delta + dbias) · Wᵀ + bias), or "
        "act(LN(wte[idx] + wpe[pos]) · Wᵀ + bias) with the embedding rows written to resid_out");
  m.def("decode_gemv_pair", &decode_gemv_pair, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("out"),
        pybind11::arg("mode"), pybind11::arg("kind") = 0, pybind11::arg("D") = 0, pybind11::arg("nrot") = 0,
        pybind11::arg("cos") = pybind11::none(), pybind11::arg("sin") = pybind11::none(),
        pybind11::arg("pairs_per_wave") = 0,
        "paired-row decode GEMV for 1..4 rows: gated MLP (mode 1) or RoPE QKV (mode 2) epilogue");
  m.def("decode_gemm_acc", &decode_gemm_acc, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("bias"),
        pybind11::arg("resid"), pybind11::arg("flags") = 0,
        "batched decode: resid += x·wᵀ + bias (fp32 residual, in place)");
  m.def("decode_gemm", &decode_gemm, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("out"),
        pybind11::arg("kind") = -1,
        "batched decode (16-64 rows): out = x·wᵀ, or the gated MLP act(x·Wgᵀ)·(x·Wuᵀ) of a packed [gate; up] weight");
  m.def("update_moments", &update_moments, "per-epoch weight-update diagnostics: [n, 2] (std(w - prev), std(w))");
  m.def("gemm_nt_supported", &gemm_nt_supported, "shapes the native NT GEMM takes (M % 256, N % 128, K % 32, K >= 160)");
  m.def("gemm_nt", &gemm_nt, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("bias"), pybind11::arg("out"),
        pybind11::arg("act") = pybind11::none(), pybind11::arg("approx") = 0, pybind11::arg("group_m") = 0,
        pybind11::arg("grid") = 0, pybind11::arg("ablate") = 0,
        "out = a·bᵀ (+ bias) (bf16, both operands reduction-contiguous); with act: act = GELU(out)");
  m.def("wgrad_gemm", &wgrad_gemm, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("grad"),
        pybind11::arg("tile") = 256, pybind11::arg("variant") = 8, pybind11::arg("accumulate") = true,
        "grad (+)= dyᵀ·x (fp32 gradient, bf16 operands); accumulate=False overwrites grad");
  m.def("flash_attn_fwd", &flash_attn_fwd);
  m.def("flash_fwd_variant", &flash_fwd_variant, pybind11::arg("variant") = 0,
        "select the forward kernel (1 single-stage, 2 tile-pipelined); returns the previous one");
  m.def("flash_attn_bwd", &flash_attn_bwd, pybind11::arg("dout"), pybind11::arg("qkv"), pybind11::arg("out"),
        pybind11::arg("lse"), pybind11::arg("dqkv"), pybind11::arg("H"), pybind11::arg("Hkv"), pybind11::arg("D"),
        pybind11::arg("scale"), pybind11::arg("p_drop"), pybind11::arg("seed"), pybind11::arg("dbias") = pybind11::none(),
        "causal flash-attention backward (head_dim 64) into dqkv; dbias += column sums of dqkv when given");
  m.def("cu_masked_stream", &cu_masked_stream, "stream restricted to a CU mask (raw hipStream_t)");
  m.def("cu_count", &cu_count, "compute units of a device");
  m.def("flash_bwd_stamps", &flash_bwd_stamps, pybind11::arg("buf") = pybind11::none(),
        "diagnostic: s_memtime phase sums of the dK/dV kernel into an int64 [6] GPU tensor (None: off)");
  m.def("flash_attn_gen_fwd", &flash_attn_gen_fwd, "causal flash attention forward, head_dim 128 / 256");
  m.def("flash_attn_gen_bwd", &flash_attn_gen_bwd, "causal flash attention backward, head_dim 128 / 256");
}
