// Python binding of the gfx950 kernels: adapts at::Tensor arguments to the extern "C" launchers in
// csrc/kernels/*.hip and launches them on torch's current HIP stream (so they order with hipBLASLt
// GEMMs and RCCL work issued by torch, and are captured by torch.cuda.graphs).
//
// Every entry point validates device, dtype, contiguity and the shape assumptions of its kernel on
// the host before launching -- a wrong shape must be a Python exception, never a GPU fault.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int ftc_rmsnorm_fwd(const void* x, const void* res, const void* w, void* h_out, void* y, float* rstd, int rows, int d,
                    float eps, long long y_rs, hipStream_t stream);
int ftc_rmsnorm_bwd_grid(int rows);
int ftc_rmsnorm_bwd(const void* dy, const void* h, const void* w, const float* rstd, const void* dres, void* dx,
                    float* dw_part, float* dw, int rows, int d, long long dres_rs, long long dx_rs,
                    hipStream_t stream);
int ftc_rope(void* qkv, const float* cosT, const float* sinT, const int* positions, long long rows, int ld,
             int n_rot_heads, int head_dim, int seq_len, int inverse, int max_pos, hipStream_t stream);
int ftc_swiglu_fwd(const void* gu, void* a, long long rows, int F, long long a_rs, hipStream_t stream);
int ftc_swiglu_bwd(const void* da, const void* gu, void* dgu, long long rows, int F, long long dgu_rs,
                   hipStream_t stream);
int ftc_swiglu_fwd_lora(const void* gu, void* h, long long rows, int F, long long h_rs, const void* Am, long long lda,
                        int nct, int Rp, hipStream_t stream);
int ftc_swiglu_bwd_lora(const void* da, long long da_rs, const void* gu, void* dgu, long long rows, int F,
                        long long dgu_rs, const void* Bt, long long ldb, int nct, int split, int Rp,
                        hipStream_t stream);
int ftc_swiglu_wgrad_plan(long long T, int F, int* rb, long long* ws_floats);
int ftc_swiglu_bwd_wgrad(const void* da, long long da_rs, const void* gu, void* dgu, long long dgu_rs, long long T,
                         int F, const void* bt, long long ldb, const void* xa, long long xa_rs, const void* dyb,
                         long long dyb_rs, float* ws, void* mgB, long long ldB, float alphaB, void* mgA, long long ldA,
                         float alphaA, int Rp, hipStream_t stream);
int ftc_tail_gemm(void* x, long long ldx, long long rows, int K, const void* Bm, long long ldb, int nct, int Rp,
                  hipStream_t stream);
int ftc_transpose(const void* x, long long ldx, void* y, long long ldy, int R, int C, hipStream_t stream);
int ftc_copy2d_batched(const void* jobs, int njobs, long long max_elems, hipStream_t stream);
int ftc_splitk_sum(const float* parts, int nsplit, long long pstride, void* c, int c_fp32, long long rows, int cols,
                   long long ldc, float beta, hipStream_t stream);
int ftc_ce_fwd_bwd(void* logits, const long long* labels, float* loss, float* lse, long long rows, int V, long long ld,
                   float gscale, long long ignore_index, hipStream_t stream);
int ftc_adamw(void* param_bf16, float* master, float* m, float* v, const void* grad, int grad_is_fp32, long long n,
              float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, const float* gscale,
              const float* hpdev, hipStream_t stream);
int ftc_sumsq_partials();
int ftc_sumsq(const void* x, int is_fp32, long long n, float* partial, float* out, float* coef, float max_norm,
              float scale, hipStream_t stream);
int ftc_flash_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int H, int KV, int D,
                  long long q_row_stride, long long kv_row_stride, long long o_row_stride, float scale, int causal,
                  int window, const int* doc_start, int kv_valid, hipStream_t stream);
int ftc_flash_bwd_workspace(int B, int S, int H, int D, long long* bytes);
long long ftc_decode_workspace_floats(int B, int H, int KV, int D, int max_len);
int ftc_decode_attention(const void* q, void* kc, void* vc, const void* knew, const void* vnew, long long new_rs,
                         const int* lens, void* out, float* workspace, int B, int H, int KV, int D, int max_len,
                         long long q_rs, long long kv_rs, long long b_rs, long long o_rs, float scale, int window,
                         hipStream_t stream);
int ftc_flash_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout, const float* lse,
                  void* dq, void* dk, void* dv, void* workspace, int B, int S, int H, int KV, int D,
                  long long q_row_stride, long long kv_row_stride, long long o_row_stride, long long do_row_stride,
                  long long dq_row_stride,
                  long long dkv_row_stride, float scale, int causal, int window, const int* doc_start,
                  const int* doc_end, int kv_valid, const float* rope_cos, const float* rope_sin,
                  const int* rope_pos, hipStream_t stream);
int ftc_nf4_dequant(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale, float absmax_offset,
                    void* out, long long n, int block, int block2, hipStream_t stream);
int ftc_nf4_quant(const void* w, uint8_t* packed, float* absmax, long long n, int block, hipStream_t stream);
int ftc_nf4_dequant_aug(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale, float absmax_offset,
                        void* out, int rows, int cols, long long ldo, int block, int block2, int transpose, const void* B,
                        long long ldb, void* out_b, long long ldob, const void* A, long long lda, void* out_a,
                        long long ldoa, float s, int R, hipStream_t stream);
int ftc_nf4_dequant_into(const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                         float absmax_offset, void* out, int rows, int cols, long long ldo, int block, int block2,
                         int transpose, hipStream_t stream);
int ftc_nf4_gemm(const void* x, const uint8_t* packed, const uint8_t* absmax_q, const float* absmax_scale,
                 float absmax_offset, void* y, int M, int N, int K, int block, int block2, hipStream_t stream);
int ftc_lora_merge(void* w, const void* a, const void* b, int out_f, int in_f, int r, int seg_rows, float scale,
                   hipStream_t stream);
int ftc_lora_wgrad_splits(int T, int M);
int ftc_lora_wgrad(const void* x, long long ldx, const void* y, long long ldy, float* ws, int T, int M, int R,
                   void* out, long long out_sm, long long out_sr, float alpha, float beta, int nseg, const int* m_end,
                   const int* ycol, const int* ocol, hipStream_t stream);
}

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline void check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed with code ", rc, (rc > 0 ? std::string(": ") + hipGetErrorString((hipError_t)rc) : std::string(" (shape/argument rejected)")));
}

inline void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

inline void need_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1 && t.stride(0) == t.size(1), name, " must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

// ---------------- RMSNorm ----------------
// pad > 0: y is returned as the [rows, d] column view of a [rows, d + pad] buffer (LoRA "augmented" GEMM input)
std::vector<at::Tensor> rmsnorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& res, const at::Tensor& w,
                                    double eps, int64_t pad) {
  need(x, at::kBFloat16, "x");
  need(w, at::kBFloat16, "w");
  need_rows(x, "x");
  const int rows = (int)x.size(0), d = (int)x.size(1);
  TORCH_CHECK(w.numel() == d && w.is_contiguous(), "w must be [d] contiguous");
  TORCH_CHECK(d % 8 == 0 && d <= 8192, "rmsnorm: d must be a multiple of 8 and <= 8192");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0, "rmsnorm: pad must be a multiple of 8");
  auto ybuf = at::empty({rows, d + pad}, x.options());
  auto y = pad ? ybuf.narrow(1, 0, d) : ybuf;
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  at::Tensor h;
  const void* rp = nullptr;
  if (res.has_value()) {
    need(*res, at::kBFloat16, "res");
    need_rows(*res, "res");
    TORCH_CHECK(res->sizes() == x.sizes(), "res shape mismatch");
    h = at::empty_like(x);
    rp = res->data_ptr();
  } else {
    h = x;
  }
  check(ftc_rmsnorm_fwd(x.data_ptr(), rp, w.data_ptr(), rp ? h.data_ptr() : nullptr, y.data_ptr(),
                        rstd.data_ptr<float>(), rows, d, (float)eps, (long long)(d + pad), cur_stream()),
        "rmsnorm_fwd");
  return {y, rstd, h};
}

// dres may be a row-padded view; pad > 0 returns dx as the [rows, d] view of a [rows, d + pad] buffer
std::vector<at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& h, const at::Tensor& w,
                                    const at::Tensor& rstd, const c10::optional<at::Tensor>& dres, bool need_dw,
                                    int64_t pad) {
  need(dy, at::kBFloat16, "dy");
  need(h, at::kBFloat16, "h");
  need(w, at::kBFloat16, "w");
  need(rstd, at::kFloat, "rstd");
  need_rows(dy, "dy");
  need_rows(h, "h");
  TORCH_CHECK(dy.sizes() == h.sizes(), "dy/h shape mismatch");
  const int rows = (int)h.size(0), d = (int)h.size(1);
  TORCH_CHECK(rstd.numel() == rows && w.numel() == d, "rstd/w shape mismatch");
  TORCH_CHECK(d % 8 == 0 && d <= 8192, "rmsnorm: bad d");
  const void* drp = nullptr;
  if (dres.has_value()) {
    need(*dres, at::kBFloat16, "dres");
    TORCH_CHECK(dres->dim() == 2 && dres->stride(1) == 1 && dres->stride(0) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(dres->data_ptr()) % 16 == 0,
                "dres must be a 16-byte aligned row view");
    TORCH_CHECK(dres->sizes() == h.sizes(), "dres shape mismatch");
    drp = dres->data_ptr();
  }
  TORCH_CHECK(pad >= 0 && pad % 8 == 0, "rmsnorm_bwd: pad must be a multiple of 8");
  auto dxbuf = at::empty({rows, d + pad}, h.options());
  auto dx = pad ? dxbuf.narrow(1, 0, d) : dxbuf;
  at::Tensor dw, part;
  if (need_dw) {
    const int g = ftc_rmsnorm_bwd_grid(rows);
    part = at::empty({g, d}, h.options().dtype(at::kFloat));
    dw = at::empty({d}, h.options().dtype(at::kFloat));
  }
  check(ftc_rmsnorm_bwd(dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(), drp, dx.data_ptr(),
                        need_dw ? part.data_ptr<float>() : nullptr, need_dw ? dw.data_ptr<float>() : nullptr, rows, d,
                        drp ? dres->stride(0) : d, d + pad, cur_stream()),
        "rmsnorm_bwd");
  if (need_dw) return {dx, dw};
  return {dx};
}

// ---------------- RoPE (in place) ----------------
void rope_(at::Tensor& qkv, const at::Tensor& cos, const at::Tensor& sin, const c10::optional<at::Tensor>& positions,
           int64_t n_rot_heads, int64_t head_dim, int64_t seq_len, bool inverse) {
  need(qkv, at::kBFloat16, "qkv");
  need(cos, at::kFloat, "cos");
  need(sin, at::kFloat, "sin");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be 2-D with unit column stride");
  TORCH_CHECK(head_dim % 16 == 0, "rope: head_dim must be a multiple of 16");
  TORCH_CHECK(qkv.size(1) >= n_rot_heads * head_dim, "rope: qkv too narrow");
  TORCH_CHECK(qkv.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0, "rope: alignment");
  TORCH_CHECK(cos.is_contiguous() && sin.is_contiguous() && cos.size(1) == head_dim / 2, "rope: tables [P, D/2]");
  const int* pp = nullptr;
  const long long rows = qkv.size(0);
  if (positions.has_value()) {
    need(*positions, at::kInt, "positions");
    TORCH_CHECK(positions->numel() == rows && positions->is_contiguous(), "positions length");
    pp = positions->data_ptr<int>();  // clamped to the table in the kernel (no host read)
  } else {
    TORCH_CHECK(seq_len <= cos.size(0), "rope: seq_len beyond table");
  }
  check(ftc_rope(qkv.data_ptr(), cos.data_ptr<float>(), sin.data_ptr<float>(), pp, rows, (int)qkv.stride(0),
                 (int)n_rot_heads, (int)head_dim, (int)seq_len, inverse ? 1 : 0, (int)cos.size(0), cur_stream()),
        "rope");
}

// ---------------- SwiGLU ----------------
at::Tensor swiglu_fwd(const at::Tensor& gu, int64_t pad) {
  need(gu, at::kBFloat16, "gu");
  need_rows(gu, "gu");
  const long long rows = gu.size(0);
  const int F = (int)(gu.size(1) / 2);
  TORCH_CHECK(gu.size(1) % 16 == 0, "swiglu: 2F must be a multiple of 16");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0, "swiglu: pad must be a multiple of 8");
  auto abuf = at::empty({rows, F + pad}, gu.options());
  check(ftc_swiglu_fwd(gu.data_ptr(), abuf.data_ptr(), rows, F, F + pad, cur_stream()), "swiglu_fwd");
  return pad ? abuf.narrow(1, 0, F) : abuf;
}

at::Tensor swiglu_bwd(const at::Tensor& da, const at::Tensor& gu, int64_t pad) {
  need(da, at::kBFloat16, "da");
  need(gu, at::kBFloat16, "gu");
  need_rows(da, "da");
  need_rows(gu, "gu");
  TORCH_CHECK(da.size(0) == gu.size(0) && gu.size(1) == 2 * da.size(1), "swiglu_bwd shapes");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0, "swiglu_bwd: pad must be a multiple of 8");
  auto dbuf = at::empty({gu.size(0), gu.size(1) + pad}, gu.options());
  check(ftc_swiglu_bwd(da.data_ptr(), gu.data_ptr(), dbuf.data_ptr(), gu.size(0), (int)da.size(1), gu.size(1) + pad,
                       cur_stream()),
        "swiglu_bwd");
  return pad ? dbuf.narrow(1, 0, gu.size(1)) : dbuf;
}

// SwiGLU fused with the LoRA rank product of its output (fwd: h (sA)^T, bwd: dgu B) written into the
// tail columns of the row-padded result (csrc/kernels/swiglu_lora.hip).  `am` / `bt` are row views
// [>= 16 nct, F] / [>= 16 nct, 2F] with unit column stride; Rp = pad (all pad columns are written).
inline void need_rowview(const at::Tensor& t, int64_t min_rows, int64_t cols, const char* name) {
  need(t, at::kBFloat16, name);
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= min_rows && t.size(1) == cols, name,
              " must be a [>=", min_rows, ", ", cols, "] row view");
  TORCH_CHECK(t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name,
              " rows must be 16-byte aligned");
}

at::Tensor swiglu_fwd_lora(const at::Tensor& gu, int64_t pad, const at::Tensor& am, int64_t nct) {
  need(gu, at::kBFloat16, "gu");
  need_rows(gu, "gu");
  const long long rows = gu.size(0);
  const int F = (int)(gu.size(1) / 2);
  TORCH_CHECK(F % 128 == 0, "swiglu_fwd_lora: F must be a multiple of 128");
  TORCH_CHECK(nct >= 1 && nct <= 4 && pad >= 16 * nct && pad % 16 == 0, "swiglu_fwd_lora: bad nct/pad");
  need_rowview(am, 16 * nct, F, "am");
  auto abuf = at::empty({rows, F + pad}, gu.options());
  check(ftc_swiglu_fwd_lora(gu.data_ptr(), abuf.data_ptr(), rows, F, F + pad, am.data_ptr(), am.stride(0), (int)nct,
                            (int)pad, cur_stream()),
        "swiglu_fwd_lora");
  return abuf.narrow(1, 0, F);
}

at::Tensor swiglu_bwd_lora(const at::Tensor& da, const at::Tensor& gu, int64_t pad, const at::Tensor& bt,
                           int64_t nct, bool split) {
  need(da, at::kBFloat16, "da");
  need(gu, at::kBFloat16, "gu");
  need_rows(gu, "gu");
  TORCH_CHECK(da.dim() == 2 && da.stride(1) == 1 && da.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(da.data_ptr()) % 16 == 0,
              "swiglu_bwd_lora: da must be a 16-byte aligned row view");
  TORCH_CHECK(da.size(0) == gu.size(0) && gu.size(1) == 2 * da.size(1), "swiglu_bwd_lora shapes");
  const int F = (int)da.size(1);
  TORCH_CHECK(F % 128 == 0, "swiglu_bwd_lora: F must be a multiple of 128");
  TORCH_CHECK(!split || nct % 2 == 0, "swiglu_bwd_lora: split needs an even tile count");
  TORCH_CHECK(nct >= 1 && nct <= 4 && pad >= 16 * nct && pad % 16 == 0, "swiglu_bwd_lora: bad nct/pad");
  need_rowview(bt, 16 * nct, 2 * F, "bt");
  auto dbuf = at::empty({gu.size(0), gu.size(1) + pad}, gu.options());
  check(ftc_swiglu_bwd_lora(da.data_ptr(), da.stride(0), gu.data_ptr(), dbuf.data_ptr(), gu.size(0), F,
                            gu.size(1) + pad, bt.data_ptr(), bt.stride(0), (int)nct, split ? 1 : 0, (int)pad,
                            cur_stream()),
        "swiglu_bwd_lora");
  return dbuf.narrow(1, 0, gu.size(1));
}

// SwiGLU backward + row tail dgu B_gu + LoRA weight gradients dB_gu (+=) and dA_down (+=) in one pass
// (csrc/kernels/swiglu_lora.hip).  Per-segment rank 16: bt [>=32, 2F], xa [T, 32] view, dyb [T, 16] view,
// mgB = B_gu.main_grad [2F, 32], mgA = A_down.main_grad [16, F] (both bf16, updated in place).
bool swiglu_wgrad_ok(const at::Tensor& gu, int64_t pad) {
  int rb;
  long long wsf;
  const long long T = gu.size(0), F = gu.size(1) / 2;
  return gu.dim() == 2 && ftc_swiglu_wgrad_plan(T, (int)F, &rb, &wsf) == 0 && pad >= 32 && pad % 8 == 0;
}

at::Tensor swiglu_bwd_wgrad(const at::Tensor& da, const at::Tensor& gu, int64_t pad, const at::Tensor& bt,
                            const at::Tensor& xa, const at::Tensor& dyb, at::Tensor& mgB, at::Tensor& mgA,
                            double alphaB, double alphaA) {
  need(gu, at::kBFloat16, "gu");
  need_rows(gu, "gu");
  const long long T = gu.size(0);
  const int F = (int)(gu.size(1) / 2);
  TORCH_CHECK(swiglu_wgrad_ok(gu, pad), "swiglu_bwd_wgrad: unsupported shape");
  TORCH_CHECK(da.dim() == 2 && da.size(0) == T && da.size(1) == F && da.stride(1) == 1 && da.stride(0) % 8 == 0,
              "swiglu_bwd_wgrad: da must be a [T, F] row view");
  need(da, at::kBFloat16, "da");
  need_rowview(bt, 32, 2 * F, "bt");
  need(xa, at::kBFloat16, "xa");
  need(dyb, at::kBFloat16, "dyb");
  TORCH_CHECK(xa.dim() == 2 && xa.size(0) == T && xa.size(1) == 32 && xa.stride(1) == 1 && xa.stride(0) % 8 == 0,
              "swiglu_bwd_wgrad: xa must be a [T, 32] row view");
  TORCH_CHECK(dyb.dim() == 2 && dyb.size(0) == T && dyb.size(1) == 16 && dyb.stride(1) == 1 && dyb.stride(0) % 8 == 0,
              "swiglu_bwd_wgrad: dyb must be a [T, 16] row view");
  for (const at::Tensor* t : {&da, &xa, &dyb})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "swiglu_bwd_wgrad: 16-byte aligned rows");
  need(mgB, at::kBFloat16, "mgB");
  need(mgA, at::kBFloat16, "mgA");
  TORCH_CHECK(mgB.dim() == 2 && mgB.size(0) == 2 * F && mgB.size(1) == 32 && mgB.stride(1) == 1,
              "swiglu_bwd_wgrad: mgB must be [2F, 32]");
  TORCH_CHECK(mgA.dim() == 2 && mgA.size(0) == 16 && mgA.size(1) == F && mgA.stride(1) == 1,
              "swiglu_bwd_wgrad: mgA must be [16, F]");
  int rb;
  long long wsf;
  ftc_swiglu_wgrad_plan(T, F, &rb, &wsf);
  auto ws = at::empty({wsf}, gu.options().dtype(at::kFloat));
  auto dbuf = at::empty({T, 2 * F + pad}, gu.options());
  check(ftc_swiglu_bwd_wgrad(da.data_ptr(), da.stride(0), gu.data_ptr(), dbuf.data_ptr(), dbuf.stride(0), T, F,
                             bt.data_ptr(), bt.stride(0), xa.data_ptr(), xa.stride(0), dyb.data_ptr(), dyb.stride(0),
                             ws.data_ptr<float>(), mgB.data_ptr(), mgB.stride(0), (float)alphaB, mgA.data_ptr(),
                             mgA.stride(0), (float)alphaA, (int)pad, cur_stream()),
        "swiglu_bwd_wgrad");
  return dbuf.narrow(1, 0, 2 * F);
}

// tail[:, 0:Rp] = x[:, 0:K] Bm[0:Rp]^T into x's own spare columns (x: [T, K] view with row stride >= K + Rp)
bool tail_gemm_ok(const at::Tensor& x, int64_t Rp) {
  return x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1 &&
         x.size(1) % 128 == 0 && x.stride(0) % 8 == 0 && x.stride(0) >= x.size(1) + Rp &&
         reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
}

void tail_gemm_(at::Tensor& x, const at::Tensor& bm, int64_t nct, int64_t Rp) {
  TORCH_CHECK(tail_gemm_ok(x, Rp), "tail_gemm_: x must be a [T, K] bf16 row view with Rp spare columns");
  TORCH_CHECK(nct >= 1 && nct <= 4 && Rp >= 16 * nct && Rp % 16 == 0, "tail_gemm_: bad nct / Rp");
  need_rowview(bm, 16 * nct, x.size(1), "bm");
  check(ftc_tail_gemm(x.data_ptr(), x.stride(0), x.size(0), (int)x.size(1), bm.data_ptr(), bm.stride(0), (int)nct,
                      (int)Rp, cur_stream()),
        "tail_gemm_");
}

// ---------------- batched strided copy / scale (LoRA operand refresh) ----------------
// jobs: device table of njobs 64-byte records built by ops/linear.py from live bf16 tensor views (so
// every address and stride it holds is inside its tensor); checked here for size and placement only.
void copy2d_batched_(const at::Tensor& jobs, int64_t njobs, int64_t max_elems) {
  TORCH_CHECK(jobs.is_cuda() && jobs.is_contiguous() && jobs.scalar_type() == at::kLong, "copy2d_batched: jobs");
  TORCH_CHECK(jobs.numel() * 8 == njobs * 64 && njobs > 0 && njobs <= 65535, "copy2d_batched: job table size");
  check(ftc_copy2d_batched(jobs.data_ptr(), (int)njobs, (long long)max_elems, cur_stream()), "copy2d_batched");
}

// ---------------- transpose ----------------
// out[C, R] = x[R, C]^T for a 2-D bf16 row view x (unit column stride); out: contiguous [C, R] or None
at::Tensor transpose2d(const at::Tensor& x, const c10::optional<at::Tensor>& out) {
  need(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "transpose2d: x must be a 2-D row view");
  TORCH_CHECK(x.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "transpose2d: x rows must be 16-byte aligned");
  const int64_t R = x.size(0), C = x.size(1);
  TORCH_CHECK(R % 8 == 0 && C % 8 == 0, "transpose2d: both dims must be multiples of 8");
  at::Tensor y;
  if (out.has_value()) {
    y = *out;
    need(y, at::kBFloat16, "out");
    need_rows(y, "out");
    TORCH_CHECK(y.size(0) == C && y.size(1) == R, "transpose2d: out must be [C, R]");
  } else {
    y = at::empty({C, R}, x.options());
  }
  check(ftc_transpose(x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), (int)R, (int)C, cur_stream()),
        "transpose2d");
  return y;
}

// ---------------- split-K partials: c = beta c + sum_s parts[s] ----------------
// parts [S, M, N] fp32 contiguous; c [M, N] bf16 or fp32 row view (unit column stride)
void splitk_sum_(at::Tensor& c, const at::Tensor& parts, double beta) {
  TORCH_CHECK(parts.is_cuda() && c.is_cuda() && parts.dim() == 3 && c.dim() == 2 && parts.is_contiguous() &&
                  parts.scalar_type() == at::kFloat && c.stride(1) == 1 && parts.size(1) == c.size(0) &&
                  parts.size(2) == c.size(1) && (c.scalar_type() == at::kBFloat16 || c.scalar_type() == at::kFloat),
              "splitk_sum_: parts [S, M, N] fp32 contiguous, c [M, N] bf16/fp32 row view");
  check(ftc_splitk_sum(parts.data_ptr<float>(), (int)parts.size(0), parts.size(1) * parts.size(2), c.data_ptr(),
                       c.scalar_type() == at::kFloat, c.size(0), (int)c.size(1), c.stride(0), (float)beta,
                       cur_stream()),
        "splitk_sum_");
}


// ---------------- cross entropy (in place on logits) ----------------
at::Tensor ce_fwd_bwd_(at::Tensor& logits, const at::Tensor& labels, double gscale, int64_t ignore_index) {
  need(logits, at::kBFloat16, "logits");
  need(labels, at::kLong, "labels");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be 2-D row-major");
  TORCH_CHECK(labels.numel() == logits.size(0) && labels.is_contiguous(), "labels length");
  auto loss = at::empty({logits.size(0)}, logits.options().dtype(at::kFloat));
  check(ftc_ce_fwd_bwd(logits.data_ptr(), (const long long*)labels.data_ptr<int64_t>(), loss.data_ptr<float>(), nullptr, logits.size(0),
                       (int)logits.size(1), logits.stride(0), (float)gscale, ignore_index, cur_stream()),
        "ce_fwd_bwd");
  return loss;
}

// ---------------- AdamW / grad norm ----------------
void adamw_(const c10::optional<at::Tensor>& param, at::Tensor& master, at::Tensor& m, at::Tensor& v,
            const at::Tensor& grad, double lr, double b1, double b2, double eps, double wd, int64_t step,
            const c10::optional<at::Tensor>& gscale, const c10::optional<at::Tensor>& hpdev) {
  need(master, at::kFloat, "master");
  need(m, at::kFloat, "m");
  need(v, at::kFloat, "v");
  TORCH_CHECK(master.is_contiguous() && m.is_contiguous() && v.is_contiguous() && grad.is_contiguous(),
              "adamw: flat contiguous buffers required");
  const long long n = master.numel();
  TORCH_CHECK(m.numel() == n && v.numel() == n && grad.numel() == n, "adamw: size mismatch");
  TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16, "adamw: grad dtype");
  void* pp = nullptr;
  if (param.has_value()) {
    need(*param, at::kBFloat16, "param");
    TORCH_CHECK(param->is_contiguous() && param->numel() == n, "adamw: param size");
    pp = param->data_ptr();
  }
  const float* gs = nullptr;
  if (gscale.has_value()) {
    need(*gscale, at::kFloat, "gscale");
    gs = gscale->data_ptr<float>();
  }
  const float* hp = nullptr;
  if (hpdev.has_value() && hpdev->defined()) {
    need(*hpdev, at::kFloat, "hp");
    TORCH_CHECK(hpdev->is_contiguous() && hpdev->numel() == 3, "adamw: hp = [lr, 1 - b1^t, 1 - b2^t]");
    hp = hpdev->data_ptr<float>();
  }
  const double bc1 = 1.0 - std::pow(b1, (double)step);
  const double bc2 = 1.0 - std::pow(b2, (double)step);
  check(ftc_adamw(pp, master.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), grad.data_ptr(),
                  grad.scalar_type() == at::kFloat, n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd,
                  (float)bc1, (float)bc2, gs, hp, cur_stream()),
        "adamw");
}

// returns [sumsq, coef] (fp32, on device): coef = scale * min(1, max_norm/||scale*g||)
at::Tensor grad_sumsq(const at::Tensor& g, double max_norm, double scale) {
  TORCH_CHECK(g.is_cuda() && g.is_contiguous(), "grad_sumsq: contiguous GPU tensor");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "grad_sumsq: dtype");
  auto part = at::empty({ftc_sumsq_partials()}, g.options().dtype(at::kFloat));
  auto out = at::empty({2}, g.options().dtype(at::kFloat));
  check(ftc_sumsq(g.data_ptr(), g.scalar_type() == at::kFloat, g.numel(), part.data_ptr<float>(),
                  out.data_ptr<float>(), out.data_ptr<float>() + 1, (float)max_norm, (float)scale, cur_stream()),
        "grad_sumsq");
  return out;
}

// ---------------- flash attention ----------------
// optional packed-sequence document bounds: int32 [B*S], doc_start[t] = first position of t's document,
// doc_end[t] = one past its last position (causal attention only)
static const int* doc_ptr(const c10::optional<at::Tensor>& t, int64_t n, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->is_contiguous() && t->numel() == n, what,
              ": int32 contiguous [B*S] device tensor");
  return t->data_ptr<int>();
}

// q: [B*S, >=H*D] view (row stride q_rs), k/v: [B*S, >=KV*D] views; all bf16 with unit column stride.
std::vector<at::Tensor> flash_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, int64_t B, int64_t S,
                                  int64_t H, int64_t KV, int64_t D, double scale, bool causal, int64_t window,
                                  int64_t pad, const c10::optional<at::Tensor>& doc_start, int64_t kv_valid) {
  need(q, at::kBFloat16, "q");
  need(k, at::kBFloat16, "k");
  need(v, at::kBFloat16, "v");
  TORCH_CHECK(q.dim() == 2 && k.dim() == 2 && v.dim() == 2, "flash_fwd: 2-D row views");
  TORCH_CHECK(q.stride(1) == 1 && k.stride(1) == 1 && v.stride(1) == 1, "flash_fwd: unit column stride");
  TORCH_CHECK(q.size(0) == B * S && k.size(0) == B * S && v.size(0) == B * S, "flash_fwd: rows != B*S");
  TORCH_CHECK(q.size(1) >= H * D && k.size(1) >= KV * D && v.size(1) >= KV * D, "flash_fwd: width");
  TORCH_CHECK(k.stride(0) == v.stride(0), "flash_fwd: k/v strides must match");
  TORCH_CHECK(D == 128 || D == 64, "flash_fwd: head_dim 64 or 128");
  TORCH_CHECK(H % KV == 0, "flash_fwd: H % KV");
  TORCH_CHECK(S % 64 == 0, "flash_fwd: S must be a multiple of 64");
  TORCH_CHECK(q.stride(0) % 8 == 0 && k.stride(0) % 8 == 0, "flash_fwd: row strides must be 16B multiples");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0, "flash_fwd: pad must be a multiple of 8");
  auto obuf = at::empty({B * S, H * D + pad}, q.options());
  auto o = pad ? obuf.narrow(1, 0, H * D) : obuf;
  auto lse = at::empty({B, H, S}, q.options().dtype(at::kFloat));
  check(ftc_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), (int)B, (int)S,
                      (int)H, (int)KV, (int)D, q.stride(0), k.stride(0), o.stride(0), (float)scale, causal ? 1 : 0,
                      (int)window, doc_ptr(doc_start, B * S, "doc_start"), (int)kv_valid, cur_stream()),
        "flash_fwd");
  return {o, lse};
}

// writes dq/dk/dv into the given views (packed dqkv buffer)
void flash_bwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
               const at::Tensor& dout, const at::Tensor& lse, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv,
               int64_t B, int64_t S, int64_t H, int64_t KV, int64_t D, double scale, bool causal, int64_t window,
               const c10::optional<at::Tensor>& doc_start, const c10::optional<at::Tensor>& doc_end,
               int64_t kv_valid, const c10::optional<at::Tensor>& rope_cos,
               const c10::optional<at::Tensor>& rope_sin, const c10::optional<at::Tensor>& rope_pos) {
  TORCH_CHECK(doc_start.has_value() == doc_end.has_value(), "flash_bwd: doc_start and doc_end go together");
  TORCH_CHECK(rope_cos.has_value() == rope_sin.has_value() && (!rope_pos.has_value() || rope_cos.has_value()),
              "flash_bwd: rope_cos / rope_sin go together");
  const float* rc = nullptr;
  const float* rsn = nullptr;
  const int* rp = nullptr;
  if (rope_cos.has_value()) {
    for (auto* t : {&*rope_cos, &*rope_sin}) {
      need(*t, at::kFloat, "rope cos/sin");
      TORCH_CHECK(t->dim() == 2 && t->size(1) == 64 && t->is_contiguous(), "flash_bwd: rope tables [max_pos, 64]");
    }
    TORCH_CHECK(D == 128, "flash_bwd: the RoPE epilogue needs head_dim 128");
    rc = rope_cos->data_ptr<float>();
    rsn = rope_sin->data_ptr<float>();
    if (rope_pos.has_value()) {
      need(*rope_pos, at::kInt, "rope_pos");
      TORCH_CHECK(rope_pos->numel() == B * S, "flash_bwd: rope_pos [B*S]");
      rp = rope_pos->data_ptr<int>();
    } else {
      TORCH_CHECK(rope_cos->size(0) >= S, "flash_bwd: rope tables shorter than the sequence");
    }
  }
  for (auto* t : {&q, &k, &v, &o, &dout}) need(*t, at::kBFloat16, "flash_bwd input");
  need(lse, at::kFloat, "lse");
  TORCH_CHECK(D == 128 || D == 64, "flash_bwd: head_dim");
  TORCH_CHECK(S % 256 == 0 && H % KV == 0, "flash_bwd: S must be a multiple of 256, H of KV");
  TORCH_CHECK(o.stride(1) == 1 && dout.stride(1) == 1 && o.stride(0) % 8 == 0 && dout.stride(0) % 8 == 0,
              "flash_bwd: o/dout must be row views with 16-byte row strides");
  TORCH_CHECK(dk.stride(0) == dv.stride(0) && k.stride(0) == v.stride(0), "flash_bwd: k/v strides");
  TORCH_CHECK(lse.numel() == B * H * S, "flash_bwd: lse size");
  long long ws = 0;
  check(ftc_flash_bwd_workspace((int)B, (int)S, (int)H, (int)D, &ws), "flash_bwd_workspace");
  auto work = at::empty({ws}, q.options().dtype(at::kByte));
  check(ftc_flash_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr<float>(),
                      dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), work.data_ptr(), (int)B, (int)S, (int)H, (int)KV,
                      (int)D, q.stride(0), k.stride(0), o.stride(0), dout.stride(0), dq.stride(0), dk.stride(0),
                      (float)scale,
                      causal ? 1 : 0, (int)window, doc_ptr(doc_start, B * S, "doc_start"),
                      doc_ptr(doc_end, B * S, "doc_end"), (int)kv_valid, rc, rsn, rp, cur_stream()),
        "flash_bwd");
}

// ---------------- decode attention (generation) ----------------
// qkv: [B, >=(H+2KV)*D] row view of the current token's packed projection (q | k | v); k_cache /
// v_cache: [B, Lmax, KV*D] contiguous; lens: int32 [B] valid keys (current token included, <= max_len
// <= Lmax).  The current token's K/V rows are appended at position lens-1 by the kernel itself.
at::Tensor decode_attention(const at::Tensor& q, at::Tensor& k_cache, at::Tensor& v_cache,
                            const at::Tensor& lens, int64_t H, int64_t KV, int64_t D, int64_t max_len, double scale,
                            int64_t window) {
  need(q, at::kBFloat16, "q");
  need(k_cache, at::kBFloat16, "k_cache");
  need(v_cache, at::kBFloat16, "v_cache");
  TORCH_CHECK(lens.is_cuda() && lens.scalar_type() == at::kInt && lens.is_contiguous(), "lens: int32 device tensor");
  TORCH_CHECK(k_cache.dim() == 3 && k_cache.is_contiguous() && v_cache.sizes() == k_cache.sizes() &&
                  v_cache.is_contiguous(), "decode_attention: caches [B, Lmax, KV*D] contiguous");
  const int64_t B = k_cache.size(0), Lmax = k_cache.size(1);
  TORCH_CHECK(D == 64 || D == 128, "decode_attention: head_dim 64 or 128");
  TORCH_CHECK(H % KV == 0 && H / KV <= 8 && k_cache.size(2) == KV * D, "decode_attention: heads / cache width");
  TORCH_CHECK(q.dim() == 2 && q.size(0) == B && q.size(1) >= (H + 2 * KV) * D && q.stride(1) == 1 &&
                  q.stride(0) % 8 == 0,
              "decode_attention: qkv [B, >=(H+2KV)*D] row view with 16-byte rows");
  TORCH_CHECK(lens.numel() == B && max_len >= 1 && max_len <= Lmax, "decode_attention: lens / max_len");
  auto out = at::empty({B, H * D}, q.options());
  auto ws = at::empty({ftc_decode_workspace_floats((int)B, (int)H, (int)KV, (int)D, (int)max_len)},
                      q.options().dtype(at::kFloat));
  const auto* qp = static_cast<const uint16_t*>(q.data_ptr());
  check(ftc_decode_attention(qp, k_cache.data_ptr(), v_cache.data_ptr(), qp + H * D, qp + (H + KV) * D, q.stride(0),
                             lens.data_ptr<int>(), out.data_ptr(), ws.data_ptr<float>(), (int)B, (int)H, (int)KV,
                             (int)D, (int)max_len,
                             q.stride(0), KV * D, Lmax * KV * D, out.stride(0), (float)scale, (int)window,
                             cur_stream()),
        "decode_attention");
  return out;
}

// ---------------- NF4 (QLoRA) ----------------
std::vector<at::Tensor> nf4_quantize(const at::Tensor& w, int64_t block) {
  need(w, at::kBFloat16, "w");
  TORCH_CHECK(w.is_contiguous() && w.numel() % block == 0 && block % 2 == 0, "nf4_quantize: shape");
  const long long n = w.numel();
  auto packed = at::empty({n / 2}, w.options().dtype(at::kByte));
  auto absmax = at::empty({n / block}, w.options().dtype(at::kFloat));
  check(ftc_nf4_quant(w.data_ptr(), packed.data_ptr<uint8_t>(), absmax.data_ptr<float>(), n, (int)block,
                      cur_stream()),
        "nf4_quant");
  return {packed, absmax};
}

at::Tensor nf4_dequantize(const at::Tensor& packed, const at::Tensor& absmax_q, const at::Tensor& absmax_scale,
                          double absmax_offset, int64_t rows, int64_t cols, int64_t block, int64_t block2) {
  need(packed, at::kByte, "packed");
  need(absmax_q, at::kByte, "absmax_q");
  need(absmax_scale, at::kFloat, "absmax_scale");
  const long long n = rows * cols;
  TORCH_CHECK(packed.numel() * 2 == n && absmax_q.numel() * block == n, "nf4_dequantize: sizes");
  TORCH_CHECK(absmax_scale.numel() * block2 >= absmax_q.numel(), "nf4_dequantize: second-level scales");
  auto out = at::empty({rows, cols}, packed.options().dtype(at::kBFloat16));
  check(ftc_nf4_dequant(packed.data_ptr<uint8_t>(), absmax_q.data_ptr<uint8_t>(), absmax_scale.data_ptr<float>(),
                        (float)absmax_offset, out.data_ptr(), n, (int)block, (int)block2, cur_stream()),
        "nf4_dequant");
  return out;
}

// dequantise W [rows, cols] into a row view `out` (row stride out.stride(0)); transpose=True writes W^T
// into a [cols, >= rows] view (the TN backward operand)
void nf4_dequantize_into(const at::Tensor& packed, const at::Tensor& absmax_q, const at::Tensor& absmax_scale,
                         double absmax_offset, at::Tensor& out, int64_t rows, int64_t cols, int64_t block,
                         int64_t block2, bool transpose) {
  need(packed, at::kByte, "packed");
  need(absmax_q, at::kByte, "absmax_q");
  need(absmax_scale, at::kFloat, "absmax_scale");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(packed.numel() * 2 == rows * cols && absmax_q.numel() * block == rows * cols, "nf4_dequantize_into: sizes");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.stride(0) % 8 == 0, "nf4_dequantize_into: out row view");
  TORCH_CHECK(transpose ? (out.size(0) == cols && out.size(1) >= rows) : (out.size(0) == rows && out.size(1) >= cols),
              "nf4_dequantize_into: out shape");
  check(ftc_nf4_dequant_into(packed.data_ptr<uint8_t>(), absmax_q.data_ptr<uint8_t>(), absmax_scale.data_ptr<float>(),
                             (float)absmax_offset, out.data_ptr(), (int)rows, (int)cols, out.stride(0), (int)block,
                             (int)block2, transpose ? 1 : 0, cur_stream()),
        "nf4_dequant_into");
}

// nf4_dequantize_into plus the rank-r operand parts in the same launch (csrc/kernels/nf4.hip AugTail):
// out_b = B ([N, R] views), out_a = s * A ([R, K] views; transposed: out_a is a [K, R] view = (s A)^T).
void nf4_dequantize_aug(const at::Tensor& packed, const at::Tensor& absmax_q, const at::Tensor& absmax_scale,
                        double absmax_offset, at::Tensor& out, int64_t rows, int64_t cols, int64_t block,
                        int64_t block2, bool transpose, const c10::optional<at::Tensor>& B,
                        const c10::optional<at::Tensor>& out_b, const c10::optional<at::Tensor>& A,
                        const c10::optional<at::Tensor>& out_a, double s) {
  need(packed, at::kByte, "packed");
  need(absmax_q, at::kByte, "absmax_q");
  need(absmax_scale, at::kFloat, "absmax_scale");
  need(out, at::kBFloat16, "out");
  TORCH_CHECK(packed.numel() * 2 == rows * cols && absmax_q.numel() * block == rows * cols, "nf4_dequantize_aug: sizes");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.stride(0) % 8 == 0, "nf4_dequantize_aug: out row view");
  TORCH_CHECK(transpose ? (out.size(0) == cols && out.size(1) >= rows) : (out.size(0) == rows && out.size(1) >= cols),
              "nf4_dequantize_aug: out shape");
  TORCH_CHECK(B.has_value() == out_b.has_value() && A.has_value() == out_a.has_value(), "nf4_dequantize_aug: pairs");
  int R = 0;
  auto row_view = [](const at::Tensor& t, const char* name) {
    need(t, at::kBFloat16, name);
    TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "nf4_dequantize_aug: ", name, " must be a row view");
  };
  if (B) {
    row_view(*B, "B");
    row_view(*out_b, "out_b");
    R = (int)B->size(1);
    TORCH_CHECK(B->size(0) == rows && out_b->size(0) == rows && out_b->size(1) == R, "nf4_dequantize_aug: B shapes");
  }
  if (A) {
    row_view(*A, "A");
    row_view(*out_a, "out_a");
    TORCH_CHECK(!B || A->size(0) == R, "nf4_dequantize_aug: rank of A and B");
    R = (int)A->size(0);
    TORCH_CHECK(A->size(1) == cols, "nf4_dequantize_aug: A shape");
    TORCH_CHECK(transpose ? (out_a->size(0) == cols && out_a->size(1) == R) : (out_a->size(0) == R && out_a->size(1) == cols),
                "nf4_dequantize_aug: out_a shape");
  }
  check(ftc_nf4_dequant_aug(packed.data_ptr<uint8_t>(), absmax_q.data_ptr<uint8_t>(), absmax_scale.data_ptr<float>(),
                            (float)absmax_offset, out.data_ptr(), (int)rows, (int)cols, out.stride(0), (int)block,
                            (int)block2, transpose ? 1 : 0, B ? B->data_ptr() : nullptr, B ? B->stride(0) : 0,
                            out_b ? out_b->data_ptr() : nullptr, out_b ? out_b->stride(0) : 0,
                            A ? A->data_ptr() : nullptr, A ? A->stride(0) : 0, out_a ? out_a->data_ptr() : nullptr,
                            out_a ? out_a->stride(0) : 0, (float)s, R, cur_stream()),
        "nf4_dequant_aug");
}

// y[M,N] = x[M,K] @ dequant(W)[N,K]^T  with the NF4 decode fused into the MFMA operand load
at::Tensor nf4_linear(const at::Tensor& x, const at::Tensor& packed, const at::Tensor& absmax_q,
                      const at::Tensor& absmax_scale, double absmax_offset, int64_t N, int64_t block, int64_t block2) {
  need(x, at::kBFloat16, "x");
  need_rows(x, "x");
  const int M = (int)x.size(0), K = (int)x.size(1);
  TORCH_CHECK(packed.numel() * 2 == (long long)N * K, "nf4_linear: packed size");
  TORCH_CHECK(K % 64 == 0 && N % 32 == 0 && block == 64, "nf4_linear: K multiple of 64, N of 32, block 64");
  auto y = at::empty({M, N}, x.options());
  check(ftc_nf4_gemm(x.data_ptr(), packed.data_ptr<uint8_t>(), absmax_q.data_ptr<uint8_t>(),
                     absmax_scale.data_ptr<float>(), (float)absmax_offset, y.data_ptr(), M, (int)N, K, (int)block,
                     (int)block2, cur_stream()),
        "nf4_gemm");
  return y;
}

// ---------------- LoRA merge ----------------
// W[out,in] += scale * B[out, r_total] @ A[r_total, in]; with seg_rows > 0 the product is block diagonal:
// output rows [s*seg_rows, (s+1)*seg_rows) only see rank slice s (packed qkv / gate_up projections)
void lora_merge_(at::Tensor& w, const at::Tensor& a, const at::Tensor& b, double scale, int64_t seg_rows) {
  need(w, at::kBFloat16, "w");
  need(a, at::kBFloat16, "a");
  need(b, at::kBFloat16, "b");
  need_rows(w, "w");
  TORCH_CHECK(a.is_contiguous() && b.is_contiguous(), "lora_merge: contiguous A/B");
  const int out_f = (int)w.size(0), in_f = (int)w.size(1), r = (int)a.size(0);
  TORCH_CHECK(a.size(1) == in_f && b.size(0) == out_f && b.size(1) == r, "lora_merge: shapes");
  TORCH_CHECK(in_f % 8 == 0, "lora_merge: in_features % 8");
  check(ftc_lora_merge(w.data_ptr(), a.data_ptr(), b.data_ptr(), out_f, in_f, r, (int)seg_rows, (float)scale,
                       cur_stream()),
        "lora_merge");
}

// ---------------- LoRA weight gradient ----------------
// out[m, ocol(m) + r] = beta * out + alpha * sum_t X[t, m] Y[t, ycol(m) + r]  (r < R) for X [T, M] and Y [T, *]
// (row-strided views, unit column stride).  Segments (m_end, ycol, ocol) describe the block-diagonal B of a
// packed projection; empty lists = one segment (ycol = ocol = 0).  out is any strided 2-D bf16 view (pass
// main_grad.t() for dA [R, K]).
bool lora_wgrad_ok(const at::Tensor& x, const at::Tensor& y, int64_t R) {
  auto al = [](const at::Tensor& t) {
    return t.scalar_type() == at::kBFloat16 && t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 &&
           t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
  };
  if (!al(x) || !al(y)) return false;
  const int64_t T = x.size(0), M = x.size(1);
  return y.size(0) == T && T % 64 == 0 && M % 128 == 0 && R % 8 == 0 && R > 0 && R <= 64 && R <= y.size(1);
}

void lora_wgrad_(at::Tensor& out, const at::Tensor& x, const at::Tensor& y, int64_t R, double alpha, double beta,
                 std::vector<int64_t> m_end, std::vector<int64_t> ycol, std::vector<int64_t> ocol) {
  TORCH_CHECK(lora_wgrad_ok(x, y, R), "lora_wgrad: unsupported operands (bf16, T%64, M%128, R%8, R<=64, aligned rows)");
  need(out, at::kBFloat16, "out");
  const int T = (int)x.size(0), M = (int)x.size(1);
  if (m_end.empty()) {
    m_end = {M};
    ycol = {0};
    ocol = {0};
  }
  const int nseg = (int)m_end.size();
  TORCH_CHECK(nseg <= 4 && (int)ycol.size() == nseg && (int)ocol.size() == nseg, "lora_wgrad: <= 4 segments");
  int me[4], yc[4], oc[4];
  for (int i = 0; i < nseg; ++i) {
    me[i] = (int)m_end[i];
    yc[i] = (int)ycol[i];
    oc[i] = (int)ocol[i];
    TORCH_CHECK(yc[i] + R <= y.size(1), "lora_wgrad: segment reads past Y");
    TORCH_CHECK(oc[i] + R <= out.size(1), "lora_wgrad: segment writes past out");
  }
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M, "lora_wgrad: out must have M rows");
  const int splits = ftc_lora_wgrad_splits(T, M);
  auto ws = at::empty({(int64_t)splits * M * R}, x.options().dtype(at::kFloat));
  check(ftc_lora_wgrad(x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0), ws.data_ptr<float>(), T, M, (int)R,
                       out.data_ptr(), out.stride(0), out.stride(1), (float)alpha, (float)beta, nseg, me, yc, oc,
                       cur_stream()),
        "lora_wgrad");
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "finetune_controller_amd gfx950 kernels";
  namespace py = pybind11;
  m.def("rmsnorm_fwd", &rmsnorm_fwd, py::arg("x"), py::arg("res"), py::arg("w"), py::arg("eps"), py::arg("pad") = 0);
  m.def("rmsnorm_bwd", &rmsnorm_bwd, py::arg("dy"), py::arg("h"), py::arg("w"), py::arg("rstd"), py::arg("dres"),
        py::arg("need_dw"), py::arg("pad") = 0);
  m.def("rope_", &rope_);
  m.def("copy2d_batched_", &copy2d_batched_);
  m.def("swiglu_fwd", &swiglu_fwd, py::arg("gu"), py::arg("pad") = 0);
  m.def("swiglu_bwd", &swiglu_bwd, py::arg("da"), py::arg("gu"), py::arg("pad") = 0);
  m.def("swiglu_fwd_lora", &swiglu_fwd_lora, py::arg("gu"), py::arg("pad"), py::arg("am"), py::arg("nct"));
  m.def("swiglu_bwd_lora", &swiglu_bwd_lora, py::arg("da"), py::arg("gu"), py::arg("pad"), py::arg("bt"),
        py::arg("nct"), py::arg("split") = false);
  m.def("swiglu_wgrad_ok", &swiglu_wgrad_ok);
  m.def("swiglu_bwd_wgrad", &swiglu_bwd_wgrad);
  m.def("tail_gemm_ok", &tail_gemm_ok);
  m.def("tail_gemm_", &tail_gemm_);
  m.def("transpose2d", &transpose2d, py::arg("x"), py::arg("out") = py::none());
  m.def("splitk_sum_", &splitk_sum_);
  m.def("ce_fwd_bwd_", &ce_fwd_bwd_);
  m.def("adamw_", &adamw_, py::arg("param"), py::arg("master"), py::arg("m"), py::arg("v"), py::arg("grad"),
        py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("step"),
        py::arg("gscale") = py::none(), py::arg("hp") = py::none());
  m.def("grad_sumsq", &grad_sumsq);
  m.def("flash_fwd", &flash_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("B"), py::arg("S"), py::arg("H"),
        py::arg("KV"), py::arg("D"), py::arg("scale"), py::arg("causal"), py::arg("window"), py::arg("pad") = 0,
        py::arg("doc_start") = py::none(), py::arg("kv_valid") = -1);
  m.def("flash_bwd", &flash_bwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"), py::arg("dout"),
        py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("B"), py::arg("S"), py::arg("H"),
        py::arg("KV"), py::arg("D"), py::arg("scale"), py::arg("causal"), py::arg("window"),
        py::arg("doc_start") = py::none(), py::arg("doc_end") = py::none(), py::arg("kv_valid") = -1,
        py::arg("rope_cos") = py::none(), py::arg("rope_sin") = py::none(), py::arg("rope_pos") = py::none());
  m.def("decode_attention", &decode_attention);
  m.def("nf4_quantize", &nf4_quantize);
  m.def("nf4_dequantize", &nf4_dequantize);
  m.def("nf4_linear", &nf4_linear);
  m.def("lora_merge_", &lora_merge_);
  m.def("lora_wgrad_ok", &lora_wgrad_ok);
  m.def("lora_wgrad_", &lora_wgrad_, py::arg("out"), py::arg("x"), py::arg("y"), py::arg("R"), py::arg("alpha"),
        py::arg("beta") = 1.0, py::arg("m_end") = std::vector<int64_t>{}, py::arg("ycol") = std::vector<int64_t>{},
        py::arg("ocol") = std::vector<int64_t>{});
  m.def("nf4_gemm_ready", [] { return true; });
  m.def("nf4_dequantize_into", &nf4_dequantize_into);
  m.def("nf4_dequantize_aug", &nf4_dequantize_aug, py::arg("packed"), py::arg("absmax_q"), py::arg("absmax_scale"),
        py::arg("absmax_offset"), py::arg("out"), py::arg("rows"), py::arg("cols"), py::arg("block"), py::arg("block2"),
        py::arg("transpose"), py::arg("B") = py::none(), py::arg("out_b") = py::none(), py::arg("A") = py::none(),
        py::arg("out_a") = py::none(), py::arg("s") = 1.0);
}
