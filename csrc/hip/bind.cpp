// SPDX-License-Identifier: Apache-2.0
// pybind11 / PyTorch binding of the paddle_operator_amd HIP kernels.
// Compiled by hipcc for gfx950 (tools/build.py) — no hipify, no CUDA names.
// Every entry point checks device, dtype, contiguity and shape before launch:
// a kernel never sees a shape its grid does not assume.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cmath>

#include "kernels.h"

namespace {

using pdo::bf16;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_I64(t) TORCH_CHECK((t).scalar_type() == at::kLong, #t " must be int64")
#define CHECK_IN(t) \
  CHECK_DEV(t);     \
  CHECK_CONTIG(t)
#define CHECK_RC(rc, what) TORCH_CHECK((rc) == 0, what " rejected the shape (code ", rc, ")")

inline bf16* bp(const at::Tensor& t) { return reinterpret_cast<bf16*>(t.data_ptr()); }
inline float* fp(const at::Tensor& t) { return t.data_ptr<float>(); }

// ---------------------------------------------------------------- deferred column sums
// The bias / norm-weight gradients that kernels reduce into the gradient arena
// (LayerNorm γ/β and the fused residual bias, fc1's bias in the dGELU epilogue,
// the QKV bias in the attention backward) are column sums of fp32 partial rows.
// Inside a colsum_defer(true) window (the trainer's backward) they are queued
// with their partial buffers kept alive and run by colsum_flush() as a few
// batched launches — before each bucket all-reduce and at the end of the
// backward — instead of two launches per parameter group (194 per GPT-2-medium
// step).  Only arena destinations (accumulate) are deferred.
struct PendingColsum {
  at::Tensor keep;
  pdo::ColsumJob job;
};
static std::vector<PendingColsum> g_colsum_q;
static bool g_colsum_defer = false;

static void colsum_or_defer(const at::Tensor& part, int G, int C, int ld, const pdo::ColOut& co, bool defer_ok) {
  const float* p = fp(part);
  float* scratch = fp(part) + (size_t)G * ld;
  if (g_colsum_defer && defer_ok) {
    g_colsum_q.push_back({part, pdo::ColsumJob{p, scratch, G, C, ld, co}});
    return;
  }
  pdo::colsum(p, G, C, ld, co, scratch, cur_stream());
}

// destinations of two jobs overlap (both accumulate into the same arena slice,
// e.g. a LayerNorm run by two graphs before one backward)
static bool colsum_overlap(const pdo::ColsumJob& a, const pdo::ColsumJob& b) {
  auto segs = [](const pdo::ColsumJob& j, int k, const bf16*& lo, const bf16*& hi) {
    if (!j.co.p[k]) return false;
    const int n = j.C < (k + 1) * j.co.seg ? j.C - k * j.co.seg : j.co.seg;
    lo = j.co.p[k];
    hi = j.co.p[k] + (n > 0 ? n : 0);
    return n > 0;
  };
  for (int i = 0; i < 3; ++i) {
    const bf16 *alo, *ahi;
    if (!segs(a, i, alo, ahi)) continue;
    for (int k = 0; k < 3; ++k) {
      const bf16 *blo, *bhi;
      if (segs(b, k, blo, bhi) && alo < bhi && blo < ahi) return true;
    }
  }
  return false;
}

void colsum_flush() {
  if (g_colsum_q.empty()) return;
  // jobs of one batched launch run concurrently: a job whose destination another
  // job of the batch also accumulates into starts the next batch (launch order
  // keeps the read-modify-writes ordered)
  std::vector<pdo::ColsumJob> jobs;
  jobs.reserve(g_colsum_q.size());
  for (const auto& q : g_colsum_q) {
    bool clash = false;
    for (const auto& j : jobs) clash = clash || colsum_overlap(j, q.job);
    if (clash) {
      CHECK_RC(pdo::colsum_batched(jobs.data(), (int)jobs.size(), cur_stream()), "colsum_batched");
      jobs.clear();
    }
    jobs.push_back(q.job);
  }
  CHECK_RC(pdo::colsum_batched(jobs.data(), (int)jobs.size(), cur_stream()), "colsum_batched");
  g_colsum_q.clear();  // the partial buffers return to the caching allocator in stream order
}

// returns the previous mode; turning deferral off flushes the queue
bool colsum_defer(bool on) {
  const bool prev = g_colsum_defer;
  if (!on) colsum_flush();
  g_colsum_defer = on;
  return prev;
}

int64_t colsum_pending() { return (int64_t)g_colsum_q.size(); }

// ---------------------------------------------------------------- layernorm
std::vector<at::Tensor> layernorm_fwd(at::Tensor x, at::Tensor w, at::Tensor b, double eps) {
  CHECK_IN(x); CHECK_IN(w); CHECK_IN(b); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(b);
  TORCH_CHECK(x.dim() == 2 && w.numel() == x.size(1) && b.numel() == x.size(1));
  const int N = x.size(0), C = x.size(1);
  auto y = at::empty_like(x);
  auto mean = at::empty({N}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({N}, x.options().dtype(at::kFloat));
  CHECK_RC(pdo::layernorm_fwd(bp(x), nullptr, nullptr, bp(w), bp(b), nullptr, bp(y), fp(mean), fp(rstd), N, C,
                              (float)eps, cur_stream()), "layernorm_fwd");
  return {y, mean, rstd};
}

std::vector<at::Tensor> add_layernorm_fwd(at::Tensor x, at::Tensor r, at::Tensor w, at::Tensor b, double eps,
                                          c10::optional<at::Tensor> rbias) {
  CHECK_IN(x); CHECK_IN(r); CHECK_IN(w); CHECK_IN(b);
  CHECK_BF16(x); CHECK_BF16(r); CHECK_BF16(w); CHECK_BF16(b);
  TORCH_CHECK(x.dim() == 2 && x.sizes() == r.sizes() && w.numel() == x.size(1) && b.numel() == x.size(1));
  const bf16* rb = nullptr;
  if (rbias.has_value()) {
    CHECK_IN((*rbias)); CHECK_BF16((*rbias));
    TORCH_CHECK(rbias->numel() == x.size(1));
    rb = bp(*rbias);
  }
  const int N = x.size(0), C = x.size(1);
  auto h = at::empty_like(x);
  auto y = at::empty_like(x);
  auto mean = at::empty({N}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({N}, x.options().dtype(at::kFloat));
  CHECK_RC(pdo::layernorm_fwd(bp(x), bp(r), rb, bp(w), bp(b), bp(h), bp(y), fp(mean), fp(rstd), N, C, (float)eps,
                              cur_stream()), "add_layernorm_fwd");
  return {h, y, mean, rstd};
}

// grads (optional): destination tensors for dgamma, dbeta (, drbias) — e.g. the
// parameters' slices of the flat gradient arena — accumulated in place; the
// result then holds dx only
std::vector<at::Tensor> ln_bwd_impl(at::Tensor dy, at::Tensor x, at::Tensor w, at::Tensor mean, at::Tensor rstd,
                                    c10::optional<at::Tensor> dres, bool rbias,
                                    c10::optional<std::vector<at::Tensor>> grads) {
  CHECK_IN(dy); CHECK_IN(x); CHECK_IN(w); CHECK_IN(mean); CHECK_IN(rstd);
  CHECK_BF16(dy); CHECK_BF16(x); CHECK_BF16(w); CHECK_F32(mean); CHECK_F32(rstd);
  TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes() && w.numel() == x.size(1));
  const int N = x.size(0), C = x.size(1);
  TORCH_CHECK(mean.numel() == N && rstd.numel() == N);
  const bf16* dr = nullptr;
  if (dres.has_value()) {
    CHECK_IN((*dres)); CHECK_BF16((*dres));
    TORCH_CHECK(dres->sizes() == x.sizes());
    dr = bp(*dres);
  }
  auto dx = at::empty_like(x);
  const int G = pdo::layernorm_bwd_grid(N);
  const int NA = rbias ? 3 : 2;
  auto part = at::empty({G * NA * C + pdo::colsum_scratch_floats(G, NA * C)}, x.options().dtype(at::kFloat));
  pdo::ColOut co;
  co.seg = C;
  at::Tensor out;
  if (grads.has_value()) {
    TORCH_CHECK((int)grads->size() == NA, "layernorm_bwd: need ", NA, " gradient destinations");
    for (int i = 0; i < NA; ++i) {
      const at::Tensor& g = (*grads)[i];
      CHECK_IN(g); CHECK_BF16(g);
      TORCH_CHECK(g.numel() == C);
      co.p[i] = bp(g);
    }
    co.acc = 1;
  } else {
    out = at::empty({NA, C}, w.options());
    for (int i = 0; i < NA; ++i) co.p[i] = bp(out) + (size_t)i * C;
  }
  CHECK_RC(pdo::layernorm_bwd(bp(dy), bp(x), bp(w), fp(mean), fp(rstd), dr, bp(dx), fp(part),
                              fp(part) + (size_t)G * NA * C, co, rbias, N, C, cur_stream(), false), "layernorm_bwd");
  // scratch must follow the partial rows (colsum_or_defer's layout): ld = NA·C
  colsum_or_defer(part, G, NA * C, NA * C, co, grads.has_value());
  if (grads.has_value()) return {dx};
  if (rbias) return {dx, out[0], out[1], out[2]};
  return {dx, out[0], out[1]};
}

std::vector<at::Tensor> layernorm_bwd(at::Tensor dy, at::Tensor x, at::Tensor w, at::Tensor mean, at::Tensor rstd,
                                      c10::optional<std::vector<at::Tensor>> grads) {
  return ln_bwd_impl(dy, x, w, mean, rstd, c10::nullopt, false, grads);
}

std::vector<at::Tensor> layernorm_bwd_add(at::Tensor dy, at::Tensor h, at::Tensor w, at::Tensor mean,
                                          at::Tensor rstd, at::Tensor dres, bool rbias,
                                          c10::optional<std::vector<at::Tensor>> grads) {
  return ln_bwd_impl(dy, h, w, mean, rstd, dres, rbias, grads);
}

// ---------------------------------------------------------------- bias + gelu
at::Tensor bias_gelu_fwd(at::Tensor x, at::Tensor b) {
  CHECK_IN(x); CHECK_IN(b); CHECK_BF16(x); CHECK_BF16(b);
  TORCH_CHECK(x.dim() == 2 && b.numel() == x.size(1));
  auto y = at::empty_like(x);
  CHECK_RC(pdo::bias_gelu_fwd(bp(x), bp(b), bp(y), x.size(0), x.size(1), cur_stream()), "bias_gelu_fwd");
  return y;
}

// db_out (optional): accumulate the bias gradient there (arena slice); returns {dx} then
std::vector<at::Tensor> bias_gelu_bwd(at::Tensor dy, at::Tensor x, at::Tensor b, c10::optional<at::Tensor> db_out) {
  CHECK_IN(dy); CHECK_IN(x); CHECK_IN(b); CHECK_BF16(dy); CHECK_BF16(x); CHECK_BF16(b);
  TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes() && b.numel() == x.size(1));
  const long long N = x.size(0);
  const int F = x.size(1);
  auto dx = at::empty_like(x);
  const int G = pdo::bias_gelu_bwd_groups(N, F);
  auto part = at::empty({(int64_t)G * F + pdo::colsum_scratch_floats(G, F)}, x.options().dtype(at::kFloat));
  at::Tensor db;
  if (db_out.has_value()) {
    db = *db_out;
    CHECK_IN(db); CHECK_BF16(db);
    TORCH_CHECK(db.numel() == F);
  } else {
    db = at::empty_like(b);
  }
  CHECK_RC(pdo::bias_gelu_bwd(bp(dy), bp(x), bp(b), bp(dx), fp(part), fp(part) + (size_t)G * F, bp(db), N, F,
                              cur_stream(), db_out.has_value() ? 1 : 0), "bias_gelu_bwd");
  if (db_out.has_value()) return {dx};
  return {dx, db};
}

// db = colsum(dy) for a [N, F] bf16 gradient; with `out`, accumulated into it
at::Tensor bias_grad(at::Tensor dy, c10::optional<at::Tensor> out) {
  CHECK_IN(dy); CHECK_BF16(dy);
  TORCH_CHECK(dy.dim() == 2);
  const long long N = dy.size(0);
  const int F = dy.size(1);
  auto scratch = at::empty({pdo::bias_grad_scratch_floats(N, F)}, dy.options().dtype(at::kFloat));
  at::Tensor db;
  if (out.has_value()) {
    db = *out;
    CHECK_IN(db); CHECK_BF16(db);
    TORCH_CHECK(db.numel() == F);
  } else {
    db = at::empty({F}, dy.options());
  }
  CHECK_RC(pdo::bias_grad(bp(dy), N, F, bp(db), fp(scratch), cur_stream(), out.has_value() ? 1 : 0), "bias_grad");
  return db;
}

// ---------------------------------------------------------------- cross entropy
std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor tgt, int64_t V) {
  CHECK_IN(logits); CHECK_IN(tgt); CHECK_BF16(logits); CHECK_I64(tgt);
  TORCH_CHECK(logits.dim() == 2 && tgt.numel() == logits.size(0) && V <= logits.size(1));
  const int N = logits.size(0), Vp = logits.size(1);
  auto row_loss = at::empty({N}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({N}, logits.options().dtype(at::kFloat));
  auto stats = at::empty({2}, logits.options().dtype(at::kFloat));
  CHECK_RC(pdo::xent_fwd(bp(logits), tgt.data_ptr<int64_t>(), fp(row_loss), fp(lse), fp(stats), N, Vp, (int)V,
                         cur_stream()), "xent_fwd");
  return {stats.select(0, 0), lse, stats};
}

at::Tensor xent_bwd(at::Tensor logits, at::Tensor tgt, at::Tensor lse, at::Tensor dloss, at::Tensor stats, int64_t V,
                    bool inplace) {
  CHECK_IN(logits); CHECK_IN(tgt); CHECK_IN(lse); CHECK_IN(dloss); CHECK_IN(stats);
  CHECK_BF16(logits); CHECK_F32(lse); CHECK_F32(dloss); CHECK_F32(stats);
  const int N = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(lse.numel() == N && tgt.numel() == N && dloss.numel() == 1 && stats.numel() == 2);
  auto out = inplace ? logits : at::empty_like(logits);
  CHECK_RC(pdo::xent_bwd(bp(logits), tgt.data_ptr<int64_t>(), fp(lse), fp(dloss), fp(stats), bp(out), N, Vp, (int)V,
                         cur_stream()), "xent_bwd");
  return out;
}

// logits → dlogits in place (for dloss = 1); returns the mean loss over valid targets
at::Tensor xent_fused(at::Tensor logits, at::Tensor tgt, at::Tensor inv_cnt, int64_t V) {
  CHECK_IN(logits); CHECK_IN(tgt); CHECK_IN(inv_cnt); CHECK_BF16(logits); CHECK_I64(tgt); CHECK_F32(inv_cnt);
  TORCH_CHECK(logits.dim() == 2 && tgt.numel() == logits.size(0) && V <= logits.size(1) && inv_cnt.numel() == 1);
  const int N = logits.size(0), Vp = logits.size(1);
  auto row_loss = at::empty({N}, logits.options().dtype(at::kFloat));
  auto loss = at::empty({}, logits.options().dtype(at::kFloat));
  CHECK_RC(pdo::xent_fused(bp(logits), tgt.data_ptr<int64_t>(), fp(inv_cnt), fp(row_loss), fp(loss), N, Vp, (int)V,
                           cur_stream()), "xent_fused");
  return loss;
}

// ---------------------------------------------------------------- embedding
at::Tensor embed_fwd(at::Tensor idx, at::Tensor wte, at::Tensor wpe) {
  CHECK_IN(idx); CHECK_IN(wte); CHECK_IN(wpe); CHECK_I64(idx); CHECK_BF16(wte); CHECK_BF16(wpe);
  TORCH_CHECK(idx.dim() == 2 && wte.dim() == 2 && wpe.dim() == 2 && wte.size(1) == wpe.size(1));
  const int B = idx.size(0), S = idx.size(1), C = wte.size(1);
  TORCH_CHECK(S <= wpe.size(0), "sequence longer than the position table");
  auto y = at::empty({B, S, C}, wte.options());
  CHECK_RC(pdo::embed_fwd(idx.data_ptr<int64_t>(), bp(wte), bp(wpe), bp(y), B, S, C, cur_stream()), "embed_fwd");
  return y;
}

std::vector<at::Tensor> embed_bwd(at::Tensor dy, at::Tensor idx, int64_t Vp, int64_t P) {
  CHECK_IN(dy); CHECK_IN(idx); CHECK_BF16(dy); CHECK_I64(idx);
  TORCH_CHECK(dy.dim() == 3 && idx.dim() == 2 && dy.size(0) == idx.size(0) && dy.size(1) == idx.size(1));
  const int B = dy.size(0), S = dy.size(1), C = dy.size(2);
  TORCH_CHECK(S <= P);
  auto acc = at::empty({Vp, C}, dy.options().dtype(at::kFloat));
  auto dwte = at::empty({Vp, C}, dy.options());
  auto dwpe = at::empty({P, C}, dy.options());
  CHECK_RC(pdo::embed_bwd(bp(dy), idx.data_ptr<int64_t>(), fp(acc), bp(dwte), bp(dwpe), B, S, C, (int)Vp, (int)P,
                          cur_stream()), "embed_bwd");
  return {dwte, dwpe};
}

// d(wte) accumulated into `dwte` (the gradient arena's bf16 [Vp, C] slice) from the
// stably sorted token ids (keys, perm = torch.sort(idx.flatten(), stable=True));
// returns d(wpe)
at::Tensor embed_bwd_sorted(at::Tensor dy, at::Tensor keys, at::Tensor perm, at::Tensor dwte, int64_t P) {
  CHECK_IN(dy); CHECK_IN(keys); CHECK_IN(perm); CHECK_IN(dwte);
  CHECK_BF16(dy); CHECK_I64(keys); CHECK_I64(perm); CHECK_BF16(dwte);
  TORCH_CHECK(dy.dim() == 3 && keys.numel() == dy.size(0) * dy.size(1) && perm.numel() == keys.numel());
  const int B = dy.size(0), S = dy.size(1), C = dy.size(2);
  TORCH_CHECK(S <= P && dwte.dim() == 2 && dwte.size(1) == C);
  auto dwpe = at::empty({P, C}, dy.options());
  auto part = at::empty({pdo::embed_sorted_part_floats(B * S, C)}, dy.options().dtype(at::kFloat));
  CHECK_RC(pdo::embed_bwd_sorted(bp(dy), keys.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), bp(dwte), bp(dwpe),
                                 fp(part), B, S, C, (int)dwte.size(0), (int)P, 1, cur_stream()), "embed_bwd_sorted");
  return dwpe;
}

// ---------------------------------------------------------------- optimizer
void sumsq(at::Tensor g, at::Tensor out, double scale) {
  CHECK_IN(g); CHECK_IN(out); CHECK_BF16(g); CHECK_F32(out);
  const int cap = 2048;
  auto part = at::empty({cap}, g.options().dtype(at::kFloat));
  CHECK_RC(pdo::sumsq(bp(g), g.numel(), fp(part), cap, (float)scale, fp(out), cur_stream()), "sumsq");
}

void sumsq_chunks(at::Tensor g, at::Tensor part, int64_t chunk, int64_t k0, int64_t k1) {
  CHECK_IN(g); CHECK_IN(part); CHECK_BF16(g); CHECK_F32(part);
  TORCH_CHECK(k0 >= 0 && k1 <= part.numel() && (k1 - 1) * chunk < g.numel(), "sumsq_chunks: chunk range");
  CHECK_RC(pdo::sumsq_chunks(bp(g), g.numel(), chunk, (int)k0, (int)k1, fp(part), cur_stream()), "sumsq_chunks");
}

void sumsq_total(at::Tensor part, at::Tensor out, double scale) {
  CHECK_IN(part); CHECK_IN(out); CHECK_F32(part); CHECK_F32(out);
  CHECK_RC(pdo::sumsq_total(fp(part), (int)part.numel(), (float)scale, fp(out), cur_stream()), "sumsq_total");
}

void adamw_flat(at::Tensor p, at::Tensor g, at::Tensor master, at::Tensor m1, at::Tensor m2, at::Tensor decay,
                at::Tensor normsq, double lr, double b1, double b2, double eps, double wd, double bc1, double bc2,
                double grad_scale, double clip) {
  CHECK_IN(p); CHECK_IN(g); CHECK_IN(master); CHECK_IN(m1); CHECK_IN(m2); CHECK_IN(decay); CHECK_IN(normsq);
  CHECK_BF16(p); CHECK_BF16(g); CHECK_F32(master); CHECK_F32(m1); CHECK_F32(m2); CHECK_F32(decay);
  const long long n = p.numel();
  TORCH_CHECK(g.numel() == n && master.numel() == n && m1.numel() == n && m2.numel() == n);
  TORCH_CHECK(n % 1024 == 0 && decay.numel() == n / 1024);
  CHECK_RC(pdo::adamw_flat(bp(p), bp(g), fp(master), fp(m1), fp(m2), fp(decay), fp(normsq), n, (float)lr, (float)b1,
                           (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2, (float)grad_scale, (float)clip,
                           cur_stream()), "adamw_flat");
}

void sgd_flat(at::Tensor w, at::Tensor g, at::Tensor buf, at::Tensor decay, double lr, double mom, double wd,
              double grad_scale) {
  CHECK_IN(w); CHECK_IN(g); CHECK_IN(buf); CHECK_IN(decay);
  CHECK_F32(w); CHECK_F32(g); CHECK_F32(buf); CHECK_F32(decay);
  const long long n = w.numel();
  TORCH_CHECK(g.numel() == n && buf.numel() == n && n % 1024 == 0 && decay.numel() == n / 1024);
  CHECK_RC(pdo::sgd_flat(fp(w), fp(g), fp(buf), fp(decay), n, (float)lr, (float)mom, (float)wd, (float)grad_scale,
                         cur_stream()), "sgd_flat");
}

// out (+)= sum over the leading dim of part [s, ...] (split-K weight gradients)
void splitk_add(at::Tensor part, at::Tensor out, bool accumulate) {
  CHECK_IN(part); CHECK_BF16(part); CHECK_BF16(out);
  TORCH_CHECK(out.is_contiguous() && part.size(0) >= 1 && part[0].numel() == out.numel());
  CHECK_RC(pdo::splitk_add(bp(part), (int)part.size(0), out.numel(), bp(out), accumulate ? 1 : 0, cur_stream()),
           "splitk_add");
}

// out[M][N] (+)= dyᵀ·x for dy [T, M], x [T, N] (bf16, contiguous); false = unsupported shape
bool gemm_dw(at::Tensor dy, at::Tensor x, at::Tensor out, bool accumulate, int64_t splits) {
  CHECK_IN(dy); CHECK_IN(x); CHECK_IN(out); CHECK_BF16(dy); CHECK_BF16(x); CHECK_BF16(out);
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0));
  const long long T = dy.size(0);
  const int M = dy.size(1), N = x.size(1);
  TORCH_CHECK(out.numel() == (int64_t)M * N, "gemm_dw: out must hold M·N elements");
  int s = pdo::gemm_dw_splits(T, M, N);
  if (s == 0) return false;
  if (splits > 0) s = (int)splits;
  at::Tensor ws;
  if (s > 1) ws = at::empty({(int64_t)s * M * N}, dy.options());
  CHECK_RC(pdo::gemm_dw(bp(dy), bp(x), T, M, N, M, N, bp(out), N, accumulate ? 1 : 0, s > 1 ? bp(ws) : nullptr, s,
                        cur_stream()), "gemm_dw");
  return true;
}

// every matrix of `table` (int64 [n, 5]: first tile, src offset, dst offset, R, C)
// transposed from src into dst in one launch (ops: the step's Wᵀ operands).
// `host` is the CPU tensor the device `table` was copied from: the entries are
// validated there, so no device → host copy runs per call.
void transpose_batched(at::Tensor src, at::Tensor dst, at::Tensor table, at::Tensor host, int64_t tiles) {
  CHECK_IN(src); CHECK_IN(dst); CHECK_IN(table); CHECK_BF16(src); CHECK_BF16(dst);
  TORCH_CHECK(table.scalar_type() == at::kLong && table.dim() == 2 && table.size(1) == 5, "table: int64 [n, 5]");
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == at::kLong && host.is_contiguous() &&
              host.sizes() == table.sizes(), "transpose_batched: host table must mirror the device table");
  const at::Tensor& t = host;
  const int64_t* e = t.data_ptr<int64_t>();
  int64_t want = 0;
  for (int64_t i = 0; i < t.size(0); ++i, e += 5) {
    TORCH_CHECK(e[0] == want && e[3] % 64 == 0 && e[4] % 64 == 0 && e[3] > 0 && e[4] > 0, "transpose_batched: bad entry ", i);
    TORCH_CHECK(e[1] >= 0 && e[1] + e[3] * e[4] <= src.numel() && e[2] >= 0 && e[2] + e[3] * e[4] <= dst.numel(),
                "transpose_batched: entry ", i, " out of range");
    want += (e[3] / 64) * (e[4] / 64);
  }
  TORCH_CHECK(want == tiles, "transpose_batched: tile count mismatch");
  CHECK_RC(pdo::transpose_bf16_batched(bp(src), bp(dst), reinterpret_cast<const long long*>(table.data_ptr<int64_t>()), (int)table.size(0), tiles,
                                       cur_stream()), "transpose_batched");
}

// ---- forward-layout GEMM with fused epilogues (gemm_nt.hip) ----
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) {
  return M < (1LL << 31) && N < (1LL << 31) && pdo::gemm_nt_ok((int)M, (int)N, (int)K, (int)K, (int)K, (int)N);
}

static void nt_check(const at::Tensor& a, const at::Tensor& b) {
  CHECK_IN(a); CHECK_IN(b); CHECK_BF16(a); CHECK_BF16(b);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.size(1) == b.size(1), "gemm_nt: a [M, K], b [N, K]");
  TORCH_CHECK(gemm_nt_supported(a.size(0), b.size(0), a.size(1)), "gemm_nt: M, N % 256 and K % 64 required");
}

// c = a·bᵀ (+ bias); into `out` ([M, N] contiguous bf16) when given
at::Tensor gemm_nt(at::Tensor a, at::Tensor b, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> out) {
  nt_check(a, b);
  const int M = a.size(0), N = b.size(0), K = a.size(1);
  at::Tensor c;
  if (out.has_value()) {
    CHECK_IN((*out)); CHECK_BF16((*out));
    TORCH_CHECK(out->dim() == 2 && out->size(0) == M && out->size(1) == N, "gemm_nt: out must be [M, N]");
    c = *out;
  } else {
    c = at::empty({M, N}, a.options());
  }
  const bf16* bptr = nullptr;
  if (bias.has_value()) {
    CHECK_IN((*bias)); CHECK_BF16((*bias)); TORCH_CHECK(bias->numel() == N);
    bptr = bp(*bias);
  }
  CHECK_RC(pdo::gemm_nt(bp(a), bp(b), M, N, K, K, K, bp(c), N, bptr ? 1 : 0, bptr, nullptr, 0, nullptr,
                        cur_stream()), "gemm_nt");
  return c;
}

// c = a·bᵀ + r (r: [M, N] contiguous bf16), one pass
// c = a·bᵀ (+ bias) + r, one rounding on the 4-wave mainloop
at::Tensor gemm_nt_add(at::Tensor a, at::Tensor b, at::Tensor r, c10::optional<at::Tensor> bias,
                       c10::optional<at::Tensor> mask) {
  nt_check(a, b);
  CHECK_IN(r); CHECK_BF16(r);
  const int M = a.size(0), N = b.size(0), K = a.size(1);
  TORCH_CHECK(r.dim() == 2 && r.size(0) == M && r.size(1) == N, "gemm_nt_add: r must be [M, N]");
  const bf16* bptr = nullptr;
  if (bias && bias->defined()) {
    CHECK_IN((*bias)); CHECK_BF16((*bias));
    TORCH_CHECK(bias->numel() == N, "gemm_nt_add: bias must have N elements");
    bptr = bp(*bias);
  }
  int epi = bptr ? 5 : 4;
  if (mask && mask->defined()) {  // c = a·bᵀ + r ⊙ keep (bit j of byte i keeps element 8i + j of r)
    TORCH_CHECK(!bptr, "gemm_nt_add: bias and mask are exclusive");
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                mask->numel() == (int64_t)M * N / 8 && N % 8 == 0, "gemm_nt_add: mask [M·N/8] uint8");
    bptr = reinterpret_cast<const bf16*>(mask->data_ptr<uint8_t>());
    epi = 6;
  }
  auto c = at::empty({M, N}, a.options());
  CHECK_RC(pdo::gemm_nt(bp(a), bp(b), M, N, K, K, K, bp(c), N, epi, bptr, bp(r), N, nullptr, cur_stream()),
           "gemm_nt_add");
  return c;
}

// (c, part): c = a·bᵀ and the BatchNorm statistics of its bf16 columns per
// row group of gemm_nt_stats_rows(K) rows, part [M / rows, 2, N] = (Σ, Σ(x − x̄)²)
// — bn_act_fwd_tiles' input
std::vector<at::Tensor> gemm_nt_stats(at::Tensor a, at::Tensor b) {
  nt_check(a, b);
  const int M = a.size(0), N = b.size(0), K = a.size(1);
  TORCH_CHECK(N % 256 == 0 || pdo::gemm_nt_epi_ok(M, N, K), "gemm_nt_stats: N % 256 = 0 on the 8-wave ring");
  auto c = at::empty({M, N}, a.options());
  auto part = at::empty({M / pdo::gemm_nt_stats_rows(K), 2, N}, a.options().dtype(at::kFloat));
  CHECK_RC(pdo::gemm_nt(bp(a), bp(b), M, N, K, K, K, bp(c), N, 9, nullptr, nullptr, 0, fp(part), cur_stream()),
           "gemm_nt_stats");
  return {c, part};
}

// (pre, y): pre = a·bᵀ, y = gelu(pre + bias); saved_grad: pre = gelu'(a·bᵀ + bias)
// instead (EPI 7, for gemm_nt_dgelu(..., saved_grad=true))
std::vector<at::Tensor> gemm_nt_gelu(at::Tensor a, at::Tensor b, at::Tensor bias, bool saved_grad) {
  nt_check(a, b);
  CHECK_IN(bias); CHECK_BF16(bias);
  const int M = a.size(0), N = b.size(0), K = a.size(1);
  TORCH_CHECK(bias.numel() == N);
  auto pre = at::empty({M, N}, a.options());
  auto y = at::empty({M, N}, a.options());
  CHECK_RC(pdo::gemm_nt(bp(a), bp(b), M, N, K, K, K, bp(pre), N, saved_grad ? 7 : 2, bp(bias), bp(y), N, nullptr,
                        cur_stream()),
           "gemm_nt_gelu");
  return {pre, y};
}

// dx = (a·bᵀ) ⊙ gelu'(pre + bias); db = colsum(dx) (accumulated into db_out when given).
// saved_grad: pre is gemm_nt_gelu(..., saved_grad=true)'s gelu' and dx = (a·bᵀ) ⊙ pre
// (EPI 8; bias unused)
std::vector<at::Tensor> gemm_nt_dgelu(at::Tensor a, at::Tensor b, at::Tensor pre, at::Tensor bias,
                                      c10::optional<at::Tensor> db_out, bool saved_grad) {
  nt_check(a, b);
  CHECK_IN(pre); CHECK_IN(bias); CHECK_BF16(pre); CHECK_BF16(bias);
  const int M = a.size(0), N = b.size(0), K = a.size(1);
  TORCH_CHECK(pre.dim() == 2 && pre.size(0) == M && pre.size(1) == N && bias.numel() == N);
  auto dx = at::empty({M, N}, a.options());
  const int G = pdo::gemm_nt_dbias_rows(M, K);
  auto part = at::empty({(int64_t)G * N + pdo::colsum_scratch_floats(G, N)}, a.options().dtype(at::kFloat));
  CHECK_RC(pdo::gemm_nt(bp(a), bp(b), M, N, K, K, K, bp(dx), N, saved_grad ? 8 : 3, bp(bias), bp(pre), N, fp(part),
                        cur_stream()),
           "gemm_nt_dgelu");
  at::Tensor db;
  pdo::ColOut co;
  if (db_out.has_value()) {
    db = *db_out;
    CHECK_IN(db); CHECK_BF16(db); TORCH_CHECK(db.numel() == N);
    co = pdo::ColOut::one(bp(db), N);
    co.acc = 1;
  } else {
    db = at::empty_like(bias);
    co = pdo::ColOut::one(bp(db), N);
  }
  colsum_or_defer(part, G, N, N, co, db_out.has_value());
  if (db_out.has_value()) return {dx};
  return {dx, db};
}

at::Tensor transpose(at::Tensor x, std::optional<at::Tensor> out) {
  CHECK_IN(x); CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && x.size(0) % 64 == 0 && x.size(1) % 64 == 0, "transpose: [R, C] with R, C % 64 == 0");
  at::Tensor y;
  if (out.has_value()) {
    y = *out;
    CHECK_IN(y); CHECK_BF16(y);
    TORCH_CHECK(y.dim() == 2 && y.size(0) == x.size(1) && y.size(1) == x.size(0), "transpose: out must be [C, R]");
  } else {
    y = at::empty({x.size(1), x.size(0)}, x.options());
  }
  CHECK_RC(pdo::transpose_bf16(bp(x), bp(y), (int)x.size(0), (int)x.size(1), cur_stream()), "transpose");
  return y;
}

// ---------------------------------------------------------------- NHWC BatchNorm + ReLU (+ residual)
// x: channels_last bf16 [N,C,H,W] (memory NHWC); w,b,running_*: fp32 [C]
std::vector<at::Tensor> bn_act_fwd(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor w, at::Tensor b,
                                   c10::optional<at::Tensor> rm, c10::optional<at::Tensor> rv, double eps,
                                   double momentum, bool relu) {
  CHECK_BF16(x); CHECK_F32(w); CHECK_F32(b);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_act_fwd: channels_last bf16 input");
  const long long C = x.size(1), M = x.numel() / C;
  auto y = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  auto mean = at::empty({C}, w.options()), invstd = at::empty({C}, w.options());
  auto scratch = at::empty({(long long)pdo::bn_fwd_scratch_floats(M, C)}, w.options());
  const bf16* rp = nullptr;
  if (res && res->defined()) {
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(at::MemoryFormat::ChannelsLast));
    CHECK_BF16((*res));
    rp = bp(*res);
  }
  float* rmp = rm && rm->defined() ? fp(*rm) : nullptr;
  float* rvp = rv && rv->defined() ? fp(*rv) : nullptr;
  // ReLU after a residual add: also the 1-bit mask the backward reads instead of y
  at::Tensor mask;
  if (relu && rp) mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  CHECK_RC(pdo::bn_fwd(bp(x), rp, fp(w), fp(b), rmp, rvp, M, (int)C, (float)eps, (float)momentum, relu ? 1 : 0,
                       bp(y), fp(mean), fp(invstd), fp(scratch), cur_stream(),
                       mask.defined() ? mask.data_ptr<uint8_t>() : nullptr), "bn_fwd");
  return {y, mean, invstd, mask};
}

// part: (Σg, Σg·(x − mean)) partials [G, 2, C] that came with dy (conv_dgrad_bn); else a stats pass
static std::vector<at::Tensor> bn_act_bwd_impl(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x,
                                               at::Tensor mean, at::Tensor invstd, at::Tensor w, at::Tensor b,
                                               bool relu, bool want_dres, c10::optional<at::Tensor> dw_into,
                                               c10::optional<at::Tensor> db_into, const at::Tensor* part) {
  CHECK_BF16(dy); CHECK_BF16(x); CHECK_F32(w); CHECK_F32(b);
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "bn_act_bwd: channels_last x");
  auto dyc = dy.contiguous(at::MemoryFormat::ChannelsLast);
  const bf16* yp = nullptr;
  int rmode = relu ? 1 : 0;
  const long long C = x.size(1), M = x.numel() / C;
  if (y && y->defined()) {
    if (y->scalar_type() == at::kByte) {  // the forward's ReLU bitmask
      TORCH_CHECK(relu && y->numel() == M * C / 8 && y->is_contiguous(), "bn_act_bwd: mask [M·C/8] uint8");
      yp = reinterpret_cast<const bf16*>(y->data_ptr<uint8_t>());
      rmode = 2;
    } else {
      CHECK_BF16((*y));
      TORCH_CHECK(y->sizes() == x.sizes() && y->is_contiguous(at::MemoryFormat::ChannelsLast));
      yp = bp(*y);
    }
  }
  TORCH_CHECK(!(relu && want_dres && !yp), "bn_act_bwd: residual + ReLU needs the saved output or its mask");
  auto dx = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  at::Tensor dres;
  if (want_dres) dres = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  // dw_into/db_into: the parameters' fp32 .grad (flat arena) — accumulated in place
  const bool into = dw_into && dw_into->defined() && db_into && db_into->defined();
  at::Tensor dw, db;
  if (into) {
    CHECK_F32((*dw_into)); CHECK_F32((*db_into));
    TORCH_CHECK(dw_into->numel() == C && db_into->numel() == C && dw_into->is_contiguous() && db_into->is_contiguous());
    dw = *dw_into;
    db = *db_into;
  } else {
    dw = at::empty({C}, w.options());
    db = at::empty({C}, w.options());
  }
  if (part) {
    CHECK_F32((*part));
    TORCH_CHECK(part->dim() == 3 && part->size(1) == 2 && part->size(2) == C && part->is_contiguous(),
                "bn_act_bwd_part: partials [G, 2, C]");
    const int mf = pdo::bn_tiles_merge_floats((int)part->size(0), (int)C);
    auto coef = at::empty({3 * C + mf}, w.options());  // + the merge region for a large partial count
    CHECK_RC(pdo::bn_bwd_part(fp(*part), (int)part->size(0), bp(dyc), yp, bp(x), fp(mean), fp(invstd), fp(w), fp(b), M,
                              (int)C, rmode, bp(dx), want_dres ? bp(dres) : nullptr, fp(dw), fp(db),
                              into ? 1 : 0, fp(coef), cur_stream(), mf ? fp(coef) + 3 * C : nullptr),
             "bn_bwd_part");
  } else {
    auto scratch = at::empty({(long long)pdo::bn_bwd_scratch_floats(M, C)}, w.options());
    CHECK_RC(pdo::bn_bwd(bp(dyc), yp, bp(x), fp(mean), fp(invstd), fp(w), fp(b), M, (int)C, rmode, bp(dx),
                         want_dres ? bp(dres) : nullptr, fp(dw), fp(db), into ? 1 : 0, fp(scratch), cur_stream()),
             "bn_bwd");
  }
  if (into) return {dx, dres, at::Tensor(), at::Tensor()};
  return {dx, dres, dw, db};
}

std::vector<at::Tensor> bn_act_bwd(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x, at::Tensor mean,
                                   at::Tensor invstd, at::Tensor w, at::Tensor b, bool relu, bool want_dres,
                                   c10::optional<at::Tensor> dw_into, c10::optional<at::Tensor> db_into) {
  return bn_act_bwd_impl(dy, y, x, mean, invstd, w, b, relu, want_dres, dw_into, db_into, nullptr);
}

std::vector<at::Tensor> bn_act_bwd_part(at::Tensor part, at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x,
                                        at::Tensor mean, at::Tensor invstd, at::Tensor w, at::Tensor b, bool relu,
                                        bool want_dres, c10::optional<at::Tensor> dw_into,
                                        c10::optional<at::Tensor> db_into) {
  return bn_act_bwd_impl(dy, y, x, mean, invstd, w, b, relu, want_dres, dw_into, db_into, &part);
}

// ---------------------------------------------------------------- NHWC implicit-GEMM convolutions (conv.hip)
// x: channels_last bf16 [N, C, H, W]; w: channels_last bf16 [K, C, R, S] (OHWI memory)
bool conv_ok(int64_t N, int64_t H, int64_t W, int64_t C, int64_t K, int64_t R, int64_t S, int64_t stride,
             int64_t pad) {
  return pdo::conv_supported((int)N, (int)H, (int)W, (int)C, (int)K, (int)R, (int)S, (int)stride, (int)pad) != 0;
}

// y = conv(x, w); with_stats: also the per-M-tile BatchNorm partials [tiles, 2, K] (+ tile rows)
std::vector<at::Tensor> conv_fwd(at::Tensor x, at::Tensor w, int64_t stride, int64_t pad, bool with_stats) {
  CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_fwd: channels_last bf16 input");
  TORCH_CHECK(w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(1) == x.size(1),
              "conv_fwd: channels_last bf16 weight [K, C, R, S]");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3);
  const int K = (int)w.size(0), R = (int)w.size(2), S = (int)w.size(3);
  const int Ho = (H + 2 * (int)pad - R) / (int)stride + 1, Wo = (W + 2 * (int)pad - S) / (int)stride + 1;
  auto y = at::empty({N, K, Ho, Wo}, x.options(), at::MemoryFormat::ChannelsLast);
  at::Tensor st;
  if (with_stats) st = at::empty({pdo::conv_fwd_tiles((long long)N * Ho * Wo, K), 2, K}, x.options().dtype(at::kFloat));
  CHECK_RC(pdo::conv_fwd_nhwc(bp(x), N, H, W, C, bp(w), K, R, S, (int)stride, (int)pad, bp(y),
                              with_stats ? fp(st) : nullptr, cur_stream()), "conv_fwd_nhwc");
  return {y, st};
}

int64_t conv_tile_rows(int64_t K) { return pdo::conv_fwd_tile_rows((int)K); }

// Wᵀ of a channels_last [K, C, R, S] weight: [C, R·S·K] (the input-gradient GEMM's B)
at::Tensor conv_weight_t(at::Tensor w) {
  CHECK_BF16(w);
  TORCH_CHECK(w.is_cuda() && w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast));
  const int K = (int)w.size(0), C = (int)w.size(1), T = (int)(w.size(2) * w.size(3));
  auto wt = at::empty({C, (int64_t)T * K}, w.options().memory_format(at::MemoryFormat::Contiguous));
  CHECK_RC(pdo::conv_weight_t(bp(w), bp(wt), K, T, C, cur_stream()), "conv_weight_t");
  return wt;
}

// dst[segment] = Wᵀ of src[segment] for every (offset, K, T, C) row of table (int32, device)
void conv_weight_t_batched(at::Tensor src, at::Tensor dst, at::Tensor table, int64_t max_tiles) {
  CHECK_BF16(src); CHECK_BF16(dst);
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.numel() == dst.numel() && table.is_cuda() &&
              table.scalar_type() == at::kInt && table.dim() == 2 && table.size(1) == 4 && table.is_contiguous(),
              "conv_weight_t_batched: bf16 arenas and an int32 [n, 4] device table");
  CHECK_RC(pdo::conv_weight_t_batched(bp(src), bp(dst), table.data_ptr<int>(), (int)table.size(0), max_tiles,
                                      cur_stream()), "conv_weight_t_batched");
}

// dx [N, C, H, W] (channels_last) of y = conv(x, w) from dy and wt = conv_weight_t(w)
// add: a same-shape channels_last bf16 gradient summed in the epilogue (dx = dgrad + add)
at::Tensor conv_dgrad(at::Tensor dy, at::Tensor wt, int64_t C, int64_t R, int64_t S, int64_t H, int64_t W,
                      int64_t stride, int64_t pad, c10::optional<at::Tensor> add) {
  CHECK_BF16(dy); CHECK_BF16(wt);
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad: channels_last bf16 dy");
  const int N = (int)dy.size(0), K = (int)dy.size(1);
  TORCH_CHECK(wt.is_contiguous() && wt.size(0) == C && wt.size(1) == R * S * K, "conv_dgrad: wt [C, R*S*K]");
  auto dx = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  const bf16* ap = nullptr;
  if (add && add->defined()) {
    CHECK_BF16((*add));
    TORCH_CHECK(add->sizes() == dx.sizes() && add->is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_dgrad: add must match dx (channels_last)");
    ap = bp(*add);
  }
  CHECK_RC(pdo::conv_dgrad_nhwc(bp(dy), N, (int)H, (int)W, (int)C, bp(wt), K, (int)R, (int)S, (int)stride, (int)pad,
                                bp(dx), cur_stream(), nullptr, ap), "conv_dgrad_nhwc");
  return dx;
}

// conv_dgrad whose input x was the output of a BatchNorm (input bx, batch mean /
// invstd, affine w / b, ReLU): also that BatchNorm's backward partials
// [tiles, 2, C] (Σg, Σg·(bx − mean), g = dx·relu'), for bn_act_bwd_part
std::vector<at::Tensor> conv_dgrad_bn(at::Tensor dy, at::Tensor wt, int64_t R, int64_t S, int64_t stride,
                                      int64_t pad, at::Tensor bx, at::Tensor mean, at::Tensor invstd, at::Tensor w,
                                      at::Tensor b, bool relu) {
  CHECK_BF16(dy); CHECK_BF16(wt); CHECK_BF16(bx);
  CHECK_F32(mean); CHECK_F32(invstd); CHECK_F32(w); CHECK_F32(b);
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 4 && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_bn: channels_last bf16 dy");
  TORCH_CHECK(bx.dim() == 4 && bx.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_dgrad_bn: channels_last bx");
  const int N = (int)dy.size(0), K = (int)dy.size(1);
  const int C = (int)bx.size(1), H = (int)bx.size(2), W = (int)bx.size(3);
  TORCH_CHECK(bx.size(0) == N, "conv_dgrad_bn: batch");
  TORCH_CHECK(wt.is_contiguous() && wt.size(0) == C && wt.size(1) == R * S * K, "conv_dgrad_bn: wt [C, R*S*K]");
  for (const at::Tensor* t : {&mean, &invstd, &w, &b})
    TORCH_CHECK(t->numel() == C && t->is_contiguous(), "conv_dgrad_bn: per-channel BatchNorm tensors");
  auto dx = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  auto part = at::empty({pdo::conv_dgrad_tiles(N, H, W, C, (int)R, (int)stride, (int)pad), 2, C},
                        dy.options().dtype(at::kFloat));
  pdo::ConvBnBwd bn{bp(bx), fp(mean), fp(invstd), fp(w), fp(b), fp(part), relu ? 1 : 0};
  CHECK_RC(pdo::conv_dgrad_nhwc(bp(dy), N, H, W, C, bp(wt), K, (int)R, (int)S, (int)stride, (int)pad, bp(dx),
                                cur_stream(), &bn), "conv_dgrad_nhwc(bn)");
  return {dx, part};
}

// dw (fp32 [K, C, R, S] channels_last, e.g. the flat arena's slice) (+)= the weight
// gradient of y = conv(x, w) for dy; without `out` a new fp32 tensor
at::Tensor conv_wgrad(at::Tensor dy, at::Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad,
                      c10::optional<at::Tensor> out) {
  CHECK_BF16(dy); CHECK_BF16(x);
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              x.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_wgrad: channels_last bf16 dy, x");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)dy.size(1);
  at::Tensor dw;
  const bool acc = out.has_value() && out->defined();
  if (acc) {
    dw = *out;
    CHECK_F32(dw);
    TORCH_CHECK(dw.numel() == (int64_t)K * C * R * S && dw.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_wgrad: out must be a channels_last fp32 [K, C, R, S]");
  } else {
    dw = at::empty({K, C, R, S}, x.options().dtype(at::kFloat), at::MemoryFormat::ChannelsLast);
  }
  auto scratch = at::empty({pdo::conv_wgrad_scratch_floats(N, H, W, C, K, (int)R, (int)S, (int)stride, (int)pad)},
                           x.options().dtype(at::kFloat));
  CHECK_RC(pdo::conv_wgrad_nhwc(bp(dy), bp(x), N, H, W, C, K, (int)R, (int)S, (int)stride, (int)pad, fp(dw),
                                acc ? 1 : 0, fp(scratch), cur_stream()), "conv_wgrad_nhwc");
  return dw;
}

// dx (channels_last [N, C, H, W]) += add at the stride-2 pixels (add: [N, C, ceil(H/2), ceil(W/2)])
void conv_stride2_add(at::Tensor dx, at::Tensor add) {
  CHECK_BF16(dx); CHECK_BF16(add);
  TORCH_CHECK(dx.is_cuda() && dx.dim() == 4 && dx.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              add.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_stride2_add: channels_last bf16");
  const int N = (int)dx.size(0), C = (int)dx.size(1), H = (int)dx.size(2), W = (int)dx.size(3);
  TORCH_CHECK(add.size(0) == N && add.size(1) == C && add.size(2) == (H - 1) / 2 + 1 && add.size(3) == (W - 1) / 2 + 1,
              "conv_stride2_add: add shape");
  CHECK_RC(pdo::conv_stride2_add(bp(dx), bp(add), N, H, W, C, cur_stream()), "conv_stride2_add");
}

// ResNet stem 7×7 / stride 2 / pad 3 (3 → 64 channels) through the space-to-depth
// 4×4 implicit GEMM: [y, BatchNorm tile statistics (with_stats), z = the 16-channel
// image the weight gradient reads]
bool stem_ok(int64_t N, int64_t H, int64_t W, int64_t C, int64_t K) {
  return pdo::stem_supported((int)N, (int)H, (int)W, (int)C, (int)K) != 0;
}

std::vector<at::Tensor> stem_fwd(at::Tensor x, at::Tensor w, bool with_stats) {
  CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_fwd: channels_last bf16 input");
  TORCH_CHECK(w.dim() == 4 && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
              w.is_contiguous(at::MemoryFormat::ChannelsLast), "stem_fwd: channels_last bf16 weight [K, 3, 7, 7]");
  const int N = (int)x.size(0), C = (int)x.size(1), H = (int)x.size(2), W = (int)x.size(3), K = (int)w.size(0);
  TORCH_CHECK(pdo::stem_supported(N, H, W, C, K), "stem_fwd: unsupported shape");
  const int IH = H / 2, IW = W / 2;
  auto z = at::empty({N, 16, IH, IW}, x.options(), at::MemoryFormat::ChannelsLast);
  auto w2 = at::empty({K, 256}, w.options().memory_format(at::MemoryFormat::Contiguous));
  auto y = at::empty({N, K, IH, IW}, x.options(), at::MemoryFormat::ChannelsLast);
  at::Tensor st;
  if (with_stats) st = at::empty({pdo::stem_fwd_tiles((long long)N * IH * IW), 2, K}, x.options().dtype(at::kFloat));
  auto s = cur_stream();
  CHECK_RC(pdo::stem_s2d(bp(x), N, H, W, bp(z), s), "stem_s2d");
  CHECK_RC(pdo::stem_weight(bp(w), bp(w2), K, s), "stem_weight");
  CHECK_RC(pdo::stem_fwd(bp(z), N, IH, IW, bp(w2), K, bp(y), with_stats ? fp(st) : nullptr, s), "stem_fwd");
  return {y, st, z};
}

// dw (fp32 [K, 3, 7, 7] channels_last) (+)= the stem's weight gradient from dy and stem_fwd's z
at::Tensor stem_wgrad(at::Tensor dy, at::Tensor z, c10::optional<at::Tensor> out) {
  CHECK_BF16(dy); CHECK_BF16(z);
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              z.is_contiguous(at::MemoryFormat::ChannelsLast) && z.size(1) == 16,
              "stem_wgrad: channels_last bf16 dy, z [N, 16, H/2, W/2]");
  const int N = (int)z.size(0), IH = (int)z.size(2), IW = (int)z.size(3), K = (int)dy.size(1);
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == IH && dy.size(3) == IW, "stem_wgrad: dy / z shapes");
  at::Tensor dw;
  const bool acc = out.has_value() && out->defined();
  if (acc) {
    dw = *out;
    CHECK_F32(dw);
    TORCH_CHECK(dw.numel() == (int64_t)K * 147 && dw.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem_wgrad: out must be a channels_last fp32 [K, 3, 7, 7]");
  } else {
    dw = at::empty({K, 3, 7, 7}, z.options().dtype(at::kFloat), at::MemoryFormat::ChannelsLast);
  }
  auto scratch = at::empty({pdo::stem_wgrad_scratch_floats(N, IH, IW, K)}, z.options().dtype(at::kFloat));
  CHECK_RC(pdo::stem_wgrad(bp(dy), bp(z), N, IH, IW, K, fp(dw), acc ? 1 : 0, fp(scratch), cur_stream()),
           "stem_wgrad");
  return dw;
}

// BatchNorm (+ residual) (+ ReLU) forward from conv_fwd's tile statistics
std::vector<at::Tensor> bn_act_fwd_tiles(at::Tensor x, at::Tensor stats, int64_t tile_rows,
                                         c10::optional<at::Tensor> res, at::Tensor w, at::Tensor b,
                                         c10::optional<at::Tensor> rm, c10::optional<at::Tensor> rv, double eps,
                                         double momentum, bool relu) {
  CHECK_BF16(x); CHECK_F32(w); CHECK_F32(b); CHECK_F32(stats);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_act_fwd_tiles: channels_last bf16 input");
  const long long C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(stats.dim() == 3 && stats.size(1) == 2 && stats.size(2) == C &&
              stats.size(0) == (M + tile_rows - 1) / tile_rows, "bn_act_fwd_tiles: stats [tiles, 2, C]");
  auto y = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  auto mean = at::empty({C}, w.options()), invstd = at::empty({C}, w.options());
  auto ss = at::empty({2 * C}, w.options());
  const bf16* rp = nullptr;
  if (res && res->defined()) {
    TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(at::MemoryFormat::ChannelsLast));
    CHECK_BF16((*res));
    rp = bp(*res);
  }
  float* rmp = rm && rm->defined() ? fp(*rm) : nullptr;
  float* rvp = rv && rv->defined() ? fp(*rv) : nullptr;
  at::Tensor mask;
  if (relu && rp) mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  const int mf = pdo::bn_tiles_merge_floats((int)stats.size(0), (int)C);
  at::Tensor merge;
  if (mf) merge = at::empty({mf}, w.options());
  CHECK_RC(pdo::bn_fwd_tiles(fp(stats), (int)stats.size(0), (int)tile_rows, bp(x), rp, fp(w), fp(b), rmp, rvp, M,
                             (int)C, (float)eps, (float)momentum, relu ? 1 : 0, bp(y), fp(mean), fp(invstd), fp(ss),
                             cur_stream(), mask.defined() ? mask.data_ptr<uint8_t>() : nullptr,
                             mf ? fp(merge) : nullptr), "bn_fwd_tiles");
  return {y, mean, invstd, mask};
}

// y = act(BN(x) + BN_r(r)) from both convolutions' tile statistics (ResNet's
// downsample block: r = the downsample conv's output, never normalised in memory):
// [y, mean, invstd, mask (ReLU bits), rmean, rinvstd]
std::vector<at::Tensor> bn_act_fwd_tiles_bnres(at::Tensor x, at::Tensor stats, int64_t tile_rows, at::Tensor w,
                                               at::Tensor b, c10::optional<at::Tensor> rm,
                                               c10::optional<at::Tensor> rv, double eps, double momentum,
                                               at::Tensor r, at::Tensor rstats, int64_t rtile_rows, at::Tensor rw,
                                               at::Tensor rb, c10::optional<at::Tensor> rrm,
                                               c10::optional<at::Tensor> rrv, double reps, double rmomentum,
                                               bool relu) {
  CHECK_BF16(x); CHECK_BF16(r); CHECK_F32(w); CHECK_F32(b); CHECK_F32(rw); CHECK_F32(rb);
  CHECK_F32(stats); CHECK_F32(rstats);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              r.sizes() == x.sizes() && r.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_act_fwd_tiles_bnres: channels_last bf16 x and r of one shape");
  const long long C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(stats.dim() == 3 && stats.size(1) == 2 && stats.size(2) == C &&
              stats.size(0) == (M + tile_rows - 1) / tile_rows, "bn_act_fwd_tiles_bnres: stats [tiles, 2, C]");
  TORCH_CHECK(rstats.dim() == 3 && rstats.size(1) == 2 && rstats.size(2) == C &&
              rstats.size(0) == (M + rtile_rows - 1) / rtile_rows, "bn_act_fwd_tiles_bnres: rstats [tiles, 2, C]");
  TORCH_CHECK(w.numel() == C && b.numel() == C && rw.numel() == C && rb.numel() == C);
  auto y = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  auto mean = at::empty({C}, w.options()), invstd = at::empty({C}, w.options());
  auto rmean = at::empty({C}, w.options()), rinvstd = at::empty({C}, w.options());
  auto ss = at::empty({2 * C}, w.options()), rss = at::empty({2 * C}, w.options());
  at::Tensor mask;
  if (relu) mask = at::empty({M * C / 8}, x.options().dtype(at::kByte));
  auto opt = [](c10::optional<at::Tensor>& t) { return t && t->defined() ? fp(*t) : nullptr; };
  const int mf = std::max(pdo::bn_tiles_merge_floats((int)stats.size(0), (int)C),
                          pdo::bn_tiles_merge_floats((int)rstats.size(0), (int)C));
  at::Tensor merge;
  if (mf) merge = at::empty({mf}, w.options());
  CHECK_RC(pdo::bn_fwd_tiles_bnres(fp(stats), (int)stats.size(0), (int)tile_rows, bp(x), fp(w), fp(b), opt(rm), opt(rv),
                                   (float)eps, (float)momentum, fp(mean), fp(invstd), fp(ss), fp(rstats),
                                   (int)rstats.size(0), (int)rtile_rows, bp(r), fp(rw), fp(rb), opt(rrm), opt(rrv),
                                   (float)reps, (float)rmomentum, fp(rmean), fp(rinvstd), fp(rss), M, (int)C,
                                   relu ? 1 : 0, bp(y), mask.defined() ? mask.data_ptr<uint8_t>() : nullptr,
                                   cur_stream(), mf ? fp(merge) : nullptr),
           "bn_fwd_tiles_bnres");
  return {y, mean, invstd, mask, rmean, rinvstd};
}

// backward of bn_act_fwd_tiles_bnres: [dx, dr, dw, db, drw, drb] from dy and the
// ReLU bitmask; parameter gradients accumulated into the *_into fp32 tensors when given
std::vector<at::Tensor> bn_act_bwd_pair(at::Tensor dy, at::Tensor mask, at::Tensor x, at::Tensor mean,
                                        at::Tensor invstd, at::Tensor w, at::Tensor r, at::Tensor rmean,
                                        at::Tensor rinvstd, at::Tensor rw, c10::optional<at::Tensor> dw_into,
                                        c10::optional<at::Tensor> db_into, c10::optional<at::Tensor> rdw_into,
                                        c10::optional<at::Tensor> rdb_into) {
  CHECK_BF16(dy); CHECK_BF16(x); CHECK_BF16(r);
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && r.sizes() == x.sizes() &&
              r.is_contiguous(at::MemoryFormat::ChannelsLast), "bn_act_bwd_pair: channels_last x, r of one shape");
  const long long C = x.size(1), M = x.numel() / C;
  TORCH_CHECK(mask.scalar_type() == at::kByte && mask.numel() == M * C / 8 && mask.is_contiguous(),
              "bn_act_bwd_pair: mask [M·C/8] uint8");
  auto dyc = dy.contiguous(at::MemoryFormat::ChannelsLast);
  auto dx = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  auto dr = at::empty_like(r, r.options(), at::MemoryFormat::ChannelsLast);
  auto grads = [&](c10::optional<at::Tensor>& wi, c10::optional<at::Tensor>& bi, at::Tensor& dw, at::Tensor& db) {
    const bool into = wi && wi->defined() && bi && bi->defined();
    if (into) {
      CHECK_F32((*wi)); CHECK_F32((*bi));
      TORCH_CHECK(wi->numel() == C && bi->numel() == C && wi->is_contiguous() && bi->is_contiguous());
      dw = *wi;
      db = *bi;
    } else {
      dw = at::empty({C}, w.options());
      db = at::empty({C}, w.options());
    }
    return into ? 1 : 0;
  };
  at::Tensor dw, db, rdw, rdb;
  const int acc = grads(dw_into, db_into, dw, db), racc = grads(rdw_into, rdb_into, rdw, rdb);
  auto scratch = at::empty({(long long)pdo::bn_bwd_scratch_pair_floats(M, C)}, w.options());
  CHECK_RC(pdo::bn_bwd_pair(bp(dyc), mask.data_ptr<uint8_t>(), bp(x), fp(mean), fp(invstd), fp(w), fp(dw), fp(db), acc,
                            bp(r), fp(rmean), fp(rinvstd), fp(rw), fp(rdw), fp(rdb), racc, M, (int)C, bp(dx), bp(dr),
                            fp(scratch), cur_stream()),
           "bn_bwd_pair");
  return {dx, dr, dw, db, rdw, rdb};
}

// ResNet stem BatchNorm + ReLU + max-pool 3×3/2 from the stem conv's tile statistics:
// [pooled y, window positions (uint8), xsel (the BatchNorm input at each maximum), mean, invstd]
std::vector<at::Tensor> bn_relu_pool_fwd_tiles(at::Tensor x, at::Tensor stats, int64_t tile_rows, at::Tensor w,
                                               at::Tensor b, c10::optional<at::Tensor> rm,
                                               c10::optional<at::Tensor> rv, double eps, double momentum) {
  CHECK_BF16(x); CHECK_F32(w); CHECK_F32(b); CHECK_F32(stats);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "bn_relu_pool_fwd_tiles: channels_last bf16 input");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), M = N * H * W;
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "bn_relu_pool_fwd_tiles: C % 8 == 0 and (C / 8) | 256");
  TORCH_CHECK(stats.dim() == 3 && stats.size(1) == 2 && stats.size(2) == C &&
              stats.size(0) == (M + tile_rows - 1) / tile_rows, "bn_relu_pool_fwd_tiles: stats [tiles, 2, C]");
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  auto y = at::empty({N, C, OH, OW}, x.options(), at::MemoryFormat::ChannelsLast);
  auto arg = at::empty({N * OH * OW * C}, x.options().dtype(at::kByte));
  auto xsel = at::empty({N, C, OH, OW}, x.options(), at::MemoryFormat::ChannelsLast);
  auto mean = at::empty({C}, w.options()), invstd = at::empty({C}, w.options());
  auto ss = at::empty({2 * C}, w.options());
  float* rmp = rm && rm->defined() ? fp(*rm) : nullptr;
  float* rvp = rv && rv->defined() ? fp(*rv) : nullptr;
  const int mf = pdo::bn_tiles_merge_floats((int)stats.size(0), (int)C);
  at::Tensor merge;
  if (mf) merge = at::empty({mf}, w.options());
  CHECK_RC(pdo::bn_relu_pool_fwd_tiles(fp(stats), (int)stats.size(0), (int)tile_rows, bp(x), fp(w), fp(b), rmp, rvp,
                                       (int)N, (int)H, (int)W, (int)C, (float)eps, (float)momentum, bp(y),
                                       arg.data_ptr<uint8_t>(), bp(xsel), fp(mean), fp(invstd), fp(ss), cur_stream(),
                                       mf ? fp(merge) : nullptr),
           "bn_relu_pool_fwd_tiles");
  return {y, arg, xsel, mean, invstd};
}

// its backward: [dx of the BatchNorm input, dgamma, dbeta] (dgamma / dbeta accumulated
// into dw_into / db_into — the parameters' fp32 arena slices — when given)
std::vector<at::Tensor> pool_bn_bwd(at::Tensor dy, at::Tensor y, at::Tensor xsel, at::Tensor arg, at::Tensor x,
                                    at::Tensor mean, at::Tensor invstd, at::Tensor w, at::Tensor b,
                                    c10::optional<at::Tensor> dw_into, c10::optional<at::Tensor> db_into) {
  CHECK_BF16(dy); CHECK_BF16(x); CHECK_BF16(y); CHECK_BF16(xsel); CHECK_F32(w); CHECK_F32(b);
  TORCH_CHECK(y.sizes() == dy.sizes() && xsel.sizes() == dy.sizes() &&
              y.is_contiguous(at::MemoryFormat::ChannelsLast) && xsel.is_contiguous(at::MemoryFormat::ChannelsLast),
              "pool_bn_bwd: y / xsel as dy");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "pool_bn_bwd: channels_last dy, x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == C && dy.size(2) == OH && dy.size(3) == OW, "pool_bn_bwd: dy shape");
  TORCH_CHECK(arg.scalar_type() == at::kByte && arg.numel() == N * OH * OW * C, "pool_bn_bwd: arg");
  auto dx = at::empty_like(x, x.options(), at::MemoryFormat::ChannelsLast);
  const bool into = dw_into && dw_into->defined() && db_into && db_into->defined();
  at::Tensor dw, db;
  if (into) {
    CHECK_F32((*dw_into)); CHECK_F32((*db_into));
    TORCH_CHECK(dw_into->numel() == C && db_into->numel() == C && dw_into->is_contiguous() && db_into->is_contiguous());
    dw = *dw_into;
    db = *db_into;
  } else {
    dw = at::empty({C}, w.options());
    db = at::empty({C}, w.options());
  }
  auto scratch = at::empty({(int64_t)pdo::pool_bn_bwd_scratch_floats((int)N, (int)H, (int)W, (int)C)}, w.options());
  CHECK_RC(pdo::pool_bn_bwd(bp(dy), bp(y), bp(xsel), arg.data_ptr<uint8_t>(), bp(x), fp(mean), fp(invstd), fp(w),
                            fp(b), (int)N,
                            (int)H, (int)W, (int)C, bp(dx), fp(dw), fp(db), into ? 1 : 0, fp(scratch), cur_stream()),
           "pool_bn_bwd");
  if (into) return {dx, at::Tensor(), at::Tensor()};
  return {dx, dw, db};
}

// ---------------------------------------------------------------- NHWC max-pool 3×3/2
std::vector<at::Tensor> maxpool3s2_fwd(at::Tensor x) {
  CHECK_BF16(x);
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0,
              "maxpool3s2_fwd: channels_last bf16 input with C % 8 == 0");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  auto y = at::empty({N, C, OH, OW}, x.options(), at::MemoryFormat::ChannelsLast);
  auto arg = at::empty({N, C, OH, OW}, x.options().dtype(at::kByte), at::MemoryFormat::ChannelsLast);
  CHECK_RC(pdo::maxpool3s2_fwd(bp(x), (int)N, (int)H, (int)W, (int)C, bp(y), arg.data_ptr<uint8_t>(), cur_stream()),
           "maxpool3s2_fwd");
  return {y, arg};
}

// dx = the global average pool's input gradient, channels_last [N, C, H, W], from dy [N, C]
at::Tensor gap_bwd(at::Tensor dy, int64_t H, int64_t W) {
  CHECK_BF16(dy);
  TORCH_CHECK(dy.is_cuda() && dy.dim() == 2 && dy.is_contiguous() && dy.size(1) % 8 == 0, "gap_bwd: dy [N, C], C % 8 == 0");
  const int64_t N = dy.size(0), C = dy.size(1);
  auto dx = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  CHECK_RC(pdo::gap_bwd(bp(dy), (int)N, (int)(H * W), (int)C, bp(dx), cur_stream()), "gap_bwd");
  return dx;
}

at::Tensor maxpool3s2_bwd(at::Tensor dy, at::Tensor arg, int64_t H, int64_t W) {
  CHECK_BF16(dy);
  auto dyc = dy.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(arg.scalar_type() == at::kByte && arg.sizes() == dy.sizes() &&
              arg.is_contiguous(at::MemoryFormat::ChannelsLast), "maxpool3s2_bwd: arg");
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(dy.size(2) == (H - 1) / 2 + 1 && dy.size(3) == (W - 1) / 2 + 1, "maxpool3s2_bwd: input size");
  auto dx = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  CHECK_RC(pdo::maxpool3s2_bwd(bp(dyc), arg.data_ptr<uint8_t>(), (int)N, (int)H, (int)W, (int)C, bp(dx),
                               cur_stream()), "maxpool3s2_bwd");
  return dx;
}

// ---------------------------------------------------------------- attention
std::vector<at::Tensor> attn_fwd(at::Tensor qkv, int64_t n_head) {
  CHECK_IN(qkv); CHECK_BF16(qkv);
  TORCH_CHECK(qkv.dim() == 3 && qkv.size(2) % (3 * n_head) == 0);
  const int B = qkv.size(0), S = qkv.size(1), C = qkv.size(2) / 3, H = n_head, D = C / H;
  TORCH_CHECK(D == 64 && S % 128 == 0, "attn_fwd supports head_dim 64 and seq % 128 == 0");
  auto o = at::empty({B, S, C}, qkv.options());
  auto lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
  CHECK_RC(pdo::attn_fwd(bp(qkv), bp(o), fp(lse), B, S, H, D, 1.f / std::sqrt((float)D), cur_stream()), "attn_fwd");
  return {o, lse};
}

// dqkv, plus (with_bias_grad) the QKV bias gradient reduced from the kernels'
// fp32 column partials — accumulated into db_out when given, else returned
std::vector<at::Tensor> attn_bwd(at::Tensor dout, at::Tensor qkv, at::Tensor o, at::Tensor lse, int64_t n_head,
                                 bool with_bias_grad, c10::optional<at::Tensor> db_out) {
  CHECK_IN(dout); CHECK_IN(qkv); CHECK_IN(o); CHECK_IN(lse);
  CHECK_BF16(dout); CHECK_BF16(qkv); CHECK_BF16(o); CHECK_F32(lse);
  const int B = qkv.size(0), S = qkv.size(1), C = qkv.size(2) / 3, H = n_head, D = C / H;
  TORCH_CHECK(dout.sizes() == o.sizes() && o.size(2) == C && lse.numel() == (int64_t)B * H * S);
  TORCH_CHECK(D == 64 && S % 128 == 0);
  auto dqkv = at::empty_like(qkv);
  auto delta = at::empty({2, B, H, S}, qkv.options().dtype(at::kFloat));  // delta | lse·log2e
  const int G = B * (S / 128), NC = 3 * C;
  at::Tensor part;
  if (with_bias_grad)
    part = at::empty({(int64_t)G * NC + pdo::colsum_scratch_floats(G, NC)}, qkv.options().dtype(at::kFloat));
  CHECK_RC(pdo::attn_bwd(bp(dout), bp(qkv), bp(o), fp(lse), fp(delta), bp(dqkv), B, S, H, D,
                         1.f / std::sqrt((float)D), cur_stream(), with_bias_grad ? fp(part) : nullptr), "attn_bwd");
  if (!with_bias_grad) return {dqkv};
  at::Tensor db;
  pdo::ColOut co;
  if (db_out.has_value()) {
    db = *db_out;
    CHECK_IN(db); CHECK_BF16(db); TORCH_CHECK(db.numel() == NC);
    co = pdo::ColOut::one(bp(db), NC);
    co.acc = 1;
  } else {
    db = at::empty({NC}, qkv.options());
    co = pdo::ColOut::one(bp(db), NC);
  }
  colsum_or_defer(part, G, NC, NC, co, db_out.has_value());
  if (db_out.has_value()) return {dqkv};
  return {dqkv, db};
}

// ---------------------------------------------------------------- bucket helpers
void scale_(at::Tensor x, double s) {
  CHECK_IN(x); CHECK_BF16(x);
  CHECK_RC(pdo::scale_bf16(bp(x), x.numel(), (float)s, cur_stream()), "scale_bf16");
}

// x *= s[0] in place (s: fp32 device scalar, e.g. the loss gradient)
void scale_dev_(at::Tensor x, at::Tensor s) {
  CHECK_IN(x); CHECK_BF16(x); CHECK_IN(s);
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.numel() >= 1, "scale must be an fp32 device scalar");
  CHECK_RC(pdo::scale_dev_bf16(bp(x), x.numel(), fp(s), cur_stream()), "scale_dev_bf16");
}

// y += s[0] · x in place (bf16, same length; s: fp32 device scalar)
void axpy_dev_(at::Tensor y, at::Tensor x, at::Tensor s) {
  CHECK_IN(y); CHECK_IN(x); CHECK_BF16(y); CHECK_BF16(x); CHECK_IN(s);
  TORCH_CHECK(y.numel() == x.numel(), "axpy_dev_: length mismatch");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.numel() >= 1, "scale must be an fp32 device scalar");
  CHECK_RC(pdo::axpy_dev_bf16(bp(y), bp(x), y.numel(), fp(s), cur_stream()), "axpy_dev_bf16");
}

// g += h; h = 0 (bf16, same length)
void fold_zero(at::Tensor g, at::Tensor h) {
  CHECK_IN(g); CHECK_IN(h); CHECK_BF16(g); CHECK_BF16(h);
  TORCH_CHECK(g.numel() == h.numel(), "fold_zero: length mismatch");
  CHECK_RC(pdo::fold_zero_bf16(bp(g), bp(h), g.numel(), cur_stream()), "fold_zero_bf16");
}

// flat[off_i : off_i + n_i] = scale * t_i for every tensor (one launch);
// reverse: t_i = flat[off_i : off_i + n_i].  bf16 or f32, all one dtype.
void flatten_scale(std::vector<at::Tensor> ts, at::Tensor flat, std::vector<int64_t> offsets, double scale,
                   bool reverse) {
  CHECK_IN(flat);
  const auto dt = flat.scalar_type();
  TORCH_CHECK(dt == at::kBFloat16 || dt == at::kFloat, "flat must be bf16 or float32");
  TORCH_CHECK(ts.size() == offsets.size());
  const int n = ts.size();
  if (n == 0) return;
  auto meta = at::empty({n, 3}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
  int64_t* mp = meta.data_ptr<int64_t>();
  int64_t prev = -1, total = 0;
  for (int i = 0; i < n; ++i) {
    CHECK_IN(ts[i]);
    TORCH_CHECK(ts[i].scalar_type() == dt, "every tensor must have the flat buffer's dtype");
    TORCH_CHECK(ts[i].device() == flat.device(), "tensors must live on the flat buffer's device");
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] >= prev, "offsets must be non-negative and increasing");
    TORCH_CHECK(offsets[i] + ts[i].numel() <= flat.numel(), "tensor overruns the flat buffer");
    TORCH_CHECK(i == 0 || offsets[i] >= offsets[i - 1] + ts[i - 1].numel(), "tensors overlap in the flat buffer");
    prev = offsets[i];
    mp[3 * i] = reinterpret_cast<int64_t>(ts[i].data_ptr());
    mp[3 * i + 1] = ts[i].numel();
    mp[3 * i + 2] = offsets[i];
    total = offsets[i] + ts[i].numel();
  }
  auto dmeta = meta.to(flat.device(), /*non_blocking=*/true);
  CHECK_RC(pdo::bucket_copy(dt == at::kFloat ? 1 : 0, !reverse, flat.data_ptr(), total, n, dmeta.data_ptr(),
                            (float)scale, cur_stream()),
           "flatten/unflatten");
  // the pinned meta must outlive the async H2D copy
  c10::hip::getCurrentHIPStream().synchronize();
}

// dst (f32) = scale * src (bf16), elementwise; numel % 8 == 0
void cast_scale_bf16_f32(at::Tensor src, at::Tensor dst, double scale) {
  CHECK_IN(src); CHECK_IN(dst); CHECK_BF16(src); CHECK_F32(dst);
  TORCH_CHECK(src.numel() == dst.numel() && src.numel() % 8 == 0, "cast: numel mismatch or not a multiple of 8");
  CHECK_RC(pdo::cast_scale_bf16_f32(bp(src), fp(dst), src.numel(), (float)scale, cur_stream()), "cast_scale_bf16_f32");
}

// dst (bf16) = src (f32); numel % 8 == 0
void cast_f32_bf16(at::Tensor src, at::Tensor dst) {
  CHECK_IN(src); CHECK_IN(dst); CHECK_F32(src); CHECK_BF16(dst);
  TORCH_CHECK(src.numel() == dst.numel() && src.numel() % 8 == 0, "cast: numel mismatch or not a multiple of 8");
  CHECK_RC(pdo::cast_f32_bf16(fp(src), bp(dst), src.numel(), cur_stream()), "cast_f32_bf16");
}

// ---------------------------------------------------------------- device / IPC bootstrap
// (launcher: hipSetDevice before any other HIP call, intra-node hipIpc handle
// exchange to probe/warm the xGMI peer links before the RCCL communicator)
#define HIP_OK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    TORCH_CHECK(e_ == hipSuccess, #x " failed: ", hipGetErrorString(e_));            \
  } while (0)

py::dict device_info(int dev) {
  hipDeviceProp_t p;
  HIP_OK(hipGetDeviceProperties(&p, dev));
  char bus[64] = {0};
  HIP_OK(hipDeviceGetPCIBusId(bus, sizeof bus, dev));
  py::dict d;
  d["name"] = std::string(p.name);
  d["gcn_arch"] = std::string(p.gcnArchName);
  d["pci_bus_id"] = std::string(bus);
  d["compute_units"] = p.multiProcessorCount;
  d["total_mem"] = (int64_t)p.totalGlobalMem;
  d["lds_per_block"] = (int64_t)p.sharedMemPerBlock;
  d["clock_khz"] = p.clockRate;
  d["l2_bytes"] = p.l2CacheSize;
  d["warp_size"] = p.warpSize;
  return d;
}

int set_device(int dev) {
  HIP_OK(hipSetDevice(dev));
  int cur = -1;
  HIP_OK(hipGetDevice(&cur));
  return cur;
}

// export a tensor for another process: (handle of the allocation that holds
// it, byte offset of the tensor inside that allocation) — the caching
// allocator sub-allocates, so the tensor need not start at the allocation base
py::tuple ipc_get_handle(at::Tensor t) {
  CHECK_DEV(t);
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  HIP_OK(hipMemGetAddressRange(&base, &size, t.data_ptr()));
  hipIpcMemHandle_t h;
  HIP_OK(hipIpcGetMemHandle(&h, base));
  const int64_t off = reinterpret_cast<char*>(t.data_ptr()) - reinterpret_cast<char*>(base);
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof h), off);
}

// map a peer's exported buffer into this process as a uint8 tensor of
// `nbytes` starting `offset` bytes into the peer's allocation
at::Tensor ipc_open_handle(py::bytes handle, int64_t nbytes, int64_t device, int64_t offset) {
  std::string hs = handle;
  TORCH_CHECK(hs.size() == sizeof(hipIpcMemHandle_t), "bad IPC handle size");
  TORCH_CHECK(offset >= 0 && nbytes >= 0, "bad IPC offset/size");
  hipIpcMemHandle_t h;
  memcpy(&h, hs.data(), sizeof h);
  void* p = nullptr;
  HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  auto opts = at::TensorOptions().dtype(at::kByte).device(at::Device(at::kCUDA, (c10::DeviceIndex)device));
  void* base = p;
  return at::from_blob(static_cast<char*>(p) + offset, {nbytes}, [base](void*) { (void)hipIpcCloseMemHandle(base); },
                       opts);
}

bool can_access_peer(int dev, int peer) {
  int ok = 0;
  HIP_OK(hipDeviceCanAccessPeer(&ok, dev, peer));
  return ok != 0;
}

bool enable_peer_access(int peer) {
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();
    return true;
  }
  return e == hipSuccess;
}

}  // namespace

PYBIND11_MODULE(_pdo_hip, m) {
  m.doc() = "paddle_operator_amd HIP/CDNA4 kernels (gfx950)";
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("add_layernorm_fwd", &add_layernorm_fwd, py::arg("x"), py::arg("r"), py::arg("w"), py::arg("b"),
        py::arg("eps"), py::arg("rbias") = py::none());
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"),
        py::arg("rstd"), py::arg("grads") = py::none());
  m.def("layernorm_bwd_add", &layernorm_bwd_add, py::arg("dy"), py::arg("h"), py::arg("w"), py::arg("mean"),
        py::arg("rstd"), py::arg("dres"), py::arg("rbias"), py::arg("grads") = py::none());
  m.def("bias_gelu_fwd", &bias_gelu_fwd);
  m.def("bias_gelu_bwd", &bias_gelu_bwd, py::arg("dy"), py::arg("x"), py::arg("b"), py::arg("db_out") = py::none());
  m.def("bias_grad", &bias_grad, py::arg("dy"), py::arg("out") = py::none());
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("xent_fused", &xent_fused);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("embed_bwd_sorted", &embed_bwd_sorted);
  m.def("sumsq", &sumsq);
  m.def("sumsq_chunks", &sumsq_chunks);
  m.def("set_adamw_variant", [](int v) { pdo::adamw_set_variant(v); });
  m.def("sumsq_total", &sumsq_total);
  m.def("adamw_flat", &adamw_flat);
  m.def("sgd_flat", &sgd_flat);
  m.def("splitk_add", &splitk_add);
  m.def("transpose", &transpose, py::arg("x"), py::arg("out") = py::none());
  m.def("transpose_batched", &transpose_batched);
  m.def("colsum_defer", &colsum_defer);
  m.def("colsum_flush", &colsum_flush);
  m.def("colsum_pending", &colsum_pending);
  m.def("axpy_dev_", &axpy_dev_);
  m.def("gemm_dw", &gemm_dw, py::arg("dy"), py::arg("x"), py::arg("out"), py::arg("accumulate") = true,
        py::arg("splits") = 0);
  m.def("gemm_dw_splits", &pdo::gemm_dw_splits);
  m.def("gemm_nt_supported", &gemm_nt_supported);
  m.def("gemm_nt_stats", &gemm_nt_stats);
  m.def("gemm_nt_stats_rows", [](int64_t K) { return pdo::gemm_nt_stats_rows((int)K); });
  // EPI 7 / 8 (the saved-GELU' pair) run on the 4-wave mainloop only
  m.def("gemm_nt_epi_ok", [](int64_t M, int64_t N, int64_t K) {
    return M < (1LL << 31) && N < (1LL << 31) && pdo::gemm_nt_epi_ok((int)M, (int)N, (int)K) != 0;
  });
  m.def("gemm_dw_impl", [](int impl) {
    const int prev = pdo::gemm_dw_get_impl();
    if (impl >= 0) pdo::gemm_dw_set_impl(impl);
    return prev;
  }, py::arg("impl") = -1, "select gemm_dw's mainloop (0 = 8-wave, 1.. = 4-wave variants); returns the previous");
  m.def("gemm_nt_impl", [](int impl) {
    const int prev = pdo::gemm_nt_get_impl();
    if (impl >= 0) pdo::gemm_nt_set_impl(impl);
    return prev;
  }, py::arg("impl") = -1, "select gemm_nt's mainloop (0 = 8-wave ring, 1 = 4-wave); returns the previous");
  m.def("gemm_nt4_dynamic", [](int on) {
    static int cur = 0;
    const int prev = cur;
    if (on >= 0) pdo::gemm_nt4_set_dynamic(cur = on);
    return prev;
  }, py::arg("on") = -1, "gemm_nt4 tile order: 1 = dynamic per-XCD counters, 0 = static (default); returns the previous");
  m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("b"), py::arg("bias") = py::none(), py::arg("out") = py::none());
  m.def("gemm_nt_gelu", &gemm_nt_gelu, py::arg("a"), py::arg("b"), py::arg("bias"), py::arg("saved_grad") = false);
  m.def("gemm_nt_dgelu", &gemm_nt_dgelu, py::arg("a"), py::arg("b"), py::arg("pre"), py::arg("bias"),
        py::arg("db_out") = py::none(), py::arg("saved_grad") = false);
  m.def("bn_act_fwd", &bn_act_fwd);
  m.def("bn_act_bwd_pair", &bn_act_bwd_pair);
  m.def("bn_act_fwd_tiles_bnres", &bn_act_fwd_tiles_bnres);
  m.def("bn_act_fwd_tiles", &bn_act_fwd_tiles);
  m.def("conv_ok", &conv_ok);
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"),
        py::arg("with_stats") = false);
  m.def("conv_tile_rows", &conv_tile_rows);
  m.def("conv_stride2_add", &conv_stride2_add);
  m.def("stem_ok", &stem_ok);
  m.def("stem_tile_rows", &pdo::stem_tile_rows);
  m.def("stem_fwd", &stem_fwd, py::arg("x"), py::arg("w"), py::arg("with_stats") = true);
  m.def("stem_wgrad", &stem_wgrad, py::arg("dy"), py::arg("z"), py::arg("out") = py::none());
  m.def("conv_weight_t", &conv_weight_t);
  m.def("conv_weight_t_batched", &conv_weight_t_batched);
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("wt"), py::arg("C"), py::arg("R"), py::arg("S"),
        py::arg("H"), py::arg("W"), py::arg("stride"), py::arg("pad"), py::arg("add") = py::none());
  m.def("gemm_nt_add", &gemm_nt_add, py::arg("a"), py::arg("b"), py::arg("r"), py::arg("bias") = py::none(),
        py::arg("mask") = py::none());
  m.def("conv_dgrad_bn", &conv_dgrad_bn);
  m.def("conv_wgrad_mode", &pdo::conv_wgrad_mode);
  m.def("conv_wgrad_c64_mode", &pdo::conv_wgrad_c64_mode);
  m.def("bn_act_bwd_part", &bn_act_bwd_part);
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("R"), py::arg("S"), py::arg("stride"),
        py::arg("pad"), py::arg("out") = py::none());
  m.def("bn_act_bwd", &bn_act_bwd);
  m.def("maxpool3s2_fwd", &maxpool3s2_fwd);
  m.def("bn_relu_pool_fwd_tiles", &bn_relu_pool_fwd_tiles);
  m.def("pool_bn_bwd", &pool_bn_bwd, py::arg("dy"), py::arg("y"), py::arg("xsel"), py::arg("arg"), py::arg("x"),
        py::arg("mean"), py::arg("invstd"),
        py::arg("w"), py::arg("b"), py::arg("dw_into") = py::none(), py::arg("db_into") = py::none());
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("qkv"), py::arg("o"), py::arg("lse"), py::arg("n_head"),
        py::arg("with_bias_grad") = false, py::arg("db_out") = py::none());
  m.def("scale_", &scale_);
  m.def("scale_dev_", &scale_dev_);
  m.def("fold_zero", &fold_zero);
  m.def("flatten_scale", &flatten_scale);
  m.def("cast_scale_bf16_f32", &cast_scale_bf16_f32);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("device_info", &device_info);
  m.def("set_device", &set_device);
  m.def("ipc_get_handle", &ipc_get_handle);
  m.def("ipc_open_handle", &ipc_open_handle, py::arg("handle"), py::arg("nbytes"), py::arg("device"),
        py::arg("offset") = 0);
  m.def("can_access_peer", &can_access_peer);
  m.def("enable_peer_access", &enable_peer_access);
  m.attr("arch") = "gfx950";
}
