// SPDX-License-Identifier: Apache-2.0
// Host-side launch API of the paddle_operator_amd HIP kernels (gfx950).
// Raw pointers + hipStream_t only: no torch headers here, so each kernel TU
// compiles in seconds; `bind.cpp` adapts torch tensors to these calls.
// Return value: 0 ok, <0 unsupported shape (caller raises).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdo {
typedef __bf16 bf16;

// Destination of a column sum: columns [k·seg, (k+1)·seg) go to p[k] (≤ 3
// segments, seg % 4 == 0); acc = add into the existing bf16 values.
struct ColOut {
  bf16* p[3] = {nullptr, nullptr, nullptr};
  int seg = 1 << 30;
  int acc = 0;
  static ColOut one(bf16* o, int C) {
    ColOut c;
    c.p[0] = o;
    c.seg = C;
    return c;
  }
};

// layernorm.hip
int layernorm_fwd(const bf16* x, const bf16* r, const bf16* rb, const bf16* w, const bf16* b, bf16* h, bf16* y,
                  float* mean, float* rstd, int N, int C, float eps, hipStream_t st);
int layernorm_bwd_grid(int N);
// out: where dgamma | dbeta | (drbias) go (ColOut segments of C columns)
// reduce = false: only the partial rows are written (the caller reduces part later)
int layernorm_bwd(const bf16* dy, const bf16* x, const bf16* w, const float* mean, const float* rstd,
                  const bf16* dres, bf16* dx, float* part, float* scratch, const ColOut& out, bool rbias, int N,
                  int C, hipStream_t st, bool reduce = true);

// reduce.hip
int colsum_scratch_floats(int G, int C);
void colsum(const float* part, int G, int C, int ld, bf16* out, float* scratch, hipStream_t st);
void colsum(const float* part, int G, int C, int ld, const ColOut& out, float* scratch, hipStream_t st);
// A column sum to run later (deferred bias / norm-weight gradients): part [G][ld]
// f32 → co; scratch ≥ colsum_scratch_floats(G, C).  colsum_batched runs n of them
// in two launches per COLSUM_BATCH jobs (the jobs are passed as kernel arguments).
struct ColsumJob {
  const float* part;
  float* scratch;
  int G, C, ld;
  ColOut co;
};
constexpr int COLSUM_BATCH = 24;
struct ColsumBatch {
  int n;
  int l1[COLSUM_BATCH + 1], l2[COLSUM_BATCH + 1];
  ColsumJob j[COLSUM_BATCH];
};
int colsum_batched(const ColsumJob* jobs, int n, hipStream_t st);
int bias_grad_scratch_floats(long long N, int F);
int bias_grad(const bf16* dy, long long N, int F, bf16* db, float* scratch, hipStream_t st, int accumulate = 0);
// NHWC BatchNorm (+ReLU, +residual) training forward / backward (batchnorm.hip)
// conv.hip: NHWC implicit-GEMM convolutions (3×3 / strided 1×1, C % 64, Kout 64 or % 128)
int conv_supported(int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad);
int conv_fwd_tiles(long long M, int Kout);
int conv_fwd_tile_rows(int Kout);
int conv_fwd_nhwc(const bf16* x, int N, int H, int W, int C, const bf16* w, int Kout, int R, int S, int stride, int pad,
                  bf16* y, float* tile_stats, hipStream_t st);
int conv_weight_t(const bf16* w, bf16* wt, int Kout, int T, int C, hipStream_t st);
// BatchNorm whose output the convolution consumed: its backward statistics ride
// on the input gradient's epilogue (part: [conv_dgrad_tiles][2][C])
struct ConvBnBwd {
  const bf16* x;
  const float *mean, *invstd, *w, *b;
  float* part;
  int relu;
};
// convolution weight gradient on gemm_dw4's mainloop with the activation gathered per tap (gemm_dw4.hip)
int conv_wgrad_dw4_splits(int Kout, int TC, long long M);
// PDO_WGRAD_DW4 routing (1 on, 0 off; < 0 only reads); returns the previous mode
int conv_wgrad_mode(int mode);
// PDO_WGRAD_C64 routing (the all-taps 64-channel 3×3 weight gradient); < 0 only reads
int conv_wgrad_c64_mode(int mode);
int conv_wgrad_dw4(const bf16* dy, const bf16* x, int N, int H, int W, int C, int Kout, int R, int S, int stride,
                   int pad, float* part, int splits, hipStream_t st);
// Wᵀ [C][T·K] of each [K][T][C] segment (table: n × (offset, K, T, C) int32, device) in one launch;
// max_tiles = the largest segment's T·⌈K/64⌉·⌈C/64⌉
int conv_weight_t_batched(const bf16* src, bf16* dst, const int* table, int n, long long max_tiles, hipStream_t st);
int conv_dgrad_tiles(int N, int H, int W, int C, int R, int stride, int pad);
int conv_dgrad_nhwc(const bf16* dy, int N, int H, int W, int C, const bf16* wt, int Kout, int R, int S, int stride,
                    int pad, bf16* dx, hipStream_t st, const ConvBnBwd* bn = nullptr, const bf16* add = nullptr);
int bn_bwd_part(const float* part, int G, const bf16* dy, const bf16* y, const bf16* x, const float* mean,
                const float* invstd, const float* w, const float* b, long long M, int C, int relu, bf16* dx,
                bf16* dres, float* dw, float* db, int accumulate, float* coef, hipStream_t st,
                float* merge = nullptr);  // merge: bn_tiles_merge_floats(G, C) floats for a large G
long long conv_wgrad_scratch_floats(int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad);
int conv_wgrad_nhwc(const bf16* dy, const bf16* x, int N, int H, int W, int C, int Kout, int R, int S, int stride,
                    int pad, float* dw, int accumulate, float* scratch, hipStream_t st);
// dx[n][2a][2b] += add[n][a][b] (NHWC bf16): a compact 1×1 stride-2 input gradient joining dX
int conv_stride2_add(bf16* dx, const bf16* add, int N, int H, int W, int C, hipStream_t st);
// ResNet stem (7×7 / stride 2 / pad 3, 3 → Kout = 64 channels) as a space-to-depth
// 4×4 stride-1 convolution over a 16-channel image on the implicit GEMM (conv.hip)
int stem_supported(int N, int H, int W, int C, int Kout);
int stem_s2d(const bf16* x, int N, int H, int W, bf16* z, hipStream_t st);
int stem_weight(const bf16* w, bf16* w2, int Kout, hipStream_t st);
int stem_fwd(const bf16* z, int N, int IH, int IW, const bf16* w2, int Kout, bf16* y, float* tile_stats,
             hipStream_t st);
long long stem_wgrad_scratch_floats(int N, int IH, int IW, int Kout);
int stem_tile_rows();              // rows per BatchNorm statistics tile of stem_fwd
int stem_fwd_tiles(long long M);
int stem_wgrad(const bf16* dy, const bf16* z, int N, int IH, int IW, int Kout, float* dw, int accumulate,
               float* scratch, hipStream_t st);
int bn_fwd_tiles(const float* tile_part, int G, int tile_rows, const bf16* x, const bf16* res, const float* w,
                 const float* b, float* running_mean, float* running_var, long long M, int C, float eps,
                 float momentum, int relu, bf16* y, float* mean, float* invstd, float* ss, hipStream_t st, unsigned char* mask = nullptr,
                 float* merge = nullptr);
// floats of the pre-merge buffer the *_tiles BatchNorm forwards take for G partial rows (0: none needed)
int bn_tiles_merge_floats(int G, int C);
// act(BN(x) + BN_r(r)): both from their convolutions' tile statistics, one apply pass
int bn_fwd_tiles_bnres(const float* tile_part, int G, int tile_rows, const bf16* x, const float* w, const float* b,
                       float* running_mean, float* running_var, float eps, float momentum, float* mean, float* invstd,
                       float* ss, const float* rtile_part, int rG, int rtile_rows, const bf16* r, const float* rw,
                       const float* rb, float* rrunning_mean, float* rrunning_var, float reps, float rmomentum,
                       float* rmean, float* rinvstd, float* rss, long long M, int C, int relu, bf16* y,
                       unsigned char* mask, hipStream_t st, float* merge = nullptr);
int bn_fwd_scratch_floats(long long M, int C);
// backward of bn_fwd_tiles_bnres's pair (ReLU bitmask `mask`): dx, dr and both
// BatchNorms' dgamma / dbeta, one statistics and one apply pass
int bn_bwd_scratch_pair_floats(long long M, int C);
int bn_bwd_pair(const bf16* dy, const unsigned char* mask, const bf16* x, const float* mean, const float* invstd,
                const float* w, float* dw, float* db, int accumulate, const bf16* r, const float* rmean,
                const float* rinvstd, const float* rw, float* rdw, float* rdb, int raccumulate, long long M, int C,
                bf16* dx, bf16* dr, float* scratch, hipStream_t st);
// ResNet stem BatchNorm + ReLU + 3×3/2 max-pool fused (batchnorm.hip): forward from
// the conv's tile statistics → pooled y and window positions; backward → dx of the
// BatchNorm input and dgamma / dbeta (scratch: pool_bn_bwd_scratch_floats)
int bn_relu_pool_fwd_tiles(const float* tile_part, int G, int tile_rows, const bf16* x, const float* w, const float* b,
                           float* running_mean, float* running_var, int N, int H, int W, int C, float eps,
                           float momentum, bf16* y, uint8_t* arg, bf16* xsel, float* mean, float* invstd, float* ss,
                           hipStream_t st, float* merge = nullptr);
int pool_bn_bwd_scratch_floats(int N, int H, int W, int C);
int pool_bn_bwd(const bf16* dy, const bf16* y, const bf16* xsel, const uint8_t* arg, const bf16* x, const float* mean,
                const float* invstd, const float* w, const float* b, int N, int H, int W, int C, bf16* dx, float* dw,
                float* db, int accumulate, float* scratch, hipStream_t st);
int bn_fwd(const bf16* x, const bf16* res, const float* w, const float* b, float* running_mean, float* running_var,
           long long M, int C, float eps, float momentum, int relu, bf16* y, float* mean, float* invstd,
           float* scratch, hipStream_t st, unsigned char* mask = nullptr);
int bn_bwd_scratch_floats(long long M, int C);
// y may be null: the ReLU mask is then recomputed from x (only valid without a residual)
int bn_bwd(const bf16* dy, const bf16* y, const bf16* x, const float* mean, const float* invstd, const float* w,
           const float* b, long long M, int C, int relu, bf16* dx, bf16* dres, float* dw, float* db, int accumulate,
           float* scratch, hipStream_t st);
// ResNet stem max-pool 3×3/2 pad 1, NHWC bf16 (pool.hip); arg = uint8 window position
int maxpool3s2_fwd(const bf16* x, int N, int H, int W, int C, bf16* y, uint8_t* arg, hipStream_t st);
int maxpool3s2_bwd(const bf16* dy, const uint8_t* arg, int N, int H, int W, int C, bf16* dx, hipStream_t st);
// global average pool backward: dy [N][C] → dx NHWC [N][HW][C] = dy / HW
int gap_bwd(const bf16* dy, int N, int HW, int C, bf16* dx, hipStream_t st);
// gemm_dw.hip: C[M][N] (+)= Aᵀ·B for token-major A [T][M], B [T][N] (weight gradients)
// splits: 0 = shape unsupported; ws: splits·M·N bf16 when splits > 1
int gemm_dw_splits(long long T, int M, int N);
int gemm_dw(const bf16* A, const bf16* B, long long T, int M, int N, int lda, int ldb, bf16* C, int ldc,
            int accumulate, bf16* ws, int splits, hipStream_t st);
// gemm_dw4.hip: the same contract on the 4-wave / 128 × 128-per-wave mainloop (-2: split count unsupported)
int gemm_dw4(const bf16* A, const bf16* B, long long T, int M, int N, int lda, int ldb, bf16* C, int ldc,
             int accumulate, bf16* ws, int splits, hipStream_t st, int variant);
// which mainloop gemm_dw() runs: 0 = 8-wave (gemm_dw.hip), 1.. = 4-wave variant impl - 1
void gemm_dw_set_impl(int impl);
int gemm_dw_get_impl();
// transpose.hip: out[C][R] = in[R][C], R and C multiples of 64
// gemm_nt.hip: C[M][N] = A[M][K]·B[N][K]ᵀ with a fused epilogue
// (0 plain, 1 +bias, 2 C = pre-activation & Y = gelu(C + bias),
//  3 C = (A·Bᵀ)⊙gelu'(Y + bias) & fp32 column partials [gemm_nt_dbias_rows(M, K)][N])
int gemm_nt_ok(int M, int N, int K, int lda, int ldb, int ldc);
// EPI 7 / 8 / 9 (the 4-wave mainloop's epilogues) apply to this product
int gemm_nt_epi_ok(int M, int N, int K);
// rows per BatchNorm partial row of EPI 9 (gemm_nt with the statistics epilogue)
int gemm_nt_stats_rows(int K);
int gemm_nt_dbias_rows(int M, int K);
int gemm_nt(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
            const bf16* bias, bf16* Y, int ldy, float* dbias_part, hipStream_t st);
// gemm_nt4.hip: the same contract on the 4-wave / 128 × 128-per-wave mainloop
int gemm_nt4(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
             const bf16* bias, bf16* Y, int ldy, float* dbias_part, hipStream_t st);
// (N % 256 = 128 allowed: half-width last tile column)
// which mainloop gemm_nt() runs: 0 = 8-wave ring (gemm_nt.hip), 1 = 4-wave
// (gemm_nt4.hip, default)
void gemm_nt_set_impl(int impl);
// gemm_nt4 tile order: 1 = dynamic per-XCD counters, 0 = static (default; experiments only)
void gemm_nt4_set_dynamic(int on);
int gemm_nt_get_impl();
int transpose_bf16(const bf16* in, bf16* out, int R, int C, hipStream_t st);
// every matrix of a table in one launch: table = n × {first tile, src offset, dst
// offset, R, C} int64 (device), elements relative to src / dst; tiles = Σ (R/64)(C/64)
int transpose_bf16_batched(const bf16* src, bf16* dst, const long long* table, int n, long long tiles,
                           hipStream_t st);
int splitk_add(const bf16* part, int s, long long n, bf16* out, int accumulate, hipStream_t st);

// gelu.hip
int bias_gelu_fwd(const bf16* x, const bf16* b, bf16* y, long long N, int F, hipStream_t st);
int bias_gelu_bwd_groups(long long N, int F);
int bias_gelu_bwd(const bf16* dy, const bf16* x, const bf16* b, bf16* dx, float* part, float* scratch, bf16* db,
                  long long N, int F, hipStream_t st, int accumulate = 0);

// xent.hip
int xent_fwd(const bf16* logits, const int64_t* tgt, float* row_loss, float* lse, float* stats, int N, int Vp, int V,
             hipStream_t st);
// xent.hip: stats + dlogits (dloss = 1, scaled by inv_cnt) in place, one kernel; loss = mean over valid targets
int xent_fused(bf16* logits, const int64_t* tgt, const float* inv_cnt, float* row_loss, float* loss, int N, int Vp,
               int V, hipStream_t st);
int xent_bwd(const bf16* logits, const int64_t* tgt, const float* lse, const float* dloss, const float* stats,
             bf16* dlogits, int N, int Vp, int V, hipStream_t st);

// embed.hip
int embed_fwd(const int64_t* idx, const bf16* wte, const bf16* wpe, bf16* y, int B, int S, int C, hipStream_t st);
int embed_bwd(const bf16* dy, const int64_t* idx, float* acc, bf16* dwte, bf16* dwpe, int B, int S, int C, int Vp,
              int P, hipStream_t st);
// part: embed_sorted_part_floats(B·S, C) fp32 scratch (partials of runs that cross segments)
int embed_sorted_part_floats(int N, int C);
int embed_bwd_sorted(const bf16* dy, const int64_t* keys, const int64_t* perm, bf16* dwte, bf16* dwpe, float* part,
                     int B, int S, int C, int Vp, int P, int accumulate, hipStream_t st);
int sgd_flat(float* w, const float* g, float* buf, const float* decay_chunks, long long n, float lr, float mom,
             float wd, float grad_scale, hipStream_t st);
int cast_f32_bf16(const float* in, bf16* out, long long n, hipStream_t st);

// optim.hip
int sumsq(const bf16* g, long long n, float* part, int part_cap, float scale, float* out, hipStream_t st);
void adamw_set_variant(int v);
// Σ g² per fixed chunk (elements [k·chunk, (k+1)·chunk)) for chunks [k0, k1) → part[k]
int sumsq_chunks(const bf16* g, long long n, long long chunk, int k0, int k1, float* part, hipStream_t st);
// out[0] = scale² · Σ part[0..K), in a fixed order
int sumsq_total(const float* part, int K, float scale, float* out, hipStream_t st);
int adamw_flat(bf16* p, const bf16* g, float* master, float* m1, float* m2, const float* decay_chunks,
               const float* normsq, long long n, float lr, float b1, float b2, float eps, float wd, float bc1,
               float bc2, float grad_scale, float clip, hipStream_t st);

// attention.hip  (qkv: [B, S, 3, H, D] bf16; o: [B, S, H, D]; lse: [B, H, S] f32)
int attn_fwd(const bf16* qkv, bf16* o, float* lse, int B, int S, int H, int D, float scale, hipStream_t st);
// dbias_part (optional): fp32 [B·S/128][3·H·64] column partial sums of dqkv
// (the QKV bias gradient before its final reduction)
int attn_bwd(const bf16* dout, const bf16* qkv, const bf16* o, const float* lse, float* delta, bf16* dqkv, int B,
             int S, int H, int D, float scale, hipStream_t st, float* dbias_part = nullptr);

// bucket.hip (DDP helpers).  bucket_copy: dtype 0 = bf16, 1 = f32; dev_meta is
// n × {ptr, numel, offset} (int64) in device memory; flatten: flat[off+k] = scale·t[k],
// else t[k] = flat[off+k]
int bucket_copy(int dtype, bool flatten, void* flat, long long total, int n, void* dev_meta, float scale,
                hipStream_t st);
int cast_scale_bf16_f32(const bf16* src, float* dst, long long n, float s, hipStream_t st);
int scale_bf16(bf16* x, long long n, float s, hipStream_t st);
int scale_dev_bf16(bf16* x, long long n, const float* s, hipStream_t st);
// y = bf16(y + s·x) with the fp32 scale read on device
int axpy_dev_bf16(bf16* y, const bf16* x, long long n, const float* s, hipStream_t st);
int fold_zero_bf16(bf16* g, bf16* h, long long n, hipStream_t st);

}  // namespace pdo
