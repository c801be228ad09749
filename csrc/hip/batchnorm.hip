// SPDX-License-Identifier: Apache-2.0
// Training-mode BatchNorm fused with its consumers for NHWC (channels_last) bf16.
//
// ResNet-50 on MI355X spent ~a third of its step in MIOpen's BatchNorm plus
// the separate ReLU / residual-add / ReLU-backward elementwise kernels around
// it.  These kernels treat an NHWC activation as a row-major [M = N·H·W, C]
// matrix and do
//   forward:  stats    — per (row group, channel) Σd, Σd² of d = x − K (K = row
//                        0 of x, a per-channel shift that keeps E[d²]−E[d]²
//                        free of cancellation), partials [G][2][C]
//             finalize — one block per 8-channel chunk sums the G partials:
//                        mean, invstd, scale/shift, running statistics
//             apply    — y = act(x·scale + shift [+ residual])
//   backward: stats    — Σg, Σg·(x−mean), g = dy·[pre-activation > 0]
//             finalize — dgamma, dbeta and the dx coefficients
//             apply    — dx = k·g − k·Σg/M − k·invstd·Σg·x̂/M  [+ dresidual = g]
// Without a residual the ReLU mask is recomputed from x (bit-identical
// x·scale + shift through the same helper), so y is neither saved nor re-read.
// Per-block fp32 atomics into one [2C] buffer were tried instead of partials +
// finalize: 512 blocks hitting the same 16 L2 lines serialised the stats
// kernel (24 → 86 µs avg), far more than the finalize launch costs.
#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int BN_THREADS = 256;
constexpr int BN_ROWS = 64;

struct Affine {
  f32x8 sc, sh;
};

// scale/shift from (mean, invstd, w, b): shared by forward and backward so the
// recomputed pre-activation has the same bits as the forward's
__device__ __forceinline__ Affine affine8(const f32x8& mean, const f32x8& inv, const float* w, const float* b) {
  const f32x8 wv = *reinterpret_cast<const f32x8*>(w);
  const f32x8 bv = *reinterpret_cast<const f32x8*>(b);
  Affine a;
  a.sc = wv * inv;
  a.sh = bv - mean * a.sc;
  return a;
}

__device__ __forceinline__ f32x8 preact(const f32x8& x, const Affine& a) { return x * a.sc + a.sh; }

// forward stats: grid (column chunks of TX·8 channels, row groups)
template <int TX>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_kernel(const bf16* __restrict__ x, long long M, int C,
                                                              long long rows_per_group, float* __restrict__ part) {
  constexpr int TY = BN_THREADS / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int c8 = blockIdx.x * TX + tx;
  const long long r0 = (long long)blockIdx.y * rows_per_group;
  const long long r1 = r0 + rows_per_group < M ? r0 + rows_per_group : M;
  f32x8 s = {0, 0, 0, 0, 0, 0, 0, 0}, q = s;
  const bool live = c8 * 8 < C;
  if (live) {
    const f32x8 k = to_f32(*reinterpret_cast<const bf16x8*>(x + c8 * 8));
#pragma unroll 4
    for (long long r = r0 + ty; r < r1; r += TY) {
      const f32x8 d = to_f32(*reinterpret_cast<const bf16x8*>(x + r * C + c8 * 8)) - k;
      s += d;
      q += d * d;
    }
  }
  __shared__ f32x8 ls[BN_THREADS], lq[BN_THREADS];
  ls[threadIdx.x] = s;
  lq[threadIdx.x] = q;
  __syncthreads();
  // tree over the TY row threads of each channel chunk
#pragma unroll
  for (int h = TY / 2; h > 0; h >>= 1) {
    if (ty < h) {
      ls[threadIdx.x] += ls[threadIdx.x + h * TX];
      lq[threadIdx.x] += lq[threadIdx.x + h * TX];
    }
    __syncthreads();
  }
  if (ty == 0 && live) {
    float* p = part + (size_t)blockIdx.y * 2 * C + c8 * 8;
    *reinterpret_cast<f32x8*>(p) = ls[tx];
    *reinterpret_cast<f32x8*>(p + C) = lq[tx];
  }
}

// sum of the G partial rows [G][2][C] for 8 channels across one 256-thread
// block (4 waves: shuffle reduction, then LDS across waves)
constexpr int FIN_THREADS = 256;
__device__ __forceinline__ void block_sum_partials(const float* __restrict__ part, int G, int C, int c, f32x8& s,
                                                   f32x8& q) {
  s = f32x8{0, 0, 0, 0, 0, 0, 0, 0};
  q = s;
#pragma unroll 4
  for (int g = threadIdx.x; g < G; g += FIN_THREADS) {
    const float* p = part + (size_t)g * 2 * C + c;
    s += *reinterpret_cast<const f32x8*>(p);
    q += *reinterpret_cast<const f32x8*>(p + C);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] = wave_sum(s[j]);
    q[j] = wave_sum(q[j]);
  }
  __shared__ f32x8 ws[FIN_THREADS / WAVE], wq[FIN_THREADS / WAVE];
  const int w = threadIdx.x / WAVE;
  if ((threadIdx.x & (WAVE - 1)) == 0) {
    ws[w] = s;
    wq[w] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 1; k < FIN_THREADS / WAVE; ++k) {
      s += ws[k];
      q += wq[k];
    }
  }
}

// forward finalize: one block per 8-channel chunk → mean, invstd, scale/shift
// [2][C], running statistics (unbiased variance, momentum)
__global__ __launch_bounds__(FIN_THREADS) void bn_finalize_kernel(const float* __restrict__ part, int G, const bf16* x,
                                                           long long M, int C, const float* __restrict__ w,
                                                           const float* __restrict__ b, float eps, float momentum,
                                                           float* __restrict__ running_mean,
                                                           float* __restrict__ running_var,
                                                           float* __restrict__ mean_out,
                                                           float* __restrict__ invstd_out, float* __restrict__ ss) {
  const int c = blockIdx.x * 8;
  f32x8 s, q;
  block_sum_partials(part, G, C, c, s, q);
  if (threadIdx.x != 0) return;
  const float Minv = 1.f / (float)M;
  const f32x8 k = to_f32(*reinterpret_cast<const bf16x8*>(x + c));  // the shift used by the stats pass
  const f32x8 md = s * Minv;
  f32x8 var, inv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    var[j] = fmaxf(q[j] * Minv - md[j] * md[j], 0.f);
    inv[j] = rsqrtf(var[j] + eps);
  }
  const f32x8 mean = k + md;
  *reinterpret_cast<f32x8*>(mean_out + c) = mean;
  *reinterpret_cast<f32x8*>(invstd_out + c) = inv;
  const Affine a = affine8(mean, inv, w + c, b + c);
  *reinterpret_cast<f32x8*>(ss + c) = a.sc;
  *reinterpret_cast<f32x8*>(ss + C + c) = a.sh;
  if (running_mean) {
    const float unb = M > 1 ? (float)M / (float)(M - 1) : 1.f;
    f32x8 rm = *reinterpret_cast<const f32x8*>(running_mean + c);
    f32x8 rv = *reinterpret_cast<const f32x8*>(running_var + c);
    rm = (1.f - momentum) * rm + momentum * mean;
    rv = (1.f - momentum) * rv + (momentum * unb) * var;
    *reinterpret_cast<f32x8*>(running_mean + c) = rm;
    *reinterpret_cast<f32x8*>(running_var + c) = rv;
  }
}

// forward apply: y = act(x·scale + shift [+ res]).  HOIST: 256 % (C/8) == 0, so
// a lane's channel chunk never changes along the grid-stride loop.
// mask (optional): bit j of byte i = [y[8i + j] > 0], the ReLU mask the backward
// reads instead of y (1/16 of the bytes; relu = 2 there)
// rss (optional, with res): the residual is itself a BatchNorm's input — res·rscale
// + rshift is added (ResNet's downsample branch: its normalised output never
// exists in memory)
template <bool HOIST>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                       const float* __restrict__ ss, long long n8, int C, int relu,
                                                       bf16* __restrict__ y, unsigned char* __restrict__ mask,
                                                       const float* __restrict__ rss) {
  const int C8 = C / 8;
  const long long i0 = blockIdx.x * 256LL + threadIdx.x;
  const long long stride = (long long)gridDim.x * 256;
  Affine a, ra;
  auto load_aff = [&](int c) {
    a.sc = *reinterpret_cast<const f32x8*>(ss + c);
    a.sh = *reinterpret_cast<const f32x8*>(ss + C + c);
    if (rss) {
      ra.sc = *reinterpret_cast<const f32x8*>(rss + c);
      ra.sh = *reinterpret_cast<const f32x8*>(rss + C + c);
    }
  };
  if (HOIST) load_aff((int)(i0 % C8) * 8);
  for (long long i = i0; i < n8; i += stride) {
    if (!HOIST) load_aff((int)(i % C8) * 8);
    f32x8 v = preact(to_f32(reinterpret_cast<const bf16x8*>(x)[i]), a);
    if (res) {
      const f32x8 r = to_f32(reinterpret_cast<const bf16x8*>(res)[i]);
      v += rss ? preact(r, ra) : r;
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    const bf16x8 yb = to_bf16(v);
    reinterpret_cast<bf16x8*>(y)[i] = yb;
    if (mask) {
      unsigned bits = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) bits |= ((float)yb[j] > 0.f ? 1u : 0u) << j;
      mask[i] = (unsigned char)bits;
    }
  }
}

// g = dy · [pre-activation > 0]: from y when a residual was added (y > 0 ⇔
// v + res > 0), else recomputed from x through the forward's affine
__device__ __forceinline__ f32x8 relu_grad(const bf16* dy, const bf16* y, const f32x8& xv, const Affine& a,
                                           long long i, int relu) {
  f32x8 g = to_f32(reinterpret_cast<const bf16x8*>(dy)[i]);
  if (relu == 2) {  // y is the forward's ReLU bitmask (bn_apply_kernel)
    const unsigned bits = reinterpret_cast<const unsigned char*>(y)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = (bits >> j) & 1u ? g[j] : 0.f;
  } else if (relu) {
    if (y) {
      const f32x8 yv = to_f32(reinterpret_cast<const bf16x8*>(y)[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
    } else {
      const f32x8 v = preact(xv, a);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = v[j] > 0.f ? g[j] : 0.f;
    }
  }
  return g;
}

// backward stats: per (row group, channel) partial Σg and Σg·(x−mean)
template <int TX>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_stats_kernel(const bf16* __restrict__ dy,
                                                                  const bf16* __restrict__ y,
                                                                  const bf16* __restrict__ x,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ invstd,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ b, long long M, int C,
                                                                  long long rows_per_group, int relu,
                                                                  float* __restrict__ part) {
  constexpr int TY = BN_THREADS / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int c8 = blockIdx.x * TX + tx;
  const long long r0 = (long long)blockIdx.y * rows_per_group;
  const long long r1 = r0 + rows_per_group < M ? r0 + rows_per_group : M;
  f32x8 s1 = {0, 0, 0, 0, 0, 0, 0, 0}, s2 = s1;
  const bool live = c8 * 8 < C;
  if (live) {
    const f32x8 mu = *reinterpret_cast<const f32x8*>(mean + c8 * 8);
    const f32x8 inv = *reinterpret_cast<const f32x8*>(invstd + c8 * 8);
    const Affine a = affine8(mu, inv, w + c8 * 8, b + c8 * 8);
    const int C8 = C / 8;
#pragma unroll 4
    for (long long r = r0 + ty; r < r1; r += TY) {
      const long long i = r * C8 + c8;
      const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
      const f32x8 g = relu_grad(dy, y, xv, a, i, relu);
      s1 += g;
      s2 += g * (xv - mu);
    }
  }
  __shared__ f32x8 l1[BN_THREADS], l2[BN_THREADS];
  l1[threadIdx.x] = s1;
  l2[threadIdx.x] = s2;
  __syncthreads();
#pragma unroll
  for (int h = TY / 2; h > 0; h >>= 1) {
    if (ty < h) {
      l1[threadIdx.x] += l1[threadIdx.x + h * TX];
      l2[threadIdx.x] += l2[threadIdx.x + h * TX];
    }
    __syncthreads();
  }
  if (ty == 0 && live) {
    float* p = part + (size_t)blockIdx.y * 2 * C + c8 * 8;
    *reinterpret_cast<f32x8*>(p) = l1[tx];
    *reinterpret_cast<f32x8*>(p + C) = l2[tx];
  }
}

// the same for two BatchNorms fed one output gradient through one ReLU bitmask
// (ResNet's downsample block tail: bn3 over x, the downsample BatchNorm over r):
// g = dy ⊙ mask is read once, partials (Σg, Σg·(x−μ)) and (Σg, Σg·(r−μr))
template <int TX>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_stats_pair_kernel(
    const bf16* __restrict__ dy, const unsigned char* __restrict__ mask, const bf16* __restrict__ x,
    const float* __restrict__ mean, const bf16* __restrict__ r, const float* __restrict__ rmean, long long M, int C,
    long long rows_per_group, float* __restrict__ part, float* __restrict__ rpart) {
  constexpr int TY = BN_THREADS / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int c8 = blockIdx.x * TX + tx;
  const long long r0 = (long long)blockIdx.y * rows_per_group;
  const long long r1 = r0 + rows_per_group < M ? r0 + rows_per_group : M;
  f32x8 s1 = {0, 0, 0, 0, 0, 0, 0, 0}, s2 = s1, s3 = s1;
  const bool live = c8 * 8 < C;
  if (live) {
    const f32x8 mu = *reinterpret_cast<const f32x8*>(mean + c8 * 8);
    const f32x8 rmu = *reinterpret_cast<const f32x8*>(rmean + c8 * 8);
    const int C8 = C / 8;
    const Affine unused{};
#pragma unroll 4
    for (long long rr = r0 + ty; rr < r1; rr += TY) {
      const long long i = rr * C8 + c8;
      const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
      const f32x8 rv = to_f32(reinterpret_cast<const bf16x8*>(r)[i]);
      const f32x8 g = relu_grad(dy, reinterpret_cast<const bf16*>(mask), xv, unused, i, 2);
      s1 += g;
      s2 += g * (xv - mu);
      s3 += g * (rv - rmu);
    }
  }
  __shared__ f32x8 l1[BN_THREADS], l2[BN_THREADS], l3[BN_THREADS];
  l1[threadIdx.x] = s1;
  l2[threadIdx.x] = s2;
  l3[threadIdx.x] = s3;
  __syncthreads();
#pragma unroll
  for (int h = TY / 2; h > 0; h >>= 1) {
    if (ty < h) {
      l1[threadIdx.x] += l1[threadIdx.x + h * TX];
      l2[threadIdx.x] += l2[threadIdx.x + h * TX];
      l3[threadIdx.x] += l3[threadIdx.x + h * TX];
    }
    __syncthreads();
  }
  if (ty == 0 && live) {
    float* p = part + (size_t)blockIdx.y * 2 * C + c8 * 8;
    float* q = rpart + (size_t)blockIdx.y * 2 * C + c8 * 8;
    *reinterpret_cast<f32x8*>(p) = l1[tx];
    *reinterpret_cast<f32x8*>(p + C) = l2[tx];
    *reinterpret_cast<f32x8*>(q) = l1[tx];
    *reinterpret_cast<f32x8*>(q + C) = l3[tx];
  }
}

// backward finalize: one block per 8-channel chunk → dgamma = Σg·x̂, dbeta = Σg
// and the dx coefficients [3][C]: k = w·invstd, k1 = k·Σg/M,
// k2 = k·invstd·(Σg·x̂)/M with Σg·x̂ = invstd·Σg(x−μ)
__global__ __launch_bounds__(FIN_THREADS) void bn_bwd_finalize_kernel(const float* __restrict__ part, int G, long long M,
                                                               int C, const float* __restrict__ w,
                                                               const float* __restrict__ invstd,
                                                               float* __restrict__ dw, float* __restrict__ db,
                                                               int accumulate, float* __restrict__ coef) {
  const int c = blockIdx.x * 8;
  f32x8 s1, s2;
  block_sum_partials(part, G, C, c, s1, s2);
  if (threadIdx.x != 0) return;
  const float Minv = 1.f / (float)M;
  const f32x8 inv = *reinterpret_cast<const f32x8*>(invstd + c);
  const f32x8 wv = *reinterpret_cast<const f32x8*>(w + c);
  const f32x8 dgamma = s2 * inv;
  f32x8* dwp = reinterpret_cast<f32x8*>(dw + c);
  f32x8* dbp = reinterpret_cast<f32x8*>(db + c);
  *dwp = accumulate ? *dwp + dgamma : dgamma;  // accumulate: dw/db are the parameters' .grad
  *dbp = accumulate ? *dbp + s1 : s1;
  const f32x8 k = wv * inv;
  *reinterpret_cast<f32x8*>(coef + c) = k;
  *reinterpret_cast<f32x8*>(coef + C + c) = k * s1 * Minv;
  *reinterpret_cast<f32x8*>(coef + 2 * C + c) = k * inv * dgamma * Minv;
}

// backward apply: dx = k·g − k1 − k2·(x−μ) (and dres = g)
template <bool HOIST>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                                                           const bf16* __restrict__ x, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           const float* __restrict__ coef, long long n8, int C,
                                                           int relu, bf16* __restrict__ dx, bf16* __restrict__ dres) {
  const int C8 = C / 8;
  const long long i0 = blockIdx.x * 256LL + threadIdx.x;
  const long long stride = (long long)gridDim.x * 256;
  f32x8 mu, k, k1, k2;
  Affine a;
  auto load = [&](int c) {
    mu = *reinterpret_cast<const f32x8*>(mean + c);
    a = affine8(mu, *reinterpret_cast<const f32x8*>(invstd + c), w + c, b + c);
    k = *reinterpret_cast<const f32x8*>(coef + c);
    k1 = *reinterpret_cast<const f32x8*>(coef + C + c);
    k2 = *reinterpret_cast<const f32x8*>(coef + 2 * C + c);
  };
  if (HOIST) load((int)(i0 % C8) * 8);
  for (long long i = i0; i < n8; i += stride) {
    if (!HOIST) load((int)(i % C8) * 8);
    const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
    const f32x8 g = relu_grad(dy, y, xv, a, i, relu);
    if (dres) reinterpret_cast<bf16x8*>(dres)[i] = to_bf16(g);
    reinterpret_cast<bf16x8*>(dx)[i] = to_bf16(k * g - k1 - k2 * (xv - mu));
  }
}

// backward apply of the pair: dx = k·g − k1 − k2·(x−μ), dr likewise, g read once
template <bool HOIST>
__global__ __launch_bounds__(256) void bn_bwd_apply_pair_kernel(
    const bf16* __restrict__ dy, const unsigned char* __restrict__ mask, const bf16* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ coef, const bf16* __restrict__ r,
    const float* __restrict__ rmean, const float* __restrict__ rcoef, long long n8, int C, bf16* __restrict__ dx,
    bf16* __restrict__ dr) {
  const int C8 = C / 8;
  const long long i0 = blockIdx.x * 256LL + threadIdx.x;
  const long long stride = (long long)gridDim.x * 256;
  f32x8 mu, k, k1, k2, rmu, rk, rk1, rk2;
  auto load = [&](int c) {
    mu = *reinterpret_cast<const f32x8*>(mean + c);
    k = *reinterpret_cast<const f32x8*>(coef + c);
    k1 = *reinterpret_cast<const f32x8*>(coef + C + c);
    k2 = *reinterpret_cast<const f32x8*>(coef + 2 * C + c);
    rmu = *reinterpret_cast<const f32x8*>(rmean + c);
    rk = *reinterpret_cast<const f32x8*>(rcoef + c);
    rk1 = *reinterpret_cast<const f32x8*>(rcoef + C + c);
    rk2 = *reinterpret_cast<const f32x8*>(rcoef + 2 * C + c);
  };
  if (HOIST) load((int)(i0 % C8) * 8);
  const Affine unused{};
  for (long long i = i0; i < n8; i += stride) {
    if (!HOIST) load((int)(i % C8) * 8);
    const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
    const f32x8 rv = to_f32(reinterpret_cast<const bf16x8*>(r)[i]);
    const f32x8 g = relu_grad(dy, reinterpret_cast<const bf16*>(mask), xv, unused, i, 2);
    reinterpret_cast<bf16x8*>(dx)[i] = to_bf16(k * g - k1 - k2 * (xv - mu));
    reinterpret_cast<bf16x8*>(dr)[i] = to_bf16(rk * g - rk1 - rk2 * (rv - rmu));
  }
}

// forward finalize from the convolution epilogue's per-M-tile partials
// ([G][2][C]: Σv and Σ(v − mean_tile)² over the tile's rows, conv.hip): a
// block per 8 channels, 256 tile lanes each reading the 8 channels as one
// 32-B vector (G = 3 136 tiles at ResNet's 56 × 56 × 64: 13 per lane).  Two
// plain reductions (no sequential merge): mean = Σ sum_i / M, then
// M2 = Σ (M2_i + n_i·(mean_i − mean)²); both by wave butterflies + one LDS
// exchange (block_sum256) instead of an 8-level LDS tree.
// a block-wide f32x8 sum by wave butterflies and one LDS exchange of the 4 wave totals
// (fixed order: deterministic); red = 4 vectors of LDS
__device__ __forceinline__ f32x8 block_sum256(f32x8 v, f32x8* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += __shfl_xor(v[k], o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const f32x8 t = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return t;
}

// Large partial counts (G > 512: layer 1's 56 × 56 convolutions, the stem) are
// first merged per 256 partial rows by a 2-D grid — (Σ, M2 about the chunk
// mean) of 256·tile_rows rows — so the finalize's one block per 8 channels
// walks G / 256 rows instead of G (its serial per-lane loads dominated: 20-74
// µs per call at those G)
constexpr int MERGE_MIN_G = 512, MERGE_CHUNK = 256;
__device__ __forceinline__ f32x8 block_sum256(f32x8 v, f32x8* red);

__global__ __launch_bounds__(256) void bn_merge_tiles_kernel(const float* __restrict__ part, int G, int tile_rows,
                                                             long long M, int C, float* __restrict__ out) {
  const int c = blockIdx.x * 8, sidx = blockIdx.y;
  const int g0 = sidx * MERGE_CHUNK, g = g0 + threadIdx.x;
  __shared__ f32x8 red[4];
  const f32x8 z = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool live = g < G;
  const f32x8 sum = live ? *reinterpret_cast<const f32x8*>(part + (size_t)g * 2 * C + c) : z;
  const f32x8 m2 = live ? *reinterpret_cast<const f32x8*>(part + (size_t)g * 2 * C + C + c) : z;
  const long long r0 = (long long)g * tile_rows, cr0 = (long long)g0 * tile_rows;
  const float n = live ? (float)(M - r0 < tile_rows ? M - r0 : tile_rows) : 1.f;
  const long long cn = M - cr0 < (long long)MERGE_CHUNK * tile_rows ? M - cr0 : (long long)MERGE_CHUNK * tile_rows;
  const f32x8 S = block_sum256(sum, red);
  const f32x8 d = sum * (1.f / n) - S * (1.f / (float)cn);
  const f32x8 Q = block_sum256(live ? m2 + n * d * d : z, red);
  if (threadIdx.x == 0) {
    *reinterpret_cast<f32x8*>(out + (size_t)sidx * 2 * C + c) = S;
    *reinterpret_cast<f32x8*>(out + (size_t)sidx * 2 * C + C + c) = Q;
  }
}

__global__ __launch_bounds__(256) void bn_finalize_tiles_kernel(const float* __restrict__ part, int G, int tile_rows,
                                                                long long M, int C, const float* __restrict__ w,
                                                                const float* __restrict__ b, float eps,
                                                                float momentum, float* __restrict__ running_mean,
                                                                float* __restrict__ running_var,
                                                                float* __restrict__ mean_out,
                                                                float* __restrict__ invstd_out,
                                                                float* __restrict__ ss) {
  const int c = blockIdx.x * 8;
  __shared__ f32x8 red[4];
  const f32x8 z = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // 4 partial rows in flight per lane (the loop is latency-bound: G / 256 ≈
  // 1-13 rows per lane at ResNet-50's shapes)
  auto row = [&](int i, int off) { return i < G ? *reinterpret_cast<const f32x8*>(part + (size_t)i * 2 * C + off + c) : z; };
  f32x8 s = z;
  for (int i = threadIdx.x; i < G; i += 1024) {
    const f32x8 a0 = row(i, 0), a1 = row(i + 256, 0), a2 = row(i + 512, 0), a3 = row(i + 768, 0);
    s += (a0 + a1) + (a2 + a3);
  }
  const f32x8 mean = block_sum256(s, red) * (1.f / (float)M);
  auto dev = [&](int i) {  // M2_i + n_i·(mean_i − mean)² of partial row i (0 past G)
    if (i >= G) return z;
    const long long r0 = (long long)i * tile_rows;
    const float n = (float)(M - r0 < tile_rows ? M - r0 : tile_rows);
    const f32x8 d = row(i, 0) * (1.f / n) - mean;
    return row(i, C) + n * d * d;
  };
  f32x8 q = z;
  for (int i = threadIdx.x; i < G; i += 1024) q += (dev(i) + dev(i + 256)) + (dev(i + 512) + dev(i + 768));
  q = block_sum256(q, red);
  if (threadIdx.x != 0) return;
  f32x8 var, inv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    var[j] = fmaxf(q[j] / (float)M, 0.f);
    inv[j] = rsqrtf(var[j] + eps);
  }
  *reinterpret_cast<f32x8*>(mean_out + c) = mean;
  *reinterpret_cast<f32x8*>(invstd_out + c) = inv;
  const Affine a = affine8(mean, inv, w + c, b + c);
  *reinterpret_cast<f32x8*>(ss + c) = a.sc;
  *reinterpret_cast<f32x8*>(ss + C + c) = a.sh;
  if (running_mean) {
    const float unb = M > 1 ? (float)M / (float)(M - 1) : 1.f;
    f32x8 rm = *reinterpret_cast<const f32x8*>(running_mean + c);
    f32x8 rv = *reinterpret_cast<const f32x8*>(running_var + c);
    rm = (1.f - momentum) * rm + momentum * mean;
    rv = (1.f - momentum) * rv + (momentum * unb) * var;
    *reinterpret_cast<f32x8*>(running_mean + c) = rm;
    *reinterpret_cast<f32x8*>(running_var + c) = rv;
  }
}

// ---------------------------------------------------------------------------
// ResNet stem: BatchNorm + ReLU + 3×3 / stride-2 / pad-1 max-pool in one pass
// each way.  Forward reads the conv output x once and writes only the pooled
// activation, its window positions and the BatchNorm input at each maximum
// (xsel; the unfused pair wrote and re-read the full-resolution activation).
// A gradient reaches only window maxima, so the backward's statistics
// (Σg, Σg·(x − mean), g = dy·[y > 0]) are bn_bwd_stats over the POOLED tensors
// (dy, y, xsel: 1/4 of the pixels); its apply pass gathers the ≤ 4 window
// gradients per input pixel (maxpool3s2_bwd's gather) straight into the
// BatchNorm input gradient.  C / 8 must divide 256 (a lane's channel chunk is
// fixed along its loop).
typedef uint8_t u8x8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(256) void bn_relu_pool_fwd_kernel(const bf16* __restrict__ x, const float* __restrict__ ss,
                                                               int N, int H, int W, int C, int OH, int OW,
                                                               bf16* __restrict__ y, uint8_t* __restrict__ arg,
                                                               bf16* __restrict__ xsel) {
  // flat grid-stride over (n, oh, ow, c8): rows of OW·C8 chunks do not fill 256 lanes evenly
  const int C8 = C / 8;
  const int c8 = threadIdx.x % C8;
  Affine a;
  a.sc = *reinterpret_cast<const f32x8*>(ss + c8 * 8);
  a.sh = *reinterpret_cast<const f32x8*>(ss + C + c8 * 8);
  const int total = N * OH * OW * C8;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < total; j += gridDim.x * 256) {
    const int t = j / C8, ow = t % OW, t2 = t / OW, oh = t2 % OH, n = t2 / OH;
    const bf16* xn = x + (long long)n * H * W * C;
    f32x8 best, xb;
    u8x8 pos;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      xb[q] = 0.f;
      pos[q] = 0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = oh * 2 - 1 + kh;
      if (h < 0 || h >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = ow * 2 - 1 + kw;
        if (w < 0 || w >= W) continue;
        const f32x8 xv = to_f32(*reinterpret_cast<const bf16x8*>(xn + ((long long)h * W + w) * C + c8 * 8));
        f32x8 v = preact(xv, a);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
        v = to_f32(to_bf16(v));  // compare the bf16 activations, as the unfused max-pool does
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (v[q] > best[q]) {  // first maximum in scan order wins ties
            best[q] = v[q];
            xb[q] = xv[q];
            pos[q] = (uint8_t)(kh * 3 + kw);
          }
        }
      }
    }
    reinterpret_cast<bf16x8*>(y)[j] = to_bf16(best);  // j = ((n·OH + oh)·OW + ow)·C8 + c8
    reinterpret_cast<u8x8*>(arg)[j] = pos;
    reinterpret_cast<bf16x8*>(xsel)[j] = to_bf16(xb);  // exact: xb is a bf16 input value
  }
}

// backward apply: a thread per 2 × 2 input block (rows 2k, 2k+1, columns 2m,
// 2m+1) and 8 channels — exactly the windows (k | k+1, m | m+1) reach it, so
// each window's dy / position vector is loaded once for the four pixels
// (pixel (2k+a, 2m+b) takes window (k+i, m+j) for i ≤ a, j ≤ b, at position
// (2 − 2i + ... ) = (a + 1 − 2i)·3 + (b + 1 − 2j)); g = the summed window
// gradients, ReLU-masked; dx = k·g − k1 − k2·(x − μ).  One block per row pair.
__global__ __launch_bounds__(256) void pool_bn_bwd_apply_kernel(const bf16* __restrict__ dy,
                                                                const uint8_t* __restrict__ arg,
                                                                const bf16* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ wgt,
                                                                const float* __restrict__ bia,
                                                                const float* __restrict__ coef, int N, int H, int W,
                                                                int C, int OH, int OW, bf16* __restrict__ dx) {
  const int C8 = C / 8;
  const int KH = (H + 1) / 2, MW = (W + 1) / 2;
  const int c8 = threadIdx.x % C8;
  const f32x8 mu = *reinterpret_cast<const f32x8*>(mean + c8 * 8);
  const Affine a = affine8(mu, *reinterpret_cast<const f32x8*>(invstd + c8 * 8), wgt + c8 * 8, bia + c8 * 8);
  const f32x8 k = *reinterpret_cast<const f32x8*>(coef + c8 * 8);
  const f32x8 k1 = *reinterpret_cast<const f32x8*>(coef + C + c8 * 8);
  const f32x8 k2 = *reinterpret_cast<const f32x8*>(coef + 2 * C + c8 * 8);
  const int total = N * KH * MW * C8;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < total; j += gridDim.x * 256) {
    const int t = j / C8, m = t % MW, t2 = t / MW, kr = t2 % KH, n = t2 / KH;
    const bf16* xn = x + (long long)n * H * W * C;
    bf16* dxn = dx + (long long)n * H * W * C;
    const long long on = (long long)n * OH;
    // the four windows (k + i, m + jj); absent ones give no gradient
    f32x8 g[2][2];
    u8x8 p[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int oh = kr + i, ow = m + jj;
        if (oh < OH && ow < OW) {
          const long long o = ((on + oh) * OW + ow) * C8 + c8;
          g[i][jj] = to_f32(reinterpret_cast<const bf16x8*>(dy)[o]);
          p[i][jj] = reinterpret_cast<const u8x8*>(arg)[o];
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            g[i][jj][q] = 0.f;
            p[i][jj][q] = 255;
          }
        }
      }
#pragma unroll
    for (int ar = 0; ar < 2; ++ar) {
      const int h = 2 * kr + ar;
      if (h >= H) continue;
#pragma unroll
      for (int bc = 0; bc < 2; ++bc) {
        const int w = 2 * m + bc;
        if (w >= W) continue;
        f32x8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i <= ar; ++i)
#pragma unroll
          for (int jj = 0; jj <= bc; ++jj) {
            // window (kr + i, m + jj) starts at (2(kr + i) − 1, 2(m + jj) − 1)
            const uint8_t me = (uint8_t)((ar + 1 - 2 * i) * 3 + (bc + 1 - 2 * jj));
#pragma unroll
            for (int q = 0; q < 8; ++q) acc[q] += p[i][jj][q] == me ? g[i][jj][q] : 0.f;
          }
        const long long e = ((long long)h * W + w) * C8 + c8;
        const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(xn)[e]);
        const f32x8 v = preact(xv, a);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = v[q] > 0.f ? acc[q] : 0.f;
        reinterpret_cast<bf16x8*>(dxn)[e] = to_bf16(k * acc - k1 - k2 * (xv - mu));
      }
    }
  }
}

int pick_tx(int C) {
  const int c8 = C / 8;
  if (c8 >= 32) return 32;
  if (c8 >= 16) return 16;
  return 8;
}

void stats_grid(long long M, int C, int TX, int* gx, int* gy, long long* rpg) {
  *gx = (C / 8 + TX - 1) / TX;
  // ~8 blocks (32 waves) per CU so enough 16-B loads are in flight to cover
  // HBM latency (2 blocks per CU read at ~3.5 TB/s), each block ≥ BN_ROWS rows
  int want = (2048 + *gx - 1) / *gx;
  long long maxg = (M + BN_ROWS - 1) / BN_ROWS;
  if (want > maxg) want = (int)maxg;
  if (want < 1) want = 1;
  *gy = want;
  *rpg = (M + want - 1) / want;
}

unsigned apply_grid(long long n8) {
  long long b = (n8 + 255) / 256;
  return (unsigned)(b < 4096 ? b : 4096);
}

}  // namespace

int bn_fwd_scratch_floats(long long M, int C) {
  int gx, gy;
  long long rpg;
  stats_grid(M, C, pick_tx(C), &gx, &gy, &rpg);
  return gy * 2 * C + 2 * C;
}

int bn_fwd(const bf16* x, const bf16* res, const float* w, const float* b, float* running_mean, float* running_var,
           long long M, int C, float eps, float momentum, int relu, bf16* y, float* mean, float* invstd,
           float* scratch, hipStream_t st, unsigned char* mask) {
  if (C % 8 != 0 || M < 1 || M * C / 8 >= (1ll << 32)) return -2;
  const int TX = pick_tx(C);
  int gx, gy;
  long long rpg;
  stats_grid(M, C, TX, &gx, &gy, &rpg);
  float* part = scratch;
  float* ss = scratch + (size_t)gy * 2 * C;
  const dim3 grid(gx, gy);
  if (TX == 32) bn_stats_kernel<32><<<grid, BN_THREADS, 0, st>>>(x, M, C, rpg, part);
  else if (TX == 16) bn_stats_kernel<16><<<grid, BN_THREADS, 0, st>>>(x, M, C, rpg, part);
  else bn_stats_kernel<8><<<grid, BN_THREADS, 0, st>>>(x, M, C, rpg, part);
  bn_finalize_kernel<<<C / 8, FIN_THREADS, 0, st>>>(part, gy, x, M, C, w, b, eps, momentum, running_mean, running_var, mean,
                                             invstd, ss);
  const long long n8 = M * C / 8;
  const unsigned g = apply_grid(n8);
  if (256 % (C / 8) == 0) bn_apply_kernel<true><<<g, 256, 0, st>>>(x, res, ss, n8, C, relu, y, mask, nullptr);
  else bn_apply_kernel<false><<<g, 256, 0, st>>>(x, res, ss, n8, C, relu, y, mask, nullptr);
  return 0;
}

// BatchNorm forward whose statistics came with the producing convolution
// (conv.hip tile partials): finalize + apply, no statistics pass over x
int bn_tiles_merge_floats(int G, int C) {
  return G > MERGE_MIN_G ? (G + MERGE_CHUNK - 1) / MERGE_CHUNK * 2 * C : 0;
}

// finalize from [G][2][C] tile partials, pre-merged through `merge`
// (bn_tiles_merge_floats floats, or nullptr) when G is large
static void finalize_tiles(const float* part, int G, int tile_rows, long long M, int C, const float* w, const float* b,
                           float eps, float momentum, float* rm, float* rv, float* mean, float* invstd, float* ss,
                           float* merge, hipStream_t st) {
  if (merge && G > MERGE_MIN_G) {
    const int S = (G + MERGE_CHUNK - 1) / MERGE_CHUNK;
    bn_merge_tiles_kernel<<<dim3(C / 8, S), 256, 0, st>>>(part, G, tile_rows, M, C, merge);
    part = merge;
    G = S;
    tile_rows *= MERGE_CHUNK;
  }
  bn_finalize_tiles_kernel<<<C / 8, 256, 0, st>>>(part, G, tile_rows, M, C, w, b, eps, momentum, rm, rv, mean, invstd,
                                                  ss);
}

int bn_fwd_tiles(const float* tile_part, int G, int tile_rows, const bf16* x, const bf16* res, const float* w,
                 const float* b, float* running_mean, float* running_var, long long M, int C, float eps,
                 float momentum, int relu, bf16* y, float* mean, float* invstd, float* ss, hipStream_t st,
                 unsigned char* mask, float* merge) {
  if (C % 8 != 0 || M < 1 || M * C / 8 >= (1ll << 32) || G < 1) return -2;
  finalize_tiles(tile_part, G, tile_rows, M, C, w, b, eps, momentum, running_mean, running_var, mean, invstd, ss, merge,
                 st);
  const long long n8 = M * C / 8;
  const unsigned g = apply_grid(n8);
  if (256 % (C / 8) == 0) bn_apply_kernel<true><<<g, 256, 0, st>>>(x, res, ss, n8, C, relu, y, mask, nullptr);
  else bn_apply_kernel<false><<<g, 256, 0, st>>>(x, res, ss, n8, C, relu, y, mask, nullptr);
  return 0;
}

// y = act(BN(x) + BN_r(r)) with both BatchNorms' statistics from their
// producing convolutions: two finalizes, one apply pass (the residual
// BatchNorm's output is never written)
int bn_fwd_tiles_bnres(const float* tile_part, int G, int tile_rows, const bf16* x, const float* w, const float* b,
                       float* running_mean, float* running_var, float eps, float momentum, float* mean, float* invstd,
                       float* ss, const float* rtile_part, int rG, int rtile_rows, const bf16* r, const float* rw,
                       const float* rb, float* rrunning_mean, float* rrunning_var, float reps, float rmomentum,
                       float* rmean, float* rinvstd, float* rss, long long M, int C, int relu, bf16* y,
                       unsigned char* mask, hipStream_t st, float* merge) {
  if (C % 8 != 0 || M < 1 || M * C / 8 >= (1ll << 32) || G < 1 || rG < 1) return -2;
  // (one merge buffer serves both: the second merge is stream-ordered after the first finalize)
  finalize_tiles(tile_part, G, tile_rows, M, C, w, b, eps, momentum, running_mean, running_var, mean, invstd, ss, merge,
                 st);
  finalize_tiles(rtile_part, rG, rtile_rows, M, C, rw, rb, reps, rmomentum, rrunning_mean, rrunning_var, rmean, rinvstd,
                 rss, merge, st);
  const long long n8 = M * C / 8;
  const unsigned g = apply_grid(n8);
  if (256 % (C / 8) == 0) bn_apply_kernel<true><<<g, 256, 0, st>>>(x, r, ss, n8, C, relu, y, mask, rss);
  else bn_apply_kernel<false><<<g, 256, 0, st>>>(x, r, ss, n8, C, relu, y, mask, rss);
  return 0;
}

// BatchNorm backward whose statistics (Σg, Σg·(x − mean) partials [G][2][C])
// came with the input gradient that produced dy (conv.hip): finalize + apply
// backward partials [G][2][C] pre-summed per 256 rows (the same large-G
// serial-load problem as the forward finalize; plain sums, no merge formula)
__global__ __launch_bounds__(256) void bn_sum_rows_kernel(const float* __restrict__ part, int G, int C,
                                                          float* __restrict__ out) {
  const int c = blockIdx.x * 8, sidx = blockIdx.y, g = sidx * MERGE_CHUNK + threadIdx.x;
  __shared__ f32x8 red[4];
  const f32x8 z = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool live = g < G;
  const f32x8 a = block_sum256(live ? *reinterpret_cast<const f32x8*>(part + (size_t)g * 2 * C + c) : z, red);
  const f32x8 b = block_sum256(live ? *reinterpret_cast<const f32x8*>(part + (size_t)g * 2 * C + C + c) : z, red);
  if (threadIdx.x == 0) {
    *reinterpret_cast<f32x8*>(out + (size_t)sidx * 2 * C + c) = a;
    *reinterpret_cast<f32x8*>(out + (size_t)sidx * 2 * C + C + c) = b;
  }
}

static void bwd_finalize(const float* part, int G, long long M, int C, const float* w, const float* invstd, float* dw,
                         float* db, int accumulate, float* coef, float* merge, hipStream_t st) {
  if (merge && G > MERGE_MIN_G) {
    const int S = (G + MERGE_CHUNK - 1) / MERGE_CHUNK;
    bn_sum_rows_kernel<<<dim3(C / 8, S), 256, 0, st>>>(part, G, C, merge);
    part = merge;
    G = S;
  }
  bn_bwd_finalize_kernel<<<C / 8, FIN_THREADS, 0, st>>>(part, G, M, C, w, invstd, dw, db, accumulate, coef);
}

int bn_bwd_part(const float* part, int G, const bf16* dy, const bf16* y, const bf16* x, const float* mean,
                const float* invstd, const float* w, const float* b, long long M, int C, int relu, bf16* dx,
                bf16* dres, float* dw, float* db, int accumulate, float* coef, hipStream_t st, float* merge) {
  if (C % 8 != 0 || M < 1 || M * C / 8 >= (1ll << 32) || G < 1) return -2;
  bwd_finalize(part, G, M, C, w, invstd, dw, db, accumulate, coef, merge, st);
  const long long n8 = M * C / 8;
  const unsigned g = apply_grid(n8);
  if (256 % (C / 8) == 0)
    bn_bwd_apply_kernel<true><<<g, 256, 0, st>>>(dy, y, x, mean, invstd, w, b, coef, n8, C, relu, dx, dres);
  else
    bn_bwd_apply_kernel<false><<<g, 256, 0, st>>>(dy, y, x, mean, invstd, w, b, coef, n8, C, relu, dx, dres);
  return 0;
}

int bn_bwd_scratch_floats(long long M, int C) {
  int gx, gy;
  long long rpg;
  stats_grid(M, C, pick_tx(C), &gx, &gy, &rpg);
  return gy * 2 * C + 3 * C + bn_tiles_merge_floats(gy, C);
}

int bn_bwd(const bf16* dy, const bf16* y, const bf16* x, const float* mean, const float* invstd, const float* w,
           const float* b, long long M, int C, int relu, bf16* dx, bf16* dres, float* dw, float* db, int accumulate,
           float* scratch, hipStream_t st) {
  if (C % 8 != 0 || M < 1 || M * C / 8 >= (1ll << 32)) return -2;
  const int TX = pick_tx(C);
  int gx, gy;
  long long rpg;
  stats_grid(M, C, TX, &gx, &gy, &rpg);
  float* part = scratch;
  float* coef = scratch + (size_t)gy * 2 * C;
  const dim3 grid(gx, gy);
  if (TX == 32)
    bn_bwd_stats_kernel<32><<<grid, BN_THREADS, 0, st>>>(dy, y, x, mean, invstd, w, b, M, C, rpg, relu, part);
  else if (TX == 16)
    bn_bwd_stats_kernel<16><<<grid, BN_THREADS, 0, st>>>(dy, y, x, mean, invstd, w, b, M, C, rpg, relu, part);
  else
    bn_bwd_stats_kernel<8><<<grid, BN_THREADS, 0, st>>>(dy, y, x, mean, invstd, w, b, M, C, rpg, relu, part);
  bwd_finalize(part, gy, M, C, w, invstd, dw, db, accumulate, coef, coef + 3 * C, st);  // merge region follows coef
  const long long n8 = M * C / 8;
  const unsigned g = apply_grid(n8);
  if (256 % (C / 8) == 0)
    bn_bwd_apply_kernel<true><<<g, 256, 0, st>>>(dy, y, x, mean, invstd, w, b, coef, n8, C, relu, dx, dres);
  else
    bn_bwd_apply_kernel<false><<<g, 256, 0, st>>>(dy, y, x, mean, invstd, w, b, coef, n8, C, relu, dx, dres);
  return 0;
}

// the backward of two BatchNorms whose outputs were summed under one ReLU (the
// forward of bn_fwd_tiles_bnres): one statistics pass and one apply pass over
// (dy, mask, x, r) instead of two of each
int bn_bwd_scratch_pair_floats(long long M, int C) { return 2 * bn_bwd_scratch_floats(M, C); }

int bn_bwd_pair(const bf16* dy, const unsigned char* mask, const bf16* x, const float* mean, const float* invstd,
                const float* w, float* dw, float* db, int accumulate, const bf16* r, const float* rmean,
                const float* rinvstd, const float* rw, float* rdw, float* rdb, int raccumulate, long long M, int C,
                bf16* dx, bf16* dr, float* scratch, hipStream_t st) {
  if (C % 8 != 0 || M < 1 || M * C / 8 >= (1ll << 32)) return -2;
  const int TX = pick_tx(C);
  int gx, gy;
  long long rpg;
  stats_grid(M, C, TX, &gx, &gy, &rpg);
  float* part = scratch;
  float* rpart = part + (size_t)gy * 2 * C;
  float* coef = rpart + (size_t)gy * 2 * C;
  float* rcoef = coef + 3 * C;
  const dim3 grid(gx, gy);
  if (TX == 32)
    bn_bwd_stats_pair_kernel<32><<<grid, BN_THREADS, 0, st>>>(dy, mask, x, mean, r, rmean, M, C, rpg, part, rpart);
  else if (TX == 16)
    bn_bwd_stats_pair_kernel<16><<<grid, BN_THREADS, 0, st>>>(dy, mask, x, mean, r, rmean, M, C, rpg, part, rpart);
  else
    bn_bwd_stats_pair_kernel<8><<<grid, BN_THREADS, 0, st>>>(dy, mask, x, mean, r, rmean, M, C, rpg, part, rpart);
  // (scratch = 2 × bn_bwd_scratch_floats: a merge region follows rcoef; stream order lets both use it)
  bwd_finalize(part, gy, M, C, w, invstd, dw, db, accumulate, coef, rcoef + 3 * C, st);
  bwd_finalize(rpart, gy, M, C, rw, rinvstd, rdw, rdb, raccumulate, rcoef, rcoef + 3 * C, st);
  const long long n8 = M * C / 8;
  const unsigned g = apply_grid(n8);
  if (256 % (C / 8) == 0)
    bn_bwd_apply_pair_kernel<true><<<g, 256, 0, st>>>(dy, mask, x, mean, coef, r, rmean, rcoef, n8, C, dx, dr);
  else
    bn_bwd_apply_pair_kernel<false><<<g, 256, 0, st>>>(dy, mask, x, mean, coef, r, rmean, rcoef, n8, C, dx, dr);
  return 0;
}

// ---- stem BatchNorm + ReLU + max-pool (see bn_relu_pool_fwd_kernel) ----
static bool pool_bn_ok(int N, int H, int W, int C) {
  return C % 8 == 0 && 256 % (C / 8) == 0 && N > 0 && H > 0 && W > 0 && (long long)N * (H + 1) * (W + 1) * C < (1ll << 31);
}

int bn_relu_pool_fwd_tiles(const float* tile_part, int G, int tile_rows, const bf16* x, const float* w, const float* b,
                           float* running_mean, float* running_var, int N, int H, int W, int C, float eps,
                           float momentum, bf16* y, uint8_t* arg, bf16* xsel, float* mean, float* invstd, float* ss,
                           hipStream_t st, float* merge) {
  if (!pool_bn_ok(N, H, W, C) || G < 1) return -2;
  const long long M = (long long)N * H * W;
  finalize_tiles(tile_part, G, tile_rows, M, C, w, b, eps, momentum, running_mean, running_var, mean, invstd, ss, merge,
                 st);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int tot = N * OH * OW * (C / 8);
  bn_relu_pool_fwd_kernel<<<(unsigned)min((tot + 255) / 256, 8192), 256, 0, st>>>(x, ss, N, H, W, C, OH, OW, y, arg,
                                                                                 xsel);
  return 0;
}

int pool_bn_bwd_scratch_floats(int N, int H, int W, int C) {
  const long long Mp = (long long)N * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
  int gx, gy;
  long long rpg;
  stats_grid(Mp, C, pick_tx(C), &gx, &gy, &rpg);
  return gy * 2 * C + 3 * C + bn_tiles_merge_floats(gy, C);
}

int pool_bn_bwd(const bf16* dy, const bf16* y, const bf16* xsel, const uint8_t* arg, const bf16* x, const float* mean,
                const float* invstd, const float* w, const float* b, int N, int H, int W, int C, bf16* dx, float* dw,
                float* db, int accumulate, float* scratch, hipStream_t st) {
  if (!pool_bn_ok(N, H, W, C)) return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long long Mp = (long long)N * OH * OW;
  const int TX = pick_tx(C);
  int gx, gy;
  long long rpg;
  stats_grid(Mp, C, TX, &gx, &gy, &rpg);
  float* part = scratch;
  float* coef = scratch + (size_t)gy * 2 * C;
  const dim3 grid(gx, gy);
  // statistics over the pooled tensors (relu 1 with y: g = dy·[y > 0]; x = xsel)
  if (TX == 32) bn_bwd_stats_kernel<32><<<grid, BN_THREADS, 0, st>>>(dy, y, xsel, mean, invstd, w, b, Mp, C, rpg, 1, part);
  else if (TX == 16) bn_bwd_stats_kernel<16><<<grid, BN_THREADS, 0, st>>>(dy, y, xsel, mean, invstd, w, b, Mp, C, rpg, 1, part);
  else bn_bwd_stats_kernel<8><<<grid, BN_THREADS, 0, st>>>(dy, y, xsel, mean, invstd, w, b, Mp, C, rpg, 1, part);
  // ... normalised by the BatchNorm's full-resolution count
  bwd_finalize(part, gy, (long long)N * H * W, C, w, invstd, dw, db, accumulate, coef, coef + 3 * C, st);
  const int tot = N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  pool_bn_bwd_apply_kernel<<<(unsigned)min((tot + 255) / 256, 8192), 256, 0, st>>>(dy, arg, x, mean, invstd, w, b,
                                                                                  coef, N, H, W, C, OH, OW, dx);
  return 0;
}
}  // namespace pdo
