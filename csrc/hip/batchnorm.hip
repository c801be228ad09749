// SPDX-License-Identifier: Apache-2.0
// Training-mode BatchNorm fused with its consumers for NHWC (channels_last) bf16.
//
// ResNet-50 on MI355X spends ~a third of its step in MIOpen's BatchNorm plus
// the separate ReLU / residual-add / ReLU-backward elementwise kernels around
// it (profiles/resnet50_r1.md).  These kernels treat an NHWC activation as a
// row-major [M = N·H·W, C] matrix and do
//   forward:  stats pass (per-channel Σx, Σx² → mean, invstd; running stats)
//             + one elementwise pass  y = act(x·scale + shift [+ residual])
//   backward: stats pass (Σg, Σg·(x−mean), g = dy·[y>0]) + one elementwise
//             pass dx = w·invstd/M·(M·g − Σg − x̂·Σg·x̂)  [+ dresidual = g]
// Per-thread partial sums over a few hundred rows are merged with Chan's
// parallel-variance formula (count, mean, M2), so the variance does not
// suffer E[x²]−E[x]² cancellation over millions of rows.
#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int BN_THREADS = 256;
constexpr int BN_ROWS = 64;  // rows per block-iteration group (row threads × unroll)

// Grid: x = column chunks of 8 channels × (256 / RT) ... simplified: each block
// covers CB = 8·TX channels (TX threads across) and TY = 256/TX row threads.
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  if (nb == 0.f) return;
  const float nt = n + nb;
  const float d = meanb - mean;
  mean += d * (nb / nt);
  m2 += m2b + d * d * (n * nb / nt);
  n = nt;
}

// pass 1 (forward): per (row-group g, channel c) partial (count, mean, M2)
template <int TX>
__global__ __launch_bounds__(BN_THREADS) void bn_stats_kernel(const bf16* __restrict__ x, long long M, int C,
                                                              long long rows_per_group, float* __restrict__ part) {
  constexpr int TY = BN_THREADS / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int c8 = blockIdx.x * TX + tx;  // 8-channel chunk
  const int g = blockIdx.y;
  const long long r0 = (long long)g * rows_per_group;
  const long long r1 = r0 + rows_per_group < M ? r0 + rows_per_group : M;
  f32x8 s = {0, 0, 0, 0, 0, 0, 0, 0}, q = s;
  float n = 0.f;
  if (c8 * 8 < C) {
#pragma unroll 4
    for (long long r = r0 + ty; r < r1; r += TY) {
      f32x8 v = to_f32(*reinterpret_cast<const bf16x8*>(x + r * C + c8 * 8));
      s += v;
      q += v * v;
      n += 1.f;
    }
  }
  // thread-local (n, mean, M2) per channel, then merge across the TY row threads in LDS
  __shared__ float sn[BN_THREADS], sm[8][BN_THREADS], s2[8][BN_THREADS];
  sn[threadIdx.x] = n;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float mu = n > 0.f ? s[j] / n : 0.f;
    sm[j][threadIdx.x] = mu;
    s2[j][threadIdx.x] = n > 0.f ? fmaxf(q[j] - n * mu * mu, 0.f) : 0.f;
  }
  __syncthreads();
  if (ty == 0 && c8 * 8 < C) {
    float tn = sn[tx];
    float tm[8], t2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      tm[j] = sm[j][tx];
      t2[j] = s2[j][tx];
    }
    for (int k = 1; k < TY; ++k) {
      const int idx = k * TX + tx;
      const float nb = sn[idx];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float nn = tn;
        chan_merge(nn, tm[j], t2[j], nb, sm[j][idx], s2[j][idx]);
      }
      tn += nb;
    }
    float* p = part + ((size_t)g * C + c8 * 8) * 3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p[3 * j] = tn;
      p[3 * j + 1] = tm[j];
      p[3 * j + 2] = t2[j];
    }
  }
}

// pass 2 (forward): merge G partials per channel → mean, invstd, scale/shift;
// running stats update (unbiased variance, momentum).  A block owns FC
// channels; its FG group-lanes each merge G/FG partials, then an LDS merge.
// (One thread per channel looping over all G partials took 130 µs at C=64,
// G=512 — longer than the elementwise pass it feeds.)
constexpr int FC = 32, FG = 8;
__global__ __launch_bounds__(FC* FG) void bn_finalize_kernel(const float* __restrict__ part, int G, int C,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ b, float eps, float momentum,
                                                            float* __restrict__ running_mean,
                                                            float* __restrict__ running_var,
                                                            float* __restrict__ mean_out,
                                                            float* __restrict__ invstd_out,
                                                            float* __restrict__ scale_shift) {
  const int tx = threadIdx.x % FC, ty = threadIdx.x / FC;
  const int c = blockIdx.x * FC + tx;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C) {
    for (int g = ty; g < G; g += FG) {
      const float* p = part + ((size_t)g * C + c) * 3;
      chan_merge(n, mu, m2, p[0], p[1], p[2]);
    }
  }
  __shared__ float sn[FG][FC], sm[FG][FC], s2[FG][FC];
  sn[ty][tx] = n;
  sm[ty][tx] = mu;
  s2[ty][tx] = m2;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  for (int k = 1; k < FG; ++k) chan_merge(n, mu, m2, sn[k][tx], sm[k][tx], s2[k][tx]);
  const float var = n > 0.f ? m2 / n : 0.f;
  const float inv = rsqrtf(var + eps);
  mean_out[c] = mu;
  invstd_out[c] = inv;
  const float sc = w[c] * inv;
  scale_shift[c] = sc;
  scale_shift[C + c] = b[c] - mu * sc;
  if (running_mean) {
    const float unb = n > 1.f ? m2 / (n - 1.f) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

// pass 3 (forward): y = act(x·scale + shift [+ res])
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                       const float* __restrict__ ss, long long n8, int C8, int relu,
                                                       bf16* __restrict__ y) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const int c = (int)((unsigned)i % (unsigned)C8) * 8;  // n8 < 2^32 (host check)
    const int C = C8 * 8;
    f32x8 v = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
    const f32x8 sc = *reinterpret_cast<const f32x8*>(ss + c);
    const f32x8 sh = *reinterpret_cast<const f32x8*>(ss + C + c);
    v = v * sc + sh;
    if (res) v += to_f32(reinterpret_cast<const bf16x8*>(res)[i]);
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
    }
    reinterpret_cast<bf16x8*>(y)[i] = to_bf16(v);
  }
}

// backward pass 1: per (row-group, channel) partial Σg and Σg·(x−mean), g = dy·[y>0]
template <int TX>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_stats_kernel(const bf16* __restrict__ dy,
                                                                  const bf16* __restrict__ y,
                                                                  const bf16* __restrict__ x,
                                                                  const float* __restrict__ mean, long long M, int C,
                                                                  long long rows_per_group, int relu,
                                                                  float* __restrict__ part) {
  constexpr int TY = BN_THREADS / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int c8 = blockIdx.x * TX + tx;
  const int g = blockIdx.y;
  const long long r0 = (long long)g * rows_per_group;
  const long long r1 = r0 + rows_per_group < M ? r0 + rows_per_group : M;
  f32x8 s1 = {0, 0, 0, 0, 0, 0, 0, 0}, s2 = s1;
  if (c8 * 8 < C) {
    const f32x8 mu = *reinterpret_cast<const f32x8*>(mean + c8 * 8);
#pragma unroll 4
    for (long long r = r0 + ty; r < r1; r += TY) {
      const long long off = r * C + c8 * 8;
      f32x8 gv = to_f32(*reinterpret_cast<const bf16x8*>(dy + off));
      if (relu) {
        const f32x8 yv = to_f32(*reinterpret_cast<const bf16x8*>(y + off));
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = yv[j] > 0.f ? gv[j] : 0.f;
      }
      const f32x8 xv = to_f32(*reinterpret_cast<const bf16x8*>(x + off));
      s1 += gv;
      s2 += gv * (xv - mu);
    }
  }
  __shared__ float a[8][BN_THREADS], bsum[8][BN_THREADS];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j][threadIdx.x] = s1[j];
    bsum[j][threadIdx.x] = s2[j];
  }
  __syncthreads();
  if (ty == 0 && c8 * 8 < C) {
    float t1[8], t2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      t1[j] = 0.f;
      t2[j] = 0.f;
    }
    for (int k = 0; k < TY; ++k) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        t1[j] += a[j][k * TX + tx];
        t2[j] += bsum[j][k * TX + tx];
      }
    }
    float* p = part + ((size_t)g * C + c8 * 8) * 2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      p[2 * j] = t1[j];
      p[2 * j + 1] = t2[j];
    }
  }
}

// backward pass 2: per-channel totals → dgamma, dbeta and the dx coefficients
// (same FC×FG block shape as bn_finalize_kernel)
__global__ __launch_bounds__(FC* FG) void bn_bwd_finalize_kernel(const float* __restrict__ part, int G, int C,
                                                                long long M, const float* __restrict__ w,
                                                                const float* __restrict__ invstd,
                                                                float* __restrict__ dw, float* __restrict__ db,
                                                                float* __restrict__ coef) {
  const int tx = threadIdx.x % FC, ty = threadIdx.x / FC;
  const int c = blockIdx.x * FC + tx;
  float s1 = 0.f, s2 = 0.f;
  if (c < C) {
    for (int g = ty; g < G; g += FG) {
      s1 += part[((size_t)g * C + c) * 2];
      s2 += part[((size_t)g * C + c) * 2 + 1];
    }
  }
  __shared__ float a1[FG][FC], a2[FG][FC];
  a1[ty][tx] = s1;
  a2[ty][tx] = s2;
  __syncthreads();
  if (ty != 0 || c >= C) return;
  for (int k = 1; k < FG; ++k) {
    s1 += a1[k][tx];
    s2 += a2[k][tx];
  }
  const float inv = invstd[c];
  const float dgamma = s2 * inv;  // Σ g·x̂
  dw[c] = dgamma;
  db[c] = s1;
  const float k = w[c] * inv;
  // dx = k·g − k·s1/M − k·inv·dgamma/M·(x−mean)
  coef[c] = k;
  coef[C + c] = k * s1 / (float)M;
  coef[2 * C + c] = k * inv * dgamma / (float)M;
}

// backward pass 3: dx (and dres = g)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ y,
                                                           const bf16* __restrict__ x, const float* __restrict__ mean,
                                                           const float* __restrict__ coef, long long n8, int C8,
                                                           int relu, bf16* __restrict__ dx, bf16* __restrict__ dres) {
  const int C = C8 * 8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const int c = (int)((unsigned)i % (unsigned)C8) * 8;
    f32x8 gv = to_f32(reinterpret_cast<const bf16x8*>(dy)[i]);
    if (relu) {
      const f32x8 yv = to_f32(reinterpret_cast<const bf16x8*>(y)[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] = yv[j] > 0.f ? gv[j] : 0.f;
    }
    if (dres) reinterpret_cast<bf16x8*>(dres)[i] = to_bf16(gv);
    const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
    const f32x8 mu = *reinterpret_cast<const f32x8*>(mean + c);
    const f32x8 k = *reinterpret_cast<const f32x8*>(coef + c);
    const f32x8 k1 = *reinterpret_cast<const f32x8*>(coef + C + c);
    const f32x8 k2 = *reinterpret_cast<const f32x8*>(coef + 2 * C + c);
    reinterpret_cast<bf16x8*>(dx)[i] = to_bf16(k * gv - k1 - k2 * (xv - mu));
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
  // enough row groups for ≥ 2 blocks per CU, each covering ≥ 64 rows per row-thread pass
  int want = (512 + *gx - 1) / *gx;
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
  return gy * C * 3 + 2 * C;
}

int bn_fwd(const bf16* x, const bf16* res, const float* w, const float* b, float* running_mean, float* running_var,
           long long M, int C, float eps, float momentum, int relu, bf16* y, float* mean, float* invstd,
           float* scratch, hipStream_t st) {
  if (C % 8 != 0 || M * C / 8 >= (1ll << 32)) return -2;
  const int TX = pick_tx(C);
  int gx, gy;
  long long rpg;
  stats_grid(M, C, TX, &gx, &gy, &rpg);
  float* part = scratch;
  float* ss = scratch + (size_t)gy * C * 3;
  dim3 grid(gx, gy);
  if (TX == 32) bn_stats_kernel<32><<<grid, BN_THREADS, 0, st>>>(x, M, C, rpg, part);
  else if (TX == 16) bn_stats_kernel<16><<<grid, BN_THREADS, 0, st>>>(x, M, C, rpg, part);
  else bn_stats_kernel<8><<<grid, BN_THREADS, 0, st>>>(x, M, C, rpg, part);
  bn_finalize_kernel<<<(C + FC - 1) / FC, FC * FG, 0, st>>>(part, gy, C, w, b, eps, momentum, running_mean, running_var,
                                                       mean, invstd, ss);
  const long long n8 = M * C / 8;
  bn_apply_kernel<<<apply_grid(n8), 256, 0, st>>>(x, res, ss, n8, C / 8, relu, y);
  return 0;
}

int bn_bwd_scratch_floats(long long M, int C) {
  int gx, gy;
  long long rpg;
  stats_grid(M, C, pick_tx(C), &gx, &gy, &rpg);
  return gy * C * 2 + 3 * C;
}

int bn_bwd(const bf16* dy, const bf16* y, const bf16* x, const float* mean, const float* invstd, const float* w,
           long long M, int C, int relu, bf16* dx, bf16* dres, float* dw, float* db, float* scratch, hipStream_t st) {
  if (C % 8 != 0 || M * C / 8 >= (1ll << 32)) return -2;
  const int TX = pick_tx(C);
  int gx, gy;
  long long rpg;
  stats_grid(M, C, TX, &gx, &gy, &rpg);
  float* part = scratch;
  float* coef = scratch + (size_t)gy * C * 2;
  dim3 grid(gx, gy);
  if (TX == 32) bn_bwd_stats_kernel<32><<<grid, BN_THREADS, 0, st>>>(dy, y, x, mean, M, C, rpg, relu, part);
  else if (TX == 16) bn_bwd_stats_kernel<16><<<grid, BN_THREADS, 0, st>>>(dy, y, x, mean, M, C, rpg, relu, part);
  else bn_bwd_stats_kernel<8><<<grid, BN_THREADS, 0, st>>>(dy, y, x, mean, M, C, rpg, relu, part);
  bn_bwd_finalize_kernel<<<(C + FC - 1) / FC, FC * FG, 0, st>>>(part, gy, C, M, w, invstd, dw, db, coef);
  const long long n8 = M * C / 8;
  bn_bwd_apply_kernel<<<apply_grid(n8), 256, 0, st>>>(dy, y, x, mean, coef, n8, C / 8, relu, dx, dres);
  return 0;
}

}  // namespace pdo
