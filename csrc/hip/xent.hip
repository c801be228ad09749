// SPDX-License-Identifier: Apache-2.0
// Softmax cross-entropy over a padded vocabulary (gfx950).
// Forward: one 256-thread block per row, single pass with an online
// (max, sum-exp) pair per thread over 16-B vectors, block combine → lse and the
// row loss; padded columns (>= V) are masked.  The mean over valid targets is
// reduced deterministically by a one-block kernel that also stores the count
// for backward.  Backward writes dlogits = (softmax - onehot) * dloss / count
// in place over the logits buffer (one read + one write of [N, Vp]).
// (Measured alternative, not kept: one fused pass holding each row in
// registers, dlogits written in the forward — 4.6 ms vs these two passes'
// 3.6 ms at [65536, 50304]: with ≤ 1 resident 50k-column row per CU the load,
// reduce and store phases serialise.)
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace pdo {

__global__ __launch_bounds__(256) void xent_fwd_kernel(const bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       float* __restrict__ row_loss, float* __restrict__ lse_out,
                                                       int Vp, int V) {
  __shared__ float red_m[4], red_s[4];
  const int row = blockIdx.x;
  const bf16x8* lv = reinterpret_cast<const bf16x8*>(logits + (size_t)row * Vp);
  const int nv = Vp >> 3;
  float m = -INFINITY, s = 0.f;
  auto acc = [&](bf16x8 raw, int i) {
    f32x8 v = to_f32(raw);
    const int c0 = i * 8;
    float vm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c0 + j >= V) v[j] = -INFINITY;
      vm = fmaxf(vm, v[j]);
    }
    if (vm > m) {
      s *= __expf(m - vm);
      m = vm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
  };
  int i = threadIdx.x;
  for (; i + 3 * 256 < nv; i += 4 * 256) {  // four loads in flight per thread
    const bf16x8 a0 = lv[i], a1 = lv[i + 256], a2 = lv[i + 512], a3 = lv[i + 768];
    acc(a0, i);
    acc(a1, i + 256);
    acc(a2, i + 512);
    acc(a3, i + 768);
  }
  for (; i < nv; i += 256) acc(lv[i], i);
  // wave combine of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red_m[w] = m;
    red_s[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red_m[0];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, red_m[i]);
    float S = 0.f;
    for (int i = 0; i < 4; ++i) S += red_m[i] == -INFINITY ? 0.f : red_s[i] * __expf(red_m[i] - M);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const int64_t t = tgt[row];
    row_loss[row] = (t >= 0 && t < V) ? lse - (float)logits[(size_t)row * Vp + t] : 0.f;
  }
}

// loss = sum(row_loss) / count(valid targets); stats[0]=loss, stats[1]=count
__global__ __launch_bounds__(1024) void xent_mean_kernel(const float* __restrict__ row_loss,
                                                         const int64_t* __restrict__ tgt, int N, int V,
                                                         float* __restrict__ stats) {
  __shared__ float red[16];
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < N; i += 1024) {
    s += row_loss[i];
    c += (tgt[i] >= 0 && tgt[i] < V) ? 1.f : 0.f;
  }
  s = block_sum<16>(s, red);
  c = block_sum<16>(c, red);
  if (threadIdx.x == 0) {
    stats[1] = c;
    stats[0] = c > 0.f ? s / c : 0.f;
  }
}

__global__ __launch_bounds__(256) void xent_bwd_kernel(const bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                       const float* __restrict__ lse, const float* __restrict__ dloss,
                                                       const float* __restrict__ stats, bf16* __restrict__ dlogits,
                                                       int Vp, int V) {
  const int row = blockIdx.x;
  const float L = lse[row];
  const int64_t t = tgt[row];
  const float cnt = stats[1];
  const float scale = (t >= 0 && t < V && cnt > 0.f) ? dloss[0] / cnt : 0.f;
  const bf16x8* lv = reinterpret_cast<const bf16x8*>(logits + (size_t)row * Vp);
  bf16x8* dv = reinterpret_cast<bf16x8*>(dlogits + (size_t)row * Vp);
  const int nv = Vp >> 3;
  auto grad = [&](bf16x8 raw, int i) {
    const f32x8 v = to_f32(raw);
    const int c0 = i * 8;
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float p = c < V ? __expf(v[j] - L) : 0.f;
      if (c == t) p -= 1.f;
      o[j] = p * scale;
    }
    dv[i] = to_bf16(o);
  };
  // four 16-B loads in flight per thread before the first use: one per thread
  // left the row pass latency-bound (≈ 5.2 TB/s for the read + write stream)
  int i = threadIdx.x;
  for (; i + 3 * 256 < nv; i += 4 * 256) {
    const bf16x8 a0 = lv[i], a1 = lv[i + 256], a2 = lv[i + 512], a3 = lv[i + 768];
    grad(a0, i);
    grad(a1, i + 256);
    grad(a2, i + 512);
    grad(a3, i + 768);
  }
  for (; i < nv; i += 256) grad(lv[i], i);
}

// Forward statistics AND dlogits in one kernel, for dloss = 1 (ops._LMHeadXentFn
// scales the downstream dX / dW by the real dloss): per row, pass 1 streams the
// logits once for (max, sum-exp) → lse and the row loss, pass 2 streams the same
// row again — from the XCD's L2 / the MALL, the 100 KB row was read microseconds
// before — and writes (softmax − onehot) / count in place.  HBM sees one read and
// one write of [N, Vp] instead of the two kernels' two reads and one write.
// inv_cnt: 1 / (number of valid targets), precomputed on device.
__global__ __launch_bounds__(256) void xent_fused_kernel(bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                         const float* __restrict__ inv_cnt, float* __restrict__ row_loss,
                                                         int Vp, int V) {
  __shared__ float red_m[4], red_s[4], lse_sh;
  const int row = blockIdx.x;
  const bf16x8* lv = reinterpret_cast<const bf16x8*>(logits + (size_t)row * Vp);
  const int nv = Vp >> 3;
  float m = -INFINITY, s = 0.f;
  auto acc = [&](bf16x8 raw, int i) {
    f32x8 v = to_f32(raw);
    const int c0 = i * 8;
    float vm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c0 + j >= V) v[j] = -INFINITY;
      vm = fmaxf(vm, v[j]);
    }
    if (vm > m) {
      s *= __expf(m - vm);
      m = vm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
  };
  int i = threadIdx.x;
  for (; i + 3 * 256 < nv; i += 4 * 256) {
    const bf16x8 a0 = lv[i], a1 = lv[i + 256], a2 = lv[i + 512], a3 = lv[i + 768];
    acc(a0, i);
    acc(a1, i + 256);
    acc(a2, i + 512);
    acc(a3, i + 768);
  }
  for (; i < nv; i += 256) acc(lv[i], i);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red_m[w] = m;
    red_s[w] = s;
  }
  __syncthreads();
  const int64_t t = tgt[row];
  if (threadIdx.x == 0) {
    float M = red_m[0];
    for (int k = 1; k < 4; ++k) M = fmaxf(M, red_m[k]);
    float S = 0.f;
    for (int k = 0; k < 4; ++k) S += red_m[k] == -INFINITY ? 0.f : red_s[k] * __expf(red_m[k] - M);
    const float lse = M + __logf(S);
    lse_sh = lse;
    row_loss[row] = (t >= 0 && t < V) ? lse - (float)logits[(size_t)row * Vp + t] : 0.f;
  }
  __syncthreads();  // also orders the target logit's read before pass 2 overwrites it
  const float L = lse_sh;
  const float scale = (t >= 0 && t < V) ? inv_cnt[0] : 0.f;
  bf16x8* dv = reinterpret_cast<bf16x8*>(logits + (size_t)row * Vp);
  auto grad = [&](bf16x8 raw, int k) {
    const f32x8 v = to_f32(raw);
    const int c0 = k * 8;
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float p = c < V ? __expf(v[j] - L) : 0.f;
      if (c == t) p -= 1.f;
      o[j] = p * scale;
    }
    dv[k] = to_bf16(o);
  };
  i = threadIdx.x;
  for (; i + 3 * 256 < nv; i += 4 * 256) {
    const bf16x8 a0 = lv[i], a1 = lv[i + 256], a2 = lv[i + 512], a3 = lv[i + 768];
    grad(a0, i);
    grad(a1, i + 256);
    grad(a2, i + 512);
    grad(a3, i + 768);
  }
  for (; i < nv; i += 256) grad(lv[i], i);
}

// The same row pass with the row held in registers: 512 threads × RV vectors
// of 8 (RV = 13: rows of up to 53,248 columns, GPT-2's 50,304) — the logits
// are read from HBM once instead of twice (statistics pass, then the dlogits
// pass re-reading them), and the row max comes first so each element takes one
// exp for the sum and one for its gradient (no running rescale).
template <int RV>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void xent_fused_reg_kernel(bf16* __restrict__ logits,
                                                             const int64_t* __restrict__ tgt,
                                                             const float* __restrict__ inv_cnt,
                                                             float* __restrict__ row_loss, int Vp, int V) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  bf16x8* lv = reinterpret_cast<bf16x8*>(logits + (size_t)row * Vp);
  const int nv = Vp >> 3;
  bf16x8 r[RV];
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int i = threadIdx.x + 512 * k;
    if (i < nv) r[k] = lv[i];
  }
  const int64_t t = tgt[row];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int i = threadIdx.x + 512 * k;
    if (i < nv) {
      const f32x8 v = to_f32(r[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (8 * i + j < V) m = fmaxf(m, v[j]);
    }
  }
  const float M = block_max<8>(m, red);
  float s = 0.f, tl = 0.f;
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int i = threadIdx.x + 512 * k;
    if (i < nv) {
      const f32x8 v = to_f32(r[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * i + j;
        if (c < V) s += __expf(v[j] - M);
        if (c == t) tl = v[j];
      }
    }
  }
  const float S = block_sum<8>(s, red);
  const float T = block_sum<8>(tl, red);  // the target logit (one lane holds it)
  const float L = M + __logf(S);
  const bool valid = t >= 0 && t < V;
  if (threadIdx.x == 0) row_loss[row] = valid ? L - T : 0.f;
  const float scale = valid ? inv_cnt[0] : 0.f;
#pragma unroll
  for (int k = 0; k < RV; ++k) {
    const int i = threadIdx.x + 512 * k;
    if (i < nv) {
      const f32x8 v = to_f32(r[k]);
      f32x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = 8 * i + j;
        float p = c < V ? __expf(v[j] - L) : 0.f;
        if (c == t) p -= 1.f;
        o[j] = p * scale;
      }
      lv[i] = to_bf16(o);
    }
  }
}

// loss = Σ row_loss · inv_cnt
__global__ __launch_bounds__(1024) void xent_sum_kernel(const float* __restrict__ row_loss, int N,
                                                        const float* __restrict__ inv_cnt, float* __restrict__ loss) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < N; i += 1024) s += row_loss[i];
  s = block_sum<16>(s, red);
  if (threadIdx.x == 0) loss[0] = s * inv_cnt[0];
}

int xent_fused(bf16* logits, const int64_t* tgt, const float* inv_cnt, float* row_loss, float* loss, int N, int Vp,
               int V, hipStream_t st) {
  if (Vp % 8) return -2;
  // register-resident rows where they fit (2530 vs 2888 µs for the two-read
  // kernel at 65536 × 50304, round 5); the two-read kernel above that width
  if (Vp / 8 <= 512 * 13)
    xent_fused_reg_kernel<13><<<N, 512, 0, st>>>(logits, tgt, inv_cnt, row_loss, Vp, V);
  else
    xent_fused_kernel<<<N, 256, 0, st>>>(logits, tgt, inv_cnt, row_loss, Vp, V);
  xent_sum_kernel<<<1, 1024, 0, st>>>(row_loss, N, inv_cnt, loss);
  return 0;
}

int xent_fwd(const bf16* logits, const int64_t* tgt, float* row_loss, float* lse, float* stats, int N, int Vp, int V,
             hipStream_t st) {
  if (Vp % 8) return -2;
  xent_fwd_kernel<<<N, 256, 0, st>>>(logits, tgt, row_loss, lse, Vp, V);
  xent_mean_kernel<<<1, 1024, 0, st>>>(row_loss, tgt, N, V, stats);
  return 0;
}

int xent_bwd(const bf16* logits, const int64_t* tgt, const float* lse, const float* dloss, const float* stats,
             bf16* dlogits, int N, int Vp, int V, hipStream_t st) {
  if (Vp % 8) return -2;
  xent_bwd_kernel<<<N, 256, 0, st>>>(logits, tgt, lse, dloss, stats, dlogits, Vp, V);
  return 0;
}

}  // namespace pdo
