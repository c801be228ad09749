// SPDX-License-Identifier: Apache-2.0
// Fused AdamW over the flat parameter arena + gradient global-norm (gfx950).
// One pass: bf16 grad → ×(grad_scale · clip_coef) → fp32 moments/master →
// bf16 compute copy.  The clip coefficient is read from device memory
// (written by `sumsq`), so clipping costs no host synchronisation.
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace pdo {

__global__ __launch_bounds__(256) void sumsq_part_kernel(const bf16* __restrict__ g, long long nvec,
                                                         float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    f32x8 v = to_f32(reinterpret_cast<const bf16x8*>(g)[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void sumsq_final_kernel(const float* __restrict__ part, int G, float scale2,
                                                           float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < G; i += 1024) s += part[i];
  s = block_sum<16>(s, red);
  if (threadIdx.x == 0) out[0] = s * scale2;
}

// one block per fixed chunk of the gradient: part[k0 + b] = Σ g² over chunk k0 + b
// (chunk boundaries independent of which call computes them, so partials taken
// bucket by bucket as each all-reduce lands sum to the same bits as one pass)
__global__ __launch_bounds__(256) void sumsq_chunk_kernel(const bf16* __restrict__ g, long long nvec, long long cvec,
                                                          int k0, float* __restrict__ part) {
  __shared__ float red[4];
  const int k = k0 + blockIdx.x;
  const long long lo = (long long)k * cvec, hi = lo + cvec < nvec ? lo + cvec : nvec;
  float s = 0.f;
  for (long long i = lo + threadIdx.x; i < hi; i += 256) {
    f32x8 v = to_f32(reinterpret_cast<const bf16x8*>(g)[i]);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) part[k] = s;
}

__global__ __launch_bounds__(256) void adamw_kernel(bf16* __restrict__ p, const bf16* __restrict__ g,
                                                    float* __restrict__ master, float* __restrict__ m1,
                                                    float* __restrict__ m2, const float* __restrict__ decay_chunks,
                                                    const float* __restrict__ normsq, long long nvec, float lr,
                                                    float b1, float b2, float eps, float wd, float inv_bc1,
                                                    float inv_sqrt_bc2, float grad_scale, float clip) {
  float coef = grad_scale;
  if (clip > 0.f) {
    const float norm = sqrtf(normsq[0]);
    coef *= fminf(1.f, clip / (norm + 1e-6f));
  }
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    const float dec = decay_chunks[i >> 7];  // 1024 elements per chunk = 128 vectors
    f32x8 gr = to_f32(reinterpret_cast<const bf16x8*>(g)[i]) * coef;
    f32x4* mp = reinterpret_cast<f32x4*>(master) + 2 * i;
    f32x4* ap = reinterpret_cast<f32x4*>(m1) + 2 * i;
    f32x4* vp = reinterpret_cast<f32x4*>(m2) + 2 * i;
    f32x4 w0 = mp[0], w1 = mp[1], a0 = ap[0], a1 = ap[1], v0 = vp[0], v1 = vp[1];
    f32x8 w = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
    f32x8 a = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    f32x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    a = b1 * a + (1.f - b1) * gr;
    v = b2 * v + (1.f - b2) * gr * gr;
    const float shrink = 1.f - lr * wd * dec;
    f32x8 upd;
#pragma unroll
    for (int j = 0; j < 8; ++j) upd[j] = (a[j] * inv_bc1) / (sqrtf(v[j]) * inv_sqrt_bc2 + eps);
    w = w * shrink - lr * upd;
    mp[0] = f32x4{w[0], w[1], w[2], w[3]};
    mp[1] = f32x4{w[4], w[5], w[6], w[7]};
    ap[0] = f32x4{a[0], a[1], a[2], a[3]};
    ap[1] = f32x4{a[4], a[5], a[6], a[7]};
    vp[0] = f32x4{v[0], v[1], v[2], v[3]};
    vp[1] = f32x4{v[4], v[5], v[6], v[7]};
    reinterpret_cast<bf16x8*>(p)[i] = to_bf16(w);
  }
}

// The same update with the hardware square root and reciprocal (v_sqrt_f32,
// v_rcp_f32: ≈ 1 ulp) instead of the IEEE-exact expansions, VEC consecutive
// 8-element vectors per lane per iteration with every load issued before any
// math (VEC = 2: 32 B of gradient and 64 B of each state array per lane).
template <int VEC>
__global__ __launch_bounds__(256) void adamw_fast_kernel(bf16* __restrict__ p, const bf16* __restrict__ g,
                                                         float* __restrict__ master, float* __restrict__ m1,
                                                         float* __restrict__ m2, const float* __restrict__ decay_chunks,
                                                         const float* __restrict__ normsq, long long ngroup, float lr,
                                                         float b1, float b2, float eps, float wd, float inv_bc1,
                                                         float inv_sqrt_bc2, float grad_scale, float clip) {
  float coef = grad_scale;
  if (clip > 0.f) {
    const float norm = sqrtf(normsq[0]);
    coef *= fminf(1.f, clip / (norm + 1e-6f));
  }
  const long long stride = (long long)gridDim.x * 256;
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q < ngroup; q += stride) {
    const long long i0 = q * VEC;
    bf16x8 gb[VEC];
    f32x4 w[VEC][2], a[VEC][2], v[VEC][2];
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const long long i = i0 + u;
      gb[u] = reinterpret_cast<const bf16x8*>(g)[i];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        w[u][h] = reinterpret_cast<const f32x4*>(master)[2 * i + h];
        a[u][h] = reinterpret_cast<const f32x4*>(m1)[2 * i + h];
        v[u][h] = reinterpret_cast<const f32x4*>(m2)[2 * i + h];
      }
    }
    const float shrink = 1.f - lr * wd * decay_chunks[i0 >> 7];  // 128 vectors per chunk; VEC | 128
#pragma unroll
    for (int u = 0; u < VEC; ++u) {
      const long long i = i0 + u;
      const f32x8 gr = to_f32(gb[u]) * coef;
      f32x8 wo;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 ah = a[u][h], vh = v[u][h], wh = w[u][h];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float gj = gr[4 * h + j];
          ah[j] = b1 * ah[j] + (1.f - b1) * gj;
          vh[j] = b2 * vh[j] + (1.f - b2) * gj * gj;
          const float den = __builtin_amdgcn_sqrtf(vh[j]) * inv_sqrt_bc2 + eps;
          wh[j] = wh[j] * shrink - lr * (ah[j] * inv_bc1) * __builtin_amdgcn_rcpf(den);
          wo[4 * h + j] = wh[j];
        }
        reinterpret_cast<f32x4*>(master)[2 * i + h] = wh;
        reinterpret_cast<f32x4*>(m1)[2 * i + h] = ah;
        reinterpret_cast<f32x4*>(m2)[2 * i + h] = vh;
      }
      reinterpret_cast<bf16x8*>(p)[i] = to_bf16(wo);
    }
  }
}

// Momentum SGD over a flat fp32 arena (ResNet-50, workloads/resnet.py): one
// pass, g' = g·grad_scale + wd·decay·w, buf = mom·buf + g', w −= lr·buf —
// the four bulk torch ops of the reference formula in one read of (w, g, buf)
// and one write of (w, buf)
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                  float* __restrict__ buf, const float* __restrict__ decay_chunks,
                                                  long long n4, float lr, float mom, float wd, float grad_scale) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const float dec = decay_chunks[i >> 8];  // 1024 elements per chunk = 256 f32x4
    const f32x4 gi = reinterpret_cast<const f32x4*>(g)[i] * grad_scale;
    f32x4 wi = reinterpret_cast<const f32x4*>(w)[i];
    f32x4 b = reinterpret_cast<const f32x4*>(buf)[i];
    b = mom * b + (gi + (wd * dec) * wi);
    wi = wi - lr * b;
    reinterpret_cast<f32x4*>(buf)[i] = b;
    reinterpret_cast<f32x4*>(w)[i] = wi;
  }
}

int sgd_flat(float* w, const float* g, float* buf, const float* decay_chunks, long long n, float lr, float mom,
             float wd, float grad_scale, hipStream_t st) {
  if (n % 1024) return -2;
  sgd_kernel<<<stream_grid(n / 4, 256), 256, 0, st>>>(w, g, buf, decay_chunks, n / 4, lr, mom, wd, grad_scale);
  return 0;
}

int sumsq(const bf16* g, long long n, float* part, int part_cap, float scale, float* out, hipStream_t st) {
  if (n % 8) return -2;
  int G = stream_grid(n / 8, 256);
  if (G > part_cap) G = part_cap;
  sumsq_part_kernel<<<G, 256, 0, st>>>(g, n / 8, part);
  sumsq_final_kernel<<<1, 1024, 0, st>>>(part, G, scale * scale, out);
  return 0;
}

int sumsq_chunks(const bf16* g, long long n, long long chunk, int k0, int k1, float* part, hipStream_t st) {
  if (k1 == k0) return 0;
  if (n % 8 || chunk % 8 || k1 < k0) return -2;
  sumsq_chunk_kernel<<<k1 - k0, 256, 0, st>>>(g, n / 8, chunk / 8, k0, part);
  return 0;
}

int sumsq_total(const float* part, int K, float scale, float* out, hipStream_t st) {
  sumsq_final_kernel<<<1, 1024, 0, st>>>(part, K, scale * scale, out);
  return 0;
}

// 2 (default) = fast math, one vector per lane: 1812.5 µs (5.75 TB/s) vs
// 1864.8 µs (5.59 TB/s) for 1 = the IEEE-exact kernel; 3 = fast math with two
// consecutive vectors per lane, 2269.4 µs (tools/adamw_probe.py, 355 M
// elements, median of 5 interleaved; profiles/r5_adamw_resnet_graph.md).
// PDO_ADAMW overrides; set_adamw_variant for the probe.
static int g_adamw = [] {
  const char* e = getenv("PDO_ADAMW");
  return e && *e ? atoi(e) : 2;
}();
void adamw_set_variant(int v) { g_adamw = v; }

int adamw_flat(bf16* p, const bf16* g, float* master, float* m1, float* m2, const float* decay_chunks,
               const float* normsq, long long n, float lr, float b1, float b2, float eps, float wd, float bc1,
               float bc2, float grad_scale, float clip, hipStream_t st) {
  if (n % 1024) return -2;
  const long long nvec = n / 8;
  const float ib1 = 1.f / bc1, isb2 = 1.f / sqrtf(bc2);
  if (g_adamw == 2) {
    adamw_fast_kernel<1><<<stream_grid(nvec, 256), 256, 0, st>>>(p, g, master, m1, m2, decay_chunks, normsq, nvec,
                                                                 lr, b1, b2, eps, wd, ib1, isb2, grad_scale, clip);
  } else if (g_adamw == 3) {
    adamw_fast_kernel<2><<<stream_grid(nvec / 2, 256), 256, 0, st>>>(p, g, master, m1, m2, decay_chunks, normsq,
                                                                     nvec / 2, lr, b1, b2, eps, wd, ib1, isb2,
                                                                     grad_scale, clip);
  } else {
    adamw_kernel<<<stream_grid(nvec, 256), 256, 0, st>>>(p, g, master, m1, m2, decay_chunks, normsq, nvec, lr, b1, b2,
                                                          eps, wd, ib1, isb2, grad_scale, clip);
  }
  return 0;
}

}  // namespace pdo
