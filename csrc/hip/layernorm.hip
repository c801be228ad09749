// LayerNorm forward/backward (optionally fused with the residual add) for
// gfx950.  One wave per row: a row of C bf16 is held in registers as VPL
// vectors of 8 (16-B loads), statistics are two-pass in registers (exact
// mean, then centred variance), reductions are 64-lane shuffles.  Backward
// computes dx per row and accumulates dgamma/dbeta per lane in registers over
// a grid-stride row loop; the 4 waves of a block combine through LDS and the
// per-block partials are summed by `colsum_kernel` (deterministic, no atomics).
#include "common.h"
#include "kernels.h"

namespace pdo {

template <int VPL, bool ADD>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                     const bf16* __restrict__ w, const bf16* __restrict__ b,
                                                     bf16* __restrict__ h, bf16* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int N, int C, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const size_t base = (size_t)row * C;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + base);
  const bf16x8* rr = reinterpret_cast<const bf16x8*>(r + base);
  const int C8 = C >> 3;
  f32x8 v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c8 = lane + i * 64;
    if (c8 < C8) {
      v[i] = to_f32(xr[c8]);
      if (ADD) v[i] += to_f32(rr[c8]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    } else {
      v[i] = f32x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  const float inv_c = 1.f / (float)C;
  const float mean = wave_sum(s) * inv_c;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c8 = lane + i * 64;
    if (c8 < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) * inv_c + eps);
  const bf16x8* wr = reinterpret_cast<const bf16x8*>(w);
  const bf16x8* br = reinterpret_cast<const bf16x8*>(b);
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c8 = lane + i * 64;
    if (c8 < C8) {
      if (ADD) reinterpret_cast<bf16x8*>(h + base)[c8] = to_bf16(v[i]);
      f32x8 wf = to_f32(wr[c8]), bf = to_f32(br[c8]);
      f32x8 o = (v[i] - mean) * rstd * wf + bf;
      reinterpret_cast<bf16x8*>(y + base)[c8] = to_bf16(o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <int VPL, bool ADD>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                     const bf16* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const bf16* __restrict__ dres,
                                                     bf16* __restrict__ dx, float* __restrict__ part, int N, int C) {
  __shared__ float red[4 * 2 * 64 * 8 * VPL];  // per wave: dw,db partial of its columns
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int C8 = C >> 3;
  const float inv_c = 1.f / (float)C;
  f32x8 wv[VPL], adw[VPL], adb[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c8 = lane + i * 64;
    wv[i] = c8 < C8 ? to_f32(reinterpret_cast<const bf16x8*>(w)[c8]) : f32x8{0, 0, 0, 0, 0, 0, 0, 0};
    adw[i] = f32x8{0, 0, 0, 0, 0, 0, 0, 0};
    adb[i] = f32x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const int nw = gridDim.x * 4;
  for (int row = blockIdx.x * 4 + wid; row < N; row += nw) {
    const size_t base = (size_t)row * C;
    const float mu = mean[row], rs = rstd[row];
    f32x8 xh[VPL], g[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c8 = lane + i * 64;
      if (c8 < C8) {
        f32x8 d = to_f32(reinterpret_cast<const bf16x8*>(dy + base)[c8]);
        f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x + base)[c8]);
        xh[i] = (xv - mu) * rs;
        g[i] = d * wv[i];
        adw[i] += d * xh[i];
        adb[i] += d;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
        }
      }
    }
    s1 = wave_sum(s1) * inv_c;
    s2 = wave_sum(s2) * inv_c;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c8 = lane + i * 64;
      if (c8 < C8) {
        f32x8 o = (g[i] - s1 - xh[i] * s2) * rs;
        if (ADD) o += to_f32(reinterpret_cast<const bf16x8*>(dres + base)[c8]);
        reinterpret_cast<bf16x8*>(dx + base)[c8] = to_bf16(o);
      }
    }
  }
  // combine the 4 waves: wave 0..3 stores, then each thread sums a slice
  float* my = red + wid * (2 * 64 * 8 * VPL);
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      my[(i * 64 + lane) * 8 + j] = adw[i][j];
      my[64 * 8 * VPL + (i * 64 + lane) * 8 + j] = adb[i][j];
    }
  __syncthreads();
  const int per = 2 * 64 * 8 * VPL;
  for (int k = threadIdx.x; k < per; k += 256) {
    float t = red[k] + red[per + k] + red[2 * per + k] + red[3 * per + k];
    // k < 64*8*VPL: dw column k ; else db column k - 64*8*VPL
    const int half = 64 * 8 * VPL;
    const int col = k < half ? k : k - half;
    if (col < C) part[(size_t)blockIdx.x * 2 * C + (k < half ? 0 : C) + col] = t;
  }
}

// out[c] = sum_g part[g*stride + c] ; 16 waves per 64 columns
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ part, int G, int C, int stride,
                                                      bf16* __restrict__ out_bf16, float* __restrict__ out_f32) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < C) {
    for (int g = wid; g < G; g += 16) s += part[(size_t)g * stride + col];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][lane];
    if (col < C) {
      if (out_bf16) out_bf16[col] = (bf16)t;
      if (out_f32) out_f32[col] = t;
    }
  }
}

void colsum(const float* part, int G, int C, int stride, bf16* out_bf16, float* out_f32, hipStream_t st) {
  colsum_kernel<<<(C + 63) / 64, 1024, 0, st>>>(part, G, C, stride, out_bf16, out_f32);
}

#define LN_DISPATCH(VPL_, ...)                  \
  switch (VPL_) {                               \
    case 1: { constexpr int V = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int V = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int V = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int V = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int V = 5; __VA_ARGS__; } break; \
    case 6: { constexpr int V = 6; __VA_ARGS__; } break; \
    case 8: { constexpr int V = 8; __VA_ARGS__; } break; \
    default: return -1;                         \
  }

static int vpl_for(int C) {
  int v = (C + 511) / 512;
  if (v == 7) v = 8;
  return v;
}

int layernorm_fwd(const bf16* x, const bf16* r, const bf16* w, const bf16* b, bf16* h, bf16* y, float* mean,
                  float* rstd, int N, int C, float eps, hipStream_t st) {
  if (C % 8 != 0 || C > 4096) return -2;
  const int grid = (N + 3) / 4;
  const int vpl = vpl_for(C);
  if (r) {
    LN_DISPATCH(vpl, ln_fwd_kernel<V, true><<<grid, 256, 0, st>>>(x, r, w, b, h, y, mean, rstd, N, C, eps))
  } else {
    LN_DISPATCH(vpl, ln_fwd_kernel<V, false><<<grid, 256, 0, st>>>(x, r, w, b, h, y, mean, rstd, N, C, eps))
  }
  return 0;
}

int layernorm_bwd_grid(int N) {
  int g = (N + 15) / 16;  // >= 4 rows per wave
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  return g;
}

int layernorm_bwd(const bf16* dy, const bf16* x, const bf16* w, const float* mean, const float* rstd,
                  const bf16* dres, bf16* dx, float* part, bf16* dw, bf16* db, int N, int C, hipStream_t st) {
  if (C % 8 != 0 || C > 4096) return -2;
  const int grid = layernorm_bwd_grid(N);
  const int vpl = vpl_for(C);
  if (vpl > 4) return -3;  // LDS budget of the in-block combine
  if (dres) {
    LN_DISPATCH(vpl, ln_bwd_kernel<V, true><<<grid, 256, 0, st>>>(dy, x, w, mean, rstd, dres, dx, part, N, C))
  } else {
    LN_DISPATCH(vpl, ln_bwd_kernel<V, false><<<grid, 256, 0, st>>>(dy, x, w, mean, rstd, dres, dx, part, N, C))
  }
  colsum(part, grid, C, 2 * C, dw, nullptr, st);
  colsum(part + C, grid, C, 2 * C, db, nullptr, st);
  return 0;
}

}  // namespace pdo
