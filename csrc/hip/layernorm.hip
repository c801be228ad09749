// SPDX-License-Identifier: Apache-2.0
// LayerNorm forward/backward (optionally fused with the residual add) for
// gfx950.  One wave per row: a row of C bf16 is held in registers as VPL
// vectors of 8 (16-B loads), statistics are two-pass in registers (exact
// mean, then centred variance), reductions are 64-lane shuffles.  Backward
// computes dx per row and accumulates dgamma/dbeta per lane in registers over
// a grid-stride row loop; the 4 waves of a block combine through LDS and the
// per-block partials are summed by the two-level `colsum` (reduce.hip).
#include "common.h"
#include "kernels.h"

namespace pdo {

template <int VPL, bool ADD>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ r,
                                                     const bf16* __restrict__ rb,
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
      if (ADD) {
        v[i] += to_f32(rr[c8]);
        if (rb) v[i] += to_f32(reinterpret_cast<const bf16x8*>(rb)[c8]);
      }
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

// NA = 2: partials (dgamma, dbeta); NA = 3: + colsum(dx) — the gradient of a
// bias folded into the residual branch (h = x + r + rbias).
template <int VPL, bool ADD, int NA>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                     const bf16* __restrict__ w, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const bf16* __restrict__ dres,
                                                     bf16* __restrict__ dx, float* __restrict__ part, int N, int C) {
  constexpr int COLS = 64 * 8 * VPL;
  __shared__ float red[NA * COLS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int C8 = C >> 3;
  const float inv_c = 1.f / (float)C;
  f32x8 wv[VPL], adw[VPL], adb[VPL], adx[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c8 = lane + i * 64;
    wv[i] = c8 < C8 ? to_f32(reinterpret_cast<const bf16x8*>(w)[c8]) : f32x8{0, 0, 0, 0, 0, 0, 0, 0};
    adw[i] = f32x8{0, 0, 0, 0, 0, 0, 0, 0};
    adb[i] = adw[i];
    adx[i] = adw[i];
  }
  const int nw = gridDim.x * 4;
  // every operand of a row (dy, x and the residual gradient) is requested
  // up front, and the NEXT row's are requested before this row's two
  // wave-wide reductions: the reductions' latency hides the loads'
  bf16x8 nd[VPL], nx[VPL], nr[VPL];
  auto fetch = [&](int row) {
    const size_t base = (size_t)row * C;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c8 = lane + i * 64;
      if (c8 < C8) {
        nd[i] = reinterpret_cast<const bf16x8*>(dy + base)[c8];
        nx[i] = reinterpret_cast<const bf16x8*>(x + base)[c8];
        if (ADD) nr[i] = reinterpret_cast<const bf16x8*>(dres + base)[c8];
      }
    }
  };
  int row = blockIdx.x * 4 + wid;
  if (row < N) fetch(row);
  for (; row < N; row += nw) {
    const size_t base = (size_t)row * C;
    const float mu = mean[row], rs = rstd[row];
    f32x8 xh[VPL], g[VPL], rr[VPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c8 = lane + i * 64;
      if (c8 < C8) {
        f32x8 d = to_f32(nd[i]);
        f32x8 xv = to_f32(nx[i]);
        if (ADD) rr[i] = to_f32(nr[i]);
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
    if (row + nw < N) fetch(row + nw);
    s1 = wave_sum(s1) * inv_c;
    s2 = wave_sum(s2) * inv_c;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c8 = lane + i * 64;
      if (c8 < C8) {
        f32x8 o = (g[i] - s1 - xh[i] * s2) * rs;
        if (ADD) o += rr[i];
        if (NA == 3) adx[i] += o;
        reinterpret_cast<bf16x8*>(dx + base)[c8] = to_bf16(o);
      }
    }
  }
  // combine the 4 waves sequentially through one [NA][COLS] LDS image
  for (int k = 0; k < 4; ++k) {
    if (wid == k) {
#pragma unroll
      for (int i = 0; i < VPL; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = (i * 64 + lane) * 8 + j;
          const float a0 = adw[i][j], a1 = adb[i][j], a2 = adx[i][j];
          if (k == 0) {
            red[c] = a0;
            red[COLS + c] = a1;
            if (NA == 3) red[2 * COLS + c] = a2;
          } else {
            red[c] += a0;
            red[COLS + c] += a1;
            if (NA == 3) red[2 * COLS + c] += a2;
          }
        }
    }
    __syncthreads();
  }
  float* pp = part + (size_t)blockIdx.x * NA * C;
  for (int k = threadIdx.x; k < NA * C; k += 256) {
    const int a = k / C, c = k - a * C;
    pp[k] = red[a * COLS + c];
  }
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

int layernorm_fwd(const bf16* x, const bf16* r, const bf16* rb, const bf16* w, const bf16* b, bf16* h, bf16* y,
                  float* mean, float* rstd, int N, int C, float eps, hipStream_t st) {
  if (C % 8 != 0 || C > 4096) return -2;
  if (rb && !r) return -4;
  const int grid = (N + 3) / 4;
  const int vpl = vpl_for(C);
  if (r) {
    LN_DISPATCH(vpl, ln_fwd_kernel<V, true><<<grid, 256, 0, st>>>(x, r, rb, w, b, h, y, mean, rstd, N, C, eps))
  } else {
    LN_DISPATCH(vpl, ln_fwd_kernel<V, false><<<grid, 256, 0, st>>>(x, r, rb, w, b, h, y, mean, rstd, N, C, eps))
  }
  return 0;
}

int layernorm_bwd_grid(int N) {
  // one resident round: ≤ 2 waves/SIMD at this kernel's register count
  // (4 waves per block, 256 CUs × 4 SIMDs × 2 / 4 = 512 blocks), ≥ 4 rows per wave
  int g = (N + 15) / 16;
  if (g > 512) g = 512;
  if (g < 1) g = 1;
  return g;
}

// out: dgamma | dbeta | (drbias) as C-column segments; part: [grid][NA*C] f32;
// scratch: colsum_scratch_floats(grid, NA*C)
int layernorm_bwd(const bf16* dy, const bf16* x, const bf16* w, const float* mean, const float* rstd,
                  const bf16* dres, bf16* dx, float* part, float* scratch, const ColOut& out, bool rbias, int N,
                  int C, hipStream_t st, bool reduce) {
  if (C % 8 != 0 || C > 4096) return -2;
  if (rbias && !dres) return -4;
  if (out.seg != C) return -5;
  const int grid = layernorm_bwd_grid(N);
  const int vpl = vpl_for(C);
  if (vpl > 4) return -3;  // register/LDS budget of the in-block combine
  const int NA = rbias ? 3 : 2;
  if (rbias) {
    LN_DISPATCH(vpl, ln_bwd_kernel<V, true, 3><<<grid, 256, 0, st>>>(dy, x, w, mean, rstd, dres, dx, part, N, C))
  } else if (dres) {
    LN_DISPATCH(vpl, ln_bwd_kernel<V, true, 2><<<grid, 256, 0, st>>>(dy, x, w, mean, rstd, dres, dx, part, N, C))
  } else {
    LN_DISPATCH(vpl, ln_bwd_kernel<V, false, 2><<<grid, 256, 0, st>>>(dy, x, w, mean, rstd, dres, dx, part, N, C))
  }
  if (reduce) colsum(part, grid, NA * C, NA * C, out, scratch, st);
  return 0;
}

}  // namespace pdo
