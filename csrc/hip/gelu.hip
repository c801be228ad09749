// SPDX-License-Identifier: Apache-2.0
// bias + GELU(tanh) forward and backward for the GPT-2 MLP (gfx950).
// The GEMM producing x runs without bias (plain hipBLASLt); the bias add, the
// activation and — in backward — the bias gradient column reduction are fused
// here, so the [N, 4C] activation makes exactly one HBM round trip per pass.
#include "common.h"
#include "kernels.h"

namespace pdo {

__device__ __forceinline__ float fast_tanh(float u) {
  // tanh(u) = 1 - 2 / (exp(2u) + 1); saturates correctly at ±inf
  return 1.f - __fdividef(2.f, __expf(2.f * u) + 1.f);
}

__device__ __forceinline__ float gelu_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + fast_tanh(k0 * (x + k1 * x * x * x)));
}

__device__ __forceinline__ float gelu_g(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float t = fast_tanh(k0 * (x + k1 * x2 * x));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
}

// grid-stride over 8-element vectors; F % 8 == 0
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ b,
                                                            bf16* __restrict__ y, long long nvec, int F8) {
  const bf16x8* xv = reinterpret_cast<const bf16x8*>(x);
  const bf16x8* bv = reinterpret_cast<const bf16x8*>(b);
  bf16x8* yv = reinterpret_cast<bf16x8*>(y);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    f32x8 v = to_f32(xv[i]) + to_f32(bv[i % F8]);
    f32x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gelu_f(v[j]);
    yv[i] = to_bf16(o);
  }
}

// block (x: 2048-column stripe, y: row group).  dx = dy * gelu'(x+b),
// partial db for the stripe written to part[blockIdx.y][col].
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const bf16* __restrict__ b, bf16* __restrict__ dx,
                                                            float* __restrict__ part, int N, int F) {
  const int c8 = blockIdx.x * 256 + threadIdx.x;
  const int F8 = F >> 3;
  const int rows_per = (N + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(N, r0 + rows_per);
  f32x8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c8 < F8) {
    const f32x8 bb = to_f32(reinterpret_cast<const bf16x8*>(b)[c8]);
#pragma unroll 4
    for (int r = r0; r < r1; ++r) {
      const size_t idx = (size_t)r * F8 + c8;
      f32x8 d = to_f32(reinterpret_cast<const bf16x8*>(dy)[idx]);
      f32x8 v = to_f32(reinterpret_cast<const bf16x8*>(x)[idx]) + bb;
      f32x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = d[j] * gelu_g(v[j]);
      reinterpret_cast<bf16x8*>(dx)[idx] = to_bf16(o);
      acc += o;
    }
    float* p = part + (size_t)blockIdx.y * F + c8 * 8;
    reinterpret_cast<f32x4*>(p)[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    reinterpret_cast<f32x4*>(p)[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
}

int bias_gelu_fwd(const bf16* x, const bf16* b, bf16* y, long long N, int F, hipStream_t st) {
  if (F % 8) return -2;
  const long long nvec = N * (long long)(F / 8);
  bias_gelu_fwd_kernel<<<stream_grid(nvec, 256), 256, 0, st>>>(x, b, y, nvec, F / 8);
  return 0;
}

int bias_gelu_bwd_groups(long long N, int F) {
  const int gx = (F / 8 + 255) / 256;
  long long gy = 2048 / gx;
  if (gy > N) gy = N;
  if (gy < 1) gy = 1;
  return (int)gy;
}

int bias_gelu_bwd(const bf16* dy, const bf16* x, const bf16* b, bf16* dx, float* part, float* scratch, bf16* db,
                  long long N, int F, hipStream_t st, int accumulate) {
  if (F % 8) return -2;
  const int gx = (F / 8 + 255) / 256;
  const int gy = bias_gelu_bwd_groups(N, F);
  bias_gelu_bwd_kernel<<<dim3(gx, gy), 256, 0, st>>>(dy, x, b, dx, part, (int)N, F);
  ColOut co = ColOut::one(db, F);
  co.acc = accumulate;
  colsum(part, gy, F, F, co, scratch, st);
  return 0;
}

}  // namespace pdo
