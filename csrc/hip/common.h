// SPDX-License-Identifier: Apache-2.0
// Shared helpers for the CDNA4 (gfx950) kernels of paddle_operator_amd.
//
// Conventions: wave = 64 lanes; bf16 is clang's native __bf16 (casts lower to
// v_cvt_pk_bf16_f32, NaN-preserving); every memory-bound kernel moves 16 B per
// lane per access (8 × bf16 / 4 × f32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdo {

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

constexpr int WAVE = 64;

__device__ __forceinline__ f32x8 to_f32(bf16x8 v) { return __builtin_convertvector(v, f32x8); }
__device__ __forceinline__ bf16x8 to_bf16(f32x8 v) { return __builtin_convertvector(v, bf16x8); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NW*64; `red` is NW floats of LDS.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  __syncthreads();
  return t;
}

template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  return 0.5f * x * (1.f + tanhf(u));
}

// d/dx gelu_tanh(x)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2 = x * x;
  float u = k0 * (x + k1 * x2 * x);
  float t = tanhf(u);
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
}

// GELU(tanh) in logistic form (gelu.hip, gemm_nt.hip epilogues):
// 0.5·x·(1 + tanh u) = x·σ(2u), u = k0(x + k1x³): one exp2 and one rcp.
constexpr float GK0 = 0.7978845608028654f, GK1 = 0.044715f;
constexpr float GL2E = 1.4426950408889634f;

__device__ __forceinline__ float gelu_sig(float x) {
  const float t = x * x;
  const float z = x * __builtin_fmaf(t, -2.f * GK0 * GK1 * GL2E, -2.f * GK0 * GL2E);  // -2u·log2(e)
  const float e = __builtin_amdgcn_exp2f(z);
  return x * __builtin_amdgcn_rcpf(1.f + e);
}

// d/dx x·σ(2u) = s + x·s·(1-s)·2u', s = σ(2u)
__device__ __forceinline__ float gelu_sig_grad(float x) {
  const float t = x * x;
  const float z = x * __builtin_fmaf(t, -2.f * GK0 * GK1 * GL2E, -2.f * GK0 * GL2E);
  const float e = __builtin_amdgcn_exp2f(z);
  const float sg = __builtin_amdgcn_rcpf(1.f + e);
  const float w = __builtin_fmaf(t, 6.f * GK0 * GK1, 2.f * GK0);  // 2u'
  const float q = x * (1.f - sg) * w;  // (1 - s), not e·s: e = inf at x ≪ 0
  return __builtin_fmaf(sg, q, sg);
}

// The same two functions on a pair of values in packed fp32 (v_pk_mul_f32 /
// v_pk_fma_f32 / v_pk_add_f32: one issue per pair; exp2 / rcp stay per value).
// The operation sequence and rounding are those of the scalar forms.  For the
// GEMM epilogues, whose VALU work runs with the matrix pipe idle (one wave per
// SIMD); beside MFMAs packed fp32 is an anti-lever (MI355X_MICROARCH.md).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 exp2_2(f32x2 z) {
  return f32x2{__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])};
}
__device__ __forceinline__ f32x2 rcp_2(f32x2 z) { return f32x2{__builtin_amdgcn_rcpf(z[0]), __builtin_amdgcn_rcpf(z[1])}; }

__device__ __forceinline__ f32x2 gelu_sig2(f32x2 x) {
  const f32x2 t = x * x;
  const f32x2 z = x * pk_fma(t, f32x2(-2.f * GK0 * GK1 * GL2E), f32x2(-2.f * GK0 * GL2E));
  return x * rcp_2(exp2_2(z) + 1.f);
}

// m1 = (-1, -1) from the caller behind an empty asm: 1 - s then stays one
// packed fma (a literal -1 is folded into 1 - s, which the backend scalarises)
__device__ __forceinline__ f32x2 gelu_sig_grad2(f32x2 x, f32x2 m1) {
  const f32x2 t = x * x;
  const f32x2 z = x * pk_fma(t, f32x2(-2.f * GK0 * GK1 * GL2E), f32x2(-2.f * GK0 * GL2E));
  const f32x2 sg = rcp_2(exp2_2(z) + 1.f);
  const f32x2 w = pk_fma(t, f32x2(6.f * GK0 * GK1), f32x2(2.f * GK0));
  const f32x2 q = x * pk_fma(sg, m1, -m1) * w;  // 1 - s (exact as an fma)
  return pk_fma(sg, q, sg);
}

// gelu(x) and gelu'(x) together (the shared t, z, s computed once): the fc1
// forward epilogue stores gelu' for fc2's input-gradient epilogue, which then
// needs one multiply per element instead of the whole derivative
__device__ __forceinline__ void gelu_and_grad2(f32x2 x, f32x2 m1, f32x2& y, f32x2& g) {
  const f32x2 t = x * x;
  const f32x2 z = x * pk_fma(t, f32x2(-2.f * GK0 * GK1 * GL2E), f32x2(-2.f * GK0 * GL2E));
  const f32x2 sg = rcp_2(exp2_2(z) + 1.f);
  y = x * sg;
  const f32x2 w = pk_fma(t, f32x2(6.f * GK0 * GK1), f32x2(2.f * GK0));
  g = pk_fma(y * w, pk_fma(sg, m1, -m1), sg);  // s + y·2u'·(1 - s), y = x·s
}

// BatchNorm partials (Σx, Σ(x − x̄)²) of two groups of n rows each, merged
// (Chan: the means differ by (sa − sb)/n, weight n·n / 2n)
__device__ __forceinline__ void chan_merge_equal(f32x8& s, f32x8& q, const f32x8& s2, const f32x8& q2, float n) {
  const f32x8 d = s - s2;
  q = q + q2 + d * d * (0.5f / n);
  s = s + s2;
}

// number of workgroups for a grid-stride memory-bound kernel (256 CUs × 8)
inline int stream_grid(long long work_items, int per_block) {
  long long g = (work_items + per_block - 1) / per_block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace pdo
