// SPDX-License-Identifier: Apache-2.0
// Token + position embedding (gfx950).
// Forward: one wave per token row, y = wte[idx] + wpe[pos] with 16-B vectors.
// Backward: d(wte) by f32 atomics shaped as 256 contiguous bytes per wave
// instruction (one row segment per instruction, the fast atomic shape on
// MI355X) into a zeroed f32 table, then one vectorised cast to bf16 — or,
// deterministic and cheaper (embed_bwd_sorted), a segmented sum over the
// stably sorted token ids straight into the gradient rows;
// d(wpe) is a deterministic per-position sum over the batch.
#include "common.h"
#include "kernels.h"

namespace pdo {

__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ idx, const bf16* __restrict__ wte,
                                                        const bf16* __restrict__ wpe, bf16* __restrict__ y, int N,
                                                        int S, int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const int64_t tok = idx[row];
  const int pos = row % S;
  const bf16x8* a = reinterpret_cast<const bf16x8*>(wte + (size_t)tok * C);
  const bf16x8* p = reinterpret_cast<const bf16x8*>(wpe + (size_t)pos * C);
  bf16x8* o = reinterpret_cast<bf16x8*>(y + (size_t)row * C);
  for (int c8 = lane; c8 < (C >> 3); c8 += 64) o[c8] = to_bf16(to_f32(a[c8]) + to_f32(p[c8]));
}

__global__ __launch_bounds__(256) void embed_bwd_wte_kernel(const bf16* __restrict__ dy, const int64_t* __restrict__ idx,
                                                            float* __restrict__ acc, int N, int C, int Vp) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const int64_t tok = idx[row];
  if (tok < 0 || tok >= Vp) return;
  const bf16* d = dy + (size_t)row * C;
  float* a = acc + (size_t)tok * C;
  for (int c = lane; c < C; c += 64) atomicAdd(a + c, (float)d[c]);
}

// dwpe[s][c] = sum_b dy[b][s][c]
__global__ __launch_bounds__(256) void embed_bwd_wpe_kernel(const bf16* __restrict__ dy, bf16* __restrict__ dwpe,
                                                            int B, int S, int C) {
  const int s = blockIdx.x;
  for (int c8 = threadIdx.x; c8 < (C >> 3); c8 += 256) {
    f32x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = 0; b < B; ++b) t += to_f32(reinterpret_cast<const bf16x8*>(dy + ((size_t)b * S + s) * C)[c8]);
    reinterpret_cast<bf16x8*>(dwpe + (size_t)s * C)[c8] = to_bf16(t);
  }
}

// d(wte) without atomics: the token ids sorted stably (keys) with their row
// indices (perm); the wave at the first position of each run of equal keys
// sums the run's dy rows in sorted (= row) order and adds the sum into that
// token's gradient row — deterministic, no [Vp, C] fp32 table, no memset, no
// cast pass; rows of tokens absent from the batch are not touched
__global__ __launch_bounds__(256) void embed_bwd_sorted_kernel(const bf16* __restrict__ dy,
                                                               const int64_t* __restrict__ keys,
                                                               const int64_t* __restrict__ perm,
                                                               bf16* __restrict__ g, int N, int C, int Vp,
                                                               int accumulate) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= N) return;
  const int64_t tok = keys[i];
  if (i > 0 && keys[i - 1] == tok) return;  // not the start of a run
  if (tok < 0 || tok >= Vp) return;
  bf16* out = g + (size_t)tok * C;
  for (int c8 = lane; c8 < (C >> 3); c8 += 64) {
    f32x8 t = accumulate ? to_f32(reinterpret_cast<const bf16x8*>(out)[c8]) : f32x8{0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = i; j < N && keys[j] == tok; ++j)
      t += to_f32(reinterpret_cast<const bf16x8*>(dy + (size_t)perm[j] * C)[c8]);
    reinterpret_cast<bf16x8*>(out)[c8] = to_bf16(t);
  }
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ in, bf16* __restrict__ out,
                                                          long long nvec) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    const f32x4* p = reinterpret_cast<const f32x4*>(in) + 2 * i;
    f32x4 a = p[0], b = p[1];
    f32x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    reinterpret_cast<bf16x8*>(out)[i] = to_bf16(v);
  }
}

int embed_fwd(const int64_t* idx, const bf16* wte, const bf16* wpe, bf16* y, int B, int S, int C, hipStream_t st) {
  if (C % 8) return -2;
  const int N = B * S;
  embed_fwd_kernel<<<(N + 3) / 4, 256, 0, st>>>(idx, wte, wpe, y, N, S, C);
  return 0;
}

int embed_bwd(const bf16* dy, const int64_t* idx, float* acc, bf16* dwte, bf16* dwpe, int B, int S, int C, int Vp,
              int P, hipStream_t st) {
  if (C % 8) return -2;
  const int N = B * S;
  hipMemsetAsync(acc, 0, (size_t)Vp * C * sizeof(float), st);
  embed_bwd_wte_kernel<<<(N + 3) / 4, 256, 0, st>>>(dy, idx, acc, N, C, Vp);
  const long long nvec = (long long)Vp * C / 8;
  f32_to_bf16_kernel<<<stream_grid(nvec, 256), 256, 0, st>>>(acc, dwte, nvec);
  hipMemsetAsync(dwpe, 0, (size_t)P * C * sizeof(bf16), st);
  embed_bwd_wpe_kernel<<<S, 256, 0, st>>>(dy, dwpe, B, S, C);
  return 0;
}

int embed_bwd_sorted(const bf16* dy, const int64_t* keys, const int64_t* perm, bf16* dwte, bf16* dwpe, int B, int S,
                     int C, int Vp, int P, int accumulate, hipStream_t st) {
  if (C % 8) return -2;
  const int N = B * S;
  embed_bwd_sorted_kernel<<<(N + 3) / 4, 256, 0, st>>>(dy, keys, perm, dwte, N, C, Vp, accumulate);
  if (dwpe) {
    hipMemsetAsync(dwpe, 0, (size_t)P * C * sizeof(bf16), st);
    embed_bwd_wpe_kernel<<<S, 256, 0, st>>>(dy, dwpe, B, S, C);
  }
  return 0;
}

int cast_f32_bf16(const float* in, bf16* out, long long n, hipStream_t st) {
  if (n % 8) return -2;
  f32_to_bf16_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(in, out, n / 8);
  return 0;
}

}  // namespace pdo
