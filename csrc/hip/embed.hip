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

constexpr int EMB_SEG = 256;  // sorted rows per segment of the deterministic embedding backward

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
                                                               bf16* __restrict__ g, float* __restrict__ part,
                                                               int N, int C, int Vp, int accumulate) {
  // One wave per PIECE = a run of equal sorted ids cut at EMB_SEG-row segment
  // boundaries, so no wave sums more than EMB_SEG rows (a frequent token —
  // EOS, padding — would otherwise be one wave's serial loop over thousands).
  // A run inside one segment is written straight into g; the pieces of a run
  // that crosses a boundary leave fp32 partial sums in `part` (segment s:
  // [first piece | last piece] × C) for embed_bwd_fold_kernel, which adds them
  // in segment order: deterministic.
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= N) return;
  const int64_t tok = keys[i];
  const bool cont = i > 0 && keys[i - 1] == tok;  // continues a run from before
  if (cont && i % EMB_SEG != 0) return;           // not the start of a piece
  if (tok < 0 || tok >= Vp) return;               // ids outside the table contribute nothing
  const int seg = i / EMB_SEG, seg_end = min(N, (seg + 1) * EMB_SEG);
  int j = i;
  while (j < seg_end && keys[j] == tok) ++j;
  const bool more = j == seg_end && j < N && keys[j] == tok;  // run goes on past the segment
  for (int c8 = lane; c8 < (C >> 3); c8 += 64) {
    f32x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = i; k < j; ++k) t += to_f32(reinterpret_cast<const bf16x8*>(dy + (size_t)perm[k] * C)[c8]);
    if (!cont && !more) {
      bf16* out = g + (size_t)tok * C;
      if (accumulate) t += to_f32(reinterpret_cast<const bf16x8*>(out)[c8]);
      reinterpret_cast<bf16x8*>(out)[c8] = to_bf16(t);
    } else {
      float* dst = part + ((size_t)seg * 2 + (cont ? 0 : 1)) * C + 8 * c8;
      reinterpret_cast<f32x4*>(dst)[0] = f32x4{t[0], t[1], t[2], t[3]};
      reinterpret_cast<f32x4*>(dst)[1] = f32x4{t[4], t[5], t[6], t[7]};
    }
  }
}

// the runs that cross segment boundaries: the wave of the run's start adds its
// last-piece partial and the following segments' first-piece partials, in order
__global__ __launch_bounds__(256) void embed_bwd_fold_kernel(const int64_t* __restrict__ keys,
                                                             const float* __restrict__ part, bf16* __restrict__ g,
                                                             int N, int C, int Vp, int accumulate) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= N) return;
  const int64_t tok = keys[i];
  if ((i > 0 && keys[i - 1] == tok) || tok < 0 || tok >= Vp) return;  // run starts only
  const int seg = i / EMB_SEG, seg_end = (seg + 1) * EMB_SEG;
  if (seg_end >= N || keys[seg_end] != tok || keys[seg_end - 1] != tok) return;  // no boundary crossed
  bf16* out = g + (size_t)tok * C;
  for (int c8 = lane; c8 < (C >> 3); c8 += 64) {
    const float* p = part + ((size_t)seg * 2 + 1) * C + 8 * c8;
    f32x8 t = {p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7]};
    for (int s2 = seg + 1; s2 * EMB_SEG < N && keys[s2 * EMB_SEG] == tok; ++s2) {
      const float* q = part + ((size_t)s2 * 2) * C + 8 * c8;
      t += f32x8{q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7]};
    }
    if (accumulate) t += to_f32(reinterpret_cast<const bf16x8*>(out)[c8]);
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

int embed_sorted_part_floats(int N, int C) { return ((N + EMB_SEG - 1) / EMB_SEG) * 2 * C; }

int embed_bwd_sorted(const bf16* dy, const int64_t* keys, const int64_t* perm, bf16* dwte, bf16* dwpe, float* part,
                     int B, int S, int C, int Vp, int P, int accumulate, hipStream_t st) {
  if (C % 8) return -2;
  const int N = B * S;
  embed_bwd_sorted_kernel<<<(N + 3) / 4, 256, 0, st>>>(dy, keys, perm, dwte, part, N, C, Vp, accumulate);
  embed_bwd_fold_kernel<<<(N + 3) / 4, 256, 0, st>>>(keys, part, dwte, N, C, Vp, accumulate);
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
