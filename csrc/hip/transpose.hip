// SPDX-License-Identifier: Apache-2.0
// bf16 matrix transpose out[C][R] = in[R][C] (gfx950), for the input-gradient
// GEMMs that run in the forward's "TN" form dX = F.linear(dY, Wᵀ) (ops.linear).
//
// One 256-thread workgroup per 64×64 tile: rows come in as 16-B vectors and go
// to LDS with the 16-B chunk index XOR-swizzled by (row/8) — the transposed
// read (each lane gathers 8 rows of one column) then hits 16 distinct banks
// per 32-lane group, and every lane stores one 16-B run of an output row.
// PyTorch's strided copy of the same transpose ran ≈0.7 TB/s on the GPT-2
// weights (2.4 ms per step); this runs at the HBM rate.
#include "common.h"
#include "kernels.h"

namespace pdo {

constexpr int TT = 64;       // tile edge
constexpr int TLD = TT + 8;  // LDS row pitch (elements): 144 B keeps 16-B alignment

// one 64×64 tile (tr, tc) of out[C][R] = in[R][C]
__device__ __forceinline__ void transpose_tile(const bf16* __restrict__ in, bf16* __restrict__ out, int R, int C,
                                               int tr, int tc, bf16* t) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int idx = tid + 256 * i, r = idx >> 3, ch = idx & 7;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(in + (size_t)(tr * TT + r) * C + tc * TT + ch * 8);
    *reinterpret_cast<bf16x8*>(t + r * TLD + ((ch ^ ((r >> 3) & 7)) << 3)) = v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    // output row c (an input column), output columns 8·rg … 8·rg+7 (input rows)
    const int idx = tid + 256 * j, c = idx >> 3, rg = idx & 7;
    const int col = (((c >> 3) ^ rg) << 3) + (c & 7);
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t[(rg * 8 + e) * TLD + col];
    *reinterpret_cast<bf16x8*>(out + (size_t)(tc * TT + c) * R + tr * TT + rg * 8) = v;
  }
}

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                             int R, int C) {
  __shared__ __attribute__((aligned(16))) bf16 t[TT * TLD];
  const int tiles_c = C / TT;
  transpose_tile(in, out, R, C, blockIdx.x / tiles_c, blockIdx.x % tiles_c, t);
}

// The step's weight transposes (every dX GEMM's Wᵀ operand, GPT-2: 97 matrices)
// in one launch: block b belongs to the table entry whose first tile is the
// last one ≤ b (binary search over the n entries).
__global__ __launch_bounds__(256) void transpose_bf16_batched_kernel(const bf16* __restrict__ src,
                                                                     bf16* __restrict__ dst,
                                                                     const long long* __restrict__ table, int n) {
  __shared__ __attribute__((aligned(16))) bf16 t[TT * TLD];
  const long long b = blockIdx.x;
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (table[5 * mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  const long long* e = table + 5 * lo;
  const int R = (int)e[3], C = (int)e[4];
  const int local = (int)(b - e[0]), tiles_c = C / TT;
  transpose_tile(src + e[1], dst + e[2], R, C, local / tiles_c, local % tiles_c, t);
}

int transpose_bf16_batched(const bf16* src, bf16* dst, const long long* table, int n, long long tiles,
                           hipStream_t st) {
  if (n < 1 || tiles < 1 || tiles > 0x7fffffffLL) return -2;
  transpose_bf16_batched_kernel<<<(unsigned)tiles, 256, 0, st>>>(src, dst, table, n);
  return 0;
}

int transpose_bf16(const bf16* in, bf16* out, int R, int C, hipStream_t st) {
  if (R % TT || C % TT || R <= 0 || C <= 0) return -2;
  const long long tiles = (long long)(R / TT) * (C / TT);
  if (tiles > 0x7fffffffLL) return -2;
  transpose_bf16_kernel<<<(unsigned)tiles, 256, 0, st>>>(in, out, R, C);
  return 0;
}

}  // namespace pdo
