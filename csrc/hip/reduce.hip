// SPDX-License-Identifier: Apache-2.0
// Column reductions (bias / norm-weight gradients) for gfx950.
//
// out[c] = Σ_r in[r][c] as a deterministic two-level tree: level 1 gives each
// workgroup a 256-column (f32) / 512-column (bf16) stripe × a slice of rows,
// 8 waves stride the slice, the waves combine in LDS and the block writes one
// partial row; level 2 folds the ≤ a few dozen partial rows and writes bf16.
// Enough workgroups to keep HBM busy (the single-level version with one
// block per 64 columns was latency-bound at ~20 µs per call).
#include "common.h"
#include "kernels.h"

namespace pdo {

constexpr int RPB = 64;  // rows per level-1 workgroup

// one level-1 / level-2 block of the column sum: columns (bx·64 + lane)·4 ..+3,
// rows [by·rpb, by·rpb + rpb); 8 waves stride the rows, combine in LDS, and
// the block writes a partial row (out_part) or the final bf16 values (co)
__device__ __forceinline__ void colsum_block(const float* __restrict__ in, int G, int C, int ld, int rpb,
                                             float* __restrict__ out_part, const ColOut& co, int bx, int by,
                                             f32x4 (*red)[64]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = (bx * 64 + lane) * 4;
  const int r0 = by * rpb;
  const int r1 = min(G, r0 + rpb);
  f32x4 s = {0, 0, 0, 0};
  if (col < C) {
#pragma unroll 4
    for (int r = r0 + w; r < r1; r += 8) s += *reinterpret_cast<const f32x4*>(in + (size_t)r * ld + col);
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < C) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int i = 1; i < 8; ++i) t += red[i][lane];
    if (co.p[0]) {
      // segment k of `co.seg` columns goes to co.p[k] (e.g. straight into the
      // parameters' slices of the flat gradient arena), optionally accumulated
      const int k = col / co.seg, c = col - k * co.seg;
      bf16* dst = co.p[k] + c;
      if (co.acc) {
        const bf16x4 old = *reinterpret_cast<const bf16x4*>(dst);
        t += f32x4{(float)old[0], (float)old[1], (float)old[2], (float)old[3]};
      }
      bf16x4 o = {(bf16)t[0], (bf16)t[1], (bf16)t[2], (bf16)t[3]};
      *reinterpret_cast<bf16x4*>(dst) = o;
    } else {
      *reinterpret_cast<f32x4*>(out_part + (size_t)by * C + col) = t;
    }
  }
}

__global__ __launch_bounds__(512) void colsum_f32_pass(const float* __restrict__ in, int G, int C, int ld, int rpb,
                                                       float* __restrict__ out_part, ColOut co) {
  __shared__ f32x4 red[8][64];
  colsum_block(in, G, C, ld, rpb, out_part, co, blockIdx.x, blockIdx.y, red);
}

__global__ __launch_bounds__(512) void colsum_bf16_pass(const bf16* __restrict__ in, int N, int F, int rpb,
                                                        float* __restrict__ out_part) {
  __shared__ f32x8 red[8][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c8 = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * rpb;
  const int r1 = min(N, r0 + rpb);
  f32x8 s = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c8 * 8 < F) {
#pragma unroll 4
    for (int r = r0 + w; r < r1; r += 8) s += to_f32(reinterpret_cast<const bf16x8*>(in + (size_t)r * F)[c8]);
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c8 * 8 < F) {
    f32x8 t = red[0][lane];
#pragma unroll
    for (int i = 1; i < 8; ++i) t += red[i][lane];
    float* o = out_part + (size_t)blockIdx.y * F + c8 * 8;
    reinterpret_cast<f32x4*>(o)[0] = f32x4{t[0], t[1], t[2], t[3]};
    reinterpret_cast<f32x4*>(o)[1] = f32x4{t[4], t[5], t[6], t[7]};
  }
}

int colsum_scratch_floats(int G, int C) { return ((G + RPB - 1) / RPB) * C; }

// part: [G][ld] f32 (first C columns used).  scratch: colsum_scratch_floats(G, C)
void colsum(const float* part, int G, int C, int ld, const ColOut& out, float* scratch, hipStream_t st) {
  const int gx = (C / 4 + 63) / 64;
  if (G <= RPB) {
    colsum_f32_pass<<<dim3(gx, 1), 512, 0, st>>>(part, G, C, ld, RPB, nullptr, out);
    return;
  }
  const int gs = (G + RPB - 1) / RPB;
  colsum_f32_pass<<<dim3(gx, gs), 512, 0, st>>>(part, G, C, ld, RPB, scratch, ColOut{});
  colsum_f32_pass<<<dim3(gx, 1), 512, 0, st>>>(scratch, gs, C, C, gs, nullptr, out);
}

void colsum(const float* part, int G, int C, int ld, bf16* out, float* scratch, hipStream_t st) {
  colsum(part, G, C, ld, ColOut::one(out, C), scratch, st);
}

// ---- many column sums in two launches (deferred bias / norm-weight gradients) ----
// Level 1: every job's (column stripe × row slice) blocks back to back in one
// grid — a job of ≤ RPB rows is finished here, the others write partial rows
// to their scratch; level 2 folds those.  Jobs travel as kernel arguments.
__device__ __forceinline__ int batch_job(const int* start, int n, int b) {
  int e = 0;
  while (e + 1 < n && b >= start[e + 1]) ++e;
  return e;
}

__global__ __launch_bounds__(512) void colsum_batch_l1(ColsumBatch bt) {
  __shared__ f32x4 red[8][64];
  const int e = batch_job(bt.l1, bt.n, blockIdx.x);
  const ColsumJob& j = bt.j[e];
  const int b = blockIdx.x - bt.l1[e], gx = (j.C / 4 + 63) / 64;
  const int gs = (j.G + RPB - 1) / RPB;
  colsum_block(j.part, j.G, j.C, j.ld, RPB, j.scratch, gs == 1 ? j.co : ColOut{}, b % gx, b / gx, red);
}

__global__ __launch_bounds__(512) void colsum_batch_l2(ColsumBatch bt) {
  __shared__ f32x4 red[8][64];
  const int e = batch_job(bt.l2, bt.n, blockIdx.x);
  const ColsumJob& j = bt.j[e];
  const int gs = (j.G + RPB - 1) / RPB;
  colsum_block(j.scratch, gs, j.C, j.C, gs, nullptr, j.co, blockIdx.x - bt.l2[e], 0, red);
}

int colsum_batched(const ColsumJob* jobs, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += COLSUM_BATCH) {
    ColsumBatch bt{};
    bt.n = n - i0 < COLSUM_BATCH ? n - i0 : COLSUM_BATCH;
    int b1 = 0, b2 = 0;
    for (int e = 0; e < bt.n; ++e) {
      const ColsumJob& j = jobs[i0 + e];
      if (j.C % 4 || j.G < 1 || !j.co.p[0]) return -2;
      bt.j[e] = j;
      const int gx = (j.C / 4 + 63) / 64, gs = (j.G + RPB - 1) / RPB;
      bt.l1[e] = b1;
      bt.l2[e] = b2;
      b1 += gx * gs;
      if (gs > 1) b2 += gx;
    }
    bt.l1[bt.n] = b1;
    bt.l2[bt.n] = b2;
    colsum_batch_l1<<<b1, 512, 0, st>>>(bt);
    if (b2) {
      // jobs finished in level 1 get no level-2 blocks: their l2 range is empty
      colsum_batch_l2<<<b2, 512, 0, st>>>(bt);
    }
  }
  return 0;
}

int bias_grad_scratch_floats(long long N, int F) {
  const int gs = (int)((N + 255) / 256);
  return gs * F;
}

// db[f] (+)= Σ_n dy[n][f]  (bf16 in, bf16 out); scratch: bias_grad_scratch_floats
int bias_grad(const bf16* dy, long long N, int F, bf16* db, float* scratch, hipStream_t st, int accumulate) {
  if (F % 8) return -2;
  const int gx = (F / 8 + 63) / 64;
  const int gs = (int)((N + 255) / 256);
  colsum_bf16_pass<<<dim3(gx, gs), 512, 0, st>>>(dy, (int)N, F, 256, scratch);
  const int gx2 = (F / 4 + 63) / 64;
  ColOut co = ColOut::one(db, F);
  co.acc = accumulate;
  colsum_f32_pass<<<dim3(gx2, 1), 512, 0, st>>>(scratch, gs, F, F, gs, nullptr, co);
  return 0;
}



// ----------------------------------------------------------------------------
// split-K combine for long-K weight-gradient GEMMs:
//   out[i] (+)= sum_s part[s][i]   (bf16 partials, fp32 sum, bf16 out)
// dW = dY^T X has K = tokens (16-64k) but only M·N/256² = 16-64 output tiles,
// too few to fill 256 CUs; the GEMM runs as a batched [s] GEMM over token
// slices and this pass folds the slices straight into the gradient arena.
// ----------------------------------------------------------------------------
template <int S_MAX>
__global__ __launch_bounds__(256) void splitk_add_kernel(const bf16* __restrict__ part, int s, long long n,
                                                         bf16* __restrict__ out, int accumulate) {
  const long long i8 = (blockIdx.x * 256LL + threadIdx.x);
  if (i8 * 8 >= n) return;
  f32x8 acc = accumulate ? to_f32(reinterpret_cast<const bf16x8*>(out)[i8]) : f32x8{0, 0, 0, 0, 0, 0, 0, 0};
  const bf16x8* p = reinterpret_cast<const bf16x8*>(part) + i8;
  const long long stride = n / 8;
#pragma unroll
  for (int k = 0; k < S_MAX; ++k)
    if (k < s) acc += to_f32(p[k * stride]);
  reinterpret_cast<bf16x8*>(out)[i8] = to_bf16(acc);
}

int splitk_add(const bf16* part, int s, long long n, bf16* out, int accumulate, hipStream_t st) {
  if (n % 8 != 0 || s < 1 || s > 16) return -2;
  const unsigned grid = (unsigned)((n / 8 + 255) / 256);
  if (s <= 8)
    splitk_add_kernel<8><<<grid, 256, 0, st>>>(part, s, n, out, accumulate);
  else
    splitk_add_kernel<16><<<grid, 256, 0, st>>>(part, s, n, out, accumulate);
  return 0;
}

}  // namespace pdo
