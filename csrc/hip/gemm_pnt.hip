// SPDX-License-Identifier: Apache-2.0
// Persistent forward-layout GEMM C[M][N] = A[M][K] · B[N][K]ᵀ (bf16, fp32 acc)
// for gfx950 — the transformer projections whose K is short (1024 for
// GPT-2-medium's QKV / proj / fc1 forward and fc2 input gradient).
//
// Why persistent: at K = 1024 a 256×256 tile has 32 k-stages of 32; a
// one-tile-per-workgroup GEMM then pays, per tile, a pipeline fill plus a
// 128 KiB output write that nothing overlaps (hipBLASLt and gemm_nt.hip both
// reach only 0.78–1.03 PF there vs ≈1.45 PF at K = 4096: profiles/
// r2_gemm_shapes_1gpu.md).  Here one workgroup per CU walks a list of tiles and
// the LDS-DMA ring runs across tile boundaries: while the last k-stages of tile
// t are multiplied, the first stages of tile t+1 are already in flight, and
// tile t's output leaves straight from the accumulators (no LDS staging —
// the ring keeps all 160 KiB) while tile t+1's k-loop starts.
//
// Mainloop (gemm_nt.hip's): 256 × 256 × 32 stages, 8 waves as 2 (M) × 4 (N),
// 5-stage LDS ring filled by global_load_lds_dwordx4 with the XOR swizzle on
// the source address, waves 4-7 one barrier behind waves 0-3 so each SIMD
// pairs an MFMA phase with an LDS-read phase.  MFMA operands swapped (D = B·Aᵀ)
// so a lane's accumulator holds 4 consecutive output columns of one row.
//
// Epilogue from registers: per 16-row fragment row i, the 4 lanes {r, r+16,
// r+32, r+48} hold a 4×4 block matrix of 4-column pieces; two rounds of
// v_permlane32_swap / v_permlane16_swap transpose it so every lane owns 16
// contiguous columns = two 16-B stores.  Variants:
//   EPI 0  C = A·Bᵀ
//   EPI 1  C = A·Bᵀ + bias
//   EPI 2  C = A·Bᵀ (pre-activation) and Y = gelu(C + bias)   (fc1 forward)
//   EPI 3  C = (A·Bᵀ) ⊙ gelu'(Y + bias), Y = saved pre-activation, plus fp32
//          column partial sums of C (bias gradient), 2 rows per M-tile
// Rounding matches gemm_nt.hip / the unfused path: the GEMM result is rounded
// to bf16 before the activation math.
//
// Ordering of the DMA ring against the epilogue's memory operations: vmcnt
// retires in issue order, so the wait for stage g+1 allows exactly the VMEM
// instructions issued after it: 4 per later stage plus, when a tile ended in
// between, at least the epilogue's 16 (EPI 0/1/3) or 32 (EPI 2) stores —
// counting fewer than were issued only waits longer.
#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int STAGES = 5;       // 5 × 32 KiB = the whole 160 KiB LDS
constexpr int TILE = 256 * BK;  // elements of one operand tile [256 rows][32]
constexpr int NTHR = 512;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 3; }

template <int EPI>
struct EpiVm {  // VMEM instructions an epilogue issues at least (per wave)
  static constexpr int n = EPI == 2 ? 32 : 16;
};

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 join(u32x2 a, u32x2 b) {
  return __builtin_bit_cast(bf16x8, u32x4{a[0], a[1], b[0], b[1]});
}

// pack 4 floats → 4 bf16 in 2 dwords
__device__ __forceinline__ u32x2 pack4(f32x4 v) {
  bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  return __builtin_bit_cast(u32x2, b);
}

__device__ __forceinline__ void swap32(u32x2& x, u32x2& y) {  // x upper half ↔ y lower half
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    auto r = __builtin_amdgcn_permlane32_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
}

__device__ __forceinline__ void swap16(u32x2& x, u32x2& y) {  // x odd rows ↔ y even rows
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    auto r = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
}

// 4×4 block transpose across lane groups q = lane>>4: in, b[j] = columns
// 16j + 4q .. +3; out, b[q'] = columns 16q + 4q' .. +3 (16 contiguous)
__device__ __forceinline__ void transpose_blocks(u32x2 (&b)[4]) {
  swap32(b[0], b[2]);
  swap32(b[1], b[3]);
  swap16(b[0], b[1]);
  swap16(b[2], b[3]);
}

template <int EPI>
__global__ __launch_bounds__(NTHR) void gemm_pnt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                        int lda, int ldb, int M, int N, int nk, bf16* __restrict__ C,
                                                        int ldc, const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                        int ldy, float* __restrict__ dbias_part, int ntiles) {
  __shared__ __attribute__((aligned(16))) bf16 smem[STAGES * 2 * TILE];  // [stage][A|B][256][32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int tiles_n = N / BN;
  const int G = gridDim.x;
  // tiles of this workgroup: T_i = round_i · G + slot, with each XCD (b % 8)
  // holding a contiguous chunk of every round — neighbouring tiles share an
  // A row panel, which then stays in that XCD's L2
  const int b = blockIdx.x;
  int slot;
  {
    const int xcd = b & 7, s = b >> 3, q = G >> 3, r = G & 7;
    slot = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + s;
  }
  const int my_tiles = ntiles > slot ? (ntiles - slot + G - 1) / G : 0;
  const int total = my_tiles * nk;  // k-stages this workgroup runs
  if (total == 0) return;

  const int wu = __builtin_amdgcn_readfirstlane(w);
  // per-lane DMA source offsets within a tile (row, swizzled chunk)
  size_t offA[2], offB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (2 * w + i) + (lane >> 2);
    const int ch = (lane & 3) ^ swz(r);
    offA[i] = (size_t)r * lda + ch * 8;
    offB[i] = (size_t)r * ldb + ch * 8;
  }
  const int fo = (lane & 15) * BK + (((lane >> 4) ^ swz(lane & 15)) << 3);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16*)smem;
  auto glds = [](const bf16* src, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_byte)
                 : "memory");
  };
  // loader cursor: global stage ld → (tile ld_t of this WG, k-stage ld_k)
  int ld_t = 0, ld_k = 0;
  const bf16* ldA = nullptr;
  const bf16* ldB = nullptr;
  auto tile_base = [&](int t) {
    const int tile = t * G + slot;
    const int tn = tile % tiles_n, tm = tile / tiles_n;
    ldA = A + (size_t)(tm * BM) * lda;
    ldB = B + (size_t)(tn * BN) * ldb;
  };
  tile_base(0);
  auto load_next = [&](int g) {  // DMA of global stage g (the cursor's stage)
    const unsigned abase = lds0 + (unsigned)((g % STAGES) * 2 * TILE) * 2u, bbase = abase + TILE * 2u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned off = (unsigned)((2 * wu + i) * 1024);
      glds(ldA + offA[i] + (size_t)ld_k * BK, abase + off);
      glds(ldB + offB[i] + (size_t)ld_k * BK, bbase + off);
    }
    if (++ld_k == nk) {
      ld_k = 0;
      if (++ld_t < my_tiles) tile_base(ld_t);
    }
  };
  // wait until this wave's DMA of a stage landed, given `after` later stages
  // issued (0..3) and whether an epilogue's stores were issued after it
  auto wait_stage = [](int after, bool epi) {
    static_assert(STAGES == 5, "0..3 stages in flight after the awaited one");
    constexpr int E = EpiVm<EPI>::n;
    if (epi) {
      if (after >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(12 + E) : "memory");
      else if (after == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + E) : "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 + E) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(E) : "memory");
    } else {
      if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // bias-gradient partials of the current tile (EPI 3): 16 columns per lane
  const int q = lane >> 4, r16 = lane & 15;

  for (int t = 0; t < STAGES - 1; ++t)
    if (t < total) load_next(t);
  wait_stage(min(total - 1, STAGES - 2), false);
  __builtin_amdgcn_s_barrier();
  const bool g1 = wu >= 4;
  if (g1) __builtin_amdgcn_s_barrier();
  int kk = 0, ti = 0;          // k-stage within the tile, tile index of this WG
  int last_epi = -(1 << 20);  // global stage whose epilogue ran last
  for (int s = 0; s < total; ++s) {
    const bf16* As = smem + (s % STAGES) * 2 * TILE + wm * 128 * BK + fo;
    const bf16* Bs = smem + (s % STAGES) * 2 * TILE + TILE + wn * 64 * BK + fo;
    bf16x8 xf[8], wf[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = *reinterpret_cast<const bf16x8*>(As + i * 16 * BK);
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(Bs + j * 16 * BK);
    if (s + STAGES - 1 < total) load_next(s + STAGES - 1);
    if (s + 1 < total) {
      // stage s+1 was issued in iteration s+2-STAGES; an epilogue after it
      // ran in one of the iterations s+2-STAGES .. s-1
      const bool epi = last_epi >= s + 2 - STAGES;
      wait_stage(min(total - 1, s + STAGES - 1) - (s + 1), epi);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j], xf[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (++kk < nk) continue;
    // ---------------- tile epilogue (registers → global) ----------------
    kk = 0;
    const int tile = ti * G + slot;
    ++ti;
    last_epi = s;
    const int tn = tile % tiles_n, tm = tile / tiles_n;
    const int ncol = tn * BN + wn * 64 + 16 * q;  // this lane's 16 columns after the transpose
    f32x8 b0, b1;
    f32x4 bq[4];  // EPI 1: bias of the accumulator's own columns, added before the rounding
    if constexpr (EPI == 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x4 v = *reinterpret_cast<const bf16x4*>(bias + tn * BN + wn * 64 + 16 * j + 4 * q);
        bq[j] = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
      }
    }
    if constexpr (EPI >= 2) {
      b0 = to_f32(*reinterpret_cast<const bf16x8*>(bias + ncol));
      b1 = to_f32(*reinterpret_cast<const bf16x8*>(bias + ncol + 8));
    }
    f32x8 cp0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, cp1 = cp0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      u32x2 blk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (EPI == 1) blk[j] = pack4(acc[i][j] + bq[j]);
        else blk[j] = pack4(acc[i][j]);
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
      transpose_blocks(blk);
      const size_t m = (size_t)(tm * BM + wm * 128 + 16 * i + r16);
      const bf16x8 v0 = join(blk[0], blk[1]), v1 = join(blk[2], blk[3]);
      bf16* crow = C + m * ldc + ncol;
      if constexpr (EPI <= 1) {
        *reinterpret_cast<bf16x8*>(crow) = v0;
        *reinterpret_cast<bf16x8*>(crow + 8) = v1;
      } else if constexpr (EPI == 2) {
        *reinterpret_cast<bf16x8*>(crow) = v0;
        *reinterpret_cast<bf16x8*>(crow + 8) = v1;
        const f32x8 x0 = to_f32(v0) + b0, x1 = to_f32(v1) + b1;
        f32x8 y0, y1;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          y0[e] = gelu_sig(x0[e]);
          y1[e] = gelu_sig(x1[e]);
        }
        bf16* yrow = Y + m * ldy + ncol;
        *reinterpret_cast<bf16x8*>(yrow) = to_bf16(y0);
        *reinterpret_cast<bf16x8*>(yrow + 8) = to_bf16(y1);
      } else {
        const bf16* yrow = Y + m * ldy + ncol;
        const f32x8 x0 = to_f32(*reinterpret_cast<const bf16x8*>(yrow)) + b0;
        const f32x8 x1 = to_f32(*reinterpret_cast<const bf16x8*>(yrow + 8)) + b1;
        const f32x8 d0f = to_f32(v0), d1f = to_f32(v1);
        f32x8 d0, d1;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          d0[e] = d0f[e] * gelu_sig_grad(x0[e]);
          d1[e] = d1f[e] * gelu_sig_grad(x1[e]);
        }
        const bf16x8 o0 = to_bf16(d0), o1 = to_bf16(d1);
        // the bias gradient sums what is stored (the rounded values)
        cp0 += to_f32(o0);
        cp1 += to_f32(o1);
        *reinterpret_cast<bf16x8*>(crow) = o0;
        *reinterpret_cast<bf16x8*>(crow + 8) = o1;
      }
    }
    if constexpr (EPI == 3) {
      // 16 lanes of a group hold 16 rows each (×8 fragments) of the same
      // columns: reduce over the group, one partial row per (M-tile, wm)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          cp0[e] += __shfl_xor(cp0[e], o, 64);
          cp1[e] += __shfl_xor(cp1[e], o, 64);
        }
      }
      if (r16 == 0) {
        float* prow = dbias_part + (size_t)(2 * tm + wm) * N + ncol;
        *reinterpret_cast<f32x4*>(prow) = f32x4{cp0[0], cp0[1], cp0[2], cp0[3]};
        *reinterpret_cast<f32x4*>(prow + 4) = f32x4{cp0[4], cp0[5], cp0[6], cp0[7]};
        *reinterpret_cast<f32x4*>(prow + 8) = f32x4{cp1[0], cp1[1], cp1[2], cp1[3]};
        *reinterpret_cast<f32x4*>(prow + 12) = f32x4{cp1[4], cp1[5], cp1[6], cp1[7]};
      }
    }
  }
  if (!g1) __builtin_amdgcn_s_barrier();  // balance the stagger
}

}  // namespace

int gemm_pnt_ok(int M, int N, int K, int lda, int ldb, int ldc) {
  return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0 && K / BK >= STAGES - 1 && lda % 8 == 0 &&
         ldb % 8 == 0 && ldc % 8 == 0 && lda >= K && ldb >= K && ldc >= N;
}

int gemm_pnt_dbias_rows(int M) { return 2 * (M / BM); }

int gemm_pnt(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
             const bf16* bias, bf16* Y, int ldy, float* dbias_part, int grid, hipStream_t st) {
  if (!gemm_pnt_ok(M, N, K, lda, ldb, ldc)) return -2;
  if (epi != 0 && !bias) return -3;
  if ((epi == 2 || epi == 3) && (!Y || ldy % 8 || ldy < N)) return -3;
  if (epi == 3 && !dbias_part) return -3;
  const long long ntiles = (long long)(M / BM) * (N / BN);
  if (ntiles > 0x7fffffffLL) return -2;
  if (grid <= 0) grid = 256;  // one workgroup per CU (160 KiB LDS each)
  if (grid > ntiles) grid = (int)ntiles;
  const int nk = K / BK;
  const int nt = (int)ntiles;
  switch (epi) {
    case 0: gemm_pnt_kernel<0><<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, nt); break;
    case 1: gemm_pnt_kernel<1><<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, nt); break;
    case 2: gemm_pnt_kernel<2><<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, nt); break;
    case 3: gemm_pnt_kernel<3><<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, nt); break;
    default: return -4;
  }
  return 0;
}

}  // namespace pdo
