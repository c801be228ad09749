// SPDX-License-Identifier: Apache-2.0
// Weight-gradient GEMM C[M][N] (+)= Σ_t A[t][M] · B[t][N]  (bf16 in, fp32 acc)
// for gfx950 — dW = dYᵀ·X with both operands in their natural token-major
// layout, the "NT" case that hipBLASLt runs at ≈1.08 PF on the GPT-2-medium
// shapes (against 1.3-1.7 PF for the forward's layout).
//
// Both MFMA operands need 8 consecutive tokens per lane while memory holds
// rows of tokens, i.e. a transpose.  Here it costs nothing: the token-major
// tiles are staged into LDS as they are in memory and every fragment is read
// with ds_read_b64_tr_b16 (the hardware transposing LDS read — the same
// recipe as attention's V operand).  A and B use the same permuted token
// order inside a 16-token MFMA step, so their products pair up.
//
// Tile: 256 (M) × 256 (N) × 64 tokens per k-step, 8 waves as 2 (M) × 4 (N),
// each wave 128 × 64 = 4 × 2 accumulators of v_mfma_f32_32x32x16_bf16.
// LDS: 2 stages × (A + B) × [64 tokens][256] bf16 = 128 KiB (one workgroup per
// CU), 16-B chunk index XOR (token & 3)·4 so the transposed reads of 4 token
// rows × 64 B per half-wave hit 4 distinct 64-B bank groups.
// Staging is LDS-DMA (global_load_lds_dwordx4, swizzle on the source
// address); the two waves of each SIMD ping-pong between MFMA and LDS-read
// phases (details at the loop).  Long token axis: split-K over token slices
// (bf16 partials + the HIP fold, reduce.hip splitk_add), sized for one resident
// round; workgroup ids remapped so the workgroups sharing an A or B panel run
// on one XCD (shared L2).  Measured: 1.05-1.21 PF vs hipBLASLt's 0.86-1.15 PF
// on the same shapes (tools/dw_probe.py --pdo-only); the register-staged and
// plain LDS-DMA 2-barrier versions of this tiling ran 0.92-0.95 PF, and a
// 16x16x32 version over a 5-deep ring of 32-token stages (gemm_nt.hip's
// schedule, which gained 5 % there) ran 8-20 % slower here: qkv 445, proj
// 165, fc1 546, fc2 523 µs (tools/dw_probe.py).
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int LROW = 256;                 // LDS row (elements) of a [BK][256] tile
constexpr int TILE = BK * LROW;           // elements per operand tile
constexpr int NTHR = 512;

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// element offset of (token row r, 16-B chunk ch) in the swizzled LDS tile
__device__ __forceinline__ int loff(int r, int ch) { return r * LROW + ((ch ^ ((r & 3) << 2)) << 3); }

// per-lane element offset of the transposed fragment for k0 = 0 and columns
// [cb, cb + 32); tokens k0 + 4·(lane>>5) + q and +8 (q = (lane>>2)&3)
__device__ __forceinline__ int frag_base(int cb, int lane) {
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int col = cb + 16 * (g & 1) + 4 * p;
  const int r0 = 4 * (g >> 1) + q;
  return loff(r0, col >> 3) + (col & 7);
}

template <int K0>
__device__ __forceinline__ bf16x8 frag(const bf16* T) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(T + K0 * LROW));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(T + (K0 + 8) * LROW));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__global__ __launch_bounds__(NTHR) void gemm_dw_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       int lda, int ldb, int M, int N, int ksteps_total, int splits,
                                                       bf16* __restrict__ C, int ldc, long long split_stride,
                                                       int accumulate) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE];  // [stage][A|B][BK][256]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int tiles_n = N / BN, tiles_m = M / BM;
  const int nwg = tiles_m * tiles_n * splits;
  // XCD remap: hardware ids go round-robin over the 8 XCDs; give each XCD a
  // contiguous range of logical ids (bijective for any nwg)
  int id = blockIdx.x;
  {
    const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tn = id % tiles_n;
  const int tm = (id / tiles_n) % tiles_m;
  const int split = id / (tiles_n * tiles_m);
  // token slice of this split: k-steps [k0, k1)
  const int kq = ksteps_total / splits, kr = ksteps_total % splits;
  const int k0 = split * kq + min(split, kr);
  const int nk = kq + (split < kr ? 1 : 0);
  const int m0 = tm * BM, n0 = tn * BN;

  const bf16* Ab = A + (size_t)k0 * BK * lda + m0;
  const bf16* Bb = B + (size_t)k0 * BK * ldb + n0;

  // LDS-DMA staging (global_load_lds_dwordx4): one wave-instruction fills 1 KiB
  // of LDS = 2 token rows, lane l → row 2·(4w+i) + (l>>5), LDS chunk l&31.  The
  // image is lane-linear, so the XOR swizzle goes on the SOURCE address: the
  // lane fetches global chunk (l&31) ^ 4·(row&3), which loff() reads back.
  const int wu = __builtin_amdgcn_readfirstlane(w);
  int src_off[4];  // element offset of this lane's source chunk, relative to the k-step's first row
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = 2 * (4 * w + i) + (lane >> 5);
    src_off[i] = (((lane & 31) ^ ((r & 3) << 2)) << 3);
  }
  const int fa[4] = {frag_base(wm * 128 + 0, lane), frag_base(wm * 128 + 32, lane), frag_base(wm * 128 + 64, lane),
                     frag_base(wm * 128 + 96, lane)};
  const int fb[2] = {frag_base(wn * 64 + 0, lane), frag_base(wn * 64 + 32, lane)};

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  // Ping-pong: waves 4-7 run one barrier interval behind waves 0-3, so on
  // every SIMD one wave issues its 8 MFMAs while the other issues the next
  // step's 12 transposed LDS reads (+ this tile's share of the next tile's
  // LDS-DMA).  Per 16-token step: R (reads [+ DMA]; lgkmcnt(0)) | barrier |
  // M (8 MFMAs) | barrier.  The next tile's DMA goes out in steps 0-1 and is
  // drained (vmcnt(0)) in step 3's R, one barrier before anyone reads it; its
  // buffer's last reads (previous tile, step 3) retired before the barrier
  // that precedes the DMA issue.
  // LDS-DMA in inline asm: hipcc does not count these, so it neither drains
  // them before every ds_read (what it does for the builtin: it cannot prove
  // the DMA target and the reads apart) nor at the raw barriers — the only
  // wait is the explicit vmcnt(0) in step 3
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16*)smem;
  auto glds = [](const bf16* src, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_byte)
                 : "memory");
  };
  auto load_half = [&](int kt, int buf, int h) {
    const unsigned abase = lds0 + (unsigned)(buf * 2 * TILE) * 2u, bbase = abase + TILE * 2u;
#pragma unroll
    for (int i = 2 * h; i < 2 * h + 2; ++i) {
      const int r = 2 * (4 * w + i) + (lane >> 5);
      const size_t row = (size_t)(kt * BK + r);
      const unsigned off = (unsigned)((4 * wu + i) * 512) * 2u;
      glds(Ab + row * lda + src_off[i], abase + off);
      glds(Bb + row * ldb + src_off[i], bbase + off);
    }
  };
  load_half(0, 0, 0);
  load_half(0, 0, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const bool g1 = wu >= 4;
  if (g1) __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    const bf16* As = smem + buf * 2 * TILE;
    const bf16* Bs = As + TILE;
#define PDO_DW_PP(KS, PRE)                                                     \
    {                                                                          \
      bf16x8 a0 = frag<16 * KS>(As + fa[0]), a1 = frag<16 * KS>(As + fa[1]);   \
      bf16x8 a2 = frag<16 * KS>(As + fa[2]), a3 = frag<16 * KS>(As + fa[3]);   \
      bf16x8 b0 = frag<16 * KS>(Bs + fb[0]), b1 = frag<16 * KS>(Bs + fb[1]);   \
      PRE                                                                      \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                       \
      __builtin_amdgcn_sched_barrier(0);                                       \
      __builtin_amdgcn_s_barrier();                                            \
      __builtin_amdgcn_sched_barrier(0);                                       \
      __builtin_amdgcn_s_setprio(1);                                           \
      acc[0][0] = mfma(a0, b0, acc[0][0]);                                     \
      acc[0][1] = mfma(a0, b1, acc[0][1]);                                     \
      acc[1][0] = mfma(a1, b0, acc[1][0]);                                     \
      acc[1][1] = mfma(a1, b1, acc[1][1]);                                     \
      acc[2][0] = mfma(a2, b0, acc[2][0]);                                     \
      acc[2][1] = mfma(a2, b1, acc[2][1]);                                     \
      acc[3][0] = mfma(a3, b0, acc[3][0]);                                     \
      acc[3][1] = mfma(a3, b1, acc[3][1]);                                     \
      __builtin_amdgcn_s_setprio(0);                                           \
      __builtin_amdgcn_sched_barrier(0);                                       \
      __builtin_amdgcn_s_barrier();                                            \
      __builtin_amdgcn_sched_barrier(0);                                       \
    }
    PDO_DW_PP(0, if (more) load_half(kt + 1, buf ^ 1, 0);)
    PDO_DW_PP(1, if (more) load_half(kt + 1, buf ^ 1, 1);)
    PDO_DW_PP(2, )
    PDO_DW_PP(3, asm volatile("s_waitcnt vmcnt(0)" ::: "memory");)
#undef PDO_DW_PP
  }
  if (!g1) __builtin_amdgcn_s_barrier();  // balance the stagger

  // epilogue: acc[mb][nb][r] = C[m0 + wm·128 + 32mb + (r&3) + 8(r>>2) + 4hh][n0 + wn·64 + 32nb + lane&31]
  bf16* Cb = C + (size_t)split * split_stride;
  const int hh = lane >> 5, li = lane & 31;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const int n = n0 + wn * 64 + 32 * nb + li;
        bf16* p = Cb + (size_t)m * ldc + n;
        float v = acc[mb][nb][r];
        if (accumulate) v += (float)*p;
        *p = (bf16)v;
      }
}

}  // namespace

// 4-wave mainloop (gemm_dw4.hip) where its contract holds: impl 1 (default) =
// the half-buffer refill schedule on 16x16x32 MFMAs, impl 2 = the same on
// 32x32x16 (isolated: qkv 333 -> 325 us, proj 125 -> 118, fc1 404 -> 400, fc2
// 409 -> 403 for impl 1; step 144.7 -> 143.4 ms, profiles/r3_dw4_m16.md);
// impl 0 = the 8-wave loop below.
// gemm_dw_impl() in the module selects one (probes and tests)
static int g_dw_impl = 1;
void gemm_dw_set_impl(int impl) { g_dw_impl = impl; }
int gemm_dw_get_impl() { return g_dw_impl; }

// gemm_dw4: k-tiles dealt to the slices in pairs, ≥ 2 pairs per slice; ≤ 256
// workgroups (one resident round, one workgroup per CU) unless the tiles alone exceed it
static int dw4_splits(long long T, int M, int N) {
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const long long ks = T / BK;
  if (tiles > 256) {
    // several rounds of one workgroup per CU: the smallest split whose last round
    // is nearly full (LM head, 788 tiles: 1 slice = 3.08 rounds in 4, 4 slices = 12.3 in 13)
    for (int s = 1; s <= 8; ++s) {
      if (ks % 2 || (ks / 2) / s < 2) continue;
      const long long wg = (long long)tiles * s, rounds = (wg + 255) / 256;
      if (wg * 100 >= rounds * 256 * 94) return s;
    }
  }
  // the most slices that keep one resident round (≤ 256 workgroups): qkv's 48 tiles
  // take 5 uneven slices (240 workgroups) instead of 4 even ones (192)
  for (int s = 16; s >= 1; --s) {
    if ((long long)tiles * s > 256 && s > 1) continue;
    if (ks % 2 == 0 && (ks / 2) / s >= 2) return s;
  }
  return 0;
}

int gemm_dw_splits(long long T, int M, int N) {
  if (M % (BM / 2) || N % BN || T % BK || T <= 0) return 0;
  if (g_dw_impl >= 1) {
    const int s = dw4_splits(T, M, N);
    if (s) return s;
  }
  if (M % BM) return 0;  // the half-height edge tile is gemm_dw4's only
  // one resident round of ≤ 256 workgroups (one per CU), as many as fit:
  // measured, 240 WGs in one round beat 768 in three (per-WG prologue, fold)
  const int tiles = (M / BM) * (N / BN);
  const long long ks = T / BK;
  int s = tiles >= 256 ? 1 : 256 / tiles;
  if (s > 16) s = 16;
  while (s > 1 && ks / s < 16) --s;
  return s;
}

int gemm_dw(const bf16* A, const bf16* B, long long T, int M, int N, int lda, int ldb, bf16* C, int ldc,
            int accumulate, bf16* ws, int splits, hipStream_t st) {
  if (M % (BM / 2) || N % BN || T % BK || splits < 1 || splits > 16) return -2;
  const long long ks = T / BK;
  if (ks < splits || ks > 0x7fffffffLL) return -2;
  if (g_dw_impl >= 1) {
    const int rc = gemm_dw4(A, B, T, M, N, lda, ldb, C, ldc, accumulate, ws, splits, st, g_dw_impl - 1);
    if (rc != -2) return rc;  // -2: this split count breaks its contract → the 8-wave loop
  }
  if (M % BM) return -2;
  const int tiles = (M / BM) * (N / BN);
  const int grid = tiles * splits;
  if (splits == 1) {
    gemm_dw_kernel<<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, (int)ks, 1, C, ldc, 0, accumulate);
    return 0;
  }
  if (!ws) return -3;
  if (ldc != N) return -4;
  const long long mn = (long long)M * N;
  gemm_dw_kernel<<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, (int)ks, splits, ws, N, mn, 0);
  return splitk_add(ws, splits, mn, C, accumulate, st);
}

}  // namespace pdo
