// SPDX-License-Identifier: Apache-2.0
// C[M][N] = A[M][K] · B[N][K]ᵀ on gfx950 — the TWO-workgroups-per-CU persistent
// mainloop for the fused-epilogue GEMMs (gemm_nt's EPI 2: fc1 + GELU, EPI 3:
// fc2 dX ⊙ GELU′ + bias-gradient partials; same contract and epilogues as
// gemm_nt4.hip).
//
// Why a second mainloop: gemm_nt4 runs one wave per SIMD with 128 × 128
// outputs per wave (256 accumulator registers), so its row epilogue — the
// GELU / GELU′ VALU work, 7-11 instructions per output element — issues with
// the matrix pipe idle (PMC, profiles/r3_nt4_deferred_drain.md: the fused
// forms take 83 / 150 µs more than the plain GEMM of the same shape).  Here a
// workgroup owns 256 × 128 outputs (4 waves × 128 × 64, 128 accumulator
// registers each) and uses 72 KiB of LDS, so two workgroups share a CU: while
// one runs its epilogue on the SIMDs' vector ALUs, the other's MFMAs keep the
// matrix pipes busy.  The two fall out of phase by themselves after the first
// epilogue and stay there.
//
// Mainloop: BK = 32 (one v_mfma_f32_16x16x32_bf16 k-step), a 3-stage LDS ring
// of [256 | 128][32] bf16 (24 KiB a stage) filled by LDS-DMA two k-steps ahead
// (6 one-KiB pieces per wave per step, swizzle applied on the source address),
// one barrier per k-step.  The k-steps of consecutive tiles form one stream:
// the ring refill at the end of a tile already fetches the next tile's first
// steps, so the next tile's loads fly under this tile's epilogue.
//
// Layouts: LDS rows are 64 B (4 chunks of 16 B); chunk c of row r sits at
// c ^ ((r >> 2) & 3), so a ds_read_b128 lane group's 16 rows cover all 64
// banks.  B's rows are permuted in LDS (physical row 16j + t of a wave's
// 64-column block holds column 4t + j): lane t's four accumulator blocks j are
// four consecutive output columns, stored as one 8-B bf16x4 per row.
// Accumulator (i, j, e): C[m0 + 128·wm + 16i + 4(l >> 4) + e][n0 + 64·wn + 4(l & 15) + j].
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int BM = 256, BN = 128, BK = 32, NS = 3, NTHR = 256;
constexpr int SA = BM * BK * 2;      // 16 KiB
constexpr int SB = BN * BK * 2;      // 8 KiB
constexpr int STG = SA + SB;         // 24 KiB per stage
constexpr int PPW = (SA + SB) / 1024 / 4;  // DMA pieces per wave per k-step (6)

template <int EPI>
__global__ __launch_bounds__(NTHR, 2) void gemm_nt2_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           int lda, int ldb, int M, int N, int nk,
                                                           bf16* __restrict__ C, int ldc,
                                                           const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                           int ldy, float* __restrict__ dbias_part, int group_m) {
  __shared__ __attribute__((aligned(16))) char smem[NS * STG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_n = N / BN, tiles_m = M / BM;
  const int nwg = tiles_m * tiles_n;
  // epilogue vector-memory operations per wave (stores, pre-activation and bias loads)
  constexpr int NVM = EPI == 0 ? 32 : EPI == 1 ? 33 : 65;
  constexpr int WEPI = PPW + NVM > 63 ? 63 : PPW + NVM;
  constexpr int WEPI0 = NVM > 63 ? 63 : NVM;

  auto coords = [&](int v, int& tm_, int& tn_) {
    int id = v;
    {  // bijective XCD remap: each XCD walks a contiguous range of tiles
      const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
      id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
    }
    // grouped order: group_m tile rows, then the next tile column (shared panels in the XCD's L2)
    const int per_group = group_m * tiles_n;
    const int g = id / per_group, first_m = g * group_m;
    const int gsz = min(tiles_m - first_m, group_m), r = id - g * per_group;
    tm_ = first_m + r % gsz;
    tn_ = r / gsz;
  };

  // ---- LDS-DMA: wave w moves A pieces w + 4i (i < 4) and B pieces w + 4i (i < 2);
  // a piece is 16 rows × 64 B; lane L → row 16p + (L >> 2), LDS chunk L & 3,
  // global chunk (L & 3) ^ ((L >> 4) & 3) (= the swizzle of that row)
  const int lch = (lane & 3) ^ ((lane >> 4) & 3);
  const unsigned voffA = (unsigned)(((lane >> 2) * lda + lch * 8) * 2);
  const unsigned voffB = (unsigned)((4 * (lane >> 2) * ldb + lch * 8) * 2);  // B rows: 4t + j
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem + (unsigned)(w * 1024);
  auto glds = [](unsigned voff, const bf16* sbase, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_byte)
                 : "memory");
  };
  // pieces of k-step kt of tile (tm, tn) into stage s
  auto issue = [&](int tm_, int tn_, int kt, int s) {
    const bf16* a = A + ((size_t)tm_ * BM + 16 * w) * lda + (size_t)kt * BK;
    // B piece p = w + 4i: wave block p >> 2 = i (64 columns), j = p & 3 = w
    const bf16* b = B + ((size_t)tn_ * BN + w) * ldb + (size_t)kt * BK;
    const unsigned base = lds0 + (unsigned)(s * STG);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds(voffA, a + (size_t)64 * i * lda, base + (unsigned)(4096 * i));
#pragma unroll
    for (int i = 0; i < 2; ++i) glds(voffB, b + (size_t)64 * i * ldb, base + (unsigned)(SA + 4096 * i));
  };

  // ---- fragments: row (l & 15) of a 16-row block, k chunk (l >> 4), swizzled
  const int pch = (lane >> 4) ^ ((lane >> 2) & 3);
  const int oA = (wm * 128 + (lane & 15)) * 64 + pch * 16;
  const int oB = SA + (wn * 64 + (lane & 15)) * 64 + pch * 16;

  f32x4 acc[8][4];

  // ---- epilogue of tile (tm, tn) from acc
  auto epilogue = [&](int tm_, int tn_) {
    const int g4 = lane >> 4;
    const int nb = tn_ * BN + wn * 64 + 4 * (lane & 15);
    const size_t mr = (size_t)tm_ * BM + wm * 128 + 4 * g4;
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI >= 1) {
      const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + nb);
      bv = f32x4{(float)b4[0], (float)b4[1], (float)b4[2], (float)b4[3]};
    }
    f32x4 colp = {0.f, 0.f, 0.f, 0.f};
    f32x2 m1 = {-1.f, -1.f};
    asm volatile("" : "+v"(m1));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      bf16x4 pre[4];
      if constexpr (EPI == 3) {
#pragma unroll
        for (int e = 0; e < 4; ++e) pre[e] = *reinterpret_cast<const bf16x4*>(Y + (mr + 16 * i + e) * ldy + nb);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x4 v = {acc[i][0][e], acc[i][1][e], acc[i][2][e], acc[i][3][e]};
        const size_t m = mr + 16 * i + e;
        bf16x4* crow = reinterpret_cast<bf16x4*>(C + m * ldc + nb);
        if constexpr (EPI <= 1) {
          const f32x4 o = v + bv;
          *crow = bf16x4{(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
        } else if constexpr (EPI == 2) {
          *crow = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          const f32x4 x = v + bv;
          const f32x2 y0 = gelu_sig2(f32x2{x[0], x[1]}), y1 = gelu_sig2(f32x2{x[2], x[3]});
          *reinterpret_cast<bf16x4*>(Y + m * ldy + nb) = bf16x4{(bf16)y0[0], (bf16)y0[1], (bf16)y1[0], (bf16)y1[1]};
        } else {
          const f32x4 x = f32x4{(float)pre[e][0], (float)pre[e][1], (float)pre[e][2], (float)pre[e][3]} + bv;
          const f32x2 d0 = f32x2{v[0], v[1]} * gelu_sig_grad2(f32x2{x[0], x[1]}, m1);
          const f32x2 d1 = f32x2{v[2], v[3]} * gelu_sig_grad2(f32x2{x[2], x[3]}, m1);
          const f32x4 d = {d0[0], d0[1], d1[0], d1[1]};
          colp += d;
          *crow = bf16x4{(bf16)d[0], (bf16)d[1], (bf16)d[2], (bf16)d[3]};
        }
      }
    }
    if constexpr (EPI == 3) {
      // partial row 4·wm + (l >> 4) of this M-tile's 8 (gemm_nt_dbias_rows layout)
      *reinterpret_cast<f32x4*>(dbias_part + (size_t)(8 * tm_ + 4 * wm + g4) * N + nb) = colp;
    }
  };

  // ---- the k-step stream over this workgroup's tiles
  int v = blockIdx.x;
  if (v >= nwg) return;
  int tm, tn;
  coords(v, tm, tn);
  // the step after the current one (tile-relative), for the ring refill two ahead
  int tm1 = tm, tn1 = tn, kt1 = 1, v1 = v;  // step g+1
  bool has1 = nk > 1;
  if (nk == 1) {  // (host contract: nk ≥ 3; kept for clarity)
    v1 = v + gridDim.x;
    has1 = v1 < nwg;
    if (has1) coords(v1, tm1, tn1);
    kt1 = 0;
  }
  issue(tm, tn, 0, 0);
  if (has1) issue(tm1, tn1, kt1, 1);
  int s = 0;          // stage of the current step
  int kt = 0;         // k-step of the current step within its tile
  bool after_epi = false;
  for (;;) {
    // ---- wait for this step's pieces: issued after them are step g+1's pieces (if
    // any) and, right after a tile boundary, the epilogue's memory operations
    if (after_epi) {
      if (has1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WEPI) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WEPI0) : "memory");
    } else {
      if (has1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // step g landed for every wave; step g-1's reads all done
    // ---- refill the stage step g-1 used with step g+2
    int tm2 = tm1, tn2 = tn1, kt2 = kt1 + 1, v2 = v1;
    bool has2 = has1;
    if (has1 && kt2 >= nk) {
      v2 = v1 + gridDim.x;
      has2 = v2 < nwg;
      if (has2) coords(v2, tm2, tn2);
      kt2 = 0;
    }
    if (has2) issue(tm2, tn2, kt2, s == 0 ? 2 : s - 1);
    // ---- 32 MFMAs on stage s: 12 fragments (B 0-3, A 0-7), A-stationary runs
    const char* st = smem + s * STG;
    bf16x8 fb[4], fa[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(st + oB + j * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(st + oA + i * 1024);
    if (kt == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    // ---- advance: step g+1 becomes current
    after_epi = false;
    if (kt + 1 == nk) {
      epilogue(tm, tn);
      after_epi = true;
    }
    if (!has1) break;
    s = s == 2 ? 0 : s + 1;
    tm = tm1;
    tn = tn1;
    kt = kt1;
    tm1 = tm2;
    tn1 = tn2;
    kt1 = kt2;
    v1 = v2;
    has1 = has2;
  }
}

}  // namespace

int gemm_nt2_ok(int M, int N, int K) { return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0 && K / BK >= 3; }

// two workgroups per CU, persistent over the tiles
int gemm_nt2(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
             const bf16* bias, bf16* Y, int ldy, float* dbias_part, hipStream_t st) {
  if (!gemm_nt2_ok(M, N, K) || lda % 8 || ldb % 8 || ldc % 4 || ldy % 4) return -2;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n >= 8 ? n / 8 * 8 : 8;
  }();
  static const int group_m = [] {
    const char* e = getenv("PDO_NT2_GROUP_M");
    const int g = e ? atoi(e) : 8;
    return g >= 1 ? g : 1;
  }();
  const long long tiles = (long long)(M / BM) * (N / BN);
  const int g = (int)(tiles < 2LL * ncu ? tiles : 2LL * ncu);
  const int nk = K / BK;
  switch (epi) {
    case 0: gemm_nt2_kernel<0><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
    case 1: gemm_nt2_kernel<1><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
    case 2: gemm_nt2_kernel<2><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
    case 3: gemm_nt2_kernel<3><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
    default: return -4;
  }
  return 0;
}

}  // namespace pdo
