// SPDX-License-Identifier: Apache-2.0
// Weight-gradient GEMM C[M][N] (+)= Σ_t A[t][M] · B[t][N] on gfx950 — the
// 4-wave, one-wave-per-SIMD mainloop (same contract as gemm_dw.hip, selected
// by gemm_dw_set_impl).  The operand handling is gemm_dw's: token-major tiles
// staged into LDS as they lie in memory (LDS-DMA, swizzle on the source
// address) and every fragment read with ds_read_b64_tr_b16; the schedule is
// gemm_nt4's (profiles/r2_gemm_nt4.md): each wave owns 128 × 128 outputs = 16
// v_mfma_f32_32x32x16_bf16 accumulators (256 registers, pinned to the
// accumulator file), and one instruction stream per wave interleaves MFMAs,
// transposed reads and DMA:
//
//   tile t (64 tokens, LDS buffer t&1), two barriers per tile: each 32-token
//   half of a buffer is refilled with tile t+2 as soon as every wave has read
//   it, so every DMA piece has ≈ 1.5 tiles of lead (hipBLASLt's gfx950 loop
//   does the same with three barriers).
//
// RAW / WAR: a buffer half is refilled only after the barrier that follows
// every wave's last read of it; a tile is read only after every wave retired
// its own DMA of it and passed a barrier.  (Round 4 housekeeping: the
// one-barrier schedules of round 2 measured slower and were removed,
// profiles/r2_gemm_nt4.md.)
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int LROW = 256;             // LDS row (elements) of a [BK][256] tile
constexpr int TILE = BK * LROW;       // elements per operand tile
constexpr int OPB = TILE * 2;         // bytes per operand tile (32 KiB)
constexpr int NTHR = 256;

// element offset of (token row r, 16-B chunk ch) in the swizzled LDS tile
__device__ __forceinline__ int loff(int r, int ch) { return r * LROW + ((ch ^ ((r & 3) << 2)) << 3); }

// per-lane element offset of the transposed 32x32x16 fragment for columns
// [cb, cb + 32) at token 0 (gemm_dw.hip frag_base)
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

__global__ __launch_bounds__(NTHR, 1) void gemm_dw4_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           int lda, int ldb, int M, int N, int ksteps_total,
                                                           int splits, bf16* __restrict__ C, int ldc,
                                                           long long split_stride, int accumulate) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE];  // [buf][A|B][BK][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;  // M % 256 == 128: a half-height last row of tiles
  const int nwg = tiles_m * tiles_n * splits;
  int id = blockIdx.x;
  {  // bijective XCD remap (gemm_dw.hip)
    const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tn = id % tiles_n;
  const int tm = (id / tiles_n) % tiles_m;
  const int split = id / (tiles_n * tiles_m);
  // k-tiles are dealt to the splits in pairs (the mainloop runs tiles in pairs):
  // the first P % splits slices take one pair more
  const int pq = (ksteps_total >> 1) / splits, pr = (ksteps_total >> 1) % splits;
  const int k0 = 2 * (split * pq + min(split, pr));
  const int nk = 2 * (pq + (split < pr ? 1 : 0));
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- LDS-DMA: a wave-instruction fills 1 KiB = 2 token rows of 512 B.  Wave
  // w's piece i (0..7) of an operand covers rows 2(4i + w) + (l >> 5), LDS chunk
  // l & 31 holding global chunk (l & 31) ^ 4·(row & 3); row & 3 = (2w + (l >> 5))
  // & 3 is fixed per lane.  Per-lane byte offset in a VGPR, wave-uniform base
  // (k-tile, piece) in SGPRs.
  const int rl = lane >> 5;
  const int cs = (lane & 31) ^ (((2 * w + rl) & 3) << 2);
  // half-height edge tile (columns m0 + 128 .. m0 + 255 of A do not exist): those
  // lanes re-fetch columns m0 .. m0 + 127 — in bounds, and the rows they feed are
  // never stored
  const int csa = (m0 + BM > M && cs >= 16) ? cs - 16 : cs;
  const unsigned voffA = (unsigned)((rl * lda + csa * 8) * 2), voffB = (unsigned)((rl * ldb + cs * 8) * 2);
  const bf16* baseA = A + ((size_t)k0 * BK + 2 * w) * lda + m0;
  const bf16* baseB = B + ((size_t)k0 * BK + 2 * w) * ldb + n0;
  const unsigned stepAb = (unsigned)(16 * lda), stepBb = (unsigned)(16 * ldb);  // 8 rows, bytes
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16*)smem + (unsigned)(w * 1024);
  // M0 is not saved around the DMA: nothing else in this kernel uses it
  auto glds = [](unsigned voff, const bf16* sbase, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_byte)
                 : "memory");
  };
  struct Src {
    const char* a;
    const char* b;
    unsigned sa, sb;
  };
  auto srcs = [&](int kt) {  // laundered per tile: pieces form their bases with scalar adds
    Src r{reinterpret_cast<const char*>(baseA + (size_t)kt * BK * lda),
          reinterpret_cast<const char*>(baseB + (size_t)kt * BK * ldb), stepAb, stepBb};
    asm volatile("" : "+s"(r.a), "+s"(r.b), "+s"(r.sa), "+s"(r.sb));
    return r;
  };
  auto dma = [&](const Src& sr, auto buf_tag, int p) {  // p < 8: A piece p, else B piece p - 8
    constexpr int BUF = decltype(buf_tag)::value;
    const unsigned base = lds0 + (unsigned)(BUF * 2 * OPB);
    if (p < 8) glds(voffA, reinterpret_cast<const bf16*>(sr.a + p * sr.sa), base + (unsigned)(4096 * p));
    else glds(voffB, reinterpret_cast<const bf16*>(sr.b + (p - 8) * sr.sb), base + OPB + (unsigned)(4096 * (p - 8)));
  };

  // ---- fragments: block half h (0: tokens 0-31, 1: 32-63) holds k-steps 2h, 2h+1;
  // slot q (0..15) = k-step q >> 3, operand (q & 7) < 4 ? A mb : B nb
  const bf16* smA[2] = {smem, smem + 2 * TILE};
  int fa[4], fb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    fa[i] = frag_base(wm * 128 + 32 * i, lane);
    fb[i] = TILE + frag_base(wn * 128 + 32 * i, lane);
  }
  auto rd = [&](auto buf_tag, int h, int q) -> bf16x8 {
    constexpr int BUF = decltype(buf_tag)::value;
    const bf16* T = smA[BUF] + ((q & 7) < 4 ? fa[q & 3] : fb[q & 3]);
    const int ks = 2 * h + (q >> 3);
    switch (ks) {
      case 0: return frag<0>(T);
      case 1: return frag<16>(T);
      case 2: return frag<32>(T);
      default: return frag<48>(T);
    }
  };
  auto mma = [](f32x16& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  };
  auto mma0 = [](f32x16& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;

  f32x16 acc[4][4];  // first written by mma0 in tile 0's block 0
  bf16x8 f0[16], f1[16];

  {
    // ---- half-buffer refill schedule: each 32-token half of a buffer is
    // refilled as soon as every wave has read it — tile t+2's first half during
    // block 0 of tile t (after barrier B0: F0(t) reads done), its second half during
    // block 1 (after B1: F1(t) reads done).  Tile t+1's data therefore has ≈1.5 tiles
    // of lead (issued during tile t-1, first read after B1 of tile t) instead of ≈0.5,
    // at the price of two barriers per tile (hipBLASLt's gfx950 loop does the same
    // with three).  Pieces: first half = A 0-3, B 8-11; second half = A 4-7, B 12-15.
    {
      const Src s0 = srcs(0), s1 = srcs(1);
#pragma unroll
      for (int p = 0; p < 16; ++p) dma(s0, B0{}, p);
#pragma unroll
      for (int p = 0; p < 16; ++p) dma(s1, B1{}, p);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed (tile 1 may fly)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) f0[q] = rd(B0{}, 0, q);
    auto tileH = [&](int t, auto buf_tag, auto more_tag, auto first_tag, auto eout_tag) {
      constexpr int BUF = decltype(buf_tag)::value;
      constexpr bool MORE = decltype(more_tag)::value;
      constexpr bool FIRST = decltype(first_tag)::value;
      constexpr bool EOUT = decltype(eout_tag)::value;
      using NB = std::integral_constant<int, BUF ^ 1>;
      using SB = std::integral_constant<int, BUF>;
      Src sn2{};
      if constexpr (EOUT) sn2 = srcs(t + 2);
      // B0: every wave's F0(t) reads (buffer BUF, tokens 0-31) are done
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int ks = g >> 3, mb = (g >> 1) & 3, nb0 = 2 * (g & 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (FIRST && ks == 0) mma0(acc[mb][nb0 + u], f0[8 * ks + mb], f0[8 * ks + 4 + nb0 + u]);
          else mma(acc[mb][nb0 + u], f0[8 * ks + mb], f0[8 * ks + 4 + nb0 + u]);
        }
        f1[g] = rd(buf_tag, 1, g);
        if constexpr (EOUT) {
          if (g & 1) dma(sn2, SB{}, (g >> 1) < 4 ? (g >> 1) : (g >> 1) + 4);  // first-half pieces
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // B1: every wave's F1(t) reads are done (tokens 32-63 of BUF free) and tile t+1
      // has landed (only tile t+2's first-half pieces may still fly)
      if constexpr (MORE || EOUT) {
        if constexpr (EOUT)
          asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int ks = g >> 3, mb = (g >> 1) & 3, nb0 = 2 * (g & 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) mma(acc[mb][nb0 + u], f1[8 * ks + mb], f1[8 * ks + 4 + nb0 + u]);
        if constexpr (MORE) f0[g] = rd(NB{}, 0, g);
        if constexpr (EOUT) {
          if (g & 1) dma(sn2, SB{}, (g >> 1) < 4 ? (g >> 1) + 4 : (g >> 1) + 8);  // second-half pieces
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    tileH(0, B0{}, T_{}, T_{}, T_{});
    tileH(1, B1{}, T_{}, F_{}, T_{});
    for (int t = 2; t < nk - 2; t += 2) {
      tileH(t, B0{}, T_{}, F_{}, T_{});
      tileH(t + 1, B1{}, T_{}, F_{}, T_{});
    }
    tileH(nk - 2, B0{}, T_{}, F_{}, F_{});
    tileH(nk - 1, B1{}, F_{}, F_{}, F_{});
  }

  // ---- epilogue: acc[mb][nb][r] = C[m0 + wm·128 + 32mb + (r&3) + 8(r>>2) + 4hh][n0 + wn·128 + 32nb + (l&31)]
  // the accumulators leave through explicit v_accvgpr_read, padded against the
  // last MFMAs (hipcc does not see into the asm): 16 wait states
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  bf16* Cb = C + (size_t)split * split_stride;
  const int hh = lane >> 5, li = lane & 31;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[r]) : "a"(acc[mb][nb][r]));
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 128 + 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m >= M) continue;  // edge tile: wave-uniform (wm = 1 holds rows m0 + 128 ..)
        const int n = n0 + wn * 128 + 32 * nb + li;
        bf16* p = Cb + (size_t)m * ldc + n;
        float x = v[r];
        if (accumulate) x += (float)*p;
        *p = (bf16)x;
      }
    }
}

// ============================================================================
// The half-buffer-refill schedule on v_mfma_f32_16x16x32_bf16 (variant 0, the default).
// Same tile (256 × 256 per workgroup, 128 × 128 per wave), same DMA and
// barriers; each wave's outputs are 8 × 8 accumulators of 16 × 16 (still 256
// AGPRs), a 32-token block is ONE k-step (8 A + 8 B fragments, 64 MFMAs of
// half the 32x32x16 cycles).  Why: on random bf16 data the chip holds a higher
// clock on the 16x16x32 shape — MI355X_MICROARCH.md 'DVFS give-back' item 7
// (1.12-1.15x FLOP/s at equal cycles per FLOP in LDS-fed loops).
//
// Fragment: lane group g = l >> 4 reads 4 token rows 4g .. 4g+3 (lo) and
// 16 + 4g .. (hi) of the 16 columns cb .. cb+15 with ds_read_b64_tr_b16, so lane
// l holds column cb + (l & 15) at tokens {4g..4g+3, 16+4g..16+4g+3} — a k
// permutation shared by both operands.  The 16 rows a wave reads per
// instruction pair up as lane groups {0,1} / {2,3} (or {0,2} / {1,3}); with the
// 32x32 swizzle rows r and r + 4 would hit the same banks, so this tile's
// swizzle XORs the 32-B column pair index with (r & 3) | bit2 = b2(r) ^ b3(r):
// 8 distinct bank octets for either pairing.  The DMA's source-side swizzle
// then depends on the piece's parity (row bit 3): two per-lane offsets per operand.
__device__ __forceinline__ int swz16(int r) { return ((r & 3) | ((((r >> 2) ^ (r >> 3)) & 1) << 2)) << 1; }
__device__ __forceinline__ int loff16(int r, int ch) { return r * LROW + ((ch ^ swz16(r)) << 3); }
__device__ __forceinline__ int frag_base16(int cb, int lane) {
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int col = cb + 4 * p;
  return loff16(4 * g + q, col >> 3) + (col & 7);
}
template <int K0>
__device__ __forceinline__ bf16x8 frag16(const bf16* T) {
  const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(T + K0 * LROW));
  const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(T + (K0 + 16) * LROW));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// GATHER (the convolution weight gradient, conv.hip's conv_wgrad): B is not a
// token-major matrix but the NHWC activation gathered per tap — column
// tap·C + ci of token t is x[pixel(t, tap)][ci], zero for a padding pixel (a
// buffer_load … lds whose offset is pushed past the buffer) — and the output
// is fp32 partials [split][M][N] (folded by conv_wgrad_reduce in split order).
struct DwGather {
  const bf16* x;
  unsigned xbytes;
  int C, S, IH, IW, TA, TB;  // forward output grid: token t = (n·TA + ho)·TB + wo
  int TC;                    // R·S·C: columns past it (padding to the 256-column tile) read zeros
  float inv_TA, inv_TB;
  int st, pad;
  float* part;
};

__device__ __forceinline__ void bufld_lds(unsigned voff, __amdgpu_buffer_rsrc_t rs, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "s"(lds_byte)
               : "memory");
}

__device__ __forceinline__ void divmodf(int x, int d, float inv, int& q, int& r) {
  q = (int)((float)x * inv);
  r = x - q * d;
  if (r < 0) {
    --q;
    r += d;
  } else if (r >= d) {
    ++q;
    r -= d;
  }
}

template <bool GATHER>
__global__ __launch_bounds__(NTHR, 1) void gemm_dw4m16_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                              int lda, int ldb, int M, int N, int ksteps_total,
                                                              int splits, bf16* __restrict__ C, int ldc,
                                                              long long split_stride, int accumulate,
                                                              const DwGather gx) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE];  // [buf][A|B][BK][256]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n * splits;
  int id = blockIdx.x;
  {  // bijective XCD remap
    const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tn = id % tiles_n;
  const int tm = (id / tiles_n) % tiles_m;
  const int split = id / (tiles_n * tiles_m);
  const int pq = (ksteps_total >> 1) / splits, pr = (ksteps_total >> 1) % splits;
  const int k0 = 2 * (split * pq + min(split, pr));
  const int nk = 2 * (pq + (split < pr ? 1 : 0));
  const int m0 = tm * BM, n0 = tn * BN;

  // LDS-DMA: piece i of an operand = rows 8i + 2w + rl (rl = l >> 5), LDS chunk
  // l & 31 ← global chunk (l & 31) ^ swz16(row); swz16 of that row is fixed per
  // lane up to the piece parity (row bit 3 = i & 1)
  const int rl = lane >> 5, rw = 2 * w + rl;
  unsigned voffA[2], voffB[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int cs = (lane & 31) ^ swz16(8 * par + rw);
    const int csa = (m0 + BM > M && cs >= 16) ? cs - 16 : cs;  // half-height edge tile (as gemm_dw4_kernel)
    voffA[par] = (unsigned)((rl * lda + csa * 8) * 2);
    voffB[par] = (unsigned)((rl * ldb + cs * 8) * 2);
  }
  const bf16* baseA = A + ((size_t)k0 * BK + 2 * w) * lda + m0;
  const bf16* baseB = GATHER ? A : B + ((size_t)k0 * BK + 2 * w) * ldb + n0;
  const unsigned stepAb = (unsigned)(16 * lda), stepBb = (unsigned)(16 * ldb);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16*)smem + (unsigned)(w * 1024);
  auto glds = [](unsigned voff, const bf16* sbase, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_byte)
                 : "memory");
  };
  // GATHER: per parity, the lane's column chunk → (tap row / column offset, channel)
  int gdh[2] = {0, 0}, gdw[2] = {0, 0}, gci[2] = {0, 0};
  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(GATHER ? gx.x : A), 0, GATHER ? (int)gx.xbytes : 0, 0x00020000);
  if constexpr (GATHER) {
#pragma unroll
    for (int par = 0; par < 2; ++par) {
      const int col = n0 + (((lane & 31) ^ swz16(8 * par + rw)) << 3);
      const int tap = col / gx.C, r = tap / gx.S;
      gci[par] = col - tap * gx.C;
      gdh[par] = col < gx.TC ? r - gx.pad : -(1 << 20);  // a padding column fails every bounds check
      gdw[par] = tap - r * gx.S - gx.pad;
    }
  }
  struct Src {
    const char* a;
    const char* b;
    unsigned sa, sb;
    int kt;
  };
  auto srcs = [&](int kt) {
    Src r{reinterpret_cast<const char*>(baseA + (size_t)kt * BK * lda),
          reinterpret_cast<const char*>(baseB + (GATHER ? 0 : (size_t)kt * BK * ldb)), stepAb, stepBb, kt};
    asm volatile("" : "+s"(r.a), "+s"(r.b), "+s"(r.sa), "+s"(r.sb));
    return r;
  };
  auto dma = [&](const Src& sr, auto buf_tag, int p) {  // p < 8: A piece p, else B piece p - 8
    constexpr int BUF = decltype(buf_tag)::value;
    const unsigned base = lds0 + (unsigned)(BUF * 2 * OPB);
    if (p < 8) {
      glds(voffA[p & 1], reinterpret_cast<const bf16*>(sr.a + p * sr.sa), base + (unsigned)(4096 * p));
    } else if constexpr (GATHER) {
      // B piece p - 8: token rows 8(p - 8) + 2w + rl of k-tile k0 + kt
      const int t = (k0 + sr.kt) * BK + 8 * (p - 8) + rw;
      int q, wo, n, ho;
      divmodf(t, gx.TB, gx.inv_TB, q, wo);
      divmodf(q, gx.TA, gx.inv_TA, n, ho);
      const int hi = ho * gx.st + gdh[p & 1], wi = wo * gx.st + gdw[p & 1];
      const unsigned off = ((unsigned)hi < (unsigned)gx.IH && (unsigned)wi < (unsigned)gx.IW)
                               ? (unsigned)((((n * gx.IH + hi) * gx.IW + wi) * gx.C + gci[p & 1]) * 2)
                               : 0x80000000u;
      bufld_lds(off, rsX, base + OPB + (unsigned)(4096 * (p - 8)));
    } else {
      glds(voffB[p & 1], reinterpret_cast<const bf16*>(sr.b + (p - 8) * sr.sb), base + OPB + (unsigned)(4096 * (p - 8)));
    }
  };

  // fragment slot q (0..15) of block h (tokens 32h .. 32h+31): q < 8 → A rows
  // wm·128 + 16q, else B columns wn·128 + 16(q - 8)
  const bf16* smA[2] = {smem, smem + 2 * TILE};
  int fo[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fo[i] = frag_base16(wm * 128 + 16 * i, lane);
    fo[8 + i] = TILE + frag_base16(wn * 128 + 16 * i, lane);
  }
  auto rd = [&](auto buf_tag, int h, int q) -> bf16x8 {
    constexpr int BUF = decltype(buf_tag)::value;
    const bf16* T = smA[BUF] + fo[q];
    return h ? frag16<32>(T) : frag16<0>(T);
  };
  auto mma = [](f32x4& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  };
  auto mma0 = [](f32x4& c, const bf16x8& a, const bf16x8& b) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(a), "v"(b));
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;

  f32x4 acc[8][8];  // first written by mma0 in tile 0's block 0
  bf16x8 f0[16], f1[16];

  {
    const Src s0 = srcs(0), s1 = srcs(1);
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(s0, B0{}, p);
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(s1, B1{}, p);
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed (tile 1 may fly)
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 16; ++q) f0[q] = rd(B0{}, 0, q);
  // group g of a block: A fragment g >> 1 against B fragments 4(g & 1) .. +3
  auto tileH = [&](int t, auto buf_tag, auto more_tag, auto first_tag, auto eout_tag) {
    constexpr int BUF = decltype(buf_tag)::value;
    constexpr bool MORE = decltype(more_tag)::value;
    constexpr bool FIRST = decltype(first_tag)::value;
    constexpr bool EOUT = decltype(eout_tag)::value;
    using NB = std::integral_constant<int, BUF ^ 1>;
    using SB = std::integral_constant<int, BUF>;
    Src sn2{};
    if constexpr (EOUT) sn2 = srcs(t + 2);
    // B0: every wave's F0(t) reads (tokens 0-31 of BUF) are done
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int mb = g >> 1, nb0 = 4 * (g & 1);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (FIRST) mma0(acc[mb][nb0 + u], f0[mb], f0[8 + nb0 + u]);
        else mma(acc[mb][nb0 + u], f0[mb], f0[8 + nb0 + u]);
      }
      f1[g] = rd(buf_tag, 1, g);
      if constexpr (EOUT) {
        if (g & 1) dma(sn2, SB{}, (g >> 1) < 4 ? (g >> 1) : (g >> 1) + 4);  // first-half pieces
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // B1: every wave's F1(t) reads are done and tile t+1 has landed
    if constexpr (MORE || EOUT) {
      if constexpr (EOUT)
        asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int mb = g >> 1, nb0 = 4 * (g & 1);
#pragma unroll
      for (int u = 0; u < 4; ++u) mma(acc[mb][nb0 + u], f1[mb], f1[8 + nb0 + u]);
      if constexpr (MORE) f0[g] = rd(NB{}, 0, g);
      if constexpr (EOUT) {
        if (g & 1) dma(sn2, SB{}, (g >> 1) < 4 ? (g >> 1) + 4 : (g >> 1) + 8);  // second-half pieces
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  tileH(0, B0{}, T_{}, T_{}, T_{});
  tileH(1, B1{}, T_{}, F_{}, T_{});
  for (int t = 2; t < nk - 2; t += 2) {
    tileH(t, B0{}, T_{}, F_{}, T_{});
    tileH(t + 1, B1{}, T_{}, F_{}, T_{});
  }
  tileH(nk - 2, B0{}, T_{}, F_{}, F_{});
  tileH(nk - 1, B1{}, F_{}, F_{}, F_{});

  // ---- epilogue: acc[mb][nb][r] = C[m0 + wm·128 + 16mb + 4(l >> 4) + r][n0 + wn·128 + 16nb + (l & 15)]
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  bf16* Cb = C + (size_t)split * split_stride;
  const int g4 = lane >> 4, li = lane & 15;
  if (m0 + wm * 128 >= M) return;  // edge tile: wm = 1 holds rows m0 + 128 .. (wave-uniform)
  if constexpr (GATHER) {
    // fp32 partials of this split (ldc = N)
    float* P = gx.part + (size_t)split * split_stride;
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[r]) : "a"(acc[mb][nb][r]));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 128 + 16 * mb + 4 * g4 + r;
          P[(size_t)m * ldc + n0 + wn * 128 + 16 * nb + li] = v[r];
        }
      }
    return;
  }
#pragma unroll
  for (int mb = 0; mb < 8; ++mb)
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v[r]) : "a"(acc[mb][nb][r]));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 128 + 16 * mb + 4 * g4 + r;
        bf16* p = Cb + (size_t)m * ldc + n0 + wn * 128 + 16 * nb + li;
        float x = v[r];
        if (accumulate) x += (float)*p;
        *p = (bf16)x;
      }
    }
}

}  // namespace

// every slice gets ≥ 2 pairs of k-tiles (uneven splits allowed: pairs are dealt
// out); returns -2 when a slice would be shorter
int gemm_dw4(const bf16* A, const bf16* B, long long T, int M, int N, int lda, int ldb, bf16* C, int ldc,
             int accumulate, bf16* ws, int splits, hipStream_t st, int variant) {
  if (M % (BM / 2) || N % BN || T % BK || splits < 1 || splits > 16) return -2;
  const long long ks = T / BK;
  if (ks > 0x7fffffffLL) return -2;
  // every split's k-tile count even and ≥ 4 (pairs dealt out, remainder to the first slices)
  if (ks % 2 || (ks / 2) / splits < 2) return -2;
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const int grid = tiles * splits;
  bf16* out = C;
  int ldo = ldc;
  long long stride = 0;
  int acc = accumulate;
  if (splits > 1) {
    if (!ws || ldc != N) return -3;
    out = ws;
    ldo = N;
    stride = (long long)M * N;
    acc = 0;
  }
  if (variant == 1)  // the same schedule on 32x32x16 MFMAs (A/B alternative)
    gemm_dw4_kernel<<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, (int)ks, splits, out, ldo, stride, acc);
  else
    gemm_dw4m16_kernel<false><<<grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, (int)ks, splits, out, ldo, stride, acc,
                                                     DwGather{});
  if (splits > 1) return splitk_add(ws, splits, (long long)M * N, C, accumulate, st);
  return 0;
}

// Convolution weight gradient on the gathered mainloop: dW [Kout][R·S·C] fp32
// partials per token slice into part ([splits][Kout][TCp], TCp = R·S·C rounded up
// to 256 columns); the caller folds them.  Contract: Kout % 128 = 0, C % 8 = 0,
// tokens % 128 = 0 with ≥ 4 64-token k-tiles per slice (pairs dealt out).
int conv_wgrad_dw4_splits(int Kout, int TC, long long M) {
  const long long tiles = (long long)((Kout + 255) / 256) * ((TC + 255) / 256);
  const long long pairs = M / 128;
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  // one workgroup per CU (128 KiB of LDS each) and no second round: ⌊CUs / tiles⌋
  long long sp = ncu / tiles;
  if (sp > pairs / 2) sp = pairs / 2;
  if (sp > 256) sp = 256;
  return sp < 1 ? 1 : (int)sp;
}

int conv_wgrad_dw4(const bf16* dy, const bf16* x, int N, int H, int W, int C, int Kout, int R, int S, int stride,
                   int pad, float* part, int splits, hipStream_t st) {
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const long long M = (long long)N * Ho * Wo;
  const int TC = R * S * C, TCp = (TC + BN - 1) / BN * BN;
  if (Kout % (BM / 2) || C % 8 || M % (2 * BK) || M >= (1LL << 31)) return -2;
  const long long ks = M / BK;
  if (splits < 1 || (ks / 2) / splits < 2) return -2;
  if ((long long)N * H * W * C * 2 >= (1LL << 31)) return -2;
  DwGather g{x, (unsigned)((long long)N * H * W * C * 2), C, S, H, W, Ho, Wo, TC, 1.f / (float)Ho, 1.f / (float)Wo,
             stride, pad, part};
  const int grid = ((Kout + BM - 1) / BM) * (TCp / BN) * splits;
  gemm_dw4m16_kernel<true><<<grid, NTHR, 0, st>>>(dy, nullptr, Kout, 0, Kout, TCp, (int)ks, splits, nullptr, TCp,
                                                  (long long)Kout * TCp, 0, g);
  return 0;
}

}  // namespace pdo
