// SPDX-License-Identifier: Apache-2.0
// C[M][N] = A[M][K] · B[N][K]ᵀ on gfx950 — the 4-wave, one-wave-per-SIMD
// mainloop (same contract and epilogues as gemm_nt.hip, selected by
// gemm_nt_set_impl).
//
// Why a second mainloop: PMC passes over gemm_nt (8 waves, 128 × 64 per wave,
// two waves per SIMD ping-ponging between an MFMA phase and a read phase) at
// [65536 × 1024] · [1024 × 4096]ᵀ show the matrix pipe busy 62 % of the
// kernel's cycles, 25 % of wave cycles parked at barriers / waits, and 0.38
// LDS instructions per MFMA; hipBLASLt's kernel on the same shape (4 waves,
// 128 × 128 per wave) keeps it 80 % busy at 0.25 (profiles/r2_gemm_pmc.md).
// Here each wave owns a 128 × 128 output block (64 16×16 accumulators = 256
// fp32 registers, in the accumulator file) and one instruction stream
// interleaves everything with its MFMAs:
//
//   tile t (BK = 64, LDS buffer t&1), 128 MFMAs per wave:
//   block 0: 16 groups of {4 MFMAs on the k 0-31 fragments F0; 1 ds_read of a
//            k 32-63 fragment F1; 2 LDS-DMA (global_load_lds_dwordx4) pieces
//            of tile t+1 into the other buffer (groups 0-7)}
//   block 1: 16 groups of {4 MFMAs on F1}; after group 11: retire this wave's
//            DMA of tile t+1 (vmcnt(0)) and its F1 reads (lgkmcnt(0)), one
//            s_barrier; groups 12-15 each read 4 fragments F0 of tile t+1.
//
// One barrier per k-tile.  RAW: tile t+1's bytes are read only after every
// wave retired its own DMA and passed that barrier.  WAR: a buffer is
// overwritten (block 0 of tile t+1 writes buffer t&1) only after the barrier
// that follows every wave's last read of it (its F1 reads in block 0 of tile
// t, retired before the barrier in block 1 of tile t).
//
// LDS: [buffer][A|B][256 rows][64 k] bf16 = 128 KiB; rows are 128 B with the
// 16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7), so the 16 rows a
// ds_read_b128 lane group touches land on 16 distinct bank slots.  The DMA
// writes LDS linearly (1 KiB = 8 rows per wave-instruction) and applies the
// swizzle on the per-lane global source address.
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NTHR = 256;

// f(integral_constant<int, I>) for I = 0 .. N-1, expanded at compile time: a
// 128-slot MFMA schedule is too large for `#pragma unroll` (hipcc gives up and
// indexes the accumulators at run time); here every slot's index is a constant
template <typename Fn, int... I>
__device__ __forceinline__ void static_for_impl(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
constexpr int OPB = 256 * BK * 2;  // bytes of one operand tile [256][64] bf16 = 32 KiB

// ---- register-epilogue helpers (SCHED & 2)
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 join(u32x2 a, u32x2 b) {
  return __builtin_bit_cast(bf16x8, u32x4{a[0], a[1], b[0], b[1]});
}
__device__ __forceinline__ u32x2 pack4(f32x4 v) {  // 4 fp32 → 4 bf16 (round to nearest even)
  const bf16x4 b = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
  return __builtin_bit_cast(u32x2, b);
}
__device__ __forceinline__ void swap32(u32x2& x, u32x2& y) {  // x's upper 32 lanes ↔ y's lower 32
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto r = __builtin_amdgcn_permlane32_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
}
__device__ __forceinline__ void swap16(u32x2& x, u32x2& y) {  // x's odd 16-lane rows ↔ y's even rows
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    const auto r = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
    x[d] = r[0];
    y[d] = r[1];
  }
}
// 4×4 block transpose across the lane groups q = lane >> 4: in, b[j] holds the
// columns 16j + 4q .. +3 of the lane's row; out, b[q'] holds 16q + 4q' .. +3,
// i.e. the lane owns 16 contiguous columns of block q
__device__ __forceinline__ void transpose_blocks(u32x2 (&b)[4]) {
  swap32(b[0], b[2]);
  swap32(b[1], b[3]);
  swap16(b[0], b[1]);
  swap16(b[2], b[3]);
}

// SCHED 0: one barrier per k-tile, tile t+1's DMA issued during tile t (lead
//          ≈ 0.6 tile), described at the top of the file.
// SCHED & 1: three barriers per k-tile and an operand-split refill — the schedule
//          of hipBLASLt's gfx950 MT256x256x64 loop (profiles/r3_gemm_nt4_sched.md).
//          Tile t's buffer is released operand by operand as the waves finish
//          reading it: after barrier 1 (every wave's last A read of it, the k
//          32-63 fragments) its A half is refilled with tile t+2, after barrier 2
//          its B half.  Barrier 3 (vmcnt = this tile's own t+2 pieces still in
//          flight) publishes tile t+1, whose k 0-31 fragments are then read
//          under the last quarter of tile t's MFMAs.  Every DMA piece has
//          ≈ 1.3-1.6 tiles of lead instead of ≈ 0.6.
// SCHED & 2: the register epilogue (below) instead of the LDS-staged one.
// SCHED & 4: row-major accumulators (with SCHED & 1).  The MFMAs take A as
//          SrcA, so a lane's 4 accumulator values of a 16×16 block are 4
//          consecutive output ROWS; and B's tile rows sit permuted in LDS
//          (physical row 128h + q holds row 128h + 8(q & 15) + (q >> 4)), so
//          column c of block j is output column 8c + j: a lane holds 8
//          consecutive columns of each of its rows across blocks j = 0-7.  The
//          epilogue then stores 16 B per lane straight from the accumulators,
//          4 rows × 256 B per instruction, no LDS round trip and no barrier (the
//          layout of hipBLASLt's MT256x256x64 epilogue: 32 dwordx4 stores per
//          wave).  The permutation costs nothing: it is the DMA source address
//          (8-row lane stride, per-piece scalar base); the LDS image and the
//          fragment reads are unchanged.
// SCHED & 8: non-temporal C stores (keep the A / B panels in L2).
// SCHED & 16: with SCHED & 4, the mirror-image schedule — runs of 8 MFMAs share
//          the SrcA operand (A fragment i) as hipBLASLt's loop does, and the
//          operands trade places in the read / release / refill order.
template <int EPI, int EPG, int BAR, int BUFLD, int SCHED = 0>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt4_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           int lda, int ldb, int M, int N, int nk,
                                                           bf16* __restrict__ C, int ldc,
                                                           const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                           int ldy, float* __restrict__ dbias_part, int group_m) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * 256 * BK];  // [buf][A|B][256][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_n = (N + BN - 1) / BN;  // SCHED & 4: N % 256 = 128 allowed (half-width last tile column)
  const int nwg = (M / BM) * tiles_n;
  // SCHED & 32: persistent workgroups (grid = one per CU), virtual tile ids
  // blockIdx.x + k·gridDim.x.  The next tile's first two k-tiles are issued
  // before this tile's register epilogue, so their HBM latency hides behind the
  // epilogue's conversions and stores, and the stores drain under the next mainloop.
  constexpr bool PERS = (SCHED & 32) != 0;
  static_assert(!PERS || (SCHED & 5) == 5, "persistent tiles: SCHED 1 mainloop with the register row epilogue");
  // SCHED & 64 (with PERS): the row epilogue's stores drain under the next
  // tile's first two k-tiles.  vmcnt retires loads, stores and LDS-DMA in issue
  // order, so "wait for the next tile's pieces" was written vmcnt(16), which
  // also waited for every store of the epilogue issued after them — the
  // epilogue's 128-256 KiB per workgroup then drained with the matrix pipe
  // idle.  Tiles 0 and 1 of the next tile were issued BEFORE the stores, so
  // their waits may leave the NST stores in flight: vmcnt(16 + NST) (capped at
  // the counter's 63).  Tile 2's pieces come after the stores; its wait drains them.
  constexpr bool DEFER = (SCHED & 64) != 0;
  static_assert(!DEFER || PERS, "deferred store drain: persistent tiles only");
  constexpr int NST = EPI == 2 ? 64 : EPI == 3 ? 34 : 32;  // vm stores one wave's row epilogue issues
  constexpr int WDEF = 16 + NST > 63 ? 63 : 16 + NST;
  int pend = 0;  // this wave has epilogue stores in flight (wave-uniform)
  auto coords = [&](int v, int& tm_, int& tn_) {
    int id = v;
    {  // bijective XCD remap: each XCD walks a contiguous range of tiles (shared A panels in its L2)
      const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
      id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
    }
    // grouped tile order: consecutive ids walk group_m tile rows, then the next
    // tile column, so the 32 tiles an XCD runs at once form a group_m × (32 /
    // group_m) block and share fewer A/B panels in that XCD's 4 MiB L2 (row-major,
    // group_m = 1: 2 rows × 16 columns on the [65536, 4096] shapes = 18 panels)
    const int tiles_m = M / BM, per_group = group_m * tiles_n;
    const int g = id / per_group, first_m = g * group_m;
    const int gsz = min(tiles_m - first_m, group_m), r = id - g * per_group;
    tm_ = first_m + r % gsz;
    tn_ = r / gsz;
  };
  int vcur = blockIdx.x;
  int tn, tm;
  coords(vcur, tm, tn);
  int m0 = tm * BM, n0 = tn * BN;
  // half-width tile (only N - n0 = 128 columns exist): the B pieces of the upper
  // half re-read the lower half's rows (in bounds), the wn = 1 waves store nothing
  bool halfn = (SCHED & 4) && n0 + BN > N;
  bool dhalfn = halfn;  // of the tile whose pieces are being issued

  // ---- LDS-DMA sources.  Wave w fills 8-row blocks b = w + 4i (i = 0..7) of
  // both operands; lane l → row 8b + (l >> 3), LDS chunk l & 7, global chunk
  // (l & 7) ^ swz(row) with swz(row) = (row >> 1) & 7 = 4(w & 1) + (l >> 4).
  // The per-lane part is a 32-bit byte offset (one VGPR per operand); the
  // wave-uniform part (tile origin, block, k-tile) is an SGPR base, so a DMA
  // piece costs scalar adds instead of 64-bit vector address arithmetic.
  const int rb = lane >> 3;
  const int csrc = (lane & 7) ^ (4 * (w & 1) + (lane >> 4));
  static_assert(!(SCHED & 4) || ((SCHED & 1) && !(BUFLD & 1)), "row-major accumulators: SCHED 1 mainloop, global_load_lds");
  // SCHED & 4: physical B row 8(w + 4p) + q' (wave w, piece p, q' = l >> 3) holds
  // row 128(p >> 2) + 64(w & 1) + (w >> 1) + 2(p & 3) + 8q' — lane stride 8 rows,
  // piece stride 2 rows (and 128 for the second half); same swizzle (physical row)
  const unsigned voffA = (unsigned)((rb * lda + csrc * 8) * 2);
  const unsigned voffB = (SCHED & 4) ? (unsigned)((8 * rb * ldb + csrc * 8) * 2) : (unsigned)((rb * ldb + csrc * 8) * 2);
  const bf16* baseA = A + ((size_t)m0 + 8 * w) * lda;
  const bf16* baseB = (SCHED & 4) ? B + ((size_t)n0 + 64 * (w & 1) + (w >> 1)) * ldb : B + ((size_t)n0 + 8 * w) * ldb;
  const unsigned stepAb = (unsigned)(64 * lda);                                                // 32 rows, bytes
  const unsigned stepBb = (SCHED & 4) ? (unsigned)(4 * ldb) : (unsigned)(64 * ldb);            // 2 / 32 rows
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16*)smem + (unsigned)(w * 1024);
  // M0 is not saved around the DMA: nothing else in this kernel uses it (check
  // the .s for other M0 readers after editing); s_nop 0 = the SALU M0 write →
  // LDS-DMA wait state
  auto glds = [](unsigned voff, const bf16* sbase, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 :
                 : "v"(voff), "s"(sbase), "s"(lds_byte)
                 : "memory");
  };
  // pieces of tile kt into buffer BUF: p < 8 → A block w + 4p, else B block w + 4(p - 8).
  // The per-tile bases and strides pass through an empty asm so hipcc forms each
  // piece's 64-bit base with two scalar adds next to its DMA instead of keeping
  // 16 precomputed bases live (they pushed the kernel past the 102-SGPR limit
  // and into AGPR shuttling)
  struct Src {
    const char* a;
    const char* b;
    unsigned sa, sb;
  };
  auto srcs = [&](int kt) {
    Src r;
    if constexpr (BUFLD & 1) {
      r = Src{reinterpret_cast<const char*>((uintptr_t)(kt * BK * 2)), nullptr, stepAb, stepBb};
    } else {
      r = Src{reinterpret_cast<const char*>(baseA + (size_t)kt * BK), reinterpret_cast<const char*>(baseB + (size_t)kt * BK),
              stepAb, stepBb};
    }
    asm volatile("" : "+s"(r.a), "+s"(r.b), "+s"(r.sa), "+s"(r.sb));
    return r;
  };
  // BUFLD: the same pieces as buffer_load_dwordx4 … offen lds (buffer
  // descriptor per operand, the per-piece offset in soffset) — A/B variant
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(baseA), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(baseB), 0, 0x7fffffff, 0x00020000);
  auto bld = [](unsigned voff, __amdgpu_buffer_rsrc_t rs, unsigned soff, unsigned lds_byte) {
    asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                 :
                 : "v"(voff), "s"(rs), "s"(soff), "s"(lds_byte)
                 : "memory");
  };
  auto dma = [&](const Src& sr, auto buf_tag, int p) {
    constexpr int BUF = decltype(buf_tag)::value;
    const unsigned base = lds0 + (unsigned)(BUF * 2 * OPB);
    if constexpr (BUFLD & 1) {
      // sr.a / sr.b carry the k-tile byte offset in this mode
      const unsigned ko = (unsigned)(uintptr_t)sr.a;
      if (p < 8) bld(voffA, rsA, ko + p * sr.sa, base + (unsigned)(4096 * p));
      else bld(voffB, rsB, ko + (p - 8) * sr.sb, base + OPB + (unsigned)(4096 * (p - 8)));
    } else {
      if (p < 8) glds(voffA, reinterpret_cast<const bf16*>(sr.a + p * sr.sa), base + (unsigned)(4096 * p));
      else {
        const int pp = p - 8;
        const unsigned mul = (SCHED & 4) ? (unsigned)((pp & 3) + (dhalfn ? 0 : 64) * (pp >> 2)) : (unsigned)pp;
        glds(voffB, reinterpret_cast<const bf16*>(sr.b + mul * sr.sb), base + OPB + (unsigned)(4096 * pp));
      }
    }
  };

  // ---- fragment reads: 16x16x32 operand = rows (l & 15), k chunk 4kk + (l >> 4)
  const unsigned char* lds = reinterpret_cast<const unsigned char*>(smem);
  const int sw = (lane >> 1) & 7;
  const int ra = (wm * 128 + (lane & 15)) * 128, rbb = (wn * 128 + (lane & 15)) * 128;
  const int oA0 = ra + ((((lane >> 4)) ^ sw) << 4), oA1 = ra + (((4 + (lane >> 4)) ^ sw) << 4);
  const int oB0 = OPB + rbb + ((((lane >> 4)) ^ sw) << 4), oB1 = OPB + rbb + (((4 + (lane >> 4)) ^ sw) << 4);
  // read order within a k-half: A0, B0..B7, A1..A7 (the order block MFMAs consume them)
  auto rd = [&](auto buf_tag, int kk, int q) -> bf16x8 {
    constexpr int BUF = decltype(buf_tag)::value;
    const int o = (q == 0) ? (kk ? oA1 : oA0) : (q <= 8) ? (kk ? oB1 : oB0) + (q - 1) * 2048
                                                          : (kk ? oA1 : oA0) + (q - 8) * 2048;
    return *reinterpret_cast<const bf16x8*>(lds + BUF * 2 * OPB + o);
  };
  // MFMA with the accumulator pinned to the accumulator file ("+a"): with the
  // builtin, hipcc kept part of the 256 accumulators in arch VGPRs and shuttled
  // them through v_accvgpr_read/write around every MFMA (≈3 VALU per MFMA).
  // hipcc does not see inside the asm, so the asm must not depend on its hazard
  // padding: the operands come from ds_read (hipcc's lgkmcnt waits cover asm
  // inputs), an accumulator is rewritten 64 MFMAs after its previous write, the
  // first write of each one takes C = 0 (mma0: no v_accvgpr_write init that a
  // following MFMA would read too early), and the epilogue pads before reading.
  auto mma = [](f32x4& c, const bf16x8& b, const bf16x8& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
  };
  auto mma0 = [](f32x4& c, const bf16x8& b, const bf16x8& a) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
  };
  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;

  f32x4 acc[8][8];  // first written by mma0 in tile 0's block 0
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // ---- epilogue ----
  // The accumulators leave the accumulator file through explicit
  // v_accvgpr_read ("a" operands): with plain VALU uses here, hipcc's register
  // classes put part of the 256 accumulators in arch VGPRs for the whole
  // kernel and shuttled them through v_accvgpr_read/write around every MFMA
  // (≈3 VALU per MFMA).  hipcc does not pad the asm against the last MFMAs:
  // 16 wait states first (≥ the 8-pass XDL D → read requirement).
  auto rd_acc = [](const f32x4& a) {
    f32x4 v;
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\tv_accvgpr_read_b32 %3, %7"
                 : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3])
                 : "a"(a[0]), "a"(a[1]), "a"(a[2]), "a"(a[3]));
    return v;
  };
  auto st16 = [](bf16* p, bf16x8 v) {
    if constexpr (SCHED & 8) __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p));
    else *reinterpret_cast<bf16x8*>(p) = v;
  };
  // the row epilogue as a callable: the persistent loop runs it per tile
  auto row_epilogue = [&]() {
    if constexpr (SCHED & 4) {
      // hipcc does not pad the asm against the last MFMAs: 16 wait states first
      asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
      // ---- row epilogue: acc[i][j][e] = C[m][n], m = wm·128 + 16i + 4(l >> 4) + e,
      // n = wn·128 + 8(l & 15) + j.  Per (i, e) a lane stores 8 consecutive
      // columns; the 64 lanes cover 4 rows × 128 columns.  Same per-element math
      // and roundings as the LDS-staged path below.
      if (halfn && wn == 1) return;
      const int g4 = lane >> 4;
      const int nb = n0 + wn * 128 + 8 * (lane & 15);
      const size_t mr = (size_t)(m0 + wm * 128 + 4 * g4);
      bf16x8 pre[EPI == 3 ? 32 : 1];
      if constexpr (EPI == 3) {
#pragma unroll
        for (int u = 0; u < 32; ++u) pre[u] = *reinterpret_cast<const bf16x8*>(Y + (mr + 16 * (u >> 2) + (u & 3)) * ldy + nb);
      }
      f32x8 bv8 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI >= 1) bv8 = to_f32(*reinterpret_cast<const bf16x8*>(bias + nb));
      f32x8 colp = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      f32x2 m1 = {-1.f, -1.f};
      asm volatile("" : "+v"(m1));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f32x4 a[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = rd_acc(acc[i][j]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x8 v = {a[0][e], a[1][e], a[2][e], a[3][e], a[4][e], a[5][e], a[6][e], a[7][e]};
          const size_t m = mr + 16 * i + e;
          bf16* crow = C + m * ldc + nb;
          if constexpr (EPI <= 1) {
            st16(crow, to_bf16(v + bv8));
          } else if constexpr (EPI == 2) {
            // GELU of the fp32 pre-activation (the bf16 copy is stored for the
            // backward, as hipBLASLt's GELU_AUX epilogue does); no bf16 round trip:
            // the fused epilogues' cost is their VALU count with the matrix pipe
            // idle (profiles/r3_nt4_deferred_drain.md, PMC section)
            st16(crow, to_bf16(v));
            const f32x8 x = v + bv8;
            f32x8 y;
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
              const f32x2 gg = gelu_sig2(f32x2{x[q], x[q + 1]});
              y[q] = gg[0];
              y[q + 1] = gg[1];
            }
            st16(Y + m * ldy + nb, to_bf16(y));
          } else {
            const f32x8 x = to_f32(pre[4 * i + e]) + bv8;
            const f32x8& dy = v;  // the fp32 product, not its bf16 rounding
            f32x8 d;
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
              const f32x2 gg = f32x2{dy[q], dy[q + 1]} * gelu_sig_grad2(f32x2{x[q], x[q + 1]}, m1);
              d[q] = gg[0];
              d[q + 1] = gg[1];
            }
            colp += d;
            st16(crow, to_bf16(d));
          }
        }
      }
      if constexpr (EPI == 3) {
        // partial row 4·wm + (l >> 4) of this M-tile's 8: the rows 16i + 4(l >> 4) + e
        float* prow = dbias_part + (size_t)(8 * tm + 4 * wm + g4) * N + nb;
        *reinterpret_cast<f32x4*>(prow) = f32x4{colp[0], colp[1], colp[2], colp[3]};
        *reinterpret_cast<f32x4*>(prow + 4) = f32x4{colp[4], colp[5], colp[6], colp[7]};
      }
    }
  };


  if constexpr (SCHED & 1) {
    constexpr bool MIR = (SCHED & 16) != 0;
    static_assert(!MIR || (SCHED & 4), "the mirrored schedule feeds A as SrcA");
    // fragment i of A (rows wm·128 + 16i + (l & 15)) / B, k half kk, from buffer BUF
    auto rdA = [&](auto buf_tag, int kk, int i) -> bf16x8 {
      constexpr int BUF = decltype(buf_tag)::value;
      return *reinterpret_cast<const bf16x8*>(lds + BUF * 2 * OPB + (kk ? oA1 : oA0) + i * 2048);
    };
    auto rdB = [&](auto buf_tag, int kk, int j) -> bf16x8 {
      constexpr int BUF = decltype(buf_tag)::value;
      return *reinterpret_cast<const bf16x8*>(lds + BUF * 2 * OPB + (kk ? oB1 : oB0) + j * 2048);
    };
    // F0 (k 0-31) reads of a tile in the order its first MFMA run consumes them:
    // B fragment 0 (the run's stationary operand), A 0-7, then B 1-7
    // (MIR: the mirror image — A fragment 0 stationary first, B 0-7, then A 1-7)
    auto rdF0 = [&](auto buf_tag, int q) {
      if constexpr (MIR) {
        if (q == 0) fa0[0] = rdA(buf_tag, 0, 0);
        else if (q <= 8) fb0[q - 1] = rdB(buf_tag, 0, q - 1);
        else fa0[q - 8] = rdA(buf_tag, 0, q - 8);
      } else {
        if (q == 0) fb0[0] = rdB(buf_tag, 0, 0);
        else if (q <= 8) fa0[q - 1] = rdA(buf_tag, 0, q - 1);
        else fb0[q - 8] = rdB(buf_tag, 0, q - 8);
      }
    };
    // ---- prologue: tiles 0 and 1 in flight (then: wait for tile 0, its F0 fragments)
    auto issue01 = [&]() {
      const Src s0 = srcs(0);
#pragma unroll
      for (int p = 0; p < 16; ++p) dma(s0, B0{}, p);
      const Src s1 = srcs(1);
#pragma unroll
      for (int p = 0; p < 16; ++p) dma(s1, B1{}, p);
    };

    // slot s = MFMA index in the tile (128); run r = s >> 3 keeps B fragment
    // (r & 7) stationary over A fragments 0-7, k half s >> 6.
    //   s  0-14 (even)  F1 A reads           s 23        lgkmcnt(0), barrier 1
    //   s 24-45 (÷3)    A pieces of t+2      s 25-46 (÷3) F1 B reads
    //   s 51            lgkmcnt(0), barrier 2
    //   s 52-87 (÷5)    B pieces of t+2      s 93        vmcnt(t+2 pieces), barrier 3
    //   s 94-124 (even) F0 reads of t+1 (other buffer)
    auto tile3 = [&](int t, auto buf_tag, auto first_tag, auto more_tag, auto load_tag) {
      constexpr int BUF = decltype(buf_tag)::value;
      constexpr bool FIRST = decltype(first_tag)::value;
      constexpr bool MORE = decltype(more_tag)::value;
      constexpr bool LOAD = decltype(load_tag)::value;
      using NB = std::integral_constant<int, BUF ^ 1>;
      using SB = std::integral_constant<int, BUF>;
      Src sn2{};
      if constexpr (LOAD) sn2 = srcs(t + 2);
      static_for<128>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        // runs of 8 MFMAs share the B fragment j (MIR: the A fragment i, = SrcA)
        constexpr int i = MIR ? (s >> 3) & 7 : s & 7, j = MIR ? s & 7 : (s >> 3) & 7;
        // SrcA / SrcB: B / A (column-major accumulators) or A / B (SCHED & 4)
        if constexpr (s < 64) {
          if constexpr (FIRST) {
            if constexpr (SCHED & 4) mma0(acc[i][j], fa0[i], fb0[j]);
            else mma0(acc[i][j], fb0[j], fa0[i]);
          } else {
            if constexpr (SCHED & 4) mma(acc[i][j], fa0[i], fb0[j]);
            else mma(acc[i][j], fb0[j], fa0[i]);
          }
        } else {
          if constexpr (SCHED & 4) mma(acc[i][j], fa1[i], fb1[j]);
          else mma(acc[i][j], fb1[j], fa1[i]);
        }
        // MIR swaps the operands' roles below: B's k 32-63 fragments first, B's
        // half of the buffer released at barrier 1 and refilled first, A's at barrier 2
        if constexpr (s < 16 && (s & 1) == 0) {
          if constexpr (MIR) fb1[s >> 1] = rdB(SB{}, 1, s >> 1);
          else fa1[s >> 1] = rdA(SB{}, 1, s >> 1);
        }
        if constexpr (LOAD && s == 23) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (LOAD && s >= 24 && s < 48 && (s - 24) % 3 == 0) dma(sn2, SB{}, (MIR ? 8 : 0) + (s - 24) / 3);
        if constexpr (s >= 25 && s < 49 && (s - 25) % 3 == 0) {
          if constexpr (MIR) fa1[(s - 25) / 3] = rdA(SB{}, 1, (s - 25) / 3);
          else fb1[(s - 25) / 3] = rdB(SB{}, 1, (s - 25) / 3);
        }
        if constexpr (LOAD && s == 51) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (LOAD && s >= 52 && s < 92 && (s - 52) % 5 == 0) dma(sn2, SB{}, (MIR ? 0 : 8) + (s - 52) / 5);
        if constexpr (MORE && s == 93) {
          // this wave's tile t+1 pieces retired (its 16 tile t+2 pieces may stay in flight;
          // DEFER: in the first tile after an epilogue, its stores too)
          if constexpr (LOAD && DEFER && FIRST) {
            if (pend) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WDEF) : "memory");
            else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          } else if constexpr (LOAD) {
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (MORE && s >= 94 && s < 126 && (s & 1) == 0) rdF0(NB{}, (s - 94) >> 1);
        __builtin_amdgcn_sched_barrier(0);
      });
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    issue01();
    for (;;) {
      // tile 0 landed (tile 1 may fly; DEFER: and the previous epilogue's stores)
      if (DEFER && pend) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WDEF) : "memory");
      else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 16; ++q) rdF0(B0{}, q);
      // nk is even and ≥ 4 (host contract)
      tile3(0, B0{}, T_{}, T_{}, T_{});
      tile3(1, B1{}, F_{}, T_{}, T_{});
      for (int t = 2; t < nk - 2; t += 2) {
        tile3(t, B0{}, F_{}, T_{}, T_{});
        tile3(t + 1, B1{}, F_{}, T_{}, T_{});
      }
      tile3(nk - 2, B0{}, F_{}, T_{}, F_{});
      tile3(nk - 1, B1{}, F_{}, F_{}, F_{});
      if constexpr (PERS) {
        const int vn = vcur + (int)gridDim.x;
        if (vn >= nwg) break;
        int ntm, ntn;
        coords(vn, ntm, ntn);
        // every wave's last LDS reads of this tile precede any wave's refill
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        baseA = A + ((size_t)ntm * BM + 8 * w) * lda;
        baseB = B + ((size_t)ntn * BN + 64 * (w & 1) + (w >> 1)) * ldb;
        dhalfn = ntn * BN + BN > N;
        issue01();
        row_epilogue();  // of this tile (m0, n0, tm, halfn)
        pend = __builtin_amdgcn_readfirstlane((halfn && wn == 1) ? 0 : 1);
        vcur = vn;
        tm = ntm;
        tn = ntn;
        m0 = tm * BM;
        n0 = tn * BN;
        halfn = dhalfn;
      } else {
        break;
      }
    }
  } else {
  // ---- prologue: tile 0 → buffer 0, F0 of tile 0
  {
    const Src s0 = srcs(0);
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(s0, B0{}, p);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const bf16x8 v = rd(B0{}, 0, q);
    if (q == 0) fa0[0] = v;
    else if (q <= 8) fb0[q - 1] = v;
    else fa0[q - 8] = v;
  }

  // one k-tile in LDS buffer BUF; MORE = a next tile exists (its DMA, the
  // barrier and its F0 reads)
  // E = DMA pieces of tile t+2 issued early, in block 1 of tile t right after
  // its barrier (buffer t&1 is free then: every wave retired its last reads
  // of it before that barrier); block 0 of tile t+1 issues the other 16 - E
  constexpr int E = EPG * (15 - BAR) < 16 ? EPG * (15 - BAR) : 16;  // EPG early pieces per group after the barrier
  // ps: MORE = tile t+1 exists; EIN = its first E pieces were issued early;
  // EOUT = issue the first E pieces of tile t+2 after this tile's barrier
  auto tile = [&](int t, auto buf_tag, auto more_tag, auto first_tag, auto ein_tag, auto eout_tag) {
    constexpr int BUF = decltype(buf_tag)::value;
    constexpr bool MORE = decltype(more_tag)::value;
    constexpr bool FIRST = decltype(first_tag)::value;
    constexpr bool EIN = decltype(ein_tag)::value;
    constexpr bool EOUT = decltype(eout_tag)::value;
    constexpr int P0 = EIN ? E : 0;  // first piece of tile t+1 block 0 issues
    using NB = std::integral_constant<int, BUF ^ 1>;
    using SB = std::integral_constant<int, BUF>;
    Src sn{}, sn2{};
    if constexpr (MORE) sn = srcs(t + 1);
    if constexpr (EOUT) sn2 = srcs(t + 2);
    // ---- block 0: MFMAs on F0, reads of F1 (this tile), DMA of tile t+1
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int i = g >> 1, j0 = 4 * (g & 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // BUFLD & 2: B-stationary order (the group's 4 MFMAs share SrcA, as hipBLASLt's loop does)
        const int ii = (BUFLD & 2) ? 4 * (g & 1) + j : i, jj = (BUFLD & 2) ? (g >> 1) : j0 + j;
        if constexpr (FIRST) mma0(acc[ii][jj], fb0[jj], fa0[ii]);
        else mma(acc[ii][jj], fb0[jj], fa0[ii]);
      }
      const bf16x8 v = rd(buf_tag, 1, g);
      if (g == 0) fa1[0] = v;
      else if (g <= 8) fb1[g - 1] = v;
      else fa1[g - 8] = v;
      if constexpr (MORE) {
        if (P0 + g < 16) dma(sn, NB{}, P0 + g);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- block 1: MFMAs on F1; barrier; reads of F0 (next tile)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int i = g >> 1, j0 = 4 * (g & 1);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ii = (BUFLD & 2) ? 4 * (g & 1) + j : i, jj = (BUFLD & 2) ? (g >> 1) : j0 + j;
        mma(acc[ii][jj], fb1[jj], fa1[ii]);
      }
      if constexpr (MORE) {
        if (g == BAR) {
          asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if (g > BAR) {
          if constexpr (EOUT) {
#pragma unroll
            for (int u = 0; u < EPG; ++u)
              if (EPG * (g - BAR - 1) + u < E) dma(sn2, SB{}, EPG * (g - BAR - 1) + u);
          }
          constexpr int RPG = 16 / (15 - BAR);  // F0 reads per remaining group
#pragma unroll
          for (int u = 0; u < RPG; ++u) {
            const int q = RPG * (g - BAR - 1) + u;
            const bf16x8 v = rd(NB{}, 0, q);
            if (q == 0) fa0[0] = v;
            else if (q <= 8) fb0[q - 1] = v;
            else fa0[q - 8] = v;
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  // nk is even and ≥ 4 (host contract): pairs of tiles keep the buffer index static
  tile(0, B0{}, T_{}, T_{}, F_{}, T_{});
  tile(1, B1{}, T_{}, F_{}, T_{}, T_{});
  for (int t = 2; t < nk - 2; t += 2) {
    tile(t, B0{}, T_{}, F_{}, T_{}, T_{});
    tile(t + 1, B1{}, T_{}, F_{}, T_{}, T_{});
  }
  tile(nk - 2, B0{}, T_{}, F_{}, T_{}, F_{});
  tile(nk - 1, B1{}, F_{}, F_{}, F_{}, F_{});
  }  // SCHED

  // ---- epilogue ----
  if constexpr (SCHED & 4) {
    row_epilogue();
    return;
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  if constexpr (SCHED & 2) {
    // ---- register epilogue: no LDS round trip, no barrier.  Per 16-row block
    // i and 4-block column group h, the 4 lanes {r, r+16, r+32, r+48} hold a
    // 4×4 matrix of 4-column pieces; transpose_blocks leaves each lane 16
    // contiguous columns (two 16-B stores).  The stores of a tile leave while
    // the workgroup drains, so the next tile's DMA prologue starts without the
    // LDS staging pass (2 barriers, 128 KiB of LDS writes + reads).
    const int q = lane >> 4, rr = lane & 15;
    auto rowp = [&](int i) { return (size_t)(m0 + wm * 128 + 16 * i + rr); };
    auto colb = [&](int h) { return n0 + wn * 128 + 16 * (4 * h + q); };  // first of the lane's 16 columns
    bf16x8 pre[EPI == 3 ? 32 : 1];
    if constexpr (EPI == 3) {
      // pre-activation rows first: their latency hides behind the transposes
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            pre[(i * 2 + h) * 2 + c] = *reinterpret_cast<const bf16x8*>(Y + rowp(i) * ldy + colb(h) + 8 * c);
    }
    f32x8 bv[EPI >= 2 ? 4 : 1];
    if constexpr (EPI >= 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 2; ++c) bv[h * 2 + c] = to_f32(*reinterpret_cast<const bf16x8*>(bias + colb(h) + 8 * c));
    }
    f32x8 colp[EPI == 3 ? 4 : 1];
    if constexpr (EPI == 3) {
#pragma unroll
      for (int u = 0; u < 4; ++u) colp[u] = f32x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    }
    f32x2 m1 = {-1.f, -1.f};
    asm volatile("" : "+v"(m1));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        u32x2 b[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          f32x4 a = rd_acc(acc[i][4 * h + jj]);
          if constexpr (EPI == 1) {
            const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n0 + wn * 128 + 16 * (4 * h + jj) + 4 * q);
            a += f32x4{(float)b4[0], (float)b4[1], (float)b4[2], (float)b4[3]};
          }
          b[jj] = pack4(a);
        }
        transpose_blocks(b);
        const bf16x8 v[2] = {join(b[0], b[1]), join(b[2], b[3])};
        bf16* crow = C + rowp(i) * ldc + colb(h);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if constexpr (EPI <= 1) {
            *reinterpret_cast<bf16x8*>(crow + 8 * c) = v[c];
          } else if constexpr (EPI == 2) {
            *reinterpret_cast<bf16x8*>(crow + 8 * c) = v[c];
            const f32x8 x = to_f32(v[c]) + bv[h * 2 + c];
            f32x8 y;
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const f32x2 g = gelu_sig2(f32x2{x[e], x[e + 1]});
              y[e] = g[0];
              y[e + 1] = g[1];
            }
            *reinterpret_cast<bf16x8*>(Y + rowp(i) * ldy + colb(h) + 8 * c) = to_bf16(y);
          } else {
            const f32x8 x = to_f32(pre[(i * 2 + h) * 2 + c]) + bv[h * 2 + c];
            const f32x8 dy = to_f32(v[c]);
            f32x8 d;
#pragma unroll
            for (int e = 0; e < 8; e += 2) {
              const f32x2 g = f32x2{dy[e], dy[e + 1]} * gelu_sig_grad2(f32x2{x[e], x[e + 1]}, m1);
              d[e] = g[0];
              d[e + 1] = g[1];
            }
            colp[h * 2 + c] += d;
            *reinterpret_cast<bf16x8*>(crow + 8 * c) = to_bf16(d);
          }
        }
      }
    }
    if constexpr (EPI == 3) {
      // fp32 column partials: the 16 row lanes of a column group reduce in
      // fours (xor 1, 2); partial row 4·wm + (rr >> 2) of this M-tile's 8
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float s = colp[u][e];
          s += __shfl_xor(s, 1);
          s += __shfl_xor(s, 2);
          colp[u][e] = s;
        }
      if ((rr & 3) == 0) {
        float* prow = dbias_part + (size_t)(8 * tm + 4 * wm + (rr >> 2)) * N;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const f32x8 s = colp[h * 2 + c];
            *reinterpret_cast<f32x4*>(prow + colb(h) + 8 * c) = f32x4{s[0], s[1], s[2], s[3]};
            *reinterpret_cast<f32x4*>(prow + colb(h) + 8 * c + 4) = f32x4{s[4], s[5], s[6], s[7]};
          }
      }
    }
    return;
  }
  // acc[i][j][e] = C[m][n], m = wm·128 + 16i + (l&15), n = wn·128 + 16j + 4(l>>4) + e.
  // Staged through LDS as bf16 [256][256] (chunk c of row m at c ^ (m & 31))
  // and written back as whole 512-B rows, 16 B per lane.
  // row phase: thread t owns 16-B column chunk t & 31 of rows 8·it + (t >> 5)
  const int c = tid & 31, r0 = tid >> 5;
  const int n = n0 + 8 * c;
  // dGELU: the tile's pre-activation rows (512 B per lane) are loaded before the
  // accumulator staging, into the registers the mainloop's fragments used — their
  // HBM latency hides behind the staging instead of stalling every row batch
  bf16x8 pre[EPI == 3 ? 32 : 1];
  if constexpr (EPI == 3) {
#pragma unroll
    for (int it = 0; it < 32; ++it) pre[it] = *reinterpret_cast<const bf16x8*>(Y + (size_t)(m0 + 8 * it + r0) * ldy + n);
  }
  __syncthreads();
  unsigned char* st = reinterpret_cast<unsigned char*>(smem);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == 1) {
      const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n0 + wn * 128 + 16 * j + 4 * (lane >> 4));
      bv = f32x4{(float)b4[0], (float)b4[1], (float)b4[2], (float)b4[3]};
    }
    const int c = wn * 16 + 2 * j + (lane >> 5);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + 16 * i + (lane & 15);
      const f32x4 a = rd_acc(acc[i][j]) + bv;
      const bf16x4 o = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
      *reinterpret_cast<bf16x4*>(st + m * 512 + ((c ^ (m & 31)) << 4) + 8 * ((lane >> 4) & 1)) = o;
    }
  }
  __syncthreads();
  f32x8 bv8;
  if constexpr (EPI >= 2) bv8 = to_f32(*reinterpret_cast<const bf16x8*>(bias + n));
  f32x8 colp = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x2 m1 = {-1.f, -1.f};
  asm volatile("" : "+v"(m1));
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int r = 8 * it + r0;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(st + r * 512 + ((c ^ (r & 31)) << 4));
    const size_t m = (size_t)(m0 + r);
    if constexpr (EPI <= 1) {
      st16(C + m * ldc + n, v);
    } else if constexpr (EPI == 2) {
      st16(C + m * ldc + n, v);
      const f32x8 x = to_f32(v) + bv8;
      f32x8 y;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {  // packed pairs (common.h)
        const f32x2 g = gelu_sig2(f32x2{x[e], x[e + 1]});
        y[e] = g[0];
        y[e + 1] = g[1];
      }
      st16(Y + m * ldy + n, to_bf16(y));
    } else {
      const f32x8 x = to_f32(pre[it]) + bv8;
      const f32x8 dy = to_f32(v);
      f32x8 d;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const f32x2 g = f32x2{dy[e], dy[e + 1]} * gelu_sig_grad2(f32x2{x[e], x[e + 1]}, m1);
        d[e] = g[0];
        d[e + 1] = g[1];
      }
      colp += d;
      st16(C + m * ldc + n, to_bf16(d));
    }
  }
  if constexpr (EPI == 3) {
    // one fp32 partial row per (M-tile, row class r0): 8 rows per M-tile, as gemm_nt
    float* prow = dbias_part + (size_t)(8 * tm + r0) * N + n;
    *reinterpret_cast<f32x4*>(prow) = f32x4{colp[0], colp[1], colp[2], colp[3]};
    *reinterpret_cast<f32x4*>(prow + 4) = f32x4{colp[4], colp[5], colp[6], colp[7]};
  }
}

}  // namespace

// the variants with row-major accumulators (SCHED & 4) take N % 256 = 128
int gemm_nt4_half_n(int variant) { return variant == 8 || variant == 9 || (variant >= 11 && variant <= 15); }

// persistent variants: one workgroup per CU (a multiple of 8: the XCD mapping)
static int persistent_grid(long long tiles) {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n >= 8 ? n / 8 * 8 : 8;
  }();
  return (int)(tiles < ncu ? tiles : ncu);
}

int gemm_nt4(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
             const bf16* bias, bf16* Y, int ldy, float* dbias_part, hipStream_t st, int variant) {
  if (N % BN && !(N % BN == BN / 2 && gemm_nt4_half_n(variant))) return -2;
  const long long grid = (long long)(M / BM) * ((N + BN - 1) / BN);
  if (grid > 0x7fffffffLL) return -2;
  const int nk = K / BK;
  if (nk < 4 || nk % 2) return -2;  // the mainloop runs k-tiles in pairs, at least two
  static const int group_m = [] {
    const char* e = getenv("PDO_NT_GROUP_M");
    // 8: group_m sweep (tools/nt4_probe.py; in the step: tools/gpu.sh stepab, 8 ahead of 4 and 16) on the GPT-2 NT shapes (row-major = 1: wide K = 1024 GEMM
    // 501 -> 451 us, fc2 dX ⊙ GELU' 642 -> 607, qkv 433 -> 419; 16 is slower; bit-identical)
    const int g = e ? atoi(e) : 8;
    return g >= 1 ? g : 1;
  }();
  auto launch = [&](auto gpg, auto bar, auto bufld, auto sched) {
    constexpr int G = decltype(gpg)::value, R = decltype(bar)::value, L = decltype(bufld)::value;
    constexpr int S = decltype(sched)::value;
    const int g = (S & 32) ? persistent_grid(grid) : (int)grid;
    switch (epi) {
      case 0: gemm_nt4_kernel<0, G, R, L, S><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
      case 1: gemm_nt4_kernel<1, G, R, L, S><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
      case 2: gemm_nt4_kernel<2, G, R, L, S><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
      case 3: gemm_nt4_kernel<3, G, R, L, S><<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m); break;
      default: return -4;
    }
    return 0;
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I7 = std::integral_constant<int, 7>;
  using I11 = std::integral_constant<int, 11>;
  using I13 = std::integral_constant<int, 13>;
  using I5 = std::integral_constant<int, 5>;
  using I9 = std::integral_constant<int, 9>;
  // schedule variants under A/B (tools/nt4_probe.py, profiles/r2_gemm_nt4.md):
  // 0 = barrier after block-1 group 11, the first 4 DMA pieces of tile t+2 after it, the rest one per
  // block-0 group, B-stationary MFMA order (each group's 4 MFMAs share SrcA; default: 1-4 % faster
  // than the A-stationary order of variant 4 on qkv_fwd / proj_dx, bit-identical)
  // 5 = SCHED 1 (three barriers, operand-split refill; default), 6 = the same with
  // the register epilogue (profiles/r3_gemm_nt4_sched.md: slower on the wide-N
  // shapes, e.g. qkv_fwd 360 -> 395 us; kept for the record and the tests)
  switch (variant) {
    case 1: return launch(I1{}, I7{}, I0{}, I0{});
    case 2: return launch(I2{}, I7{}, I0{}, I0{});   // every piece of tile t+2 right after tile t's barrier
    case 3: return launch(I4{}, I11{}, I0{}, I0{});  // the same, 4 per group after a later barrier
    case 4: return launch(I1{}, I11{}, I0{}, I0{});  // variant 0 with the A-stationary order
    case 6: return launch(I1{}, I11{}, I2{}, I3{});
    case 7: return launch(I1{}, I11{}, I2{}, I0{});  // the round-2 default (SCHED 0)
    case 8: return launch(I1{}, I11{}, I2{}, I5{});   // row-major accumulators, direct row epilogue
    case 9: return launch(I1{}, I11{}, I2{}, I13{});  // the same with non-temporal stores
    case 10: return launch(I1{}, I11{}, I2{}, I9{});  // LDS-staged epilogue, non-temporal stores
    case 11: return launch(I1{}, I11{}, I2{}, std::integral_constant<int, 29>{});  // impl 10 + mirrored schedule
    case 12: return launch(I1{}, I11{}, I2{}, std::integral_constant<int, 61>{});  // variant 11, persistent
    case 13: return launch(I1{}, I11{}, I2{}, std::integral_constant<int, 45>{});  // variant 9, persistent
    case 14: return launch(I1{}, I11{}, I2{}, std::integral_constant<int, 125>{});  // variant 12, deferred store drain
    case 15: return launch(I1{}, I11{}, I2{}, std::integral_constant<int, 109>{});  // variant 13, deferred store drain
    default: return launch(I1{}, I11{}, I2{}, I1{});
  }
  return 0;
}

}  // namespace pdo
