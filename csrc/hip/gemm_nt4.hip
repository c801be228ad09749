// SPDX-License-Identifier: Apache-2.0
// C[M][N] = A[M][K] · B[N][K]ᵀ on gfx950 — the 4-wave, one-wave-per-SIMD
// persistent mainloop behind gemm_nt() for K % 128 = 0, K ≥ 256 (same contract
// and epilogues as gemm_nt.hip's 8-wave ring, which keeps the short-K shapes).
//
// Each wave owns a 128 × 128 output block (64 16×16 accumulators = 256 fp32
// registers, pinned to the accumulator file) and one instruction stream
// interleaves everything with its 128 MFMAs per k-tile (BK = 64): three
// barriers per k-tile and an operand-split refill (the schedule of hipBLASLt's
// gfx950 MT256x256x64 loop, profiles/r3_gemm_nt4_sched.md).  Tile t's buffer
// is released operand by operand as the waves finish reading it: after barrier
// 1 (every wave's last A read of it, the k 32-63 fragments) its A half is
// refilled with tile t+2, after barrier 2 its B half.  Barrier 3 (vmcnt = this
// tile's own t+2 pieces still in flight) publishes tile t+1, whose k 0-31
// fragments are then read under the last quarter of tile t's MFMAs.  Every DMA
// piece has ≈ 1.3-1.6 tiles of lead.
//
// Row-major accumulators: the MFMAs take A as SrcA, so a lane's 4 accumulator
// values of a 16×16 block are 4 consecutive output ROWS, and B's tile rows sit
// permuted in LDS (physical row 128h + q holds row 128h + 8(q & 15) + (q >> 4)),
// so column c of block j is output column 8c + j: a lane holds 8 consecutive
// columns of each of its rows across blocks j = 0-7.  The epilogue stores 16 B
// per lane straight from the accumulators, 4 rows × 256 B per instruction, no
// LDS round trip and no barrier; the permutation is the DMA source address
// (8-row lane stride, per-piece scalar base).  C stores are non-temporal (the
// A / B panels stay in L2).
//
// Persistent workgroups (grid = one per CU, virtual tile ids blockIdx.x +
// k·gridDim.x): the next tile's first two k-tiles are issued inside this
// tile's last k-tile, right after its last LDS reads (round 6; before: at the
// tile boundary), so their HBM latency hides behind the last MFMAs and the
// register epilogue's conversions and stores.  Runs of 8 MFMAs share the B fragment (K ≤ 1024) or,
// mirrored, the A fragment (K > 1024) — tools/nt4_probe.py,
// profiles/r3_gemm_nt4_rows.md.
//
// LDS: [buffer][A|B][256 rows][64 k] bf16 = 128 KiB; rows are 128 B with the
// 16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7), so the 16 rows a
// ds_read_b128 lane group touches land on 16 distinct bank slots.  The DMA
// writes LDS linearly (1 KiB = 8 rows per wave-instruction) and applies the
// swizzle on the per-lane global source address.
//
// Measured and removed (numbers in profiles/): the round-2/3 schedule variants
// — one barrier per k-tile, LDS-staged and permlane-transposed epilogues,
// buffer_load DMA, non-persistent grids (r2_gemm_nt4.md, r3_gemm_nt4_*.md) —,
// the deferred store drain (r3_nt4_deferred_drain.md) and, in round 5, the
// deferred activation epilogue that ran the GELU / GELU′ pass one element
// stage per MFMA slot under the next tile's k-loop: fc1 + GELU 565 vs 496 µs,
// fc2 dX ⊙ GELU′ 730 vs 552 µs (r5_deferred_activation_epilogue.md).
#include <atomic>
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


// MIR: runs of 8 MFMAs share the SrcA operand (A fragment i, as hipBLASLt's
//      loop does) and the operands trade places in the read / release / refill
//      order; otherwise runs share the B fragment.
template <int EPI, bool MIR>
__global__ __launch_bounds__(NTHR, 1) void gemm_nt4_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           int lda, int ldb, int M, int N, int nk,
                                                           bf16* __restrict__ C, int ldc,
                                                           const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                           int ldy, float* __restrict__ dbias_part, int group_m,
                                                           unsigned* __restrict__ sched) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * 256 * BK];  // [buf][A|B][256][64]
  __shared__ int s_next;  // dynamic order: the next virtual tile id, wave 0 → all
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_n = (N + BN - 1) / BN;  // N % 256 = 128 allowed (half-width last tile column)
  const int nwg = (M / BM) * tiles_n;
  auto coords = [&](int v, int& tm_, int& tn_) {
    int id = v;
    {  // bijective XCD remap: each XCD walks a contiguous range of tiles (shared A panels in its L2)
      const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
      id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
    }
    // grouped tile order: consecutive ids walk group_m tile rows, then the next
    // tile column, so the 32 tiles an XCD runs at once form a group_m × (32 /
    // group_m) block and share fewer A/B panels in that XCD's 4 MiB L2
    const int tiles_m = M / BM, per_group = group_m * tiles_n;
    const int g = id / per_group, first_m = g * group_m;
    const int gsz = min(tiles_m - first_m, group_m), r = id - g * per_group;
    tm_ = first_m + r % gsz;
    tn_ = r / gsz;
  };
  // Tile order.  First tile: virtual id blockIdx.x.  Static (sched = nullptr):
  // then + k·gridDim.x.  Dynamic: the next id of this workgroup's XCD comes
  // from that XCD's counter sched[xcd] (ids xcd + 8j past the first round), so
  // a workgroup that starts late — its CU held by another kernel, e.g. an RCCL
  // all-reduce on the overlap stream at N > 1 — leaves its tiles to the running
  // ones instead of extending the kernel by the hold (tools/overlap_probe.py:
  // one CU held for 267 µs took the static fc1 dX GEMM from 397 to 592 µs).
  // The ticket is taken with the last DMA pieces of the tile (k-tile nk − 3)
  // and waited for with them; the last workgroup out resets the counters.
  const bool dyn = sched != nullptr;
  const int xq = blockIdx.x & 7, j0 = ((int)gridDim.x - xq + 7) >> 3;
  unsigned ticket = 0;
  int vnext = 0;
  int vcur = blockIdx.x;
  int tn, tm;
  coords(vcur, tm, tn);
  int m0 = tm * BM, n0 = tn * BN;
  // half-width tile (only N - n0 = 128 columns exist): the B pieces of the upper
  // half re-read the lower half's rows (in bounds), the wn = 1 waves store nothing
  bool halfn = n0 + BN > N;
  bool dhalfn = halfn;  // of the tile whose pieces are being issued

  // ---- LDS-DMA sources.  Wave w fills 8-row blocks b = w + 4i (i = 0..7) of
  // both operands; lane l → physical row 8b + (l >> 3), LDS chunk l & 7, global
  // chunk (l & 7) ^ swz(row) with swz(row) = (row >> 1) & 7 = 4(w & 1) + (l >> 4).
  // The per-lane part is a 32-bit byte offset (one VGPR per operand); the
  // wave-uniform part (tile origin, block, k-tile) is an SGPR base, so a DMA
  // piece costs scalar adds instead of 64-bit vector address arithmetic.
  // B: physical row 8(w + 4p) + q' (wave w, piece p, q' = l >> 3) holds row
  // 128(p >> 2) + 64(w & 1) + (w >> 1) + 2(p & 3) + 8q' — lane stride 8 rows,
  // piece stride 2 rows (and 128 for the second half); same swizzle (physical row)
  const int rb = lane >> 3;
  const int csrc = (lane & 7) ^ (4 * (w & 1) + (lane >> 4));
  const unsigned voffA = (unsigned)((rb * lda + csrc * 8) * 2);
  const unsigned voffB = (unsigned)((8 * rb * ldb + csrc * 8) * 2);
  const bf16* baseA = A + ((size_t)m0 + 8 * w) * lda;
  const bf16* baseB = B + ((size_t)n0 + 64 * (w & 1) + (w >> 1)) * ldb;
  const unsigned stepAb = (unsigned)(64 * lda);  // 32 rows, bytes
  const unsigned stepBb = (unsigned)(4 * ldb);   // 2 rows, bytes
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
    Src r{reinterpret_cast<const char*>(baseA + (size_t)kt * BK), reinterpret_cast<const char*>(baseB + (size_t)kt * BK),
          stepAb, stepBb};
    asm volatile("" : "+s"(r.a), "+s"(r.b), "+s"(r.sa), "+s"(r.sb));
    return r;
  };
  auto dma = [&](const Src& sr, auto buf_tag, int p) {
    constexpr int BUF = decltype(buf_tag)::value;
    const unsigned base = lds0 + (unsigned)(BUF * 2 * OPB);
    if (p < 8) {
      glds(voffA, reinterpret_cast<const bf16*>(sr.a + p * sr.sa), base + (unsigned)(4096 * p));
    } else {
      const int pp = p - 8;
      const unsigned mul = (unsigned)((pp & 3) + (dhalfn ? 0 : 64) * (pp >> 2));
      glds(voffB, reinterpret_cast<const bf16*>(sr.b + mul * sr.sb), base + OPB + (unsigned)(4096 * pp));
    }
  };

  // ---- fragment reads: 16x16x32 operand = rows (l & 15), k chunk 4kk + (l >> 4)
  const unsigned char* lds = reinterpret_cast<const unsigned char*>(smem);
  const int sw = (lane >> 1) & 7;
  const int ra = (wm * 128 + (lane & 15)) * 128, rbb = (wn * 128 + (lane & 15)) * 128;
  const int oA0 = ra + ((((lane >> 4)) ^ sw) << 4), oA1 = ra + (((4 + (lane >> 4)) ^ sw) << 4);
  const int oB0 = OPB + rbb + ((((lane >> 4)) ^ sw) << 4), oB1 = OPB + rbb + (((4 + (lane >> 4)) ^ sw) << 4);
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
  // the last k-tile of a tile issues the NEXT tile's first two k-tiles (after its
  // own last LDS reads, s ≥ 49) instead of the tile boundary doing it: ≈ 80 MFMAs
  // more lead for those pieces.  EPI 8 also loads the first 16 of the epilogue's
  // 32 gelu' rows there (into fa0 / fb0's registers, dead after slot 63)
  constexpr bool EARLY8 = EPI == 8;
  bool has_next = false;
  int ntm = 0, ntn = 0;
  Src nx0{}, nx1{};
  bf16x8 pre_early[EARLY8 ? 16 : 1];

  // ---- epilogue ----
  // The accumulators leave the accumulator file through explicit
  // v_accvgpr_read ("a" operands): with plain VALU uses here, hipcc's register
  // classes put part of the 256 accumulators in arch VGPRs for the whole
  // kernel and shuttled them through v_accvgpr_read/write around every MFMA
  // (≈3 VALU per MFMA).
  auto rd_acc = [](const f32x4& a) {
    f32x4 v;
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\tv_accvgpr_read_b32 %3, %7"
                 : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3])
                 : "a"(a[0]), "a"(a[1]), "a"(a[2]), "a"(a[3]));
    return v;
  };
  auto st16 = [](bf16* p, bf16x8 v) { __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p)); };
  // the row epilogue of the current tile (m0, n0, tm, halfn)
  auto row_epilogue = [&]() {
    // hipcc does not pad the asm against the last MFMAs: 16 wait states first
    // (≥ the 8-pass XDL D → read requirement)
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    // acc[i][j][e] = C[m][n], m = wm·128 + 16i + 4(l >> 4) + e,
    // n = wn·128 + 8(l & 15) + j.  Per (i, e) a lane stores 8 consecutive
    // columns; the 64 lanes cover 4 rows × 128 columns.
    if (halfn && wn == 1) return;
    const int g4 = lane >> 4;
    const int nb = n0 + wn * 128 + 8 * (lane & 15);
    const size_t mr = (size_t)(m0 + wm * 128 + 4 * g4);
    // EPI 3: the GELU pre-activation; EPI 4 / 5 / 6: the addend; EPI 8: the saved GELU'
    constexpr bool PRE = EPI >= 3 && EPI != 7 && EPI != 9;
    bf16x8 pre[PRE ? 32 : 1];
    unsigned char mk[EPI == 6 ? 32 : 1];  // EPI 6: the addend's keep bits (8 columns per byte)
    if constexpr (PRE) {
#pragma unroll
      for (int u = 0; u < 32; ++u) {
        if constexpr (EARLY8) {
          if (u < 16) {
            pre[u] = pre_early[u];
            continue;
          }
        }
        pre[u] = *reinterpret_cast<const bf16x8*>(Y + (mr + 16 * (u >> 2) + (u & 3)) * ldy + nb);
      }
    }
    if constexpr (EPI == 6) {
      const unsigned char* mask = reinterpret_cast<const unsigned char*>(bias);
#pragma unroll
      for (int u = 0; u < 32; ++u) mk[u] = mask[((mr + 16 * (u >> 2) + (u & 3)) * ldy + nb) >> 3];
    }
    f32x8 bv8 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr ((EPI >= 1 && EPI <= 3) || EPI == 5 || EPI == 7) bv8 = to_f32(*reinterpret_cast<const bf16x8*>(bias + nb));
    f32x8 colp = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    f32x2 m1 = {-1.f, -1.f};
    asm volatile("" : "+v"(m1));
    // EPI 9: BatchNorm statistics of the bf16 outputs — per lane its 8 columns
    // over the 32 rows it holds (16i + 4(l >> 4) + e), shifted by the first row
    // (x0) so Σd² − (Σd)²/32 does not cancel when |mean| ≫ std
    f32x8 x0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ssum = x0, ssq = x0;
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
        } else if constexpr (EPI == 9) {
          const bf16x8 o = to_bf16(v);
          st16(crow, o);
          const f32x8 r = to_f32(o);
          if (i == 0 && e == 0) x0 = r;
          const f32x8 d = r - x0;
          ssum += d;
          ssq += d * d;
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
        } else if constexpr (EPI == 7) {
          // fc1 with the derivative saved instead of the pre-activation: C =
          // gelu'(x), Y = gelu(x), x = the fp32 product + bias
          const f32x8 x = v + bv8;
          f32x8 y, g;
#pragma unroll
          for (int q = 0; q < 8; q += 2) {
            f32x2 yy, gg;
            gelu_and_grad2(f32x2{x[q], x[q + 1]}, m1, yy, gg);
            y[q] = yy[0];
            y[q + 1] = yy[1];
            g[q] = gg[0];
            g[q + 1] = gg[1];
          }
          st16(crow, to_bf16(g));
          st16(Y + m * ldy + nb, to_bf16(y));
        } else if constexpr (EPI == 8) {
          // fc2's input gradient against the saved GELU': C = (A·Bᵀ) ⊙ Y, + bias-gradient partials
          const f32x8 d = v * to_f32(pre[4 * i + e]);
          colp += d;
          st16(crow, to_bf16(d));
        } else if constexpr (EPI == 4) {
          st16(crow, to_bf16(v + to_f32(pre[4 * i + e])));  // C = A·Bᵀ + Y, one rounding
        } else if constexpr (EPI == 5) {
          st16(crow, to_bf16(v + bv8 + to_f32(pre[4 * i + e])));  // C = A·Bᵀ + bias + Y (residual stream)
        } else if constexpr (EPI == 6) {
          // C = A·Bᵀ + Y ⊙ keep: a branch gradient whose ReLU mask is applied here
          const unsigned bits = mk[4 * i + e];
          f32x8 r = to_f32(pre[4 * i + e]);
#pragma unroll
          for (int q = 0; q < 8; ++q) r[q] = (bits >> q) & 1u ? r[q] : 0.f;
          st16(crow, to_bf16(v + r));
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
    if constexpr (EPI == 9) {
      // this lane's 32 rows, then the four lane groups (same columns, rows
      // 4·g4 + …) merged by xor-16 / xor-32 exchanges: one 128-row group per
      // (M-tile, wm), partial row 2·tm + wm of [M/128][2][N]
      f32x8 sum = ssum + 32.f * x0, m2 = ssq - ssum * ssum * (1.f / 32.f);
      float n = 32.f;
#pragma unroll
      for (int x = 16; x <= 32; x *= 2) {
        f32x8 s2, q2;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          s2[k] = __shfl_xor(sum[k], x, 64);
          q2[k] = __shfl_xor(m2[k], x, 64);
        }
        chan_merge_equal(sum, m2, s2, q2, n);
        n *= 2.f;
      }
      if (g4 == 0) {
        float* prow = dbias_part + (size_t)(2 * tm + wm) * 2 * N + nb;
        *reinterpret_cast<f32x4*>(prow) = f32x4{sum[0], sum[1], sum[2], sum[3]};
        *reinterpret_cast<f32x4*>(prow + 4) = f32x4{sum[4], sum[5], sum[6], sum[7]};
        *reinterpret_cast<f32x4*>(prow + N) = f32x4{m2[0], m2[1], m2[2], m2[3]};
        *reinterpret_cast<f32x4*>(prow + N + 4) = f32x4{m2[4], m2[5], m2[6], m2[7]};
      }
    }
    if constexpr (EPI == 3 || EPI == 8) {
      // the four lane groups (same 8 columns, rows 4·g4 + …) merged by xor-16 /
      // xor-32 exchanges: partial row 2·tm + wm (gemm_nt4_dbias_rows) holds this
      // wave's 128 rows — a quarter of the partial bytes of one row per lane group
#pragma unroll
      for (int x = 16; x <= 32; x *= 2)
#pragma unroll
        for (int k = 0; k < 8; ++k) colp[k] += __shfl_xor(colp[k], x, 64);
      if (g4 == 0) {
        float* prow = dbias_part + (size_t)(2 * tm + wm) * N + nb;
        *reinterpret_cast<f32x4*>(prow) = f32x4{colp[0], colp[1], colp[2], colp[3]};
        *reinterpret_cast<f32x4*>(prow + 4) = f32x4{colp[4], colp[5], colp[6], colp[7]};
      }
    }
  };

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
  // (r & 7) stationary over A fragments 0-7 (MIR: A stationary), k half s >> 6.
  //   s  0-14 (even)  F1 A reads           s 23        lgkmcnt(0), barrier 1
  //   s 24-45 (÷3)    A pieces of t+2      s 25-46 (÷3) F1 B reads
  //   s 51            lgkmcnt(0), barrier 2
  //   s 52-87 (÷5)    B pieces of t+2      s 93        vmcnt(t+2 pieces), barrier 3
  //   s 94-124 (even) F0 reads of t+1 (other buffer)
  auto tile3 = [&](int t, auto buf_tag, auto first_tag, auto more_tag, auto load_tag,
                   auto lastk_tag, bool tk = false) {
    constexpr int BUF = decltype(buf_tag)::value;
    constexpr bool FIRST = decltype(first_tag)::value;
    constexpr bool MORE = decltype(more_tag)::value;
    constexpr bool LOAD = decltype(load_tag)::value;
    constexpr bool LASTK = decltype(lastk_tag)::value;
    using NB = std::integral_constant<int, BUF ^ 1>;
    using SB = std::integral_constant<int, BUF>;
    Src sn2{};
    if constexpr (LOAD) sn2 = srcs(t + 2);
    static_for<128>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      constexpr int i = MIR ? (s >> 3) & 7 : s & 7, j = MIR ? s & 7 : (s >> 3) & 7;
      if constexpr (s < 64) {
        if constexpr (FIRST) mma0(acc[i][j], fa0[i], fb0[j]);
        else mma(acc[i][j], fa0[i], fb0[j]);
      } else {
        mma(acc[i][j], fa1[i], fb1[j]);
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
      if constexpr (LOAD && s == 92) {
        if (dyn && tk && w == 0 && lane == 0) ticket = atomicAdd(sched + xq, 1u);
      }
      if constexpr (MORE && s == 93) {
        // this wave's tile t+1 pieces retired (its 16 tile t+2 pieces may stay in
        // flight; wave 0 of a ticket tile: those and the ticket's atomic)
        if constexpr (LOAD) {
          if (dyn && tk && w == 0)
            asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
          else
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
      }
      if constexpr (MORE && s >= 94 && s < 126 && (s & 1) == 0) rdF0(NB{}, (s - 94) >> 1);
      if constexpr (MORE && !LOAD && s == 95) {  // k-tile nk − 2: the ticket has returned (vmcnt(0) at 93)
        if (dyn && w == 0) s_next = xq + 8 * (j0 + (int)__builtin_amdgcn_readfirstlane(ticket));
      }
      if constexpr (LASTK) {
        if constexpr (s == 49) {
          // every wave's last LDS reads of this tile precede any wave's refill
          if (dyn) {  // (the barrier also publishes s_next)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            vnext = __builtin_amdgcn_readfirstlane(s_next);
            has_next = vnext < nwg;
            if (has_next) coords(vnext, ntm, ntn);
          } else if (has_next) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
          }
          if (has_next) {
            baseA = A + ((size_t)ntm * BM + 8 * w) * lda;
            baseB = B + ((size_t)ntn * BN + 64 * (w & 1) + (w >> 1)) * ldb;
            dhalfn = ntn * BN + BN > N;
            nx0 = srcs(0);
            nx1 = srcs(1);
          }
        }
        if constexpr (s >= 50 && s < 66) {
          if (has_next) dma(nx0, B0{}, s - 50);
        }
        if constexpr (s >= 66 && s < 82) {
          if (has_next) dma(nx1, B1{}, s - 66);
        }
        if constexpr (EARLY8 && s >= 83 && s < 115 && (s & 1)) {
          constexpr int u = (s - 83) >> 1;
          const int g4 = lane >> 4;
          const size_t mr = (size_t)(m0 + wm * 128 + 4 * g4);
          // a half-width tile's wn = 1 waves store nothing: their (unused) rows stay in bounds
          const int nb = n0 + ((halfn && wn == 1) ? 0 : wn * 128) + 8 * (lane & 15);
          pre_early[u] = *reinterpret_cast<const bf16x8*>(Y + (mr + 16 * (u >> 2) + (u & 3)) * ldy + nb);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  issue01();
  for (;;) {
    // tile 0 landed (tile 1 may fly)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) rdF0(B0{}, q);
    // nk is even and ≥ 4 (host contract): pairs of tiles keep the buffer index static
    tile3(0, B0{}, T_{}, T_{}, T_{}, F_{});
    tile3(1, B1{}, F_{}, T_{}, T_{}, F_{}, nk == 4);
    for (int t = 2; t < nk - 2; t += 2) {
      tile3(t, B0{}, F_{}, T_{}, T_{}, F_{});
      tile3(t + 1, B1{}, F_{}, T_{}, T_{}, F_{}, t + 1 == nk - 3);
    }
    tile3(nk - 2, B0{}, F_{}, T_{}, F_{}, F_{});
    if (!dyn) {
      vnext = vcur + (int)gridDim.x;
      has_next = vnext < nwg;
      if (has_next) coords(vnext, ntm, ntn);
    }
    tile3(nk - 1, B1{}, F_{}, F_{}, F_{}, T_{});  // issues the next tile's k-tiles 0 and 1 (has_next)
    if (!has_next) break;
    row_epilogue();  // of this tile (m0, n0, tm, halfn)
    vcur = vnext;
    tm = ntm;
    tn = ntn;
    m0 = tm * BM;
    n0 = tn * BN;
    halfn = dhalfn;
  }
  row_epilogue();
  if (dyn && w == 0) {
    // the last workgroup out resets this launch slot's counters (vector stores)
    unsigned done = 0;
    if (lane == 0) done = atomicAdd(sched + 8, 1u);
    done = __builtin_amdgcn_readfirstlane(done);
    if (done == gridDim.x - 1 && lane < 9) sched[lane] = 0u;
  }
}

}  // namespace

// dynamic tile order: launch slots of 9 counters (8 XCDs + the exit count) in
// a ring, zero between launches (the kernel's last workgroup resets its slot);
// a launch inside a graph capture keeps its slot, which every replay leaves
// zeroed again.  No slot (allocation failed, or a first launch inside a
// capture): the static order.  Off (gemm_nt4_set_dynamic, for experiments):
// on one GPU the static order is 0.5 ms/step faster (GPT-2-medium 141.35 vs
// 141.87 ms), and in a step with CU-holding side kernels launched where the
// bucketed DDP launches its all-reduces the dynamic order did not recover any
// of the delay (tools/overlap_step_probe.py: +3.7 ms static vs +4.1 ms dynamic)
// — a side kernel gets its CU at a kernel boundary and delays whichever kernel
// comes next, most often not a gemm_nt4 (profiles/r6r_overlap_probe.md)
static int g_nt4_dynamic = 0;
void gemm_nt4_set_dynamic(int on) { g_nt4_dynamic = on; }
static unsigned* sched_slot(hipStream_t st) {
  constexpr int SLOTS = 256, SLOT_U32 = 16;  // one 64-B line per launch
  static unsigned* ring = nullptr;
  static std::atomic<unsigned> next{0};
  if (!g_nt4_dynamic) return nullptr;
  if (!ring) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    static unsigned* const r = [] {
      void* p = nullptr;
      if (hipMalloc(&p, SLOTS * SLOT_U32 * sizeof(unsigned)) != hipSuccess) return (unsigned*)nullptr;
      if (hipMemset(p, 0, SLOTS * SLOT_U32 * sizeof(unsigned)) != hipSuccess) return (unsigned*)nullptr;
      return (unsigned*)p;
    }();
    ring = r;
    if (!ring) return nullptr;
  }
  return ring + SLOT_U32 * (next.fetch_add(1, std::memory_order_relaxed) % SLOTS);
}

// one workgroup per CU (a multiple of 8: the XCD mapping)
static int persistent_grid(long long tiles) {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n >= 8 ? n / 8 * 8 : 8;
  }();
  return (int)(tiles < ncu ? tiles : ncu);
}

// B-stationary runs for K ≤ 1024, mirrored above (tools/nt4_probe.py,
// profiles/r3_gemm_nt4_rows.md)
int gemm_nt4(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
             const bf16* bias, bf16* Y, int ldy, float* dbias_part, hipStream_t st) {
  if (N % BN && N % BN != BN / 2) return -2;
  const long long tiles = (long long)(M / BM) * ((N + BN - 1) / BN);
  if (tiles > 0x7fffffffLL) return -2;
  const int nk = K / BK;
  if (nk < 4 || nk % 2) return -2;  // the mainloop runs k-tiles in pairs, at least two
  // 4 since round 5 (with the saved-gelu' / BatchNorm-statistics epilogues): GPT-2-medium step 145.511 /
  // 145.624 / 145.680 / 145.716 (8) vs 145.498 / 145.392 / 145.501 / 145.406 ms (4), 16 +3.2 ms
  // (soab, profiles/r5gd_saved_gelu_grad.md); round 3 had 8 ahead of 4 and 16 on the older epilogues
  constexpr int group_m = 4;
  const int g = persistent_grid(tiles);
  unsigned* sched = sched_slot(st);
  auto go = [&](auto kern) {
    kern<<<g, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part, group_m, sched);
    return 0;
  };
  auto launch = [&](auto mir_tag) -> int {
    constexpr bool MI = decltype(mir_tag)::value;
    switch (epi) {
      case 0: return go(gemm_nt4_kernel<0, MI>);
      case 1: return go(gemm_nt4_kernel<1, MI>);
      case 2: return go(gemm_nt4_kernel<2, MI>);
      case 3: return go(gemm_nt4_kernel<3, MI>);
      case 4: return go(gemm_nt4_kernel<4, MI>);
      case 5: return go(gemm_nt4_kernel<5, MI>);
      case 6: return go(gemm_nt4_kernel<6, MI>);
      case 7: return go(gemm_nt4_kernel<7, MI>);
      case 8: return go(gemm_nt4_kernel<8, MI>);
      case 9: return go(gemm_nt4_kernel<9, MI>);
      default: return -4;
    }
  };
  return K > 1024 ? launch(std::true_type{}) : launch(std::false_type{});
}

}  // namespace pdo
