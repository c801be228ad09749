// SPDX-License-Identifier: Apache-2.0
// Causal flash attention forward / backward for head_dim 64 on gfx950.
//
// Layout: the QKV GEMM output is consumed in place, qkv = [B, S, 3, H, 64]
// (row stride 3·H·64 between positions); o = [B, S, H, 64]; lse = [B, H, S].
//
// MFMA: v_mfma_f32_32x32x16_bf16 throughout (one wave = 32 rows).
// Forward (FA2 structure, one workgroup = 4 waves = 128 queries of one (b,h)):
//   S^T = K·Q^T with the query on the lane, so the online-softmax row
//   statistics are lane-local (one cross-half exchange for the max), and the
//   S^T accumulator is directly the B operand of O^T = V^T·P^T (no LDS round
//   trip for P; k order permuted as in cdna_hip_programming.md §3).  V^T
//   fragments come from ds_read_b64_tr_b16 transposed LDS reads.
// Backward: two kernels without atomics.
//   dK/dV: workgroup = 128 keys (32 per wave, key on the lane), S and dP are
//     computed as [q × key] so P and dS are the B operands of dV^T = dO^T·P
//     and dK^T = Q^T·dS; Q / dO / lse / delta tiles reach LDS by LDS-DMA
//     through a 3-slot ring (no register staging: 196 instead of 222 VGPRs).
//   dQ:   workgroup = 128 queries, S^T / dP^T with the query on the lane,
//     dQ^T = K^T·dS^T; K / V tiles stream through LDS (register-staged).  Runs
//     first and also writes delta = rowsum(dO ∘ O) (its dO fragments are
//     already in registers) and lse·log2e, which dK/dV then DMAs: no
//     separate delta pass.
// Staging choice per kernel measured in the training step (profiled with tools/gpu.sh step / soab:
// rocprofv3 per-kernel times of extension variants in one session): LDS-DMA
// wins for dK/dV (427.7 vs 448.0 µs) but not for the forward (DMA 2-slot ring at
// 4 waves/SIMD 278.5 µs, 3-slot 275.6, register staging 267.4 — although the
// microbenchmark on random inputs ranked them the other way) nor for dQ
// (365.6 vs 358.6 µs; 373.0 vs 369.9 on a second box).
// LDS tiles are [64 rows][64 bf16] with one XOR swizzle of the 16-B chunk
// index, chosen so BOTH the row reads (ds_read_b128, 16 rows per lane group)
// and the transposed reads (4 rows × 64 B per half-wave) are conflict-free.
// The forward's V tile is only read transposed and uses a swizzle that repeats
// every 8 rows, so its fragment addresses are per-lane constants plus
// ds_read immediates (toff_v; 1.6 % on the forward, bitwise-identical output).
#include <math.h>
#include <stdlib.h>

#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace pdo {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int HD = 64;     // head dim
constexpr int TROWS = 64;  // rows per LDS tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

__device__ __forceinline__ int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
// element offset of (row r, 16-B chunk ch) in a swizzled [64][64] bf16 tile
__device__ __forceinline__ int toff(int r, int ch) { return r * HD + ((ch ^ swz(r)) << 3); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ f32x16 bcast16(float v) {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = v;
  return z;
}

// operand prescale: x ← bf16(c · x), once per workgroup on the register-resident
// operand, so every score MFMA yields c2·q·k directly (log2-domain logits) and
// the softmax needs no per-score multiply.  Rounds c·x to bf16 once (the score's
// relative error grows from 2^-9 to ≈ 1.4 · 2^-9).
template <int N>
__device__ __forceinline__ void prescale(bf16x8 (&v)[N], float c) {
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = to_bf16(to_f32(v[i]) * c);
}

// row fragment: lane reads row (rbase + lane&31), chunk (2ks + lane>>5)
__device__ __forceinline__ bf16x8 row_frag(const bf16* T, int rbase, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(T + toff(rbase + (lane & 31), 2 * ks + (lane >> 5)));
}

// transposed fragment: A[row = cbase + lane&31][k permuted] = T[k0 + 8(j>>2) + 4hh + (j&3)][cbase + lane&31]
__device__ __forceinline__ bf16x8 tr_frag(const bf16* T, int k0, int cbase, int lane) {
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int col = cbase + 16 * (g & 1) + 4 * p;
  const int r0 = k0 + 4 * (g >> 1) + q;
  const int ch = col >> 3, in = col & 7;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(T + toff(r0, ch) + in));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(T + toff(r0 + 8, ch) + in));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// transposed fragment from two precomputed per-lane addresses (rows k0 and k0 + 8)
__device__ __forceinline__ bf16x8 ld_tr(const bf16* lo_p, const bf16* hi_p) {
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)lo_p);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)hi_p);
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// 8 accumulator registers [8s, 8s+8) → bf16 B-operand fragment
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)x[8 * s + j];
  return r;
}

// lane l ↔ lane l ^ 32 combine through v_permlane32_swap (a VALU op; __shfl_xor
// by 32 is a ds_bpermute LDS round trip on the softmax critical path)
__device__ __forceinline__ float xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Retire loop-invariant operand loads BEFORE the tile loop.  Otherwise
// hipcc's waitcnt pass treats them as possibly pending at the loop's first
// MFMA; vmcnt is in-order, so every iteration then waits for its own K/V
// prefetch (issued just before) — the global-load latency lands on the
// critical path of every tile.  An empty asm use forces the wait here.
template <int N>
__device__ __forceinline__ void retire(const bf16x8 (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(v[i]));
}
__device__ __forceinline__ void retire(float x) { asm volatile("" ::"v"(x)); }

// Work order of the (b, h) × block grid: heaviest blocks first across every
// (b, h) (r = 0 is the heaviest block of the pair).  ``order`` is reserved
// (0); the XCD-grouped alternative was measured and removed (attn_order).
__device__ __forceinline__ void attn_block(int order, int nb, int BH, int& bh, int& r) {
  (void)order;
  (void)nb;
  const int id = blockIdx.x;
  bh = id % BH;
  r = id / BH;
}

// ----- global → register → LDS staging of a [64 rows][64] tile (256 threads) -----
struct Stage {
  bf16x8 v[2];
};

__device__ __forceinline__ void stage_load(Stage& st, const bf16* base, size_t row_stride, int row0, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    st.v[i] = *reinterpret_cast<const bf16x8*>(base + (size_t)(row0 + r) * row_stride + ch * 8);
  }
}

// the same tile by buffer loads: per-thread byte offsets are loop-invariant
// VGPRs, the tile's row offset a scalar soffset — no per-tile 64-bit address math
__device__ __forceinline__ void stage_voff(unsigned (&vo)[2], size_t row_stride, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    vo[i] = (unsigned)(((size_t)r * row_stride + ch * 8) * 2);
  }
}
__device__ __forceinline__ void stage_load_buf(Stage& st, __amdgpu_buffer_rsrc_t rsrc, const unsigned (&vo)[2],
                                               unsigned soff) {
#pragma unroll
  for (int i = 0; i < 2; ++i) st.v[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo[i], soff, 0));
}

__device__ __forceinline__ void stage_store(const Stage& st, bf16* T, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *reinterpret_cast<bf16x8*>(T + toff(r, ch)) = st.v[i];
  }
}

// ----- global → LDS by LDS-DMA: no register staging, no ds_write -----
// A [64 rows][64] bf16 tile in the toff() image is 8 pieces of 8 rows; a piece
// is one wave-instruction (1 KiB: lane l → row 8p + (l >> 3), LDS chunk l & 7).
// The XOR swizzle is applied on the SOURCE side: the lane fetches logical chunk
// (l & 7) ^ swz(row), which toff() places at chunk l & 7.  Wave w moves pieces
// 2w and 2w + 1 of every tile; swz() only sees row bits 1-3, so the per-lane
// byte offsets of an even and an odd piece are two loop-invariant VGPRs.  M0
// carries the piece's LDS address (nothing else in these kernels reads M0);
// s_nop 0 = the SALU M0 write → LDS-DMA wait state.  The DMA counts in vmcnt:
// consumers wait with s_waitcnt vmcnt(N) for their own pieces, then barrier.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ unsigned dma_voff(int lane, size_t row_stride, int odd) {
  const int rr = lane >> 3;
  return (unsigned)(((size_t)rr * row_stride + (size_t)(((lane & 7) ^ swz(8 * odd + rr)) << 3)) * 2);
}
__device__ __forceinline__ void glds16(unsigned voff, const void* sbase, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ void glds4(unsigned voff, const void* sbase, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_byte)
               : "memory");
}
// rows [row0 + 16w, row0 + 16w + 16) of a [rows][64] bf16 matrix → the wave's 2 pieces of an LDS tile
__device__ __forceinline__ void dma_tile(const bf16* base, size_t row_stride, int row0, int wu, unsigned v_even,
                                         unsigned v_odd, unsigned lds_tile) {
  const bf16* src = base + (size_t)(row0 + 16 * wu) * row_stride;
  glds16(v_even, src, lds_tile + 2048 * wu);
  glds16(v_odd, src + 8 * row_stride, lds_tile + 2048 * wu + 1024);
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// store a 32x32 f32 accumulator (lane col = row index `rowv`, regs = 32 columns
// starting at c0) as bf16 into dst[rowv][c0 + ...] with scale
__device__ __forceinline__ void store_acc_rows(bf16* dst_row, const f32x16& acc, int c0, int hh, float s) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    bf16x4 v = {(bf16)(acc[4 * g] * s), (bf16)(acc[4 * g + 1] * s), (bf16)(acc[4 * g + 2] * s),
                (bf16)(acc[4 * g + 3] * s)};
    *reinterpret_cast<bf16x4*>(dst_row + c0 + 8 * g + 4 * hh) = v;
  }
}

// Column sums over the workgroup's 128 token rows (the QKV bias gradient,
// fused into the backward kernels).  Lane (li, hh) holds row li, columns
// 32a + 8g + 4hh + e in pair member a, register 4g + e — per half-wave 32
// values for 32 distinct columns.  A butterfly reduce-scatter (send one half
// of the vector to the xor partner, add the partner's other half) needs 16
// shuffles per accumulator instead of 16 × 5.  The 4 waves then add through LDS
// (free at the call: after the loop's last barrier).
// one 32x32 accumulator (columns c0 + 8g + 4hh + e in register 4g + e) →
// this wave's 32 column sums in red[c0 + …].  Butterfly over lane bits 3..0
// (16 live values at most), then one xor-16 add joins the two 16-row groups.
template <int O>
__device__ __forceinline__ void bfly_step(float (&v)[16], int li) {
  // compile-time O: every v[] index is a constant (a runtime step count would
  // turn them into 16-way select chains)
  const bool hi = li & O;
#pragma unroll
  for (int k = 0; k < O; ++k) {
    const float send = hi ? v[k] : v[k + O];
    const float keep = hi ? v[k + O] : v[k];
    v[k] = keep + __shfl_xor(send, O, 64);
  }
}

__device__ __forceinline__ void colsum_acc(const f32x16& acc, int c0, float sc, float* red, int lane) {
  const int hh = lane >> 5, li = lane & 31;
  float v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = acc[r];
  bfly_step<8>(v, li);
  bfly_step<4>(v, li);
  bfly_step<2>(v, li);
  bfly_step<1>(v, li);
  const float t = v[0] + __shfl_xor(v[0], 16, 64);
  // lane li (< 16) holds register index li = 4g + e → column c0 + 8g + 4hh + e
  if (li < 16) red[c0 + 8 * (li >> 2) + 4 * hh + (li & 3)] = t * sc;
}

// after colsum_acc of NP 64-column slots by every wave (red = [4 waves][NP·64]): add the
// 4 waves and write slot p's 64 sums to out[p]
template <int NP>
__device__ __forceinline__ void colsum_finish(const float* red, float* const (&out)[NP], int tid) {
  __syncthreads();
  for (int c = tid; c < 64 * NP; c += 256) {
    const float t = red[c] + red[64 * NP + c] + red[2 * 64 * NP + c] + red[3 * 64 * NP + c];
    out[c >> 6][c & 63] = t;
  }
}

// ============================================================================
// forward
// ============================================================================
// ----- V tile: a transposed-read-only swizzle -----
// V is only ever read transposed (ds_read_b64_tr_b16, 4 rows × 64 B per
// 32-lane half).  Rows r and r+2 share banks, so the 16-B chunk index is XORed
// with 4·bit1(r) only: a row's swizzle then repeats every 8 rows, every
// transposed fragment of the tile is ONE per-lane base address (two: V columns
// 0-31 / 32-63) plus a compile-time row offset, i.e. a ds_read immediate — no
// per-tile address arithmetic.  K keeps the row-read swizzle (toff).
__device__ __forceinline__ int toff_v(int r, int ch) { return r * HD + ((ch ^ (((r >> 1) & 1) << 2)) << 3); }

__device__ __forceinline__ void stage_store_v(const Stage& st, bf16* T, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + 256 * i, r = c >> 3, ch = c & 7;
    *reinterpret_cast<bf16x8*>(T + toff_v(r, ch)) = st.v[i];
  }
}

// per-lane element offset of the tr fragment rows k0 = 0 (lo) for V columns cbase
__device__ __forceinline__ int tr_base_v(int cbase, int lane) {
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  const int col = cbase + 16 * (g & 1) + 4 * p;
  const int r0 = 4 * (g >> 1) + q;
  return toff_v(r0, col >> 3) + (col & 7);
}

template <int K0>
__device__ __forceinline__ bf16x8 tr_frag_v(const bf16* Tlane) {
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Tlane + K0 * HD));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Tlane + (K0 + 8) * HD));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// causal triangle of a 32x32 block whose first key and first query coincide:
// element r of lane (li, hh) holds key c(r) + 4hh of query li, masked iff
// c(r) + 4hh > li — a compile-time 64-bit lane mask per register, applied as
// the SGPR condition of one v_cndmask (no per-element compares)
__device__ __forceinline__ constexpr unsigned long long tri_mask(int r) {
  const int c = (r & 3) + 8 * (r >> 2);
  return ((unsigned long long)((1u << (c + 4)) - 1) << 32) | ((1u << c) - 1);
}

// the transposed block's mask (key on the lane, query c(r) + 4hh on the
// register): masked iff c(r) + 4hh < li
__device__ __forceinline__ constexpr unsigned long long tri_mask_before(int r) {
  const int c = (r & 3) + 8 * (r >> 2);
  const unsigned long long lo = ~((1ull << (c + 1)) - 1) & 0xffffffffull;
  const unsigned long long hi = ~((1ull << (c + 5)) - 1) & 0xffffffffull;
  return (hi << 32) | lo;
}

__device__ __forceinline__ unsigned cvt_pk(float a, float b) {
  unsigned r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// store_acc_rows with the scale applied to register pairs and packed by v_cvt_pk
__device__ __forceinline__ void store_acc_rows_pk(bf16* dst_row, const f32x16& acc, int c0, int hh, float s) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    uint2 v;
    v.x = cvt_pk(acc[4 * g] * s, acc[4 * g + 1] * s);
    v.y = cvt_pk(acc[4 * g + 2] * s, acc[4 * g + 3] * s);
    *reinterpret_cast<uint2*>(dst_row + c0 + 8 * g + 4 * hh) = v;
  }
}

typedef bf16 bf16x2 __attribute__((ext_vector_type(2)));
// l += Σ of the 8 bf16 P values of a B-operand fragment (the values P·V uses)
__device__ __forceinline__ float rowsum8(bf16x8 p, float acc) {
  const bf16x2 one = {(bf16)1.f, (bf16)1.f};
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(p, p, 0, 1), one, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(p, p, 2, 3), one, acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(p, p, 4, 5), one, acc, false);
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(p, p, 6, 7), one, acc, false);
}

// Variant bits (A/B in one build, PDO_ATTN_FWDV): 1 = diagonal mask by lane-mask
// constants (and the fully masked half skipped as −inf), two v_max3 chains
// for the tile max, packed epilogue; 2 = row sums by v_dot2 over the packed P.
template <int V>
__device__ __forceinline__ void attn_fwd_body(const bf16* __restrict__ qkv, bf16* __restrict__ out,
                                              float* __restrict__ lse, int B, int S, int H, float c2, int order) {
  constexpr bool NEW = V & 1, DOT = V & 2;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TROWS * HD];  // [buf][K|V][64][64]
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, li = lane & 31;
  const int w = NEW ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int nqb = S / 128;
  int bh, r_;
  attn_block(order, nqb, B * H, bh, r_);
  const int qb = nqb - 1 - r_;  // heaviest query blocks first
  const int b = bh / H, h = bh % H;
  const size_t rs = (size_t)3 * H * HD;
  const bf16* qbase = qkv + (size_t)b * S * rs + (size_t)h * HD;
  const bf16* kbase = qbase + (size_t)H * HD;
  const bf16* vbase = qbase + (size_t)2 * H * HD;

  const int q = qb * 128 + w * 32 + li;
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * ks + 8 * hh);
  retire(qf);
  prescale(qf, c2);

  const int vb0 = tr_base_v(0, lane), vb1 = tr_base_v(32, lane);
  f32x16 o0 = zero16(), o1 = zero16();
  // m: running max in log2 units; nm16 = −m in every register is the score
  // MFMAs' initial accumulator, so they produce s' = c2·q·k − m directly
  float m = 0.f, l = 0.f;
  f32x16 nm16 = zero16();
  const int ntiles = (qb * 128 + 128) / TROWS;
  const int wave_qmax = qb * 128 + w * 32 + 31;

  Stage sk, sv;
  unsigned vo[2];
  __amdgpu_buffer_rsrc_t rk, rv;
  if constexpr (NEW) {
    const int nbytes = (int)((size_t)S * rs * 2 - (size_t)H * HD * 2 * 2 - (size_t)h * HD * 2);
    rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(kbase), 0, nbytes, 0x00020000);
    rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(vbase), 0, nbytes, 0x00020000);
    stage_voff(vo, rs, tid);
    stage_load_buf(sk, rk, vo, 0);
    stage_load_buf(sv, rv, vo, 0);
  } else {
    stage_load(sk, kbase, rs, 0, tid);
    stage_load(sv, vbase, rs, 0, tid);
  }
  stage_store(sk, smem, tid);
  stage_store_v(sv, smem + TROWS * HD, tid);
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const bf16* Kt = smem + (t & 1) * 2 * TROWS * HD;
    const bf16* Vt = Kt + TROWS * HD;
    const bool more = t + 1 < ntiles;
    if (more) {
      if constexpr (NEW) {
        const unsigned so = (unsigned)((t + 1) * TROWS * rs * 2);
        stage_load_buf(sk, rk, vo, so);
        stage_load_buf(sv, rv, vo, so);
      } else {
        stage_load(sk, kbase, rs, (t + 1) * TROWS, tid);
        stage_load(sv, vbase, rs, (t + 1) * TROWS, tid);
      }
    }
    const int key0 = t * TROWS;
    if (key0 <= wave_qmax) {
      f32x16 s0 = nm16, s1 = nm16;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s0 = mfma(row_frag(Kt, 0, ks, lane), qf[ks], s0);
        s1 = mfma(row_frag(Kt, 32, ks, lane), qf[ks], s1);
      }
      if (key0 + TROWS - 1 > qb * 128 + w * 32) {  // diagonal tile (wave-uniform)
        if constexpr (NEW) {
          // odd wave: keys of s0 precede every query, s1 is the triangle; even
          // wave: s0 is the triangle, s1 follows every query
          if (w & 1) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s1[r] = __builtin_amdgcn_inverse_ballot_w64(tri_mask(r)) ? -INFINITY : s1[r];
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) s0[r] = __builtin_amdgcn_inverse_ballot_w64(tri_mask(r)) ? -INFINITY : s0[r];
            s1 = bcast16(-INFINITY);
          }
        } else {
          // element r holds key key0 + c(r) + 4hh (+32 in s1): masked iff c(r) > q - key0 - 4hh
          const int d = q - key0 - 4 * hh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int c = (r & 3) + 8 * (r >> 2);
            s0[r] = c > d ? -INFINITY : s0[r];
            s1[r] = c + 32 > d ? -INFINITY : s1[r];
          }
        }
      }
      // tile max of s' (relative to m): only a growth past 2^8 rescales
      // (defer-max, cdna_hip_programming.md T13); the first tile sets m
      float tmax;
      if constexpr (NEW) {
        float ta = fmaxf(s0[0], s1[0]), tb = fmaxf(s0[1], s1[1]);
#pragma unroll
        for (int r = 2; r < 16; r += 2) {
          ta = fmaxf(fmaxf(ta, s0[r]), s1[r]);
          tb = fmaxf(fmaxf(tb, s0[r + 1]), s1[r + 1]);
        }
        tmax = xhalf_max(fmaxf(ta, tb));
      } else {
        tmax = -INFINITY;
#pragma unroll
        for (int r = 0; r < 16; r += 2) tmax = fmaxf(fmaxf(tmax, fmaxf(s0[r], s1[r])), fmaxf(s0[r + 1], s1[r + 1]));
        tmax = xhalf_max(tmax);
      }
      if (t == 0) {  // every query has key 0 unmasked here: tmax is finite
        m = tmax;
        s0 -= tmax;
        s1 -= tmax;
        nm16 = bcast16(-m);
      } else if (__any(tmax > 8.f)) {
        const float d = tmax > 8.f ? tmax : 0.f;
        const float alpha = __builtin_amdgcn_exp2f(-d);
        m += d;
        l *= alpha;
        o0 *= alpha;
        o1 *= alpha;
        s0 -= d;
        s1 -= d;
        nm16 = bcast16(-m);
      }
      if constexpr (DOT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s0[r] = __builtin_amdgcn_exp2f(s0[r]);
          s1[r] = __builtin_amdgcn_exp2f(s1[r]);
        }
      } else {
        f32x2 ls2 = {0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          s0[r] = __builtin_amdgcn_exp2f(s0[r]);
          s0[r + 1] = __builtin_amdgcn_exp2f(s0[r + 1]);
          s1[r] = __builtin_amdgcn_exp2f(s1[r]);
          s1[r + 1] = __builtin_amdgcn_exp2f(s1[r + 1]);
          ls2 += f32x2{s0[r], s0[r + 1]} + f32x2{s1[r], s1[r + 1]};
        }
        l += ls2[0] + ls2[1];
      }
      const bf16* V0 = Vt + vb0;
      const bf16* V1 = Vt + vb1;
      float la = 0.f, lb = 0.f;
      {
        const bf16x8 p0 = pack8(s0, 0), p1 = pack8(s1, 0);
        if constexpr (DOT) {
          la = rowsum8(p0, la);
          lb = rowsum8(p1, lb);
        }
        o0 = mfma(tr_frag_v<0>(V0), p0, o0);
        o1 = mfma(tr_frag_v<0>(V1), p0, o1);
        o0 = mfma(tr_frag_v<32>(V0), p1, o0);
        o1 = mfma(tr_frag_v<32>(V1), p1, o1);
      }
      {
        const bf16x8 p0 = pack8(s0, 1), p1 = pack8(s1, 1);
        if constexpr (DOT) {
          la = rowsum8(p0, la);
          lb = rowsum8(p1, lb);
        }
        o0 = mfma(tr_frag_v<16>(V0), p0, o0);
        o1 = mfma(tr_frag_v<16>(V1), p0, o1);
        o0 = mfma(tr_frag_v<48>(V0), p1, o0);
        o1 = mfma(tr_frag_v<48>(V1), p1, o1);
      }
      if constexpr (DOT) l += la + lb;
    }
    if (more) {
      bf16* Kn = smem + ((t + 1) & 1) * 2 * TROWS * HD;
      stage_store(sk, Kn, tid);
      stage_store_v(sv, Kn + TROWS * HD, tid);
    }
    __syncthreads();
  }
  const float lt = xhalf_sum(l);
  bf16* orow = out + ((size_t)(b * S + q) * H + h) * HD;
  if constexpr (NEW) {
    // lt ≥ 1: the key that set m contributes exp2(0)
    const float inv = __builtin_amdgcn_rcpf(lt);
    store_acc_rows_pk(orow, o0, 0, hh, inv);
    store_acc_rows_pk(orow, o1, 32, hh, inv);
    if (hh == 0) lse[(size_t)bh * S + q] = (m + __builtin_amdgcn_logf(lt)) * LN2;
  } else {
    const float inv = 1.f / lt;
    store_acc_rows(orow, o0, 0, hh, inv);
    store_acc_rows(orow, o1, 32, hh, inv);
    if (hh == 0) lse[(size_t)bh * S + q] = (m + log2f(lt)) * LN2;
  }
}

// 168 registers for 3 waves per SIMD: 142.20 / 142.32 vs 142.49 / 142.61 ms per
// GPT-2-medium step for the 2-wave build of the same body (since removed); a
// 4-wave cap spills (29 VGPRs).  A 256-query workgroup (64 rows per wave: each
// LDS K/V fragment feeds two sub-blocks, half the K/V traffic, LDS reads and
// barriers per query) measured no faster (309.6 vs 312.5 µs, 301.5 vs 302.3)
// and was removed: the forward is VALU-issue bound (rocprofv3 --pmc:
// SQ_INSTS_VALU ≈ 12 per MFMA), not LDS- or barrier-bound.
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void attn_fwd3_d64(
    const bf16* __restrict__ qkv, bf16* __restrict__ out, float* __restrict__ lse, int B, int S, int H, float c2,
    int order) {
  attn_fwd_body<V>(qkv, out, lse, B, S, H, c2, order);
}

// ============================================================================
// backward dK / dV: workgroup = 128 keys of one (b,h); loop over query tiles
// ============================================================================
// V (PDO_ATTN_DKDVV): 1 = each sub-block's 4 Q and 4 dO row fragments read
// before its first score MFMA (the reads overlap; otherwise every MFMA waits
// for its own LDS round trip), and the diagonal triangle by lane-mask constants.
template <int V>
__device__ __forceinline__ void dkdv_body(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                          const float* __restrict__ lse, const float* __restrict__ delta,
                                          bf16* __restrict__ dqkv, int B, int S, int H, float c2,
                                          float scale, float* __restrict__ dbias_part, int order) {
  // ring of 3 slots × {Q [64][64] bf16, dO [64][64] bf16, lse·log2e [64] f32, delta [64] f32}
  constexpr int SLOT = 2 * TROWS * HD + 2 * TROWS * 2;  // bf16 units (16896 B)
  __shared__ __attribute__((aligned(16))) bf16 smem[3 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hh = lane >> 5, li = lane & 31;
  const int nkb = S / 128;
  int bh, kb;
  attn_block(order, nkb, B * H, bh, kb);  // lowest key blocks have the most query tiles: issue first
  const int b = bh / H, h = bh % H;
  const size_t rs = (size_t)3 * H * HD;
  const size_t ors = (size_t)H * HD;
  const bf16* qbase = qkv + (size_t)b * S * rs + (size_t)h * HD;
  const bf16* kbase = qbase + (size_t)H * HD;
  const bf16* vbase = qbase + (size_t)2 * H * HD;
  const bf16* dobase = dout + (size_t)b * S * ors + (size_t)h * HD;
  const float* lse2_bh = delta + (size_t)B * H * S + (size_t)bh * S;  // −lse·log2e, written by the dQ kernel
  const float* del_bh = delta + (size_t)bh * S;
  (void)lse;

  const int key = kb * 128 + w * 32 + li;  // this lane's key (column of S / dP)
  bf16x8 kf[4], vf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    kf[ks] = *reinterpret_cast<const bf16x8*>(kbase + (size_t)key * rs + 16 * ks + 8 * hh);
    vf[ks] = *reinterpret_cast<const bf16x8*>(vbase + (size_t)key * rs + 16 * ks + 8 * hh);
  }
  retire(kf);
  retire(vf);
  prescale(kf, c2);  // s' = q·bf16(c2·k): log2-domain logits straight from the MFMA
  f32x16 dv0 = zero16(), dv1 = zero16(), dk0 = zero16(), dk1 = zero16();
  const int qt0 = (kb * 128) / TROWS;
  const int nqt = S / TROWS;
  const int wave_kmin = kb * 128 + w * 32;

  // tile qt → ring slot: Q and dO pieces (2 + 2 per wave) and one stats row per
  // wave (waves 0/2 lse·log2e, 1/3 delta — the pairs write identical bytes), so
  // every wave issues 5 DMAs per tile and waits with the same vmcnt
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const unsigned lds0 = lds_addr(smem);
  const unsigned vq0 = dma_voff(lane, rs, 0), vq1 = dma_voff(lane, rs, 1);
  const unsigned vd0 = dma_voff(lane, ors, 0), vd1 = dma_voff(lane, ors, 1);
  auto issue = [&](int qt, int slot) {
    const unsigned base = lds0 + (unsigned)(slot * SLOT * 2);
    dma_tile(qbase, rs, qt * TROWS, wu, vq0, vq1, base);
    dma_tile(dobase, ors, qt * TROWS, wu, vd0, vd1, base + TROWS * HD * 2);
    glds4((unsigned)lane * 4, ((wu & 1) ? del_bh : lse2_bh) + qt * TROWS,
          base + 2 * TROWS * HD * 2 + (unsigned)(wu & 1) * 256);
  };
  issue(qt0, 0);
  if (qt0 + 1 < nqt) issue(qt0 + 1, 1);
  int sl = 0;

  for (int qt = qt0; qt < nqt; ++qt) {
    if (qt + 1 < nqt)
      vm_wait<5>();  // this wave's pieces of tile qt have landed (qt + 1's 5 may still fly)
    else
      vm_wait<0>();
    __syncthreads();  // ... and every other wave's; slot (sl + 2) % 3 is free again
    if (qt + 2 < nqt) issue(qt + 2, sl == 0 ? 2 : sl - 1);
    const bf16* Qt = smem + sl * SLOT;
    const bf16* Dt = Qt + TROWS * HD;
    const float* L2 = reinterpret_cast<const float*>(Qt + 2 * TROWS * HD);
    const float* DL = L2 + TROWS;
    const int q0 = qt * TROWS;
    if (q0 + TROWS - 1 >= wave_kmin) {
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const int qb0 = q0 + 32 * qs;
        if (qb0 + 31 < wave_kmin) continue;  // all queries before this wave's keys
        // rows r: q = qb0 + (r&3) + 8(r>>2) + 4hh.  The accumulators start at the
        // rows' −lse·log2e and −delta (stored negated by the dQ kernel): the chains
        // end at s' = c2·q·k − lse·log2e and dp' = dO·v − delta
        f32x16 sacc, dpacc;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int qr = 32 * qs + 8 * g + 4 * hh;
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(L2 + qr);
          const f32x4 d4 = *reinterpret_cast<const f32x4*>(DL + qr);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            sacc[4 * g + e] = l4[e];
            dpacc[4 * g + e] = d4[e];
          }
        }
        if constexpr (V == 1) {
          // two k-steps of fragments in flight (16 VGPRs)
          bf16x8 qa0 = row_frag(Qt, 32 * qs, 0, lane), da0 = row_frag(Dt, 32 * qs, 0, lane);
          bf16x8 qa1 = row_frag(Qt, 32 * qs, 1, lane), da1 = row_frag(Dt, 32 * qs, 1, lane);
          sacc = mfma(qa0, kf[0], sacc);
          dpacc = mfma(da0, vf[0], dpacc);
          qa0 = row_frag(Qt, 32 * qs, 2, lane);
          da0 = row_frag(Dt, 32 * qs, 2, lane);
          sacc = mfma(qa1, kf[1], sacc);
          dpacc = mfma(da1, vf[1], dpacc);
          qa1 = row_frag(Qt, 32 * qs, 3, lane);
          da1 = row_frag(Dt, 32 * qs, 3, lane);
          sacc = mfma(qa0, kf[2], sacc);
          dpacc = mfma(da0, vf[2], dpacc);
          sacc = mfma(qa1, kf[3], sacc);
          dpacc = mfma(da1, vf[3], dpacc);
        } else {
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            sacc = mfma(row_frag(Qt, 32 * qs, ks, lane), kf[ks], sacc);
            dpacc = mfma(row_frag(Dt, 32 * qs, ks, lane), vf[ks], dpacc);
          }
        }
        // The causal mask only touches the diagonal sub-tile (wave-uniform): a
        // separate body keeps its compares and selects out of every other tile
        auto softmax_grad = [&](auto masked) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int qr = 32 * qs + 8 * g + 4 * hh;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * g + e;
              float p = __builtin_amdgcn_exp2f(sacc[r]);
              if constexpr (decltype(masked)::value) {
                if constexpr (V == 1) {
                  // diagonal block: query c(r) + 4hh (+ qb0) before key li (+ qb0) is masked
                  p = __builtin_amdgcn_inverse_ballot_w64(tri_mask_before(r)) ? 0.f : p;
                } else {
                  p = (q0 + qr + e) < key ? 0.f : p;
                }
              }
              sacc[r] = p;
              dpacc[r] = p * dpacc[r];
            }
          }
        };
        if (qb0 < wave_kmin + 31)
          softmax_grad(std::true_type{});
        else
          softmax_grad(std::false_type{});
#pragma unroll
        for (int sst = 0; sst < 2; ++sst) {
          if constexpr (V == 1) {  // the four transposed fragments in flight together
            const bf16x8 t0 = tr_frag(Dt, 32 * qs + 16 * sst, 0, lane), t1 = tr_frag(Dt, 32 * qs + 16 * sst, 32, lane);
            const bf16x8 t2 = tr_frag(Qt, 32 * qs + 16 * sst, 0, lane), t3 = tr_frag(Qt, 32 * qs + 16 * sst, 32, lane);
            const bf16x8 pb = pack8(sacc, sst);
            const bf16x8 db = pack8(dpacc, sst);
            dv0 = mfma(t0, pb, dv0);
            dv1 = mfma(t1, pb, dv1);
            dk0 = mfma(t2, db, dk0);
            dk1 = mfma(t3, db, dk1);
          } else {
            const bf16x8 pb = pack8(sacc, sst);
            const bf16x8 db = pack8(dpacc, sst);
            dv0 = mfma(tr_frag(Dt, 32 * qs + 16 * sst, 0, lane), pb, dv0);
            dv1 = mfma(tr_frag(Dt, 32 * qs + 16 * sst, 32, lane), pb, dv1);
            dk0 = mfma(tr_frag(Qt, 32 * qs + 16 * sst, 0, lane), db, dk0);
            dk1 = mfma(tr_frag(Qt, 32 * qs + 16 * sst, 32, lane), db, dk1);
          }
        }
      }
    }
    sl = sl == 2 ? 0 : sl + 1;
  }
  __syncthreads();  // the epilogue's column sums reuse the ring
  // dK = scale * dS^T Q ; dV = P^T dO.  dqkv row `key`, slot 1 (k) and 2 (v)
  bf16* krow = dqkv + (size_t)(b * S + key) * rs + (size_t)H * HD + (size_t)h * HD;
  bf16* vrow = krow + (size_t)H * HD;
  store_acc_rows(krow, dk0, 0, hh, scale);
  store_acc_rows(krow, dk1, 32, hh, scale);
  store_acc_rows(vrow, dv0, 0, hh, 1.f);
  store_acc_rows(vrow, dv1, 32, hh, 1.f);
  if (dbias_part) {  // fp32 partial row b·(S/128) + kb of the QKV bias gradient, k and v slots
    float* prow = dbias_part + (size_t)(b * (S / 128) + kb) * (3 * H * HD) + (size_t)h * HD;
    float* red = reinterpret_cast<float*>(smem);
    colsum_acc(dk0, 0, scale, red + w * 128, lane);
    colsum_acc(dk1, 32, scale, red + w * 128, lane);
    colsum_acc(dv0, 0, 1.f, red + w * 128 + 64, lane);
    colsum_acc(dv1, 32, 1.f, red + w * 128 + 64, lane);
    float* const out[2] = {prow + (size_t)H * HD, prow + (size_t)2 * H * HD};
    colsum_finish<2>(red, out, tid);
  }
}

#define PDO_DKDV_ARGS                                                                                             \
  const bf16 *__restrict__ qkv, const bf16 *__restrict__ dout, const float *__restrict__ lse,                        \
      const float *__restrict__ delta, bf16 *__restrict__ dqkv, int B, int S, int H, float c2, float scale,          \
      float *__restrict__ dbias_part, int order
// capped at 168 VGPRs: 3 waves per SIMD (the LDS ring, 49.5 KiB per
// workgroup, allows 3 workgroups per CU)
template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void attn_bwd_dkdv3_d64(PDO_DKDV_ARGS) {
  dkdv_body<V>(qkv, dout, lse, delta, dqkv, B, S, H, c2, scale, dbias_part, order);
}
#undef PDO_DKDV_ARGS

// ============================================================================
// backward dQ: workgroup = 128 queries of one (b,h); loop over key tiles
// ============================================================================
// Variant bits (PDO_ATTN_DQV): 1 = K/V staging by buffer loads (scalar tile
// offset), per-lane LDS fragment offsets computed once (rows advance in
// multiples of 16, which the swizzle does not see: the tile loop adds only
// immediates), the diagonal tile's triangle masked by lane-mask constants and
// its fully masked 32-key half skipped.
template <int V>
__device__ __forceinline__ void dq_body(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                        const bf16* __restrict__ o, const float* __restrict__ lse,
                                        float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int S, int H,
                                        float c2, float scale, float* __restrict__ dbias_part, int order) {
  constexpr bool NEW = V & 1;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TROWS * HD];
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, li = lane & 31;
  const int w = NEW ? __builtin_amdgcn_readfirstlane(tid >> 6) : tid >> 6;
  const int nqb = S / 128;
  int bh, r_;
  attn_block(order, nqb, B * H, bh, r_);
  const int qb = nqb - 1 - r_;
  const int b = bh / H, h = bh % H;
  const size_t rs = (size_t)3 * H * HD;
  const size_t ors = (size_t)H * HD;
  const bf16* qbase = qkv + (size_t)b * S * rs + (size_t)h * HD;
  const bf16* kbase = qbase + (size_t)H * HD;
  const bf16* vbase = qbase + (size_t)2 * H * HD;
  const bf16* dobase = dout + (size_t)b * S * ors + (size_t)h * HD;

  const int q = qb * 128 + w * 32 + li;
  bf16x8 qf[4], df[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = *reinterpret_cast<const bf16x8*>(qbase + (size_t)q * rs + 16 * ks + 8 * hh);
    df[ks] = *reinterpret_cast<const bf16x8*>(dobase + (size_t)q * ors + 16 * ks + 8 * hh);
  }
  const float lq = lse[(size_t)bh * S + q] * LOG2E;
  // delta = rowsum(dO ∘ O) for this lane's query, from the dO fragments already
  // in registers (this half-wave's 32 dims) + the other half's via one swap;
  // written for the dK/dV kernel, which runs after this one
  float dpart = 0.f;
  {
    const bf16* orow = o + ((size_t)(b * S + q) * H + h) * HD;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const f32x8 a = to_f32(df[ks]), c = to_f32(*reinterpret_cast<const bf16x8*>(orow + 16 * ks + 8 * hh));
#pragma unroll
      for (int j = 0; j < 8; ++j) dpart = __builtin_fmaf(a[j], c[j], dpart);
    }
  }
  const float dq_delta = xhalf_sum(dpart);
  if (hh == 0) {
    // negated: the dK/dV kernel DMAs them straight into its accumulators' initial values
    delta[(size_t)bh * S + q] = -dq_delta;
    delta[(size_t)B * H * S + (size_t)bh * S + q] = -lq;  // −lse·log2e
  }
  retire(qf);
  retire(df);
  retire(lq);
  retire(dq_delta);
  // (no operand prescale / row-constant accumulators here: the 16-register
  // −lse block pushes this 3-waves-per-SIMD kernel into spills; the per-score
  // FMA stays)
  f32x16 a0 = zero16(), a1 = zero16();
  const int ntiles = (qb * 128 + 128) / TROWS;
  const int wave_qmax = qb * 128 + w * 32 + 31;

  Stage sk, sv;
  unsigned vo[2];
  __amdgpu_buffer_rsrc_t rk, rv;
  // per-lane fragment offsets (NEW): row reads roff[ks] = toff(li, 2ks + hh);
  // transposed reads of V-columns half c: rows 4(g>>1) + q (lo) and + 8 (hi)
  int roff[4], tlo[2], thi[2];
  if constexpr (NEW) {
    const int nbytes = (int)((size_t)S * rs * 2 - (size_t)H * HD * 2 * 2 - (size_t)h * HD * 2);
    rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(kbase), 0, nbytes, 0x00020000);
    rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(vbase), 0, nbytes, 0x00020000);
    stage_voff(vo, rs, tid);
    stage_load_buf(sk, rk, vo, 0);
    stage_load_buf(sv, rv, vo, 0);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) roff[ks] = toff(li, 2 * ks + hh);
    const int g = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int col = 32 * c + 16 * (g & 1) + 4 * pp, r0 = 4 * (g >> 1) + qq;
      tlo[c] = toff(r0, col >> 3) + (col & 7);
      thi[c] = toff(r0 + 8, col >> 3) + (col & 7);
    }
  } else {
    stage_load(sk, kbase, rs, 0, tid);
    stage_load(sv, vbase, rs, 0, tid);
  }
  stage_store(sk, smem, tid);
  stage_store(sv, smem + TROWS * HD, tid);
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    const bool more = t + 1 < ntiles;
    const bf16* Kt = smem + (t & 1) * 2 * TROWS * HD;
    const bf16* Vt = Kt + TROWS * HD;
    if (more) {
      if constexpr (NEW) {
        const unsigned so = (unsigned)((t + 1) * TROWS * rs * 2);
        stage_load_buf(sk, rk, vo, so);
        stage_load_buf(sv, rv, vo, so);
      } else {
        stage_load(sk, kbase, rs, (t + 1) * TROWS, tid);
        stage_load(sv, vbase, rs, (t + 1) * TROWS, tid);
      }
    }
    const int key0 = t * TROWS;
    if (key0 <= wave_qmax) {
      const bool diag = key0 + TROWS - 1 > qb * 128 + w * 32;
#pragma unroll
      for (int ksub = 0; ksub < 2; ++ksub) {
        // diagonal tile: an even wave's second 32 keys follow all its queries
        if (NEW && ksub == 1 && diag && !(w & 1)) continue;
        f32x16 s = zero16(), dp = zero16();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          if constexpr (NEW) {
            s = mfma(*reinterpret_cast<const bf16x8*>(Kt + 32 * ksub * HD + roff[ks]), qf[ks], s);
            dp = mfma(*reinterpret_cast<const bf16x8*>(Vt + 32 * ksub * HD + roff[ks]), df[ks], dp);
          } else {
            s = mfma(row_frag(Kt, 32 * ksub, ks, lane), qf[ks], s);
            dp = mfma(row_frag(Vt, 32 * ksub, ks, lane), df[ks], dp);
          }
        }
        auto softmax_grad = [&](auto masked) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r], c2, -lq));
            if constexpr (decltype(masked)::value) {
              if constexpr (NEW) {
                p = __builtin_amdgcn_inverse_ballot_w64(tri_mask(r)) ? 0.f : p;
              } else {
                const int kr = key0 + 32 * ksub + (r & 3) + 8 * (r >> 2) + 4 * hh;
                p = kr > q ? 0.f : p;
              }
            }
            s[r] = p * (dp[r] - dq_delta);  // dS^T
          }
        };
        // wave-uniform: only the diagonal 32 × 32 block pays for the mask (NEW: the
        // triangle — the even wave's first half, the odd wave's second)
        if (NEW ? (diag && (w & 1) == ksub) : diag)
          softmax_grad(std::true_type{});
        else
          softmax_grad(std::false_type{});
#pragma unroll
        for (int sst = 0; sst < 2; ++sst) {
          const bf16x8 dsb = pack8(s, sst);
          if constexpr (NEW) {
            const bf16* T = Kt + (32 * ksub + 16 * sst) * HD;
            a0 = mfma(ld_tr(T + tlo[0], T + thi[0]), dsb, a0);
            a1 = mfma(ld_tr(T + tlo[1], T + thi[1]), dsb, a1);
          } else {
            a0 = mfma(tr_frag(Kt, 32 * ksub + 16 * sst, 0, lane), dsb, a0);
            a1 = mfma(tr_frag(Kt, 32 * ksub + 16 * sst, 32, lane), dsb, a1);
          }
        }
      }
    }
    if (more) {
      bf16* Kn = smem + ((t + 1) & 1) * 2 * TROWS * HD;
      stage_store(sk, Kn, tid);
      stage_store(sv, Kn + TROWS * HD, tid);
    }
    __syncthreads();
  }
  bf16* qrow = dqkv + (size_t)(b * S + q) * rs + (size_t)h * HD;
  if constexpr (NEW) {
    store_acc_rows_pk(qrow, a0, 0, hh, scale);
    store_acc_rows_pk(qrow, a1, 32, hh, scale);
  } else {
    store_acc_rows(qrow, a0, 0, hh, scale);
    store_acc_rows(qrow, a1, 32, hh, scale);
  }
  if (dbias_part) {  // q slot of the QKV bias-gradient partial row b·(S/128) + qb
    float* prow = dbias_part + (size_t)(b * (S / 128) + qb) * (3 * H * HD) + (size_t)h * HD;
    float* red = reinterpret_cast<float*>(smem);
    colsum_acc(a0, 0, scale, red + w * 64, lane);
    colsum_acc(a1, 32, scale, red + w * 64, lane);
    float* const out[1] = {prow};
    colsum_finish<1>(red, out, tid);
  }
}

template <int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void attn_bwd_dq_d64(
    const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const bf16* __restrict__ o,
    const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv, int B, int S, int H, float c2,
    float scale, float* __restrict__ dbias_part, int order) {
  dq_body<V>(qkv, dout, o, lse, delta, dqkv, B, S, H, c2, scale, dbias_part, order);
}

// Heaviest-first order (attn_block).  The XCD-grouped order cut the kernels'
// L2 misses 2-3× (forward TCC_EA0_RDREQ 3.1e6 vs 1.05e7 per call) and won the
// isolated microbenchmark (backward 761 / 754 vs 775 / 777 µs), but lost in
// the GPT-2-medium step: 144.20 / 144.02 / 144.19 vs 143.88 / 143.78 / 143.81
// ms (stepab, round 5) — its last workgroups end unevenly; removed in round 6.
// 4-wave-per-SIMD builds of the forward and dQ spilled and ran 401 / 1068 µs
// (removed).
static int attn_order() { return 0; }

int attn_fwd(const bf16* qkv, bf16* o, float* lse, int B, int S, int H, int D, float scale, hipStream_t st) {
  if (D != HD || S % 128 != 0) return -2;
  // variant 3 (lane-mask diagonal, v_max3 chains, buffer-load staging, v_dot2
  // row sums, packed epilogue): 285.1 / 289.0 vs 302.6 / 303.1 µs for variant 0
  // (tools/attn_ab.sh, B64 H16 S1024, 2 interleaved rounds; variant 1 alone
  // 290.2 / 290.3, variant 2 alone 298.2 / 300.1).  Variant 0 (pointer
  // staging) remains for a (b, h) slice past 31-bit buffer offsets
  const int grid = B * H * (S / 128);
  const float c2 = scale * LOG2E;
  // buffer-load variants address the (b, h) slice with 31-bit byte offsets
  const bool fits = (size_t)S * 3 * H * HD * 2 < (1ull << 31);
  if (fits)
    attn_fwd3_d64<3><<<grid, 256, 0, st>>>(qkv, o, lse, B, S, H, c2, attn_order());
  else
    attn_fwd3_d64<0><<<grid, 256, 0, st>>>(qkv, o, lse, B, S, H, c2, attn_order());
  return 0;
}

int attn_bwd(const bf16* dout, const bf16* qkv, const bf16* o, const float* lse, float* delta, bf16* dqkv, int B,
             int S, int H, int D, float scale, hipStream_t st, float* dbias_part) {
  if (D != HD || S % 128 != 0) return -2;
  const int grid = B * H * (S / 128);
  // dQ first: it also produces delta = rowsum(dO ∘ O), which dK/dV reads
  // variant 1: forward + backward 772.7 / 769.1 vs 786.9 / 784.3 µs with
  // variant 0 (tools/attn_ab.sh), which remains for slices past 31-bit buffer offsets
  const bool fits = (size_t)S * 3 * H * HD * 2 < (1ull << 31);
  if (fits)
    attn_bwd_dq_d64<1><<<grid, 256, 0, st>>>(qkv, dout, o, lse, delta, dqkv, B, S, H, scale * LOG2E, scale,
                                             dbias_part, attn_order());
  else
    attn_bwd_dq_d64<0><<<grid, 256, 0, st>>>(qkv, dout, o, lse, delta, dqkv, B, S, H, scale * LOG2E, scale,
                                             dbias_part, attn_order());
  // 3 waves per SIMD (168 VGPRs): bwd 799 -> 768 us isolated, -0.55 ms/step
  // against the 2-wave build; variant 1 (fragments prefetched two k-steps / four
  // transposed reads deep, lane-mask triangle): forward + backward 759.4 / 763.0
  // vs 766.8 / 764.8 µs (tools/attn_ab.sh).  The 2-wave build and variant 0
  // were removed in round 6 (settled A/Bs).
  attn_bwd_dkdv3_d64<1><<<grid, 256, 0, st>>>(qkv, dout, lse, delta, dqkv, B, S, H, scale * LOG2E, scale,
                                              dbias_part, attn_order());
  return 0;
}

}  // namespace pdo
