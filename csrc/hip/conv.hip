// SPDX-License-Identifier: Apache-2.0
// NHWC implicit-GEMM convolutions (3×3 and strided 1×1) for ResNet-50 on gfx950.
//
// The reference's ResNet-50 configs (deploy/examples/resnet.yaml:1-29,
// deploy/elastic/resnet.yaml:1-37) launch a training image; here that data
// plane runs on hand-written CDNA4 kernels instead of MIOpen's igemm solvers
// and their zero-fill / cast passes.
//
// One mainloop serves the forward and the input gradient: the output is a
// [tokens × Kout] GEMM whose A operand is gathered from an NHWC activation by
// a per-launch TAP TABLE (per tap: the input-pixel offset relative to the
// token's base pixel, and the column of B where that tap's weights start):
//
//   forward      token (n, ho, wo), base pixel (ho·st − pad, wo·st − pad),
//                taps (r, s), B = W [Kout][R][S][C] (channels_last OHWI)
//   dgrad, st 1  token (n, h, w), taps (pad − r, pad − s), B = Wᵀ [C][R·S][Kout]
//   dgrad, st 2  one launch per output parity class (h % 2, w % 2): token
//                (n, a, b) → pixel (2a + ph, 2b + pw); only the taps with
//                (ph + pad − r) even reach it, at dY pixel a + (ph + pad − r)/2
//                — no MFMA is spent on the zeros of a strided transposed conv
//
// Mainloop (gemm_nt4's operand handling at a smaller tile): a workgroup of 4
// waves owns BM × BN outputs (256 × 64 for Kout = 64, else 128 × 128), each
// wave 64 × 64 = 4 × 4 blocks of v_mfma_f32_16x16x32_bf16; k-step = 64
// channels of one tap.  Both operands reach LDS by LDS-DMA (1 KiB = 8 rows of
// 128 B per wave-instruction), two stages, one tile of lead:
//   * A rows are gathered: every lane of a piece computes its row's source
//     pixel for the k-step's tap; the load is a buffer_load … lds whose offset
//     is pushed past the buffer's range for a padding pixel or a row past the
//     last token, so the hardware writes zeros — no zero-fill pass;
//   * B rows are weight rows, permuted in LDS (physical row 16j + c of a wave's
//     64-column slice holds column 4c + j) so a lane's accumulators hold 4
//     consecutive output channels: the epilogue stores 8 B per lane straight
//     from registers, 128 B per row.
// LDS rows are 128 B with the 16-B chunk c of row r at c ^ ((r >> 1) & 7) (the
// swizzle is applied on the per-lane source address): the 16 rows a
// ds_read_b128 lane group touches land on 16 distinct bank slots.
//
// BatchNorm statistics in the forward epilogue: per M-tile and channel the
// sum and the centred sum of squares of the bf16-rounded outputs
// ([tiles][2][Kout], batchnorm.hip bn_fwd_tiles merges them), so the
// BatchNorm forward needs no statistics pass over the activation.
#include <stdlib.h>

#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int CNT = 256;
constexpr unsigned OOB = 0x80000000u;  // ≥ any buffer's num_records: the load returns zeros
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

template <typename Fn, int... I>
__device__ __forceinline__ void static_for_impl(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

struct ConvArgs {
  const bf16* x;         // A source, NHWC [N][IH][IW][C]
  const bf16* w;         // B [Kout][ldb], row = output channel
  bf16* y;               // output rows [N][OH][OW][Kout]
  float* stats;          // nullptr, or per-M-tile BatchNorm partials [tiles][2][Kout]
  long long M;           // tokens
  int C, Kout, ldb;
  int IH, IW;
  int TA, TB;            // token t = (n·TA + a)·TB + b
  float inv_TA, inv_TB;  // for the float-reciprocal divisions below
  int ist, ipad;         // base pixel (a·ist − ipad, b·ist − ipad)
  int OH, OW, ost, oph, opw;  // output pixel (a·ost + oph, b·ost + opw)
  int ident;             // output row = token (forward)
  // input gradient with the backward statistics of the BatchNorm that produced
  // x (its input bx, batch mean / invstd, affine w / b, ReLU): per M-tile Σg and
  // Σg·(bx − mean), g = dy·[bx·sc + sh > 0], into bpart[tile_off + tile][2][Kout]
  const bf16* bx;
  const bf16* add;  // y = conv + add (same layout as y): a branch gradient joining this one
  const float *bmean, *binv, *bw, *bb;
  float* bpart;
  int brelu, tile_off;
  unsigned xbytes;
  int ntaps;
  int dh[9], dw[9], bcol[9];
};

// q = x / d, r = x - q·d for 0 ≤ x < 2^24 (exact via a float reciprocal + one correction)
__device__ __forceinline__ void divmod(int x, int d, float inv, int& q, int& r) {
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

__device__ __forceinline__ void bufld(unsigned voff, __amdgpu_buffer_rsrc_t rs, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ void glds(unsigned voff, const void* sbase, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase),
               "s"(lds_byte)
               : "memory");
}

// Epilogue shared by the implicit-GEMM mainloops: acc[i][j][e] =
// C[m = wm·RW + 16i + 4(l >> 4) + e][col n0 + wn·64 + 4(l & 15) + j] (RW = BM / WM
// rows per wave): bf16 stores (+ a joining gradient), and the BatchNorm
// forward tile statistics or the consumed BatchNorm's backward partials.
template <int MI, int BM, int BN, int WM>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[MI][4], char* smem, int wm, int wn,
                                              int lane, long long m0, long long tm, int n0) {
  constexpr int RW = BM / WM;
  const int g4 = lane >> 4;
  const int col = n0 + wn * 64 + 4 * (lane & 15);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  f32x4 bsc, bsh, bmu;
  const bool bnb = a.bx != nullptr;
  if (bnb) {
    bmu = *reinterpret_cast<const f32x4*>(a.bmean + col);
    const f32x4 inv = *reinterpret_cast<const f32x4*>(a.binv + col);
    bsc = *reinterpret_cast<const f32x4*>(a.bw + col) * inv;
    bsh = *reinterpret_cast<const f32x4*>(a.bb + col) - bmu * bsc;
  }
  // per 4-row group: the rows' addresses and their joining-gradient / BatchNorm
  // input loads first (8 loads in flight), then the math and the stores
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    long long rowv[4];
    bf16x4 adv[4], xbv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long t = m0 + wm * RW + 16 * i + 4 * g4 + e;
      rowv[e] = -1;
      if (t >= a.M) continue;
      if (a.ident) {
        rowv[e] = t;
      } else {
        int q, bb, n, aa;
        divmod((int)t, a.TB, a.inv_TB, q, bb);
        divmod(q, a.TA, a.inv_TA, n, aa);
        rowv[e] = ((long long)n * a.OH + aa * a.ost + a.oph) * a.OW + bb * a.ost + a.opw;
      }
      if (a.add) adv[e] = *reinterpret_cast<const bf16x4*>(a.add + rowv[e] * a.Kout + col);
      if (bnb) xbv[e] = *reinterpret_cast<const bf16x4*>(a.bx + rowv[e] * a.Kout + col);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long row = rowv[e];
      if (row < 0) continue;
      f32x4 o = {acc[i][0][e], acc[i][1][e], acc[i][2][e], acc[i][3][e]};
      if (a.add) o += f32x4{(float)adv[e][0], (float)adv[e][1], (float)adv[e][2], (float)adv[e][3]};
      const bf16x4 v = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      *reinterpret_cast<bf16x4*>(a.y + row * a.Kout + col) = v;
#pragma unroll
      for (int j = 0; j < 4; ++j) cs[j] += (float)v[j];
      if (bnb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xv = (float)xbv[e][j];
          // the forward's pre-activation through the same fp32 ops (bit-identical mask)
          const float g = (!a.brelu || xv * bsc[j] + bsh[j] > 0.f) ? (float)v[j] : 0.f;
          s1[j] += g;
          s2[j] += g * (xv - bmu[j]);
        }
      }
    }
  }
  if (!a.stats && !bnb) return;
  const int rows = (int)(a.M - m0 < BM ? a.M - m0 : BM);
  float* red = reinterpret_cast<float*>(smem);  // [WM][BN] (the last k-step's barrier freed the stages)
  // LDS-only barriers (lgkmcnt, no memory fence): __syncthreads() would also
  // wait for every global store of this epilogue and, in the persistent stem
  // kernel, for the next tile's LDS-DMA pieces (vmcnt(0))
  auto lds_barrier = [] {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  auto tile_sum = [&](float (&v)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] += __shfl_xor(v[j], 16, 64);
      v[j] += __shfl_xor(v[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wm * BN + wn * 64 + 4 * lane + j] = v[j];
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = 0.f;
#pragma unroll
      for (int u = 0; u < WM; ++u) s += red[u * BN + wn * 64 + 4 * (lane & 15) + j];
      v[j] = s;
    }
    lds_barrier();
  };
  if (bnb) {
    // ---- BatchNorm backward partials of this M-tile: Σg, Σg·(x − mean) per channel
    tile_sum(s1);
    tile_sum(s2);
    if (wm == 0 && lane < 16) {
      float* p = a.bpart + (size_t)(a.tile_off + tm) * 2 * a.Kout + col;
      *reinterpret_cast<f32x4*>(p) = f32x4{s1[0], s1[1], s1[2], s1[3]};
      *reinterpret_cast<f32x4*>(p + a.Kout) = f32x4{s2[0], s2[1], s2[2], s2[3]};
    }
    return;
  }
  // ---- BatchNorm forward partials of this M-tile: Σv and Σ(v − mean_tile)² per channel
  tile_sum(cs);
  float mean[4], cq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) mean[j] = cs[j] / (float)rows;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long t = m0 + wm * RW + 16 * i + 4 * g4 + e;
      if (t >= a.M) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = (float)(bf16)acc[i][j][e] - mean[j];
        cq[j] += d * d;
      }
    }
  tile_sum(cq);
  if (wm == 0 && lane < 16) {
    float* p = a.stats + (size_t)tm * 2 * a.Kout + col;
    *reinterpret_cast<f32x4*>(p) = f32x4{cs[0], cs[1], cs[2], cs[3]};
    *reinterpret_cast<f32x4*>(p + a.Kout) = f32x4{cq[0], cq[1], cq[2], cq[3]};
  }
}

template <int BM, int BN>
__global__ __launch_bounds__(CNT, 2) void conv_igemm_kernel(const ConvArgs a) {
  constexpr int WN = BN / 64, WM = BM / 64;
  static_assert(WM * WN == 4, "4 waves of 64 × 64");
  constexpr int PA = BM / 8, PB = BN / 8;   // 1-KiB pieces per k-step
  constexpr int NA = PA / 4, NB = PB / 4;   // per wave
  constexpr int STAGE = (BM + BN) * 128;    // bytes per stage
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WN, wn = w % WN;
  const int ntn = a.Kout / BN;
  const long long ntm = (a.M + BM - 1) / BM;
  // bijective XCD remap: blocks b and b + 8 share an XCD, so each XCD walks a
  // contiguous range of tiles — the ntn tiles of one token range share its L2
  long long id = blockIdx.x;
  {
    const long long nwg = ntm * ntn, q = nwg >> 3, r = nwg & 7, x = id & 7, slot = id >> 3;
    id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + slot;
  }
  const int tn = (int)(id % ntn);
  const long long tm = id / ntn;
  const long long m0 = tm * BM;
  const int n0 = tn * BN;

  // ---- A pieces: this wave's pieces p = w + 4i (i < NA): rows 8p + (l >> 3)
  int hb[NA], wb[NA], base[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = 8 * (w + 4 * i) + (lane >> 3);
    const long long t = m0 + m;
    const int cg = (lane & 7) ^ ((m >> 1) & 7);
    if (t < a.M) {
      int q, bb, n, aa;
      divmod((int)t, a.TB, a.inv_TB, q, bb);
      divmod(q, a.TA, a.inv_TA, n, aa);
      hb[i] = aa * a.ist - a.ipad;
      wb[i] = bb * a.ist - a.ipad;
      base[i] = ((n * a.IH + hb[i]) * a.IW + wb[i]) * a.C + cg * 8;
      // 16-channel input (the space-to-depth stem): a 128-B row is 4 pixels, the
      // lane's chunk cg lies in pixel cg / 2 of them (bounds checked per lane)
      if (a.C == 16) wb[i] += cg >> 1;
    } else {
      hb[i] = -(1 << 20);  // fails every bounds check
      wb[i] = 0;
      base[i] = 0;
    }
  }
  // ---- B pieces: p = w + 4(NA + i) - PA of the B tile; physical row pr ↔ column
  unsigned voffB[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int pr = 8 * (w + 4 * i) + (lane >> 3);
    const int q = pr & 63;
    const int col = n0 + 64 * (pr >> 6) + 4 * (q & 15) + (q >> 4);
    const int cg = (lane & 7) ^ ((pr >> 1) & 7);
    voffB[i] = (unsigned)((col * a.ldb + cg * 8) * 2);
  }
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int CC = a.C >= 64 ? a.C >> 6 : 1;  // C = 16: one k-step per tap (a row of 4 pixels)
  const int nk = a.ntaps * CC;

  auto issue = [&](int kt, int stage) {
    const int tap = kt / CC, cc = kt - tap * CC;
    const int dh = a.dh[tap], dw = a.dw[tap];
    const int coff = (dh * a.IW + dw) * a.C + cc * 64;
    const unsigned sb = lds0 + (unsigned)(stage * STAGE);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int hi = hb[i] + dh, wi = wb[i] + dw;
      const bool ok = (unsigned)hi < (unsigned)a.IH && (unsigned)wi < (unsigned)a.IW;
      const unsigned v = ok ? (unsigned)((base[i] + coff) * 2) : OOB;
      bufld(v, rsX, sb + (unsigned)((w + 4 * i) * 1024));
    }
    const bf16* bsrc = a.w + a.bcol[tap] + cc * 64;
#pragma unroll
    for (int i = 0; i < NB; ++i) glds(voffB[i], bsrc, sb + (unsigned)(BM * 128 + (w + 4 * i) * 1024));
  };

  // ---- fragment offsets (bytes within a stage)
  const int sw = (lane >> 1) & 7;
  const int ch0 = ((lane >> 4) ^ sw) << 4, ch1 = ((4 + (lane >> 4)) ^ sw) << 4;
  const int rA = (wm * 64 + (lane & 15)) * 128, rB = BM * 128 + (wn * 64 + (lane & 15)) * 128;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      issue(kt + 1, (kt + 1) & 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA + NB) : "memory");  // k-step kt landed (kt + 1 flies)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... for every wave's pieces
    const char* st = smem + (kt & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk ? ch1 : ch0;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(st + rA + i * 2048 + ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(st + rB + j * 2048 + ch);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's reads of this stage precede its refill (k-step kt + 2)
  }

  conv_epilogue<4, BM, BN, WM>(a, acc, smem, wm, wn, lane, m0, tm, n0);
}

// Wᵀ for the input gradient: w [K][T][C] → wt [C][T][K] (T = R·S taps), bf16
__global__ __launch_bounds__(256) void conv_wt_kernel(const bf16* __restrict__ w, bf16* __restrict__ wt, int K, int T,
                                                      int C) {
  const long long n = (long long)K * T * C;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long kt = i / C;
    const int t = (int)(kt % T), k = (int)(kt / T);
    wt[((long long)c * T + t) * K + k] = w[i];
  }
}

// ============================================================================
// weight gradient: dW[co][tap][ci] = Σ_t dY[t][co] · X[pixel(t, tap)][ci]
// Token-major GEMM (the reduction runs over the forward's output tokens): a
// workgroup owns BMW output channels × BNW input channels of ONE tap and a
// slice of the tokens (split-K, fp32 partials [slice][Kout][T·C] folded by
// conv_wgrad_reduce in a fixed order — deterministic).  Per 64-token k-step
// both operands reach LDS as they lie in memory, rows = tokens: dY rows
// straight, X rows gathered per token for the tap (buffer_load … lds, zeros
// for padding pixels and tokens past M).  Fragments are read with
// ds_read_b64_tr_b16 (lane group g takes tokens 4g..4g+3 and 16+4g.. of 16
// columns — the same token permutation for both operands), so the MFMA
// v_mfma_f32_16x16x32_bf16 sums over tokens.  LDS rows of 128 / 256 B with
// the 32-B column group XORed by the row (128 B: bits of (r >> 1) & 3, 256 B:
// r & 7): the 8 rows a transposed read touches per half-wave hit 8 distinct
// bank groups.
// ============================================================================
struct WgradArgs {
  const bf16* dy;        // [M][Kout]
  const bf16* x;         // NHWC [N][IH][IW][C]
  float* part;           // [splits][Kout][T·C]
  long long M;
  int Kout, C, T, S;     // T taps, S = kernel width (tap = r·S + s)
  int IH, IW, TA, TB;    // forward output grid: token t = (n·TA + ho)·TB + wo
  float inv_TA, inv_TB;
  int st, pad;
  unsigned xbytes, dybytes;
  int splits, ksteps;
};

template <int ROWB>
__device__ __forceinline__ int wswz(int r) {
  return ROWB == 256 ? ((r & 7) << 1) : (((r >> 1) & 3) << 1);
}

template <int BMW, int BNW>
__global__ __launch_bounds__(CNT, 2) void conv_wgrad_kernel(const WgradArgs a) {
  constexpr int RA = BMW * 2, RB = BNW * 2;          // LDS row bytes
  constexpr int LA = BMW / 8, LB = BNW / 8;          // lanes per row (16 B each)
  constexpr int PA = BMW / 8, PB = BNW / 8;          // 1-KiB pieces per 64-token k-step
  constexpr int NA = PA / 4, NB = PB / 4;            // per wave
  constexpr int SA = 64 * RA, STAGE = 64 * (RA + RB);
  constexpr int MI = BMW / 32, NJ = BNW / 32;        // 16×16 blocks per wave (wave tile BMW/2 × BNW/2)
  // ring depth: the small tiles do little MFMA work per k-step, so the stream
  // needs more 64-token steps in flight (2 workgroups per CU: ≤ 80 KiB each)
  constexpr int NS = STAGE <= 16384 ? 4 : STAGE <= 24576 ? 3 : 2;
  constexpr int PER = NA + NB;                       // DMA pieces per wave per k-step
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int tiles_m = a.Kout / BMW, tiles_n = a.T * a.C / BNW;
  int id = blockIdx.x;
  const int split = id / (tiles_m * tiles_n);
  id -= split * tiles_m * tiles_n;
  const int tm = id % tiles_m, tn = id / tiles_m;
  const int co0 = tm * BMW;
  const int ncol0 = tn * BNW, tap = ncol0 / a.C, ci0 = ncol0 - tap * a.C;
  const int r = tap / a.S, s = tap - r * a.S;
  const int kq = a.ksteps / a.splits, kr = a.ksteps % a.splits;
  const int k0 = split * kq + min(split, kr), nk = kq + (split < kr ? 1 : 0);

  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.dy), 0, (int)a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // per-lane constant parts of the pieces: row in the tile, source chunk
  auto issue = [&](int kt, int stage) {
    const long long t0 = (long long)kt * 64;
    const unsigned sb = lds0 + (unsigned)(stage * STAGE);
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int p = w + 4 * i;
      const int row = p * (64 / LA) + lane / LA;
      const int c = (lane % LA) ^ wswz<RA>(row);
      const long long t = t0 + row;
      const unsigned v = t < a.M ? (unsigned)((t * a.Kout + co0 + c * 8) * 2) : OOB;
      bufld(v, rsY, sb + (unsigned)(p * 1024));
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int p = w + 4 * i;
      const int row = p * (64 / LB) + lane / LB;
      const int c = (lane % LB) ^ wswz<RB>(row);
      const long long t = t0 + row;
      unsigned v = OOB;
      if (t < a.M) {
        int q, wo, n, ho;
        divmod((int)t, a.TB, a.inv_TB, q, wo);
        divmod(q, a.TA, a.inv_TA, n, ho);
        const int hi = ho * a.st - a.pad + r, wi = wo * a.st - a.pad + s;
        if ((unsigned)hi < (unsigned)a.IH && (unsigned)wi < (unsigned)a.IW)
          v = (unsigned)(((((long long)n * a.IH + hi) * a.IW + wi) * a.C + ci0 + c * 8) * 2);
      }
      bufld(v, rsX, sb + (unsigned)(SA + p * 1024));
    }
  };
  // transposed fragment of the 16 columns cb..cb+15, tokens 32kk + {4g..4g+3, 16+4g..}
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  auto frag = [&](const char* T, int cb, int kk, auto rowb) -> bf16x8 {
    constexpr int RW = decltype(rowb)::value;
    const int col = cb + 4 * p4;
    const int r0 = 32 * kk + 4 * g + q4, r1 = r0 + 16;
    const char* a0 = T + r0 * RW + (((col >> 3) ^ wswz<RW>(r0)) << 4) + (col & 7) * 2;
    const char* a1 = T + r1 * RW + (((col >> 3) ^ wswz<RW>(r1)) << 4) + (col & 7) * 2;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a0);
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a1);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  using IRA = std::integral_constant<int, RA>;
  using IRB = std::integral_constant<int, RB>;

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: k-steps 0 .. NS-2 in flight; step k refills the stage step k-1 used
  // (every wave's reads of it retired at the barrier that closed step k-1)
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nk) issue(k0 + j, j);
  for (int k = 0; k < nk; ++k) {
    if (k + NS - 1 < nk) issue(k0 + k + NS - 1, (k + NS - 1) % NS);
    // steps issued after k (in flight behind it): min(NS - 1, nk - 1 - k)
    const int after = nk - 1 - k < NS - 1 ? nk - 1 - k : NS - 1;
    if (after >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory");
    else if (after == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const char* TA_ = smem + (k % NS) * STAGE;
    const char* TB_ = TA_ + SA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[MI], fb[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = frag(TA_, wm * (BMW / 2) + 16 * i, kk, IRA{});
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = frag(TB_, wn * (BNW / 2) + 16 * j, kk, IRB{});
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // acc[i][j][e] = dW[co0 + wm·BMW/2 + 16i + 4g + e][tap·C + ci0 + wn·BNW/2 + 16j + (l & 15)]
  const long long ldo = (long long)a.T * a.C;
  float* out = a.part + (size_t)split * a.Kout * ldo;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = co0 + wm * (BMW / 2) + 16 * i + 4 * g + e;
      float* orow = out + co * ldo + ncol0 + wn * (BNW / 2) + (lane & 15);
#pragma unroll
      for (int j = 0; j < NJ; ++j) orow[16 * j] = acc[i][j][e];
    }
}

// ============================================================================
// weight gradient, C = Kout = CH, 3×3 (ResNet layers 1 and 2): NT taps in one
// workgroup (CH 64: all nine; CH 128: one kernel row of three, grid × 3).  The
// per-tap kernels re-read dY once per tap tile; here each 64-token k-step stages
// dY once ([64 tok][CH]) and the NT gathered X sub-tiles (each token row's pixel
// computed once, the taps as offsets) — 160 KiB (CH 64) / 128 KiB (CH 128) for
// two stages, one workgroup per CU.  Wave w owns output columns
// [w·NT·CH/4, (w + 1)·NT·CH/4) of the group's NT·CH, all CH rows; fragments are
// transposed LDS reads as in conv_wgrad_kernel.
struct WgradTapsArgs {
  const bf16* dy;
  const bf16* x;
  float* part;  // [splits][CH][9·CH]
  long long M;
  int IH, IW, TA, TB;
  float inv_TA, inv_TB;
  int st, pad;
  unsigned xbytes, dybytes;
  int splits, ksteps;
};

// S2D (the space-to-depth stem, CH = 64, NT = 4): X is the 16-channel image
// [N][IH][IW][16] of stem_s2d; tap u = kernel row u of the 4 × 4 stride-1
// convolution, a 128-B X row = 4 pixels × 16 channels from the token's pixel
// (ho − 2 + u, wo − 2), each lane's 16-B chunk bounds-checked on its own pixel.
template <int CH, int NT, bool S2D>
__global__ __launch_bounds__(CNT, 1) void conv_wgrad_taps_kernel(const WgradTapsArgs a) {
  constexpr int RB = CH * 2;                 // LDS row bytes
  constexpr int TS = 64 * RB;                // bytes of one [64 tok][CH] sub-tile
  constexpr int STAGE = (1 + NT) * TS;
  constexpr int RPP = 1024 / RB;             // rows per 1-KiB piece
  constexpr int LPR = RB / 16;               // lanes per row
  constexpr int PW = 64 / RPP / 4;           // pieces per wave per sub-tile
  constexpr int WC = NT * CH / 4;            // output columns per wave
  constexpr int NJ = WC / 16, MI = CH / 16;  // accumulator blocks
  constexpr int PER = PW * (1 + NT);         // DMA pieces per wave per k-step
  constexpr int XC = S2D ? 16 : CH;          // X channels per pixel
  constexpr int TOT = S2D ? NT * CH : 9 * CH;  // output columns (all tap groups)
  static_assert(!S2D || (CH == 64 && NT == 4), "stem: 64 channels, 4 kernel rows");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int split = blockIdx.x % a.splits, grp = blockIdx.x / a.splits;  // tap group: taps NT·grp ..
  const int kq = a.ksteps / a.splits, kr = a.ksteps % a.splits;
  const int k0 = split * kq + min(split, kr), nk = kq + (split < kr ? 1 : 0);
  const __amdgpu_buffer_rsrc_t rsY = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.dy), 0, (int)a.dybytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // this lane's rows in pieces p = w + 4i: row RPP·p + l / LPR, chunk (l % LPR) ^ swz
  int prow[PW], pch[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    prow[i] = RPP * (w + 4 * i) + lane / LPR;
    pch[i] = (lane % LPR) ^ wswz<RB>(prow[i]);
  }
  auto issue = [&](int kt, int stage) {
    const unsigned sb = lds0 + (unsigned)(stage * STAGE);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const long long t = (long long)kt * 64 + prow[i];
      const unsigned p = (unsigned)((w + 4 * i) * 1024);
      bufld(t < a.M ? (unsigned)((t * CH + pch[i] * 8) * 2) : OOB, rsY, sb + p);
      int hb = -(1 << 20), wb = 0, base = 0;
      if (t < a.M) {
        int q, wo, n, ho;
        divmod((int)t, a.TB, a.inv_TB, q, wo);
        divmod(q, a.TA, a.inv_TA, n, ho);
        hb = ho * a.st - a.pad;
        wb = wo * a.st - a.pad;
        base = ((n * a.IH + hb) * a.IW + wb) * XC + pch[i] * 8;
        if (S2D) wb += pch[i] >> 1;  // this lane's pixel of the 4
      }
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int tap = NT * grp + u, dh = S2D ? u : tap / 3, dw = S2D ? 0 : tap - 3 * dh;
        const bool ok = (unsigned)(hb + dh) < (unsigned)a.IH && (unsigned)(wb + dw) < (unsigned)a.IW;
        bufld(ok ? (unsigned)((base + (dh * a.IW + dw) * XC) * 2) : OOB, rsX, sb + (unsigned)((1 + u) * TS) + p);
      }
    }
  };
  const int g = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3;
  auto frag = [&](const char* T, int cb, int kk) -> bf16x8 {
    const int col = cb + 4 * p4;
    const int r0 = 32 * kk + 4 * g + q4, r1 = r0 + 16;
    const char* a0 = T + r0 * RB + (((col >> 3) ^ wswz<RB>(r0)) << 4) + (col & 7) * 2;
    const char* a1 = T + r1 * RB + (((col >> 3) ^ wswz<RB>(r1)) << 4) + (col & 7) * 2;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a0);
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a1);
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) issue(k0, 0);
  for (int k = 0; k < nk; ++k) {
    if (k + 1 < nk) {
      issue(k0 + k + 1, (k + 1) & 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");  // step k landed (step k + 1 flies)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* S0 = smem + (k & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = frag(S0, 16 * i, kk);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int gc = WC * w + 16 * j, u = gc / CH;  // the group's column → sub-tile u, channel gc % CH
        const bf16x8 fb = frag(S0 + (1 + u) * TS, gc % CH, kk);
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  // acc[i][j][e] = dW[co = 16i + 4g + e][TOT column NT·CH·grp + WC·w + 16j + (l & 15)]
  float* out = a.part + (size_t)split * CH * TOT + NT * CH * grp;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* orow = out + (size_t)(16 * i + 4 * g + e) * TOT + WC * w + (lane & 15);
#pragma unroll
      for (int j = 0; j < NJ; ++j) orow[16 * j] = acc[i][j][e];
    }
}

// out[i] (+)= Σ_s part[s][i] (fp32, 4 per lane).  A block owns 256 / G
// consecutive f32x4 outputs; lane group g sums splits g, g + G, … in order and
// the G group sums join in order through LDS — deterministic, and G-way
// parallel over the splits (a 64 × 64 1×1 weight has 1 024 f32x4 outputs but
// up to 256 splits: one lane per output would walk all of them serially).
// part rows may be padded: output f32x4 i = row i / cols4, column i % cols4 reads
// part f32x4 (i / cols4)·ldp4 + i % cols4 of each split (pn4 f32x4 per split)
template <int G>
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float* __restrict__ part, int splits,
                                                                long long n4, float* __restrict__ out,
                                                                int accumulate, int cols4, int ldp4, long long pn4) {
  constexpr int OB = 256 / G;
  __shared__ f32x4 red[G][OB];
  const int o = threadIdx.x % OB, g = threadIdx.x / OB;
  const long long i = (long long)blockIdx.x * OB + o;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    const long long row = i / cols4, src = row * ldp4 + (i - row * cols4);
#pragma unroll 4
    for (int k = g; k < splits; k += G) v += reinterpret_cast<const f32x4*>(part)[(long long)k * pn4 + src];
  }
  red[g][o] = v;
  __syncthreads();
  if (g == 0 && i < n4) {
    f32x4 t = accumulate ? reinterpret_cast<const f32x4*>(out)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < G; ++k) t += red[k][o];
    reinterpret_cast<f32x4*>(out)[i] = t;
  }
}

template <int BM, int BN>
int launch_igemm(const ConvArgs& a, hipStream_t st) {
  const long long tiles = ((a.M + BM - 1) / BM) * (a.Kout / BN);
  if (tiles > 0x7fffffffLL) return -2;
  conv_igemm_kernel<BM, BN><<<(unsigned)tiles, CNT, 0, st>>>(a);
  return 0;
}

int run_igemm(ConvArgs& a, hipStream_t st, int* tile_rows) {
  a.inv_TA = 1.f / (float)a.TA;
  a.inv_TB = 1.f / (float)a.TB;
  if (a.Kout == 64) {
    if (tile_rows) *tile_rows = 256;
    return launch_igemm<256, 64>(a, st);
  }
  if (tile_rows) *tile_rows = 128;
  return launch_igemm<128, 128>(a, st);
}

bool shape_ok(int C, int Kout, int R, int S, int stride, int pad) {
  return C % 64 == 0 && Kout % 64 == 0 && (Kout == 64 || Kout % 128 == 0) && R == S && (R == 1 || R == 3) &&
         (stride == 1 || stride == 2) && pad == (R - 1) / 2;
}

}  // namespace

int conv_supported(int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad) {
  if (!shape_ok(C, Kout, R, S, stride, pad)) return 0;
  const long long xb = (long long)N * H * W * C * 2;
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const long long M = (long long)N * Ho * Wo;
  if (xb >= (1ll << 31) || M >= (1 << 24) || (long long)N * H * W >= (1 << 24)) return 0;
  const long long yb = M * Kout * 2;
  return yb < (1ll << 31);
}

int conv_fwd_tile_rows(int Kout) { return Kout == 64 ? 256 : 128; }
int conv_fwd_tiles(long long M, int Kout) {
  const int r = conv_fwd_tile_rows(Kout);
  return (int)((M + r - 1) / r);
}

int conv_fwd_nhwc(const bf16* x, int N, int H, int W, int C, const bf16* w, int Kout, int R, int S, int stride, int pad,
                  bf16* y, float* tile_stats, hipStream_t st) {
  if (!conv_supported(N, H, W, C, Kout, R, S, stride, pad)) return -2;
  ConvArgs a{};
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  a.x = x;
  a.w = w;
  a.y = y;
  a.stats = tile_stats;
  a.M = (long long)N * Ho * Wo;
  a.C = C;
  a.Kout = Kout;
  a.ldb = R * S * C;
  a.IH = H;
  a.IW = W;
  a.TA = Ho;
  a.TB = Wo;
  a.ist = stride;
  a.ipad = pad;
  a.OH = Ho;
  a.OW = Wo;
  a.ost = 1;
  a.ident = 1;
  a.xbytes = (unsigned)((long long)N * H * W * C * 2);
  a.ntaps = R * S;
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < S; ++s) {
      const int t = r * S + s;
      a.dh[t] = r;
      a.dw[t] = s;
      a.bcol[t] = t * C;
    }
  return run_igemm(a, st, nullptr);
}

// Wᵀ of many convolution weights in one launch: segment j (blockIdx.y) =
// table[j] = (element offset, K, T, C) in both arenas (bf16 shadow → its Wᵀ
// image).  Per tap t the segment is a K × C → C × K transpose; a block moves one
// 64 × 64 tile through LDS (reads along C, writes along K, both coalesced);
// blockIdx.x enumerates (t, k-tile, c-tile), blocks past a segment's tiles exit.
__global__ __launch_bounds__(256) void conv_wt_batched_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                              const int* __restrict__ table) {
  __shared__ bf16 tile[64][65];
  const int* e = table + 4 * blockIdx.y;
  const long long off = e[0];
  const int K = e[1], T = e[2], C = e[3];
  const int kt = (K + 63) / 64, ct = (C + 63) / 64;
  const int b = blockIdx.x;
  if (b >= T * kt * ct) return;
  const int t = b / (kt * ct), r = b - t * kt * ct, k0 = (r / ct) * 64, c0 = (r % ct) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {  // src [K][T][C]: row k0 + i, columns c0 + tx
    const int k = k0 + i, c = c0 + tx;
    if (k < K && c < C) tile[i][tx] = src[off + ((long long)k * T + t) * C + c];
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {  // dst [C][T][K]: row c0 + i, columns k0 + tx
    const int c = c0 + i, k = k0 + tx;
    if (k < K && c < C) dst[off + ((long long)c * T + t) * K + k] = tile[tx][i];
  }
}

int conv_weight_t_batched(const bf16* src, bf16* dst, const int* table, int n, long long max_tiles,
                          hipStream_t st) {
  if (n < 1 || n > 65535 || max_tiles < 1 || max_tiles > 0x7fffffffLL) return -2;
  conv_wt_batched_kernel<<<dim3((unsigned)max_tiles, (unsigned)n), 256, 0, st>>>(src, dst, table);
  return 0;
}

int conv_weight_t(const bf16* w, bf16* wt, int Kout, int T, int C, hipStream_t st) {
  conv_wt_kernel<<<stream_grid((long long)Kout * T * C, 256), 256, 0, st>>>(w, wt, Kout, T, C);
  return 0;
}

// tiles the input gradient writes BatchNorm-backward partials for (conv_dgrad_nhwc with bn)
int conv_dgrad_tiles(int N, int H, int W, int C, int R, int stride, int pad) {
  const int bm = conv_fwd_tile_rows(C);
  if (stride == 1) return (int)(((long long)N * H * W + bm - 1) / bm);
  long long t = 0;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      int n = 0;
      for (int r = 0; r < R; ++r)
        for (int s = 0; s < R; ++s)
          if (((ph + pad - r) & 1) == 0 && ((pw + pad - s) & 1) == 0) ++n;
      const long long ta = (H - ph + 1) / 2, tb = (W - pw + 1) / 2;
      if (n && ta > 0 && tb > 0) t += ((long long)N * ta * tb + bm - 1) / bm;
    }
  return (int)t;
}

// dx [N][H][W][C] from dy [N][Ho][Wo][Kout] and wt = Wᵀ [C][R·S][Kout]; every
// element of dx is written (parity classes without taps get zeros by a memset,
// which also contribute nothing to the BatchNorm partials)
int conv_dgrad_nhwc(const bf16* dy, int N, int H, int W, int C, const bf16* wt, int Kout, int R, int S, int stride,
                    int pad, bf16* dx, hipStream_t st, const ConvBnBwd* bn, const bf16* add) {
  if (!conv_supported(N, H, W, C, Kout, R, S, stride, pad)) return -2;
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  if ((long long)N * Ho * Wo * Kout * 2 >= (1ll << 31)) return -2;
  ConvArgs a{};
  a.x = dy;
  a.w = wt;
  a.y = dx;
  a.C = Kout;      // A channels = dY's
  a.Kout = C;      // output columns = dX's channels
  a.ldb = R * S * Kout;
  a.IH = Ho;
  a.IW = Wo;
  a.ist = 1;
  a.ipad = 0;
  a.OH = H;
  a.OW = W;
  a.xbytes = (unsigned)((long long)N * Ho * Wo * Kout * 2);
  a.add = add;
  if (bn) {
    a.bx = bn->x;
    a.bmean = bn->mean;
    a.binv = bn->invstd;
    a.bw = bn->w;
    a.bb = bn->b;
    a.bpart = bn->part;
    a.brelu = bn->relu;
  }
  if (!shape_ok(Kout, C, R, S, 1, pad)) return -2;  // the roles of C and Kout swap here
  if (stride == 1) {
    a.M = (long long)N * H * W;
    a.TA = H;
    a.TB = W;
    a.ost = 1;
    a.ident = 1;
    a.ntaps = R * S;
    for (int r = 0; r < R; ++r)
      for (int s = 0; s < S; ++s) {
        const int t = r * S + s;
        a.dh[t] = pad - r;
        a.dw[t] = pad - s;
        a.bcol[t] = t * Kout;
      }
    return run_igemm(a, st, nullptr);
  }
  // stride 2: one launch per parity class of the output pixel
  bool zero_needed = false;
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      int n = 0;
      for (int r = 0; r < R; ++r)
        for (int s = 0; s < S; ++s)
          if (((ph + pad - r) & 1) == 0 && ((pw + pad - s) & 1) == 0) ++n;
      if (n == 0) zero_needed = true;
    }
  // rows no class writes: zeros (or the addend itself)
  if (zero_needed) {
    const hipError_t e = add ? hipMemcpyAsync(dx, add, (size_t)N * H * W * C * 2, hipMemcpyDeviceToDevice, st)
                             : hipMemsetAsync(dx, 0, (size_t)N * H * W * C * 2, st);
    if (e != hipSuccess) return -5;
  }
  for (int ph = 0; ph < 2; ++ph)
    for (int pw = 0; pw < 2; ++pw) {
      ConvArgs c = a;
      c.TA = (H - ph + 1) / 2;
      c.TB = (W - pw + 1) / 2;
      if (c.TA <= 0 || c.TB <= 0) continue;
      c.M = (long long)N * c.TA * c.TB;
      c.ost = 2;
      c.oph = ph;
      c.opw = pw;
      c.ident = 0;
      c.ntaps = 0;
      for (int r = 0; r < R; ++r)
        for (int s = 0; s < S; ++s) {
          if (((ph + pad - r) & 1) || ((pw + pad - s) & 1)) continue;
          c.dh[c.ntaps] = (ph + pad - r) / 2;
          c.dw[c.ntaps] = (pw + pad - s) / 2;
          c.bcol[c.ntaps] = (r * S + s) * Kout;
          ++c.ntaps;
        }
      if (c.ntaps == 0) continue;
      int rows = 0;
      const int rc = run_igemm(c, st, &rows);
      if (rc) return rc;
      a.tile_off += (int)((c.M + rows - 1) / rows);  // the next class's BatchNorm partial rows
    }
  return 0;
}

// split count of conv_wgrad: ≈ 2 workgroups per CU over the output tiles, ≥ 8
// 64-token k-steps per slice, ≤ 256 slices (the fold reads splits × outputs fp32)
static void wgrad_cfg(int Kout, int C, int T, long long M, int* bmw, int* bnw, int* splits) {
  *bmw = Kout % 128 == 0 ? 128 : 64;
  *bnw = C % 128 == 0 ? 128 : 64;
  const long long tiles = (long long)(Kout / *bmw) * (T * C / *bnw);
  const long long ks = (M + 63) / 64;
  long long sp = (512 + tiles - 1) / tiles;
  if (sp > ks / 8) sp = ks / 8;
  if (sp > 256) sp = 256;  // one or two output tiles (64-channel 1×1 at 56×56): still ≥ 256 workgroups
  if (sp < 1) sp = 1;
  *splits = (int)sp;
}

// split fold of the weight-gradient partials ([splits][rows][ldp] fp32, rows × cols outputs)
static void wgrad_fold(const float* part, int splits, int rows, int cols, int ldp, float* dw, int accumulate,
                       hipStream_t st) {
  const long long n4 = (long long)rows * cols / 4, pn4 = (long long)rows * ldp / 4;
  const int c4 = cols / 4, l4 = ldp / 4;
  if (splits >= 16 && n4 < 1024LL * 64)
    conv_wgrad_reduce_kernel<16><<<(unsigned)((n4 + 15) / 16), 256, 0, st>>>(part, splits, n4, dw, accumulate, c4, l4, pn4);
  else if (splits >= 4)
    conv_wgrad_reduce_kernel<4><<<(unsigned)((n4 + 63) / 64), 256, 0, st>>>(part, splits, n4, dw, accumulate, c4, l4, pn4);
  else
    conv_wgrad_reduce_kernel<1><<<(unsigned)((n4 + 255) / 256), 256, 0, st>>>(part, splits, n4, dw, accumulate, c4, l4, pn4);
}

// the weight gradient on gemm_dw4's 256 × 256 mainloop (B gathered per tap) where
// its contract holds: ≥ 128 output channels, R·S·C % 256 = 0 (conv_wgrad_mode(0):
// off, for the probes and tests)
static int g_wgrad_dw4 = 1;
static int wgrad_dw4_splits(int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad) {
  // (R·S·C) % 128: at most half of the last 256-column tile is padding.  A 1×1
  // stride-1 product with half-height or half-padded tiles stays on the 128 × 128
  // kernel (measured faster there: profiles/r4i_conv_probe.jsonl)
  if (!g_wgrad_dw4 || Kout % 128 || (R * S * C) % 128 || C % 8) return 0;
  if (R == 1 && stride == 1 && (Kout % 256 || C % 256)) return 0;
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const long long M = (long long)N * Ho * Wo;
  if (M % 128 || M >= (1LL << 31) || (long long)N * H * W * C * 2 >= (1LL << 31)) return 0;
  const int sp = conv_wgrad_dw4_splits(Kout, R * S * C, M);
  return (M / 128) / sp >= 2 ? sp : 0;
}

int conv_wgrad_mode(int mode) {
  const int prev = g_wgrad_dw4;
  if (mode >= 0) g_wgrad_dw4 = mode;
  return prev;
}

// the tap-group 3×3 kernels for 64 / 128 channels (ahead of the per-tap / dw4
// kernels on every such shape: profiles/r4i_conv_probe.jsonl); conv_wgrad_c64_mode(0)
// selects those for the probes and tests
static int g_wgrad_c64 = 1;
// splits of the tap-group kernel (grid = splits × tap groups ≈ one workgroup per CU); 0: not taken
static int wgrad_c64_splits(int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad) {
  if (!g_wgrad_c64 || C != Kout || (C != 64 && C != 128) || R != 3 || S != 3 || pad != 1) return 0;
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  const long long ks = ((long long)N * Ho * Wo + 63) / 64;
  long long sp = C == 64 ? 256 : 85;  // 9 / NT tap groups per split
  if (sp > ks / 4) sp = ks / 4;
  return sp < 1 ? 1 : (int)sp;
}

int conv_wgrad_c64_mode(int mode) {
  const int prev = g_wgrad_c64;
  if (mode >= 0) g_wgrad_c64 = mode;
  return prev;
}

long long conv_wgrad_scratch_floats(int N, int H, int W, int C, int Kout, int R, int S, int stride, int pad) {
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  if (const int sp64 = wgrad_c64_splits(N, H, W, C, Kout, R, S, stride, pad)) return (long long)sp64 * C * 9 * C;
  const int sp4 = wgrad_dw4_splits(N, H, W, C, Kout, R, S, stride, pad);
  if (sp4) return (long long)sp4 * Kout * ((R * S * C + 255) / 256 * 256);
  int bm, bn, sp;
  wgrad_cfg(Kout, C, R * S, (long long)N * Ho * Wo, &bm, &bn, &sp);
  return (long long)sp * Kout * R * S * C;
}

// dw [Kout][R][S][C] fp32 (+)= Σ_t dy[t] ⊗ x[pixel(t, tap)]; scratch: conv_wgrad_scratch_floats
int conv_wgrad_nhwc(const bf16* dy, const bf16* x, int N, int H, int W, int C, int Kout, int R, int S, int stride,
                    int pad, float* dw, int accumulate, float* scratch, hipStream_t st) {
  if (!conv_supported(N, H, W, C, Kout, R, S, stride, pad)) return -2;
  if (const int sp64 = wgrad_c64_splits(N, H, W, C, Kout, R, S, stride, pad)) {
    WgradTapsArgs g{};
    const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
    g.dy = dy;
    g.x = x;
    g.part = scratch;
    g.M = (long long)N * Ho * Wo;
    g.IH = H;
    g.IW = W;
    g.TA = Ho;
    g.TB = Wo;
    g.inv_TA = 1.f / (float)Ho;
    g.inv_TB = 1.f / (float)Wo;
    g.st = stride;
    g.pad = pad;
    g.xbytes = (unsigned)((long long)N * H * W * C * 2);
    g.dybytes = (unsigned)(g.M * C * 2);
    g.splits = sp64;
    g.ksteps = (int)((g.M + 63) / 64);
    if (C == 64) conv_wgrad_taps_kernel<64, 9, false><<<(unsigned)sp64, CNT, 0, st>>>(g);
    else conv_wgrad_taps_kernel<128, 3, false><<<(unsigned)(sp64 * 3), CNT, 0, st>>>(g);
    wgrad_fold(scratch, sp64, C, 9 * C, 9 * C, dw, accumulate, st);
    return 0;
  }
  const int sp4 = wgrad_dw4_splits(N, H, W, C, Kout, R, S, stride, pad);
  if (sp4) {
    const int rc = conv_wgrad_dw4(dy, x, N, H, W, C, Kout, R, S, stride, pad, scratch, sp4, st);
    if (rc) return rc;
    const int TC = R * S * C;
    wgrad_fold(scratch, sp4, Kout, TC, (TC + 255) / 256 * 256, dw, accumulate, st);
    return 0;
  }
  WgradArgs a{};
  const int Ho = (H + 2 * pad - R) / stride + 1, Wo = (W + 2 * pad - S) / stride + 1;
  a.dy = dy;
  a.x = x;
  a.part = scratch;
  a.M = (long long)N * Ho * Wo;
  a.Kout = Kout;
  a.C = C;
  a.T = R * S;
  a.S = S;
  a.IH = H;
  a.IW = W;
  a.TA = Ho;
  a.TB = Wo;
  a.inv_TA = 1.f / (float)Ho;
  a.inv_TB = 1.f / (float)Wo;
  a.st = stride;
  a.pad = pad;
  a.xbytes = (unsigned)((long long)N * H * W * C * 2);
  a.dybytes = (unsigned)(a.M * Kout * 2);
  a.ksteps = (int)((a.M + 63) / 64);
  int bm, bn;
  wgrad_cfg(Kout, C, a.T, a.M, &bm, &bn, &a.splits);
  const long long grid = (long long)(Kout / bm) * (a.T * C / bn) * a.splits;
  if (grid > 0x7fffffffLL) return -2;
  if (bm == 128 && bn == 128) conv_wgrad_kernel<128, 128><<<(unsigned)grid, CNT, 0, st>>>(a);
  else if (bm == 128) conv_wgrad_kernel<128, 64><<<(unsigned)grid, CNT, 0, st>>>(a);
  else if (bn == 128) conv_wgrad_kernel<64, 128><<<(unsigned)grid, CNT, 0, st>>>(a);
  else conv_wgrad_kernel<64, 64><<<(unsigned)grid, CNT, 0, st>>>(a);
  wgrad_fold(scratch, a.splits, Kout, a.T * C, a.T * C, dw, accumulate, st);
  return 0;
}

// dx[n][2a][2b][:] += add[n][a][b][:] — the input gradient of a 1×1 stride-2
// convolution (ResNet's downsample branch) joining the forking convolution's dX
// at the pixels it reaches: the downsample's dX stays compact ([N][Ho][Wo][C],
// a plain GEMM), no zero-filled full-resolution tensor is written or re-read
namespace {
__global__ __launch_bounds__(256) void stride2_add_kernel(bf16* __restrict__ dx, const bf16* __restrict__ add, int H,
                                                         int W, int Ho, int Wo, int C8, long long total) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c8 = (int)(i % C8);
    const long long t = i / C8;
    const int b = (int)(t % Wo);
    const long long t2 = t / Wo;
    const int a = (int)(t2 % Ho);
    const long long n = t2 / Ho;
    bf16x8* d = reinterpret_cast<bf16x8*>(dx) + ((n * H + 2 * a) * W + 2 * b) * C8 + c8;
    *d = to_bf16(to_f32(*d) + to_f32(reinterpret_cast<const bf16x8*>(add)[i]));
  }
}
}  // namespace

int conv_stride2_add(bf16* dx, const bf16* add, int N, int H, int W, int C, hipStream_t st) {
  if (C % 8) return -2;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long long total = (long long)N * Ho * Wo * (C / 8);
  stride2_add_kernel<<<stream_grid(total, 256), 256, 0, st>>>(dx, add, H, W, Ho, Wo, C / 8, total);
  return 0;
}

// ============================================================================
// ResNet stem: y = conv7×7/2(x, w), pad 3, C = 3 → 64 channels.  With
// z[n][i][j][(2p + q)·3 + c] = x[n][2i + p][2j + q][c] (channels 12-15 zero) and
// the weight padded to 8 × 8 at the top / left (w8[r + 1][s + 1] = w[r][s]),
//   y[oh][ow] = Σ_{a,b<4} Σ_{p,q,c} z[oh − 2 + a][ow − 2 + b][(2p + q)·3 + c] · w8[2a + p][2b + q][c]
// — a 4×4 stride-1 convolution over a 16-channel image (pad 2 before, 1 after):
// K = 4 kernel rows × (4 pixels × 16 channels) = 256, every tap row one 128-B
// chunk of z, so the implicit GEMM (forward, BatchNorm statistics in the
// epilogue) and the tap-group weight gradient run it with no 3-channel gathers
// (MIOpen's igemm fwd / wrw solvers did, at ≈ 360 µs each for batch 256).
namespace {

// one z pixel (32 B) per thread from the two 12-B pixel pairs of x (4-B aligned: W even)
__global__ __launch_bounds__(256) void stem_s2d_kernel(const bf16* __restrict__ x, bf16* __restrict__ z, int H, int W,
                                                      long long npix) {
  const int IW = W >> 1, IH = H >> 1;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < npix; i += (long long)gridDim.x * 256) {
    const int j = (int)(i % IW);
    const long long ni = i / IW;
    const int ii = (int)(ni % IH);
    const long long n = ni / IH;
    const unsigned* r0 = reinterpret_cast<const unsigned*>(x + ((n * H + 2 * ii) * W + 2 * j) * 3);
    const unsigned* r1 = r0 + (W * 3) / 2;
    uint4 lo = {r0[0], r0[1], r0[2], r1[0]};
    uint4 hi = {r1[1], r1[2], 0u, 0u};
    uint4* o = reinterpret_cast<uint4*>(z + i * 16);
    o[0] = lo;
    o[1] = hi;
  }
}

// w [Kout][7][7][3] (OHWI) → w2 [Kout][4 a][4 b][16 ch] (bf16)
__global__ __launch_bounds__(256) void stem_weight_kernel(const bf16* __restrict__ w, bf16* __restrict__ w2, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int co = i >> 8, k = i & 255, aa = k >> 6, b = (k >> 4) & 3, ch = k & 15;
  bf16 v = (bf16)0.f;
  if (ch < 12) {
    const int pq = ch / 3, c = ch - 3 * pq;
    const int r = 2 * aa + (pq >> 1) - 1, s = 2 * b + (pq & 1) - 1;
    if (r >= 0 && s >= 0) v = w[((co * 7 + r) * 7 + s) * 3 + c];
  }
  w2[i] = v;
}

// dw [Kout][7][7][3] fp32 (+)= the stem entries of dw2 [Kout][256]
__global__ __launch_bounds__(256) void stem_dw_kernel(const float* __restrict__ dw2, float* __restrict__ dw, int n,
                                                     int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = i % 3, rs = (i / 3) % 49, co = i / 147, r = rs / 7, s = rs - 7 * r;
  const int aa = (r + 1) >> 1, p = (r + 1) & 1, b = (s + 1) >> 1, q = (s + 1) & 1;
  const float v = dw2[co * 256 + aa * 64 + b * 16 + (2 * p + q) * 3 + c];
  dw[i] = accumulate ? dw[i] + v : v;
}

// split count of the stem weight gradient: two workgroups per CU, ≥ 8 k-steps each
int stem_splits(long long M) {
  const long long ks = (M + 63) / 64;
  long long sp = 512;
  if (sp > ks / 8) sp = ks / 8;
  return sp < 1 ? 1 : (int)sp;
}

}  // namespace

int stem_supported(int N, int H, int W, int C, int Kout) {
  if (C != 3 || Kout != 64 || (H & 1) || (W & 1) || H < 8 || W < 8) return 0;
  const long long M = (long long)N * (H / 2) * (W / 2);
  return M < (1 << 24) && M * 16 * 2 < (1ll << 31) && M * Kout * 2 < (1ll << 31);
}

int stem_s2d(const bf16* x, int N, int H, int W, bf16* z, hipStream_t st) {
  if (!stem_supported(N, H, W, 3, 64)) return -2;
  const long long npix = (long long)N * (H / 2) * (W / 2);
  stem_s2d_kernel<<<stream_grid(npix, 256), 256, 0, st>>>(x, z, H, W, npix);
  return 0;
}

int stem_weight(const bf16* w, bf16* w2, int Kout, hipStream_t st) {
  const int n = Kout * 256;
  stem_weight_kernel<<<(n + 255) / 256, 256, 0, st>>>(w, w2, n);
  return 0;
}

int stem_fwd(const bf16* z, int N, int IH, int IW, const bf16* w2, int Kout, bf16* y, float* tile_stats,
             hipStream_t st) {
  if (!stem_supported(N, 2 * IH, 2 * IW, 3, Kout)) return -2;
  ConvArgs a{};
  a.x = z;
  a.w = w2;
  a.y = y;
  a.stats = tile_stats;
  a.M = (long long)N * IH * IW;
  a.C = 16;
  a.Kout = Kout;
  a.ldb = 256;
  a.IH = IH;
  a.IW = IW;
  a.TA = IH;
  a.TB = IW;
  a.ist = 1;
  a.ipad = 2;
  a.OH = IH;
  a.OW = IW;
  a.ost = 1;
  a.ident = 1;
  a.xbytes = (unsigned)((long long)N * IH * IW * 16 * 2);
  a.ntaps = 4;
  for (int t = 0; t < 4; ++t) {
    a.dh[t] = t;
    a.dw[t] = 0;
    a.bcol[t] = t * 64;
  }
  return run_igemm(a, st, nullptr);
}

int stem_tile_rows() { return conv_fwd_tile_rows(64); }
int stem_fwd_tiles(long long M) { return conv_fwd_tiles(M, 64); }

long long stem_wgrad_scratch_floats(int N, int IH, int IW, int Kout) {
  return (long long)(stem_splits((long long)N * IH * IW) + 1) * Kout * 256;
}

// dw [Kout][7][7][3] fp32 (+)= the stem's weight gradient from dy [N][IH][IW][Kout] and z
int stem_wgrad(const bf16* dy, const bf16* z, int N, int IH, int IW, int Kout, float* dw, int accumulate,
               float* scratch, hipStream_t st) {
  if (!stem_supported(N, 2 * IH, 2 * IW, 3, Kout)) return -2;
  WgradTapsArgs g{};
  g.dy = dy;
  g.x = z;
  g.part = scratch;
  g.M = (long long)N * IH * IW;
  g.IH = IH;
  g.IW = IW;
  g.TA = IH;
  g.TB = IW;
  g.inv_TA = 1.f / (float)IH;
  g.inv_TB = 1.f / (float)IW;
  g.st = 1;
  g.pad = 2;
  g.xbytes = (unsigned)(g.M * 16 * 2);
  g.dybytes = (unsigned)(g.M * Kout * 2);
  g.splits = stem_splits(g.M);
  g.ksteps = (int)((g.M + 63) / 64);
  conv_wgrad_taps_kernel<64, 4, true><<<(unsigned)g.splits, CNT, 0, st>>>(g);
  float* dw2 = scratch + (size_t)g.splits * Kout * 256;
  wgrad_fold(scratch, g.splits, Kout, 256, 256, dw2, 0, st);
  const int n = Kout * 147;
  stem_dw_kernel<<<(n + 255) / 256, 256, 0, st>>>(dw2, dw, n, accumulate);
  return 0;
}

}  // namespace pdo
