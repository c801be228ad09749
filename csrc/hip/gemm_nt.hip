// SPDX-License-Identifier: Apache-2.0
// Forward-layout GEMM C[M][N] = A[M][K] · B[N][K]ᵀ (bf16 in, fp32 acc) for
// gfx950 with fused epilogues — the transformer's projections (A = tokens ×
// features, B = weight [out][in]) and their input gradients (B = Wᵀ).
//
// Both operands are K-contiguous, so every MFMA fragment is a plain 16-B row
// read.  The tile machinery is gemm_dw.hip's: 256 × 256 × 64 per workgroup,
// 8 waves as 2 (M) × 4 (N), LDS-DMA staging (global_load_lds_dwordx4, the
// XOR swizzle applied to the source address), two LDS stages = 128 KiB, and
// the two waves of each SIMD ping-ponging between an MFMA phase and an
// LDS-read phase.  LDS rows are 128 B ([256][64] bf16) with attention's
// swizzle (chunk ^ swz(row)): the 16 rows a ds_read_b128 lane group touches
// land on 16 distinct bank slots.
//
// The MFMA runs with the operands swapped, D = W·Xᵀ, so an accumulator holds
// 4 consecutive output features of one token per register group (8-B LDS
// writes); the tile then leaves through LDS as whole rows, where the
// per-feature terms (GELU, GELU', bias gradient) apply to 16-B vectors with
// coalesced loads of the saved pre-activation.  Epilogues:
//   EPI_PLAIN  C = A·Bᵀ
//   EPI_BIAS   C = A·Bᵀ + bias
//   EPI_GELU   C = A·Bᵀ (the pre-activation, saved for backward) and
//              Y = gelu(C + bias) — the fc1 forward with the bias-GELU pass fused
//   EPI_DGELU  C = (A·Bᵀ) ⊙ gelu'(X + bias), X = the saved pre-activation (read
//              through Y), and fp32 column partial sums of C for the bias
//              gradient (one row per (M-tile, wave)) — the fc2 input-gradient
//              GEMM with the bias-GELU backward pass fused
//   EPI_ADD    C = A·Bᵀ + Y (EPI 5: + bias too — a projection writing the residual
//              stream x + proj(a) + b) — or an input gradient that joins another branch's
//              (ResNet's block input: conv1 dX + the identity / downsample dX);
//              EPI 6: + Y ⊙ keep bits (a ReLU mask)
//   EPI 7 / 8  (4-wave mainloop only) the GELU pair with the derivative saved:
//              fc1 writes C = gelu'(A·Bᵀ + bias), Y = gelu(A·Bᵀ + bias); fc2's
//              input gradient is then C = (A·Bᵀ) ⊙ Y plus the bias-gradient
//              partials — one multiply per element instead of the derivative
//   EPI 9      C = A·Bᵀ and the BatchNorm statistics of the bf16 outputs per
//              row group: [groups][2][N] (Σ, Σ(x − x̄)²), gemm_nt_stats_rows
//              rows each, merged by batchnorm.hip bn_fwd_tiles — a 1×1
//              convolution's forward without a statistics pass over its output
// Rounding matches the unfused path bit for bit: the GEMM result is rounded to
// bf16 before the activation math, as when it made an HBM round trip.
#include <stdlib.h>

#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int STAGES = 5;  // 5 × 32 KiB = the whole 160 KiB LDS
constexpr int TILE = 256 * BK;  // elements of one operand tile [256 rows][32]
constexpr int NTHR = 512;

// 16-B chunk swizzle of a 64-B LDS row: a ds_read_b128 lane group reads the
// 4 chunks of 4 rows ({0-3,12-15,20-27}-style groups); chunk ^= (r>>1)&3 puts
// every group's 16 (row & 3, chunk) pairs on 16 distinct bank slots
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 3; }

template <int EPI>
__global__ __launch_bounds__(NTHR) void gemm_nt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                       int lda, int ldb, int M, int N, int nk, bf16* __restrict__ C,
                                                       int ldc, const bf16* __restrict__ bias, bf16* __restrict__ Y,
                                                       int ldy, float* __restrict__ dbias_part) {
  __shared__ __attribute__((aligned(16))) bf16 smem[STAGES * 2 * TILE];  // [stage][A|B][256][32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int li = lane & 31, hh = lane >> 5;
  const int tiles_n = N / BN;
  const int nwg = (M / BM) * tiles_n;
  // XCD remap (gemm_dw.hip): each XCD gets a contiguous range of logical ids,
  // i.e. the N-tiles of a few A row panels, which then share its L2
  int id = blockIdx.x;
  {
    const int xcd = id & 7, slot = id >> 3, q = nwg >> 3, r = nwg & 7;
    id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
  }
  const int tn = id % tiles_n, tm = id / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // LDS-DMA: one wave-instruction fills 1 KiB = 16 rows of 64 B; lane l →
  // row 16·(2w+i) + (l>>2), LDS chunk l&3, holding global chunk (l&3) ^ swz(row)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const bf16* srcA[2];
  const bf16* srcB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 16 * (2 * w + i) + (lane >> 2);
    const int ch = (lane & 3) ^ swz(r);
    srcA[i] = A + (size_t)(m0 + r) * lda + ch * 8;
    srcB[i] = B + (size_t)(n0 + r) * ldb + ch * 8;
  }
  // 16x16x32 fragment: lane reads row rbase + (l&15), chunk l>>4 (the whole
  // 32-k row); swz depends on row bits 1-2 only, so rbase (% 16) is a ds_read
  // immediate and every fragment of an operand shares one per-lane offset
  const int fo = (lane & 15) * BK + (((lane >> 4) ^ swz(lane & 15)) << 3);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) bf16*)smem;
  auto glds = [](const bf16* src, unsigned lds_byte) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(lds_byte)
                 : "memory");
  };
  // one 32-k stage = 4 DMA wave-instructions per wave (2 A + 2 B)
  auto load_stage = [&](int s) {
    const unsigned abase = lds0 + (unsigned)((s % STAGES) * 2 * TILE) * 2u, bbase = abase + TILE * 2u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const unsigned off = (unsigned)((2 * wu + i) * 1024);
      glds(srcA[i] + (size_t)s * BK, abase + off);
      glds(srcB[i] + (size_t)s * BK, bbase + off);
    }
  };
  // wait until this wave's DMA for stage `s` landed, given stages ≤ last issued
  auto wait_stage = [](int after) {  // after = stages issued after it (0..STAGES-2)
    static_assert(STAGES == 5, "wait_stage covers 0..3 stages in flight after the awaited one");
    if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // Ping-pong over a STAGES-deep ring of 32-k stages: waves 4-7 run one barrier
  // interval behind waves 0-3, so on every SIMD one wave issues its 32 MFMAs
  // while the other issues the next stage's 12 row reads.  Per stage s:
  // R (12 reads; DMA of stage s+STAGES-1 into the buffer of s-1, whose last reads
  // retired before the previous barrier; wait for this wave's DMA of stage
  // s+1; lgkmcnt(0)) | barrier | M (32 MFMAs) | barrier.  Stage s+1 is read
  // two barriers after every wave waited for its share of it.
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nk) load_stage(t);
  wait_stage(min(nk - 1, STAGES - 2));
  __builtin_amdgcn_s_barrier();
  const bool g1 = wu >= 4;
  if (g1) __builtin_amdgcn_s_barrier();
  for (int s = 0; s < nk; ++s) {
    const bf16* As = smem + (s % STAGES) * 2 * TILE + wm * 128 * BK + fo;
    const bf16* Bs = smem + (s % STAGES) * 2 * TILE + TILE + wn * 64 * BK + fo;
    bf16x8 xf[8], wf[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = *reinterpret_cast<const bf16x8*>(As + i * 16 * BK);
#pragma unroll
    for (int j = 0; j < 4; ++j) wf[j] = *reinterpret_cast<const bf16x8*>(Bs + j * 16 * BK);
    if (s + STAGES - 1 < nk) load_stage(s + STAGES - 1);
    if (s + 1 < nk) wait_stage(min(nk - 1, s + STAGES - 1) - (s + 1));
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
  }
  if (!g1) __builtin_amdgcn_s_barrier();  // balance the stagger

  // ---- epilogue ----
  // acc[i][j][e] = C[m][n], m = wm·128 + 16i + (l&15), n = wn·64 + 16j + 4(l>>4) + e
  // (tile-relative).  Stage the bf16 tile through LDS — [256][256] = 128 KiB,
  // the whole array, free once every wave passed the loop's last barrier — and
  // write it back as 512-B rows, 16 B per lane (the accumulator layout would
  // scatter 8-B pieces over 16 rows per instruction).  LDS image: 16-B chunk
  // c of row m at chunk c ^ (m & 31), so the 8-B writes (16 rows per lane
  // group) and the 16-B row reads are both conflict-free.
  __syncthreads();
  unsigned char* lds = reinterpret_cast<unsigned char*>(smem);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f32x4 bv = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == 1 || EPI == 5) {  // bias before the rounding, as a library bias epilogue
      const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(bias + n0 + wn * 64 + 16 * j + 4 * (lane >> 4));
      bv = f32x4{(float)b4[0], (float)b4[1], (float)b4[2], (float)b4[3]};
    }
    const int c = wn * 8 + 2 * j + (lane >> 5);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int m = wm * 128 + 16 * i + (lane & 15);
      const f32x4 a = acc[i][j] + bv;
      const bf16x4 o = {(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3]};
      *reinterpret_cast<bf16x4*>(lds + m * 512 + ((c ^ (m & 31)) << 4) + 8 * ((lane >> 4) & 1)) = o;
    }
  }
  __syncthreads();
  // row phase: thread t owns 16-B column chunk t & 31 of rows 16·it + (t >> 5)
  const int c = tid & 31, r0 = tid >> 5;
  const int n = n0 + 8 * c;
  f32x8 bv8;
  if constexpr (EPI == 2 || EPI == 3) bv8 = to_f32(*reinterpret_cast<const bf16x8*>(bias + n));
  f32x8 colp = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // EPI 9: statistics of this thread's 16 rows, shifted by its first row
  f32x8 x0 = colp, ssq = colp;
  if constexpr (EPI == 9) x0 = to_f32(*reinterpret_cast<const bf16x8*>(lds + r0 * 512 + ((c ^ (r0 & 31)) << 4)));
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int r = 16 * it + r0;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(lds + r * 512 + ((c ^ (r & 31)) << 4));
    const size_t m = (size_t)(m0 + r);
    if constexpr (EPI <= 1) {
      *reinterpret_cast<bf16x8*>(C + m * ldc + n) = v;
    } else if constexpr (EPI == 9) {
      *reinterpret_cast<bf16x8*>(C + m * ldc + n) = v;
      const f32x8 d = to_f32(v) - x0;
      colp += d;
      ssq += d * d;
    } else if constexpr (EPI == 2) {
      *reinterpret_cast<bf16x8*>(C + m * ldc + n) = v;
      const f32x8 x = to_f32(v) + bv8;
      f32x8 y;
#pragma unroll
      for (int e = 0; e < 8; ++e) y[e] = gelu_sig(x[e]);
      *reinterpret_cast<bf16x8*>(Y + m * ldy + n) = to_bf16(y);
    } else if constexpr (EPI == 4 || EPI == 5) {
      // the addend joins after the bf16 staging: two roundings (the 4-wave path has one)
      const f32x8 r = to_f32(*reinterpret_cast<const bf16x8*>(Y + m * ldy + n));
      *reinterpret_cast<bf16x8*>(C + m * ldc + n) = to_bf16(to_f32(v) + r);
    } else if constexpr (EPI == 6) {
      // the addend masked by its keep bits (8 columns per byte): a branch gradient's ReLU
      f32x8 r = to_f32(*reinterpret_cast<const bf16x8*>(Y + m * ldy + n));
      const unsigned bits = reinterpret_cast<const unsigned char*>(bias)[(m * ldy + n) >> 3];
#pragma unroll
      for (int q = 0; q < 8; ++q) r[q] = (bits >> q) & 1u ? r[q] : 0.f;
      *reinterpret_cast<bf16x8*>(C + m * ldc + n) = to_bf16(to_f32(v) + r);
    } else {
      const f32x8 x = to_f32(*reinterpret_cast<const bf16x8*>(Y + m * ldy + n)) + bv8;
      const f32x8 dy = to_f32(v);
      f32x8 d;
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = dy[e] * gelu_sig_grad(x[e]);
      colp += d;
      *reinterpret_cast<bf16x8*>(C + m * ldc + n) = to_bf16(d);
    }
  }
  if constexpr (EPI == 9) {
    // 16 rows per thread → lanes l, l + 32 (rows r0 = 2w, 2w + 1) → the 8 waves
    // through LDS (the staged tile is dead after this barrier): one 256-row
    // group per M-tile, partial row tm of [M/256][2][N]
    f32x8 sum = colp + 16.f * x0, m2 = ssq - colp * colp * (1.f / 16.f), s2, q2;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s2[k] = __shfl_xor(sum[k], 32, 64);
      q2[k] = __shfl_xor(m2[k], 32, 64);
    }
    chan_merge_equal(sum, m2, s2, q2, 16.f);
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);  // [8 waves][2][256]
    if (lane < 32) {
      *reinterpret_cast<f32x8*>(red + w * 512 + 8 * c) = sum;
      *reinterpret_cast<f32x8*>(red + w * 512 + 256 + 8 * c) = m2;
    }
    __syncthreads();
    if (tid < 256) {
      float s = red[tid], q = red[256 + tid];
#pragma unroll
      for (int k = 1; k < 8; ++k) {  // (32k rows) + (32 rows)
        const float sb = red[k * 512 + tid], qb = red[k * 512 + 256 + tid];
        const float d = sb * (1.f / 32.f) - s * (1.f / (32.f * k));
        q += qb + d * d * (32.f * k * 32.f / (32.f * (k + 1)));
        s += sb;
      }
      dbias_part[(size_t)tm * 2 * N + n0 + tid] = s;
      dbias_part[(size_t)tm * 2 * N + N + n0 + tid] = q;
    }
  }
  if constexpr (EPI == 3) {
    // lanes l and l+32 share a column chunk: one fp32 partial row per wave
#pragma unroll
    for (int e = 0; e < 8; ++e) colp[e] += __shfl_xor(colp[e], 32, 64);
    if (lane < 32) {
      float* prow = dbias_part + (size_t)(8 * tm + w) * N + n;
      *reinterpret_cast<f32x4*>(prow) = f32x4{colp[0], colp[1], colp[2], colp[3]};
      *reinterpret_cast<f32x4*>(prow + 4) = f32x4{colp[4], colp[5], colp[6], colp[7]};
    }
  }
}

}  // namespace

// impl 0 = the 8-wave ring below; impl 1 (default) = the 4-wave persistent
// mainloop (gemm_nt4.hip) wherever K allows it.  PDO_NT_IMPL overrides (A/B in
// the training step: tools/gpu.sh 'stepab:PDO_NT_IMPL=0 PDO_NT_IMPL=1')
static int g_impl = [] {
  const char* e = getenv("PDO_NT_IMPL");
  return e && *e ? atoi(e) : 1;
}();

// N % 256 = 128 (the 50304-column LM head) only on the 4-wave mainloop
static bool nt4_path(int K) { return g_impl >= 1 && K % 128 == 0 && K >= 256; }

int gemm_nt_ok(int M, int N, int K, int lda, int ldb, int ldc) {
  const bool nok = N % BN == 0 || (N % BN == BN / 2 && nt4_path(K));
  return M > 0 && N > 0 && K >= 64 && M % BM == 0 && nok && K % 64 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 4 == 0 && lda >= K && ldb >= K && ldc >= N;
}

// partial rows of the EPI 3 / 8 bias gradient: 8 per 256-row tile on the 8-wave
// ring, 2 on the 4-wave mainloop (its lane groups merge in-register)
int gemm_nt_dbias_rows(int M, int K) { return (nt4_path(K) ? 2 : 8) * (M / BM); }
int gemm_nt_epi_ok(int M, int N, int K) { return gemm_nt_ok(M, N, K, K, K, N) && nt4_path(K); }
// rows per BatchNorm partial of EPI 9: a (tile, wm) half on the 4-wave mainloop, the tile on the ring
int gemm_nt_stats_rows(int K) { return nt4_path(K) ? BM / 2 : BM; }
void gemm_nt_set_impl(int impl) { g_impl = impl; }

int gemm_nt_get_impl() { return g_impl; }

int gemm_nt(const bf16* A, const bf16* B, int M, int N, int K, int lda, int ldb, bf16* C, int ldc, int epi,
            const bf16* bias, bf16* Y, int ldy, float* dbias_part, hipStream_t st) {
  if (!gemm_nt_ok(M, N, K, lda, ldb, ldc)) return -2;
  if (((epi >= 1 && epi <= 3) || (epi >= 5 && epi <= 7)) && !bias) return -3;  // EPI 6: bias = the addend's keep mask
  if (epi == 6 && ldy % 8) return -3;
  if (epi >= 2 && epi != 9 && (!Y || ldy % 4 || ldy < N)) return -3;
  if ((epi == 3 || epi == 8 || epi == 9) && !dbias_part) return -3;
  if ((epi == 7 || epi == 8) && !nt4_path(K)) return -4;  // the saved-GELU' pair: 4-wave mainloop only
  if (nt4_path(K))
    return gemm_nt4(A, B, M, N, K, lda, ldb, C, ldc, epi, bias, Y, ldy, dbias_part, st);
  const long long grid = (long long)(M / BM) * (N / BN);
  if (grid > 0x7fffffffLL) return -2;
  const int nk = K / BK;
  switch (epi) {
    case 0: gemm_nt_kernel<0><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 1: gemm_nt_kernel<1><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 2: gemm_nt_kernel<2><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 3: gemm_nt_kernel<3><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 4: gemm_nt_kernel<4><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 5: gemm_nt_kernel<5><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 6: gemm_nt_kernel<6><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    case 9: gemm_nt_kernel<9><<<(int)grid, NTHR, 0, st>>>(A, B, lda, ldb, M, N, nk, C, ldc, bias, Y, ldy, dbias_part); break;
    default: return -4;
  }
  return 0;
}

}  // namespace pdo
