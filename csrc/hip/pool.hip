// SPDX-License-Identifier: Apache-2.0
// ResNet stem max-pool (3×3, stride 2, pad 1) for NHWC bf16, 8 channels per lane.
//
// Forward writes the pooled value and a uint8 window position (0..8) per
// output element.  Backward is a gather, not a scatter: each input pixel is
// covered by at most 2×2 windows, so every lane sums the ≤4 upstream
// gradients whose argmax is its own position — no atomics, no zero-fill, one
// coalesced write of dx (PyTorch's NHWC max_pool2d backward took 630 µs for
// the 256×64×112×112 stem on MI355X).
#include "common.h"
#include "kernels.h"

namespace pdo {

namespace {

typedef uint8_t u8x8 __attribute__((ext_vector_type(8)));

// one block per output row (n, oh); the row's (ow, channel chunk) pairs in 32-bit
// index math (64-bit divisions per element made the pass 2.5× slower than its bytes)
__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                             int OH, int OW, bf16* __restrict__ y,
                                                             uint8_t* __restrict__ arg) {
  const int C8 = C / 8;
  const int n = blockIdx.x / OH, oh = blockIdx.x - n * OH;
  const int per_row = OW * C8;
  const long long row0 = (long long)blockIdx.x * per_row;  // output vector index of (n, oh, 0, 0)
  const bf16* xn = x + (long long)n * H * W * C;
  for (int j = threadIdx.x; j < per_row; j += 256) {
    const int ow = j / C8, c8 = j - ow * C8;
    f32x8 best;
    u8x8 pos;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      best[q] = -INFINITY;
      pos[q] = 0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = oh * 2 - 1 + kh;
      if (h < 0 || h >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = ow * 2 - 1 + kw;
        if (w < 0 || w >= W) continue;
        const f32x8 v = to_f32(*reinterpret_cast<const bf16x8*>(xn + ((long long)h * W + w) * C + c8 * 8));
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if (v[q] > best[q]) {  // first maximum in scan order wins ties
            best[q] = v[q];
            pos[q] = (uint8_t)(kh * 3 + kw);
          }
        }
      }
    }
    reinterpret_cast<bf16x8*>(y)[row0 + j] = to_bf16(best);
    reinterpret_cast<u8x8*>(arg)[row0 + j] = pos;
  }
}

// one block per input row (n, h), 32-bit index math within the row
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const bf16* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg, int N, int H, int W,
                                                             int C, int OH, int OW, bf16* __restrict__ dx) {
  const int C8 = C / 8;
  const int n = blockIdx.x / H, h = blockIdx.x - n * H;
  const int per_row = W * C8;
  const long long row0 = (long long)blockIdx.x * per_row;
  // windows covering h: oh*2-1 <= h <= oh*2+1  ⇔  h/2 <= oh <= (h+1)/2
  const int oh0 = h / 2, oh1 = min((h + 1) / 2, OH - 1);
  const long long on = (long long)n * OH;
  for (int j = threadIdx.x; j < per_row; j += 256) {
    const int w = j / C8, c8 = j - w * C8;
    f32x8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ow1 = min((w + 1) / 2, OW - 1);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = h - (oh * 2 - 1);
      for (int ow = w / 2; ow <= ow1; ++ow) {
        const int kw = w - (ow * 2 - 1);
        const long long o = ((on + oh) * OW + ow) * C8 + c8;
        const u8x8 p = reinterpret_cast<const u8x8*>(arg)[o];
        const f32x8 g = to_f32(reinterpret_cast<const bf16x8*>(dy)[o]);
        const uint8_t me = (uint8_t)(kh * 3 + kw);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += p[q] == me ? g[q] : 0.f;
      }
    }
    reinterpret_cast<bf16x8*>(dx)[row0 + j] = to_bf16(acc);
  }
}

// global average pool backward: dx[n][p][c] = dy[n][c] / HW for every pixel p of
// an NHWC activation — a pure 16-B-per-lane write stream (the framework's
// expand + channels_last copy of the broadcast gradient ran at ≈ 1.3 TB/s)
__global__ __launch_bounds__(256) void gap_bwd_kernel(const bf16* __restrict__ dy, long long n8, int HW, int C8,
                                                      float inv, bf16* __restrict__ dx) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    const long long n = i / ((long long)HW * C8);
    const int c8 = (int)(i % C8);
    const f32x8 g = to_f32(reinterpret_cast<const bf16x8*>(dy)[n * C8 + c8]) * inv;
    reinterpret_cast<bf16x8*>(dx)[i] = to_bf16(g);
  }
}

}  // namespace

int gap_bwd(const bf16* dy, int N, int HW, int C, bf16* dx, hipStream_t st) {
  if (C % 8 != 0 || N < 1 || HW < 1) return -2;
  const long long n8 = (long long)N * HW * (C / 8);
  gap_bwd_kernel<<<stream_grid(n8, 256), 256, 0, st>>>(dy, n8, HW, C / 8, 1.f / (float)HW, dx);
  return 0;
}

int maxpool3s2_fwd(const bf16* x, int N, int H, int W, int C, bf16* y, uint8_t* arg, hipStream_t st) {
  if (C % 8 != 0) return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if ((long long)N * OH > 0x7fffffffLL || (long long)OW * (C / 8) > (1 << 24)) return -2;
  maxpool3s2_fwd_kernel<<<(unsigned)(N * OH), 256, 0, st>>>(x, N, H, W, C, OH, OW, y, arg);
  return 0;
}

int maxpool3s2_bwd(const bf16* dy, const uint8_t* arg, int N, int H, int W, int C, bf16* dx, hipStream_t st) {
  if (C % 8 != 0) return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  if ((long long)N * H > 0x7fffffffLL || (long long)W * (C / 8) > (1 << 24)) return -2;
  maxpool3s2_bwd_kernel<<<(unsigned)(N * H), 256, 0, st>>>(dy, arg, N, H, W, C, OH, OW, dx);
  return 0;
}

}  // namespace pdo
