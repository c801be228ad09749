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

__global__ __launch_bounds__(256) void maxpool3s2_fwd_kernel(const bf16* __restrict__ x, int N, int H, int W, int C,
                                                             int OH, int OW, bf16* __restrict__ y,
                                                             uint8_t* __restrict__ arg) {
  const int C8 = C / 8;
  const long long total = (long long)N * OH * OW * C8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c8 = (int)(i % C8);
    long long t = i / C8;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int n = (int)(t / OH);
    f32x8 best;
    u8x8 pos;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      pos[j] = 0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = oh * 2 - 1 + kh;
      if (h < 0 || h >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = ow * 2 - 1 + kw;
        if (w < 0 || w >= W) continue;
        const f32x8 v = to_f32(*reinterpret_cast<const bf16x8*>(x + (((long long)n * H + h) * W + w) * C + c8 * 8));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (v[j] > best[j]) {  // first maximum in scan order wins ties
            best[j] = v[j];
            pos[j] = (uint8_t)(kh * 3 + kw);
          }
        }
      }
    }
    reinterpret_cast<bf16x8*>(y)[i] = to_bf16(best);
    reinterpret_cast<u8x8*>(arg)[i] = pos;
  }
}

__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const bf16* __restrict__ dy,
                                                             const uint8_t* __restrict__ arg, int N, int H, int W,
                                                             int C, int OH, int OW, bf16* __restrict__ dx) {
  const int C8 = C / 8;
  const long long total = (long long)N * H * W * C8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c8 = (int)(i % C8);
    long long t = i / C8;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    f32x8 acc = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows covering h: oh*2-1 <= h <= oh*2+1  ⇔  h/2 <= oh <= (h+1)/2
    const int oh1 = min((h + 1) / 2, OH - 1), ow1 = min((w + 1) / 2, OW - 1);
    for (int oh = h / 2; oh <= oh1; ++oh) {
      const int kh = h - (oh * 2 - 1);
      for (int ow = w / 2; ow <= ow1; ++ow) {
        const int kw = w - (ow * 2 - 1);
        const long long o = (((long long)n * OH + oh) * OW + ow) * C8 + c8;
        const u8x8 p = reinterpret_cast<const u8x8*>(arg)[o];
        const f32x8 g = to_f32(reinterpret_cast<const bf16x8*>(dy)[o]);
        const uint8_t me = (uint8_t)(kh * 3 + kw);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += p[j] == me ? g[j] : 0.f;
      }
    }
    reinterpret_cast<bf16x8*>(dx)[i] = to_bf16(acc);
  }
}

}  // namespace

int maxpool3s2_fwd(const bf16* x, int N, int H, int W, int C, bf16* y, uint8_t* arg, hipStream_t st) {
  if (C % 8 != 0) return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long long total = (long long)N * OH * OW * (C / 8);
  maxpool3s2_fwd_kernel<<<stream_grid(total, 256) * 2, 256, 0, st>>>(x, N, H, W, C, OH, OW, y, arg);
  return 0;
}

int maxpool3s2_bwd(const bf16* dy, const uint8_t* arg, int N, int H, int W, int C, bf16* dx, hipStream_t st) {
  if (C % 8 != 0) return -2;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long long total = (long long)N * H * W * (C / 8);
  maxpool3s2_bwd_kernel<<<stream_grid(total, 256) * 2, 256, 0, st>>>(dy, arg, N, H, W, C, OH, OW, dx);
  return 0;
}

}  // namespace pdo
