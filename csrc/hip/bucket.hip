// SPDX-License-Identifier: Apache-2.0
// Multi-tensor bucket kernels for the RCCL data-parallel path (gfx950).
//
// The flat-arena DDP needs no copies for its own gradients (a bucket is a
// slice of the arena).  These kernels serve what must still travel through a
// bucket:
//   flatten_scale: dst[off_i : off_i + n_i] = scale * src_i  (one launch for N tensors)
//   unflatten:     dst_i = src[off_i : off_i + n_i]
//     → one RCCL broadcast of all non-arena module buffers (BatchNorm running
//       statistics, workloads/resnet.py) instead of one collective per buffer;
//   cast_scale_bf16_f32: fp32 staging copy of a bf16 gradient bucket with the
//     1/world average folded in (parallel/ddp.py grad_reduce="fp32": the
//     all-reduce then accumulates in fp32 on the wire);
//   (the averaged fp32 gradients go back into the bf16 arena with
//   embed.hip's cast_f32_bf16).
// Work split of the multi-tensor kernels: one 2048-element span of the flat
// buffer per workgroup; the owning tensor is found by binary search over the
// (device-resident) offsets.  Cast kernels move 16 B of bf16 per lane.
#include "common.h"
#include "kernels.h"

namespace pdo {

struct Meta {
  long long ptr, size, offset;
};

__device__ __forceinline__ int find_tensor(const Meta* meta, int n, long long e) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (meta[mid].offset <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

template <typename T, bool FLATTEN>
__global__ __launch_bounds__(256) void bucket_kernel(const Meta* __restrict__ meta, int n, T* __restrict__ flat,
                                                     long long total, float scale) {
  const long long span0 = (long long)blockIdx.x * 2048;
  for (long long e = span0 + threadIdx.x; e < span0 + 2048 && e < total; e += 256) {
    const int i = find_tensor(meta, n, e);
    const long long k = e - meta[i].offset;
    if (k >= meta[i].size) continue;  // alignment padding between tensors
    T* t = reinterpret_cast<T*>(meta[i].ptr);
    if (FLATTEN) flat[e] = (T)((float)t[k] * scale);
    else t[k] = flat[e];
  }
}

__global__ __launch_bounds__(256) void scale_kernel(bf16* __restrict__ x, long long nvec, float s) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    bf16x8* p = reinterpret_cast<bf16x8*>(x) + i;
    *p = to_bf16(to_f32(*p) * s);
  }
}

__global__ __launch_bounds__(256) void cast_scale_bf16_f32_kernel(const bf16* __restrict__ src,
                                                                  float* __restrict__ dst, long long nvec, float s) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    const f32x8 v = to_f32(reinterpret_cast<const bf16x8*>(src)[i]) * s;
    f32x4* d = reinterpret_cast<f32x4*>(dst) + 2 * i;
    d[0] = f32x4{v[0], v[1], v[2], v[3]};
    d[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// x *= *s (an fp32 device scalar: the loss gradient, no host sync), fp32 math
__global__ __launch_bounds__(256) void scale_dev_kernel(bf16* __restrict__ x, long long nvec, const float* __restrict__ s) {
  const float f = *s;
  if (f == 1.f) return;  // bf16(f32(x) · 1) = x: the LM head's dloss of a plain loss.backward()
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    bf16x8* p = reinterpret_cast<bf16x8*>(x) + i;
    *p = to_bf16(to_f32(*p) * f);
  }
}

// g += h; h = 0 (a split parameter's head-gradient slot folded into its
// gradient after the all-reduce drain, parallel/flat.py fold_split)
__global__ __launch_bounds__(256) void fold_zero_kernel(bf16* __restrict__ g, bf16* __restrict__ h, long long nvec) {
  const bf16x8 z = to_bf16(f32x8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f});
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    bf16x8* pg = reinterpret_cast<bf16x8*>(g) + i;
    bf16x8* ph = reinterpret_cast<bf16x8*>(h) + i;
    *pg = to_bf16(to_f32(*pg) + to_f32(*ph));
    *ph = z;
  }
}

// y += *s · x in fp32, one rounding (a private gradient added into the arena,
// scaled by the loss gradient read on device)
__global__ __launch_bounds__(256) void axpy_dev_kernel(bf16* __restrict__ y, const bf16* __restrict__ x,
                                                       long long nvec, const float* __restrict__ s) {
  const float f = *s;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    bf16x8* py = reinterpret_cast<bf16x8*>(y) + i;
    const f32x8 xv = to_f32(reinterpret_cast<const bf16x8*>(x)[i]);
    f32x8 yv = to_f32(*py);
#pragma unroll
    for (int k = 0; k < 8; ++k) yv[k] = __builtin_fmaf(xv[k], f, yv[k]);
    *py = to_bf16(yv);
  }
}

int axpy_dev_bf16(bf16* y, const bf16* x, long long n, const float* s, hipStream_t st) {
  if (n % 8) return -2;
  if (n == 0) return 0;
  axpy_dev_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(y, x, n / 8, s);
  return 0;
}

int scale_dev_bf16(bf16* x, long long n, const float* s, hipStream_t st) {
  if (n % 8) return -2;
  if (n == 0) return 0;
  scale_dev_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(x, n / 8, s);
  return 0;
}

int fold_zero_bf16(bf16* g, bf16* h, long long n, hipStream_t st) {
  if (n % 8) return -2;
  if (n == 0) return 0;
  fold_zero_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(g, h, n / 8);
  return 0;
}

template <typename T>
static int multi_tensor(bool flatten, T* flat, long long total, int n, void* dev_meta, float scale, hipStream_t st) {
  if (total <= 0 || n <= 0) return 0;
  const unsigned grid = (unsigned)((total + 2047) / 2048);
  if (flatten) bucket_kernel<T, true><<<grid, 256, 0, st>>>((const Meta*)dev_meta, n, flat, total, scale);
  else bucket_kernel<T, false><<<grid, 256, 0, st>>>((const Meta*)dev_meta, n, flat, total, 1.f);
  return 0;
}

int bucket_copy(int dtype, bool flatten, void* flat, long long total, int n, void* dev_meta, float scale,
                hipStream_t st) {
  switch (dtype) {
    case 0: return multi_tensor<bf16>(flatten, (bf16*)flat, total, n, dev_meta, scale, st);
    case 1: return multi_tensor<float>(flatten, (float*)flat, total, n, dev_meta, scale, st);
    default: return -3;
  }
}

int scale_bf16(bf16* x, long long n, float s, hipStream_t st) {
  if (n % 8) return -2;
  scale_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(x, n / 8, s);
  return 0;
}

int cast_scale_bf16_f32(const bf16* src, float* dst, long long n, float s, hipStream_t st) {
  if (n % 8) return -2;
  if (n == 0) return 0;
  cast_scale_bf16_f32_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(src, dst, n / 8, s);
  return 0;
}

}  // namespace pdo
