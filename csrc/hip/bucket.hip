// SPDX-License-Identifier: Apache-2.0
// Multi-tensor bucket kernels for the RCCL data-parallel path (gfx950).
// The flat-arena DDP needs no copies for its own gradients; these kernels
// serve everything else that must travel through a bucket (parameter
// broadcast of non-arena modules, PS pushes, checkpoint packing):
//   flatten_scale: dst[off_i : off_i + n_i] = scale * src_i  (one launch for N tensors)
//   unflatten:     dst_i = src[off_i : off_i + n_i]
// Work split: one 2048-element span of the flat buffer per workgroup; the
// owning tensor is found by binary search over the (device-resident) offsets.
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

template <bool FLATTEN>
__global__ __launch_bounds__(256) void bucket_kernel(const Meta* __restrict__ meta, int n, bf16* __restrict__ flat,
                                                     long long total, float scale) {
  const long long span0 = (long long)blockIdx.x * 2048;
  for (long long e = span0 + threadIdx.x; e < span0 + 2048 && e < total; e += 256) {
    const int i = find_tensor(meta, n, e);
    const long long k = e - meta[i].offset;
    if (k >= meta[i].size) continue;  // alignment padding between tensors
    bf16* t = reinterpret_cast<bf16*>(meta[i].ptr);
    if (FLATTEN) flat[e] = (bf16)((float)t[k] * scale);
    else t[k] = flat[e];
  }
}

__global__ __launch_bounds__(256) void scale_kernel(bf16* __restrict__ x, long long nvec, float s) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nvec; i += (long long)gridDim.x * 256) {
    bf16x8* p = reinterpret_cast<bf16x8*>(x) + i;
    *p = to_bf16(to_f32(*p) * s);
  }
}

static long long total_of(const long long* sizes, const long long* offsets, int n) {
  return n ? offsets[n - 1] + sizes[n - 1] : 0;
}

int flatten_scale(const void* const* srcs, const long long* sizes, const long long* offsets, int n, bf16* dst,
                  float scale, void* dev_meta, hipStream_t st) {
  (void)srcs;
  const long long total = total_of(sizes, offsets, n);
  if (total == 0) return 0;
  bucket_kernel<true><<<(unsigned)((total + 2047) / 2048), 256, 0, st>>>((const Meta*)dev_meta, n, dst, total, scale);
  return 0;
}

int unflatten(const bf16* src, void* const* dsts, const long long* sizes, const long long* offsets, int n,
              void* dev_meta, hipStream_t st) {
  (void)dsts;
  const long long total = total_of(sizes, offsets, n);
  if (total == 0) return 0;
  bucket_kernel<false><<<(unsigned)((total + 2047) / 2048), 256, 0, st>>>((const Meta*)dev_meta, n,
                                                                          const_cast<bf16*>(src), total, 1.f);
  return 0;
}

int scale_bf16(bf16* x, long long n, float s, hipStream_t st) {
  if (n % 8) return -2;
  scale_kernel<<<stream_grid(n / 8, 256), 256, 0, st>>>(x, n / 8, s);
  return 0;
}

}  // namespace pdo
