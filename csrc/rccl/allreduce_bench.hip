// SPDX-License-Identifier: Apache-2.0
// pdo-allreduce-bench: RCCL collective bandwidth sweep over xGMI.
//
// Sizes the DDP bucket policy (utils/topology.py bucket_bytes_for) from
// measurements instead of NVSwitch folklore: on an 8×MI355X node every GPU
// pair is one xGMI hop and a ring step moves each byte over ONE link, so the
// all-reduce bus bandwidth grows with message size until RCCL runs enough
// channels (rings) to occupy all 7 links per GPU.
//
// One process drives all visible GPUs (ncclCommInitAll, one HIP stream per
// GPU, group calls).  Per size: warm-up, then `iters` collectives timed with
// HIP events on every device (max over devices), reported as JSON lines:
//   {"op":"allreduce","bytes":…,"dtype":"bf16","ranks":8,"us":…,"algbw_gbs":…,"busbw_gbs":…}
// busbw = algbw × 2(n−1)/n (all-reduce), (n−1)/n (all-gather / reduce-scatter).
//
//   pdo-allreduce-bench [--op allreduce|allgather|reducescatter|broadcast]
//                       [--min 1M] [--max 1G] [--factor 2] [--iters 20] [--dtype bf16|f32] [--gpus N]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(x)                                                                           \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)
#define NCCLCHECK(x)                                                                          \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_));      \
      exit(1);                                                                                \
    }                                                                                         \
  } while (0)

static size_t parse_size(const char* s) {
  char* end = nullptr;
  double v = strtod(s, &end);
  switch (end && *end ? *end : ' ') {
    case 'K': case 'k': v *= 1024; break;
    case 'M': case 'm': v *= 1024 * 1024; break;
    case 'G': case 'g': v *= 1024.0 * 1024 * 1024; break;
    default: break;
  }
  return (size_t)v;
}

int main(int argc, char** argv) {
  std::string op = "allreduce", dtype = "bf16";
  size_t minb = 1 << 20, maxb = 1ull << 30;
  double factor = 2.0;
  int iters = 20, warm = 5, ngpu = -1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto nxt = [&]() -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--op") op = nxt();
    else if (a == "--min") minb = parse_size(nxt());
    else if (a == "--max") maxb = parse_size(nxt());
    else if (a == "--factor") factor = atof(nxt());
    else if (a == "--iters") iters = atoi(nxt());
    else if (a == "--warmup") warm = atoi(nxt());
    else if (a == "--dtype") dtype = nxt();
    else if (a == "--gpus") ngpu = atoi(nxt());
    else if (a == "-h" || a == "--help") {
      printf("pdo-allreduce-bench [--op allreduce|allgather|reducescatter|broadcast] [--min 1M] [--max 1G]\n"
             "                    [--factor 2] [--iters 20] [--warmup 5] [--dtype bf16|f32] [--gpus N]\n");
      return 0;
    } else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  if (ngpu < 0 || ngpu > ndev) ngpu = ndev;
  if (ngpu < 1) {
    fprintf(stderr, "no GPU\n");
    return 1;
  }
  const ncclDataType_t dt = dtype == "f32" ? ncclFloat32 : ncclBfloat16;
  const size_t esz = dtype == "f32" ? 4 : 2;
  std::vector<int> devs(ngpu);
  for (int i = 0; i < ngpu; ++i) devs[i] = i;
  std::vector<ncclComm_t> comms(ngpu);
  NCCLCHECK(ncclCommInitAll(comms.data(), ngpu, devs.data()));
  std::vector<hipStream_t> streams(ngpu);
  std::vector<void*> sbuf(ngpu), rbuf(ngpu);
  std::vector<hipEvent_t> e0(ngpu), e1(ngpu);
  const size_t alloc = maxb * (op == "allgather" ? 1 : 1);
  for (int i = 0; i < ngpu; ++i) {
    HIPCHECK(hipSetDevice(i));
    HIPCHECK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&sbuf[i], alloc));
    HIPCHECK(hipMalloc(&rbuf[i], alloc));
    HIPCHECK(hipMemset(sbuf[i], 0, alloc));
    HIPCHECK(hipEventCreate(&e0[i]));
    HIPCHECK(hipEventCreate(&e1[i]));
  }
  auto launch = [&](size_t bytes) {
    const size_t count = bytes / esz;
    NCCLCHECK(ncclGroupStart());
    for (int i = 0; i < ngpu; ++i) {
      if (op == "allreduce")
        NCCLCHECK(ncclAllReduce(sbuf[i], rbuf[i], count, dt, ncclSum, comms[i], streams[i]));
      else if (op == "allgather")  // `bytes` = the gathered (output) size
        NCCLCHECK(ncclAllGather(sbuf[i], rbuf[i], count / ngpu, dt, comms[i], streams[i]));
      else if (op == "reducescatter")  // `bytes` = the input size
        NCCLCHECK(ncclReduceScatter(sbuf[i], rbuf[i], count / ngpu, dt, ncclSum, comms[i], streams[i]));
      else
        NCCLCHECK(ncclBroadcast(sbuf[i], rbuf[i], count, dt, 0, comms[i], streams[i]));
    }
    NCCLCHECK(ncclGroupEnd());
  };
  const double n = ngpu;
  const double bus = op == "allreduce" ? 2.0 * (n - 1) / n : (op == "broadcast" ? 1.0 : (n - 1) / n);
  for (double b = (double)minb; b <= (double)maxb * 1.0001; b *= factor) {
    size_t bytes = ((size_t)b / (esz * ngpu)) * esz * ngpu;
    if (bytes == 0) continue;
    for (int w = 0; w < warm; ++w) launch(bytes);
    for (int i = 0; i < ngpu; ++i) {
      HIPCHECK(hipSetDevice(i));
      HIPCHECK(hipEventRecord(e0[i], streams[i]));
    }
    for (int it = 0; it < iters; ++it) launch(bytes);
    float worst = 0.f;
    for (int i = 0; i < ngpu; ++i) {
      HIPCHECK(hipSetDevice(i));
      HIPCHECK(hipEventRecord(e1[i], streams[i]));
    }
    for (int i = 0; i < ngpu; ++i) {
      HIPCHECK(hipEventSynchronize(e1[i]));
      float ms = 0.f;
      HIPCHECK(hipEventElapsedTime(&ms, e0[i], e1[i]));
      if (ms > worst) worst = ms;
    }
    const double us = worst * 1e3 / iters;
    const double algbw = bytes / (us * 1e-6) / 1e9;
    printf("{\"op\":\"%s\",\"bytes\":%zu,\"dtype\":\"%s\",\"ranks\":%d,\"us\":%.2f,\"algbw_gbs\":%.2f,"
           "\"busbw_gbs\":%.2f}\n",
           op.c_str(), bytes, dtype.c_str(), ngpu, us, algbw, algbw * bus);
    fflush(stdout);
  }
  for (int i = 0; i < ngpu; ++i) {
    ncclCommDestroy(comms[i]);
    hipSetDevice(i);
    hipFree(sbuf[i]);
    hipFree(rbuf[i]);
  }
  return 0;
}
