// streamread2.hip -- does the size of the contiguous piece read from each chunk
// change what streaming the hot kernel's 64 GiB costs (rate, board power)?
//
// Same ownership as k_sha1_fixed: 131072 x 512 KiB chunks, a wave owns 64
// consecutive chunks and walks all of them front to back together.  Each step
// a wave fetches the next P bytes of each of its 64 chunks (64 * P bytes), 8
// dwordx4 loads per lane in flight per batch, and xor-folds them (nothing dead).
//   perlane P   lane l reads its own chunk l: P/16 loads per lane, back to back
//               (P = 128 is the hot kernel's pattern)
//   piece P     one wave instruction reads 1 KiB = 1024/P chunks x P contiguous
//               bytes, P/16 instructions per step (P = 128 is the LDS-staged
//               variant's pattern; P = 1024 reads each chunk 1 KiB at a time)
// Args: [launches per mode] (default 200).  Prints ms/launch and GB/s per mode
// with wall-clock stamps so a power sampler beside it can be matched up.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <unistd.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, unsigned nrec) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, nrec, 0x00020000);
}

constexpr unsigned kChunk = 512 * 1024;

template <int P>
__global__ __launch_bounds__(256) void k_perlane(const unsigned char *buf, unsigned *out) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc(buf + (size_t)wave * 64 * kChunk, 64 * kChunk);
  u32x4 acc = {0, 0, 0, 0};
  for (unsigned pos = 0; pos < kChunk; pos += P) {
#pragma unroll
    for (int b = 0; b < P / 128; ++b) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * kChunk + (b * 8 + j) * 16, pos, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= v[j];
    }
  }
  out[wave * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int P>
__global__ __launch_bounds__(256) void k_piece(const unsigned char *buf, unsigned *out) {
  constexpr unsigned kLanesPerChunk = P / 16, kChunksPerInstr = 64 / kLanesPerChunk;
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc(buf + (size_t)wave * 64 * kChunk, 64 * kChunk);
  // instruction i of a step covers chunks [i*kChunksPerInstr, (i+1)*kChunksPerInstr)
  const unsigned lane_off = (lane / kLanesPerChunk) * kChunk + (lane % kLanesPerChunk) * 16;
  u32x4 acc = {0, 0, 0, 0};
  for (unsigned pos = 0; pos < kChunk; pos += P) {
#pragma unroll
    for (int b = 0; b < (64 / kChunksPerInstr) / 8; ++b) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, lane_off + (b * 8 + j) * kChunksPerInstr * kChunk, pos, 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= v[j];
    }
  }
  out[wave * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main(int argc, char **argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 200;
  const size_t n = 131072, bytes = n * kChunk;
  unsigned char *buf;
  unsigned *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, n * 4));
  CK(hipMemset(buf, 0x5a, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Mode { const char *name; void (*k)(const unsigned char *, unsigned *); };
  const Mode modes[] = {
      {"perlane128", k_perlane<128>}, {"perlane256", k_perlane<256>}, {"perlane512", k_perlane<512>},
      {"perlane1024", k_perlane<1024>}, {"piece128", k_piece<128>}, {"piece256", k_piece<256>},
      {"piece512", k_piece<512>}, {"piece1024", k_piece<1024>},
  };
  for (const Mode &m : modes) {
    hipLaunchKernelGGL(m.k, dim3(n / 256), dim3(256), 0, 0, buf, out);
    CK(hipDeviceSynchronize());
    const time_t t0 = time(nullptr);
    CK(hipEventRecord(e0));
    for (int i = 0; i < launches; ++i) hipLaunchKernelGGL(m.k, dim3(n / 256), dim3(256), 0, 0, buf, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    const time_t t1 = time(nullptr);
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= launches;
    char ts[2][16];
    strftime(ts[0], sizeof ts[0], "%H:%M:%S", localtime(&t0));
    strftime(ts[1], sizeof ts[1], "%H:%M:%S", localtime(&t1));
    printf("%-12s %8.3f ms/launch  %7.1f GB/s  [%s - %s]\n", m.name, ms, bytes / (ms * 1e-3) / 1e9, ts[0], ts[1]);
    fflush(stdout);
    sleep(2);
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
