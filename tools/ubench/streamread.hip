// streamread.hip -- what does reading the hot kernel's 64 GiB cost by itself?
// Two read-only kernels over 131072 x 512 KiB chunks (no SHA-1 work; each lane
// xor-folds what it loads so nothing is dead):
//   perlane  the hot kernel's access pattern: one chunk per lane, a wave's 64
//            lanes 512 KiB apart, 128 B per lane per batch of loads
//   coalesced each wave reads a contiguous 1 MiB slab, 1 KiB per load instruction
//   groupedG  perlane's ownership with G lanes per 128-byte line (G = 2, 4, 8)
// each with default and non-temporal (nt) cache policy.  Run for ~10 s per mode so
// board power can be sampled alongside (tools/gpu_session.sh power_stream).
// Args: [launches per mode] (default 400) [mode 0..6, default all].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <ctime>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, unsigned nrec) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, nrec, 0x00020000);
}

template <int AUX>
__global__ __launch_bounds__(256) void k_perlane(const unsigned char *buf, unsigned pitch, unsigned chunk, unsigned *out) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  const unsigned char *base = buf + (size_t)wave * 64 * pitch;
  const __amdgpu_buffer_rsrc_t r = rsrc(base, 64 * pitch);
  u32x4 acc = {0, 0, 0, 0};
  for (unsigned pos = 0; pos < chunk; pos += 128) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * pitch + j * 16, pos, AUX);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j];
  }
  out[wave * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

// The hot kernel's ownership (a wave owns 64 chunks, walks them 128 B at a
// time), but G lanes share each line: instruction j reads chunk G*q + j%G of
// lane group q, 16*G contiguous bytes at 16*G*(j/G) of the 128-byte step.
// G = 1 is k_perlane; G = 8 reads whole lines (8 lines per instruction).
template <int G>
__global__ __launch_bounds__(256) void k_grouped(const unsigned char *buf, unsigned pitch, unsigned chunk, unsigned *out) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  const unsigned q = lane / G, r = lane % G;
  const unsigned char *base = buf + (size_t)wave * 64 * pitch;
  const __amdgpu_buffer_rsrc_t rs = rsrc(base, 64 * pitch);
  u32x4 acc = {0, 0, 0, 0};
  for (unsigned pos = 0; pos < chunk; pos += 128) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (G * q + j % G) * pitch + 16 * (G * (j / G) + r), pos, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc ^= v[j];
  }
  out[wave * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int AUX>
__global__ __launch_bounds__(256) void k_coalesced(const unsigned char *buf, unsigned slabs, unsigned *out) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x & 63;
  const unsigned nwaves = gridDim.x * blockDim.x / 64;
  u32x4 acc = {0, 0, 0, 0};
  for (unsigned s = wave; s < slabs; s += nwaves) {
    const __amdgpu_buffer_rsrc_t r = rsrc(buf + ((size_t)s << 20), 1u << 20);
    for (unsigned pos = 0; pos < (1u << 20); pos += 8 * 1024) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16 + j * 1024, pos, AUX);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc ^= v[j];
    }
  }
  out[wave * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

int main(int argc, char **argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 400;
  const int only = argc > 2 ? atoi(argv[2]) : -1;  // one mode (0..3), -1 all
  const size_t n = 131072, chunk = 512 * 1024, bytes = n * chunk;
  unsigned char *buf;
  unsigned *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, n * 4));
  CK(hipMemset(buf, 0x5a, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned slabs = (unsigned)(bytes >> 20);
  for (int mode = 0; mode < 7; ++mode) {
    if (only >= 0 && mode != only) continue;
    const char *names[] = {"perlane", "perlane_nt", "coalesced", "coalesced_nt", "grouped2", "grouped4", "grouped8"};
    auto launch = [&] {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_perlane<0>, dim3(n / 256), dim3(256), 0, 0, buf, chunk, chunk, out); break;
        case 1: hipLaunchKernelGGL(k_perlane<2>, dim3(n / 256), dim3(256), 0, 0, buf, chunk, chunk, out); break;
        case 2: hipLaunchKernelGGL(k_coalesced<0>, dim3(2048), dim3(256), 0, 0, buf, slabs, out); break;
        case 4: hipLaunchKernelGGL(k_grouped<2>, dim3(n / 256), dim3(256), 0, 0, buf, chunk, chunk, out); break;
        case 5: hipLaunchKernelGGL(k_grouped<4>, dim3(n / 256), dim3(256), 0, 0, buf, chunk, chunk, out); break;
        case 6: hipLaunchKernelGGL(k_grouped<8>, dim3(n / 256), dim3(256), 0, 0, buf, chunk, chunk, out); break;
        default: hipLaunchKernelGGL(k_coalesced<2>, dim3(2048), dim3(256), 0, 0, buf, slabs, out); break;
      }
    };
    launch();
    CK(hipDeviceSynchronize());
    const time_t t0 = time(nullptr);
    CK(hipEventRecord(e0));
    for (int i = 0; i < launches; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    const time_t t1 = time(nullptr);
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= launches;
    char ts[2][16];
    strftime(ts[0], sizeof ts[0], "%H:%M:%S", localtime(&t0));
    strftime(ts[1], sizeof ts[1], "%H:%M:%S", localtime(&t1));
    printf("%-13s %8.3f ms/launch  %7.1f GB/s  [%s - %s]\n", names[mode], ms, bytes / (ms * 1e-3) / 1e9, ts[0], ts[1]);
    fflush(stdout);
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
