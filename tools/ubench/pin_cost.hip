// pin_cost.hip -- what it costs to get page-locked host memory the DMA engine
// can read, per size and method, and the H2D rate out of each (the host
// pipelines' staging).  Prints one JSON line per case.
//   hipHostMalloc                    (the pipelines' staging today)
//   malloc + touch + hipHostRegister (4 KiB pages)
//   mmap + MADV_HUGEPAGE + touch + hipHostRegister (THP)
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e = (x);                                                     \
    if (e != hipSuccess) {                                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static double h2d_gbs(void *h, void *d, size_t n, hipStream_t s) {
  CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));  // warm
  CK(hipStreamSynchronize(s));
  const double t0 = now();
  for (int i = 0; i < 3; ++i) CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
  CK(hipStreamSynchronize(s));
  return 3.0 * n / (now() - t0) / 1e9;
}

int main() {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  void *d = nullptr;
  CK(hipMalloc(&d, 1ull << 30));
  const size_t sizes[] = {64ull << 20, 128ull << 20, 256ull << 20, 1ull << 30};
  for (int rep = 0; rep < 2; ++rep)
    for (size_t n : sizes) {
      {  // hipHostMalloc
        void *h = nullptr;
        double t0 = now();
        CK(hipHostMalloc(&h, n, hipHostMallocDefault));
        const double t_alloc = now() - t0;
        t0 = now();
        memset(h, 1, n);
        const double t_touch = now() - t0;
        const double bw = h2d_gbs(h, d, n, s);
        t0 = now();
        CK(hipHostFree(h));
        printf("{\"method\": \"hipHostMalloc\", \"MiB\": %zu, \"rep\": %d, \"pin_ms\": %.2f, \"first_touch_ms\": %.2f, "
               "\"free_ms\": %.2f, \"h2d_GBs\": %.2f}\n", n >> 20, rep, t_alloc * 1e3, t_touch * 1e3, (now() - t0) * 1e3, bw);
      }
      for (int thp = 0; thp < 2; ++thp) {  // mmap (+THP) + touch + register
        double t0 = now();
        void *h = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (h == MAP_FAILED) return 1;
        if (thp) madvise(h, n, MADV_HUGEPAGE);
        memset(h, 1, n);
        const double t_touch = now() - t0;
        t0 = now();
        CK(hipHostRegister(h, n, hipHostRegisterPortable));
        const double t_reg = now() - t0;
        const double bw = h2d_gbs(h, d, n, s);
        t0 = now();
        CK(hipHostUnregister(h));
        munmap(h, n);
        printf("{\"method\": \"mmap%s+touch+hipHostRegister\", \"MiB\": %zu, \"rep\": %d, \"touch_ms\": %.2f, "
               "\"register_ms\": %.2f, \"unregister_free_ms\": %.2f, \"h2d_GBs\": %.2f}\n",
               thp ? "+THP" : "", n >> 20, rep, t_touch * 1e3, t_reg * 1e3, (now() - t0) * 1e3, bw);
      }
      fflush(stdout);
    }
  return 0;
}
