// residency.cpp -- is the hot kernel bound by HBM or by the SHA-1 ALU work at the
// clock the chip sustains?  Runs the production k_sha1_fixed launcher
// (libbtsha1.so) over 131072 x 512 KiB chunks with three pitches:
//   hbm   pitch 512 KiB   64 GiB footprint, every byte read from HBM once
//   mall  pitch 1 KiB     overlapping chunks, ~128 MiB footprint (MALL/L2-resident)
//   l2    pitch 16 B      all lanes of the grid walk the same ~2.5 MiB (L2-resident)
// Same instruction stream, same grid in all three; only where the bytes come from
// differs.  Prints ms per launch, the hashed-bytes rate and the wall-clock window
// (to line up with power/clock samples).  Args: [chunks] [launches per mode] [rounds]
// [mode: 0 hbm, 1 mall, 2 l2; default all].
// Build: make ubench (links bittorrent-with-congestion-control_amd/libbtsha1.so).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include "sha1_launch.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : 131072, len = 512 * 1024;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;  // ~20 ms per launch
  const int rounds = argc > 3 ? atoi(argv[3]) : 2;
  const int only = argc > 4 ? atoi(argv[4]) : -1;  // 0 hbm, 1 mall, 2 l2; -1 all
  const uint64_t bytes = n * len;
  void *buf;
  uint8_t *dig;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMalloc(&dig, 20 * n));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(btsha1_launch_fill(buf, bytes, 0, 0x0B175EED, s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct { const char *name; uint32_t pitch; } modes[] = {{"hbm", 512 * 1024}, {"mall", 1024}, {"l2", 16}};
  for (int round = 0; round < rounds; ++round)
    for (int mi = 0; mi < 3; ++mi) {
      if (only >= 0 && mi != only) continue;
      auto &m = modes[mi];
      // footprint check: the last chunk must end inside the allocation
      if ((n - 1) * (uint64_t)m.pitch + len > bytes) { fprintf(stderr, "bad pitch\n"); return 1; }
      CK(btsha1_launch_fixed(buf, n, m.pitch, (uint32_t)len, dig, nullptr, nullptr, s, 310));  // warm
      const time_t t0 = time(nullptr);
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) CK(btsha1_launch_fixed(buf, n, m.pitch, (uint32_t)len, dig, nullptr, nullptr, s, 310));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      char ts[2][16];
      const time_t t1 = time(nullptr);
      strftime(ts[0], sizeof ts[0], "%H:%M:%S", localtime(&t0));
      strftime(ts[1], sizeof ts[1], "%H:%M:%S", localtime(&t1));
      printf("%-5s pitch %7u  %8.3f ms/launch  %8.1f GiB/s hashed  [%s - %s]\n", m.name, m.pitch, ms,
             bytes / (ms * 1e-3) / (1ull << 30), ts[0], ts[1]);
      fflush(stdout);
    }
  CK(hipFree(buf));
  CK(hipFree(dig));
  return 0;
}
