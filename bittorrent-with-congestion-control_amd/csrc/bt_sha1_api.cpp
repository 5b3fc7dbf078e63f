// bt_sha1_api.cpp -- the C-ABI of libbtsha1.so: the reference's sha.h/chunk.h
// surface re-implemented over the gfx950 kernels, plus batch / verify /
// multi-GPU entry points (include/bt_sha1.h).
//
// Reference interfaces replaced (yunfanye/Bittorrent-with-Congestion-Control):
//   SHA1Init/SHA1Update/SHA1Final  sha.c:149-163, 453-527, 529-558 (sha.h:58-60)
//   shahash                        chunk.c:33-49  (chunk.h:28)
//   make_chunks                    chunk.c:13-25  (chunk.h:25)
//   binary2hex / hex2binary        chunk.c:55-83  (chunk.h:31,34)
//   hash + memcmp of save_chunk    util.c:304-337 (batched: bt_sha1_verifier_*)
//
// Host-side work here is bookkeeping only (staging, padding-byte layout, hex
// formatting); every compression runs in a HIP kernel.  No CPU hashing path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <cerrno>

#include "bt_sha1.h"
#include "chunk.h"
#include "sha1_launch.h"

namespace {

thread_local std::string t_err;
thread_local int t_dev = 0;
std::atomic<int> g_variant{310};  // ring 3 x 128-byte slots, default cache policy

void set_err(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  t_err = buf;
}

#define BT_CK(expr)                                                                  \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) {                                                          \
      set_err("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
      return -1;                                                                     \
    }                                                                                \
  } while (0)

[[noreturn]] void die(const char *where) {
  fprintf(stderr, "libbtsha1: %s: %s\n", where, t_err.c_str());
  fflush(stderr);
  abort();
}

// Entry points that must switch devices (host pipelines, drop-in calls, the
// verifier) give the caller's thread its current device back on return, so
// a caller that drives its own HIP work (torch on cuda:N) is not moved.
struct KeepDevice {
  int prev = -1;
  KeepDevice() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~KeepDevice() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  KeepDevice(const KeepDevice &) = delete;
  KeepDevice &operator=(const KeepDevice &) = delete;
};

// Grow-only device / pinned scratch.
constexpr uint32_t kMaxColumns = 16;  // column-split tail: most columns per chunk (chunks_host_on)

struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  int ensure(size_t need) {
    if (need <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t sz = std::max<size_t>(need, 4096);
    BT_CK(hipMalloc(&p, sz));
    cap = sz;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const { return static_cast<T *>(p); }
};
struct PinBuf {
  void *p = nullptr;
  size_t cap = 0;
  int ensure(size_t need) {
    if (need <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t sz = std::max<size_t>(need, 4096);
    BT_CK(hipHostMalloc(&p, sz, hipHostMallocDefault));
    cap = sz;
    return 0;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const { return static_cast<T *>(p); }
};

// ---- NUMA placement of the host pipelines' staging ---------------------------
// The GPU hangs off one socket's PCIe root.  The staging lanes are written by
// the copy threads and read by the DMA engine; placing their pages on the
// GPU's node and running the copy threads on that node's CPUs keeps both
// local (the caller's pageable input is wherever the caller touched it).
// Topology from sysfs, no libnuma: node N's CPUs from
// /sys/devices/system/node/nodeN/cpulist, the GPU's node from
// /sys/bus/pci/devices/<bdf>/numa_node.
struct NumaTopo {
  int nodes = 1;
  std::vector<int> cpu_node;               // cpu -> node
  std::vector<std::vector<int>> node_cpus;  // node -> cpus
};

std::vector<int> parse_cpulist(const char *s) {
  std::vector<int> out;
  while (*s) {
    char *end = nullptr;
    const long a = strtol(s, &end, 10);
    if (end == s) break;
    long b = a;
    s = end;
    if (*s == '-') {
      b = strtol(s + 1, &end, 10);
      s = end;
    }
    for (long c = a; c <= b && c < 65536; ++c) out.push_back((int)c);
    while (*s == ',' || *s == '\n' || *s == ' ') ++s;
  }
  return out;
}

const NumaTopo &numa_topo() {
  static const NumaTopo t = [] {
    NumaTopo r;
    int present = 0;
    for (int n = 0; n < 256; ++n) {
      char path[96], buf[4096];
      snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", n);
      FILE *f = fopen(path, "r");
      if (!f) continue;
      const size_t got = fread(buf, 1, sizeof buf - 1, f);
      fclose(f);
      buf[got] = 0;
      ++present;
      r.node_cpus.resize(n + 1);
      r.node_cpus[n] = parse_cpulist(buf);
      for (int c : r.node_cpus[n]) {
        if ((int)r.cpu_node.size() <= c) r.cpu_node.resize(c + 1, -1);
        r.cpu_node[c] = n;
      }
    }
    r.nodes = std::max(1, present);
    return r;
  }();
  return t;
}

int node_of_cpu(int cpu) {
  const NumaTopo &t = numa_topo();
  return cpu >= 0 && cpu < (int)t.cpu_node.size() ? t.cpu_node[cpu] : -1;
}

// The NUMA node the device's PCI function reports (-1: unknown).
int gpu_numa_node(int dev) {
  char bdf[64] = {0};
  if (hipDeviceGetPCIBusId(bdf, sizeof bdf, dev) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  for (char *p = bdf; *p; ++p)
    if (*p >= 'A' && *p <= 'F') *p = (char)(*p + 32);
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bdf);
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

// Staging placement (BT_SHA1_NUMA): "off" = none (pages wherever the kernel
// puts them, copy threads unpinned); "lanes" (default) = the lanes' pages
// prefer the GPU's node, so the DMA engine reads local memory; "gpu" = that,
// and the copy threads run on the node's CPUs.  Applies only when the machine
// has more than one node and the GPU's node is known.  Measured on MI355X
// boxes (tools/numa_probe.py, profiles/r06/numa_place.md), 8 GiB images on
// either node: off 49.0-50.4, lanes 50.1-50.5 GiB/s; pinning the copy
// threads to the GPU node's cores cost 15-30 % on hosts whose cores other
// jobs share (34.5-40.7 GiB/s), so it is not the default.
enum NumaMode { kNumaOff = 0, kNumaLanes = 1, kNumaGpu = 2 };
constexpr int kNumaDefault = kNumaLanes;
int numa_mode() {
  static const int m = [] {
    const char *e = getenv("BT_SHA1_NUMA");
    if (!e || !*e) return (int)kNumaDefault;
    if (!strcmp(e, "off") || !strcmp(e, "0")) return (int)kNumaOff;
    if (!strcmp(e, "lanes")) return (int)kNumaLanes;
    return (int)kNumaGpu;
  }();
  return m;
}

// Pages of [p, p+len) sampled evenly (at most `samples`), counted per node
// (move_pages with no target nodes only queries).  Pages not yet faulted in
// count nowhere.
void page_nodes(const void *p, uint64_t len, int samples, int32_t *counts, int ncounts) {
  if (!p || !len || samples <= 0) return;
  const uint64_t pg = 4096, first = (uintptr_t)p & ~(pg - 1), last = ((uintptr_t)p + len - 1) & ~(pg - 1);
  const uint64_t npages = (last - first) / pg + 1;
  const int n = (int)std::min<uint64_t>((uint64_t)samples, npages);
  std::vector<void *> pages(n);
  std::vector<int> status(n, -1);
  for (int i = 0; i < n; ++i) pages[i] = (void *)(first + pg * (npages * (uint64_t)i / (uint64_t)n));
  if (syscall(SYS_move_pages, 0, (unsigned long)n, pages.data(), nullptr, status.data(), 0) != 0) return;
  for (int s : status)
    if (s >= 0 && s < ncounts) ++counts[s];
}

// Staging placement of one call: the node to bind the lanes to and the CPUs
// (within the calling thread's affinity mask) the copy threads run on.
struct Placement {
  int node = -1;      // -1: no placement
  int ncpus = 0;      // 0: threads unpinned
  cpu_set_t cpus;
  int mode() const { return node < 0 ? kNumaOff : ncpus > 0 ? kNumaGpu : kNumaLanes; }
};

Placement placement_for(int gpu_node) {
  Placement pl;
  CPU_ZERO(&pl.cpus);
  const NumaTopo &t = numa_topo();
  const int mode = numa_mode();
  if (mode == kNumaOff || gpu_node < 0 || t.nodes < 2 || gpu_node >= (int)t.node_cpus.size()) return pl;
  if (mode == kNumaLanes) {
    pl.node = gpu_node;
    return pl;
  }
  cpu_set_t aff;
  CPU_ZERO(&aff);
  if (sched_getaffinity(0, sizeof aff, &aff) != 0) return pl;
  for (int c : t.node_cpus[gpu_node])
    if (c < CPU_SETSIZE && CPU_ISSET(c, &aff)) {
      CPU_SET(c, &pl.cpus);
      ++pl.ncpus;
    }
  if (pl.ncpus == 0) return pl;  // none of the GPU's CPUs usable: leave placement to the kernel
  pl.node = gpu_node;
  return pl;
}

// Preferred (not strict) policy: pages go to `node` while it has memory.
void prefer_node(void *p, size_t len, int node) {
  if (node < 0 || node >= 256) return;
  unsigned long mask[4] = {0, 0, 0, 0};
  mask[node / 64] = 1ul << (node % 64);
  const int kMpolPreferred = 1;
  (void)syscall(SYS_mbind, p, (unsigned long)len, kMpolPreferred, mask, 256ul, 0u);
}

// The calling thread's current placement (set by run_pipeline for the
// duration of one call; read by the staging helpers on that thread).
thread_local const Placement *t_place = nullptr;
thread_local std::atomic<int32_t> *t_piece_nodes = nullptr;  // per-node piece tally of the call

void touch_parallel(uint8_t *p, uint64_t n);

// Grow-only staging buffer of the host pipelines, read only by the DMA engine
// (hipMemcpyAsync): anonymous memory on transparent huge pages, first-touched
// by several threads, then page-locked with hipHostRegister.  Per GiB on
// MI355X boxes (tools/ubench/pin_cost.hip): ~3 ms to register + the touch
// (65 ms on one thread), against 222-251 ms for hipHostMalloc -- the pinning
// was most of a make-chunks run on a 1 GiB file.  Same H2D rate (~57 GB/s).
struct StageBuf {
  void *p = nullptr;
  size_t cap = 0;
  void release() {
    if (!p) return;
    (void)hipHostUnregister(p);
    munmap(p, cap);
    p = nullptr;
    cap = 0;
  }
  // node >= 0: the pages prefer that NUMA node (placed at first touch).
  int ensure(size_t need, int node = -1) {
    if (need <= cap) return 0;
    release();
    const size_t sz = (std::max<size_t>(need, 4096) + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
    void *q = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) {
      set_err("staging mmap of %zu bytes failed: %s", sz, strerror(errno));
      return -1;
    }
    (void)madvise(q, sz, MADV_HUGEPAGE);  // a hint: 4 KiB pages still work
    // Not inherited by fork(): a child (e.g. a subprocess about to exec) would
    // otherwise get a copy of every page-locked page at fork time.
    (void)madvise(q, sz, MADV_DONTFORK);
    prefer_node(q, sz, node);
    touch_parallel((uint8_t *)q, sz);
    const hipError_t e = hipHostRegister(q, sz, hipHostRegisterPortable);
    if (e != hipSuccess) {
      munmap(q, sz);
      set_err("hipHostRegister of the staging buffer failed: %s", hipGetErrorString(e));
      return -1;
    }
    p = q;
    cap = sz;
    return 0;
  }
  template <class T>
  T *as() const { return static_cast<T *>(p); }
};

// One double-buffered staging lane of the host pipelines.
struct Lane {
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  hipEvent_t copied = nullptr;  // after the batch's last H2D (serial copy order)
  StageBuf h_in;  // staged input pieces, DMA'd to d_in
  PinBuf h_dig;   // the kernel stores digests straight into it
  PinBuf h_edge;  // registered-batch mode: the batch's unaligned head / tail bytes
  DevBuf d_in;
  bool busy = false;
  uint64_t first = 0, count = 0;  // chunk range in flight
};

struct DevCtx {
  int dev = 0;
  int numa_node = -2;  // the GPU's NUMA node (-1 unknown; -2 not read yet)
  std::mutex mu;
  hipStream_t s = nullptr;  // drop-in calls and NULL-stream launches (= lane[0].s)
  Lane lane[2];
  PinBuf h_msg, h_state;  // drop-in calls: message / chaining state, read and written by the chain kernel
  // Host pipelines' column-split last batch (chunks_host_on): its digests, its
  // few chunks that are not split (hashed from a pinned copy), the chunks'
  // chaining state between columns, the column and leftover streams, an event
  // per column copy and one after each stream's work.
  PinBuf h_cdig, h_cleft;
  DevBuf d_cstate;
  hipStream_t cs = nullptr, xs = nullptr;
  hipEvent_t cev[kMaxColumns] = {}, cdone = nullptr, xdone = nullptr;
  uint32_t seq = 0;       // drop-in calls: completion word the chain kernel stores at h_state + 32
};

std::mutex g_ctx_mu;
std::vector<std::unique_ptr<DevCtx>> g_ctx;

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

DevCtx *ctx_for(int dev) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  int n = device_count();
  if (n <= 0) {
    set_err("no HIP device visible (hipGetDeviceCount = 0)");
    return nullptr;
  }
  if (dev < 0 || dev >= n) {
    set_err("device %d out of range (%d visible)", dev, n);
    return nullptr;
  }
  if ((int)g_ctx.size() < n) g_ctx.resize(n);
  if (!g_ctx[dev]) {
    auto c = std::make_unique<DevCtx>();
    c->dev = dev;
    KeepDevice keep_dev;
    if (hipSetDevice(dev) != hipSuccess) {
      set_err("cannot initialise HIP device %d", dev);
      return nullptr;
    }
    g_ctx[dev] = std::move(c);
  }
  return g_ctx[dev].get();
}

// Everything a context holds: its streams (drained first), staging lanes and
// drop-in buffers.  Used for the per-call worker contexts of repeated device
// ids in bt_sha1_chunks_host_devices, which must not outlive the call.
void release_ctx(DevCtx *c) {
  if (!c) return;
  KeepDevice keep_dev;
  if (hipSetDevice(c->dev) != hipSuccess) return;
  for (auto &l : c->lane) {
    if (l.s) {
      (void)hipStreamSynchronize(l.s);
      (void)hipStreamDestroy(l.s);
    }
    if (l.ev) (void)hipEventDestroy(l.ev);
    if (l.copied) (void)hipEventDestroy(l.copied);
    l.copied = nullptr;
    l.s = nullptr;
    l.ev = nullptr;
    l.h_in.release();
    l.h_dig.release();
    l.h_edge.release();
    l.d_in.release();
  }
  c->s = nullptr;
  c->h_msg.release();
  c->h_state.release();
  c->h_cdig.release();
  c->h_cleft.release();
  c->d_cstate.release();
  for (hipEvent_t &e : c->cev) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
  }
  for (hipEvent_t *e : {&c->cdone, &c->xdone}) {
    if (*e) (void)hipEventDestroy(*e);
    *e = nullptr;
  }
  for (hipStream_t *t : {&c->cs, &c->xs}) {
    if (*t) (void)hipStreamDestroy(*t);
    *t = nullptr;
  }
}

// Streams are created on first use and kept few: HIP multiplexes streams onto
// GPU_MAX_HW_QUEUES (4) hardware queues, and two streams that share a queue
// serialise -- which silently kills the H2D/hash overlap of the pipelines.
int ensure_streams(DevCtx *c) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  if (c->s) return 0;
  for (auto &l : c->lane) {
    BT_CK(hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking));
    BT_CK(hipEventCreateWithFlags(&l.ev, hipEventDisableTiming));
    BT_CK(hipEventCreateWithFlags(&l.copied, hipEventDisableTiming));
  }
  c->s = c->lane[0].s;
  return 0;
}

// Caller streams of the device-resident entry points.  NULL is the device's
// null (default) stream, exactly as for a hipLaunchKernelGGL(..., 0, ...) of the
// caller's own: ordered after the caller's earlier default-stream work (e.g.
// torch's default stream, whose handle is 0) and before its later work.  The
// library's own non-blocking streams serve only its host pipelines.
hipStream_t pick_stream(void *stream) { return (hipStream_t)stream; }

bool fast_layout(const void *d_in, uint64_t chunk_len, uint64_t pitch, const void *d_dig) {
  return ((uintptr_t)d_in & 15) == 0 && (pitch & 15) == 0 && ((uintptr_t)d_dig & 3) == 0 &&
         chunk_len <= pitch && 64 * pitch + 4096 <= (1ull << 32);  // 32-bit buffer offsets incl. prefetch overrun
}

// Launch the right kernel(s) for n equal chunks of len bytes at pitch.
int launch_chunks(const void *d_in, uint64_t n, uint64_t len, uint64_t pitch, uint8_t *d_dig, hipStream_t s) {
  if (n == 0) return 0;
  if (fast_layout(d_in, len, pitch, d_dig)) {
    BT_CK(btsha1_launch_fixed(d_in, n, (uint32_t)pitch, (uint32_t)len, d_dig, nullptr, nullptr, s, g_variant.load()));
  } else {
    if (len >= (1ull << 32)) {
      set_err("chunk_len %llu exceeds 4 GiB", (unsigned long long)len);
      return -1;
    }
    BT_CK(btsha1_launch_ragged(d_in, nullptr, nullptr, pitch, (uint32_t)len, n, d_dig, s));
  }
  return 0;
}

// A contiguous image: full chunks through the hot kernel, a short last chunk
// (make_chunks' final fread, chunk.c:20) in the same launch as its tail wave
// when the layout allows, else through the ragged kernel after it.
int launch_image(const uint8_t *d_img, uint64_t bytes, uint64_t chunk_len, uint8_t *d_dig, hipStream_t s) {
  const uint64_t nfull = bytes / chunk_len, rem = bytes % chunk_len;
  if (fast_layout(d_img, chunk_len, chunk_len, d_dig)) {
    BT_CK(btsha1_launch_fixed(d_img, nfull, (uint32_t)chunk_len, (uint32_t)chunk_len, d_dig, nullptr, nullptr, s,
                              g_variant.load(), (uint32_t)rem));
    return 0;
  }
  if (launch_chunks(d_img, nfull, chunk_len, chunk_len, d_dig, s)) return -1;
  if (rem) BT_CK(btsha1_launch_ragged(d_img + nfull * chunk_len, nullptr, nullptr, 0, (uint32_t)rem, 1,
                                      d_dig + 20 * nfull, s));
  return 0;
}

// Staging batch: ~1 GiB per lane keeps >= 2048 chunks in flight per launch,
// enough that the per-chunk hash latency (~10 ms, 8193 dependent blocks at one
// wave per SIMD) still outruns PCIe; capped by the input size when known.  An
// input of 64 MiB - 2 GiB is cut in two batches so both lanes work (the second
// lane's pinning overlaps the first batch, see run_pipeline).
// Direct-DMA input (pinned / registered) uses the same 1 GiB batches, DMA'd
// straight from the caller's memory into the kept lanes.  Round 2 chose 4 GiB
// batches under overlapping copies (40.2 / 45.9 / 48.9 GiB/s with 1 / 2 / 4
// GiB); with round 3's serial copy order bigger batches gain nothing, and
// because they exceed the kept lanes they were allocated and freed on every
// call -- and a re-allocated 4 GiB batch ran the copies at 41.1-41.4 GiB/s call
// after call on three of three boxes (tools/dma_repeat.py;
// profiles/r04/dma_batch.md) where 1 GiB kept lanes hold 48.9-50.7 (8 GiB
// image) and 52.4-52.5 (32 GiB) against a ~53.6 raw copy.  BT_SHA1_DMA_BATCH_MB overrides the 1024 MiB
// default; batches above 1 GiB are freed after the call.
uint64_t dma_batch_target() {
  static const uint64_t v = [] {
    const char *e = getenv("BT_SHA1_DMA_BATCH_MB");
    const long mb = e ? atol(e) : 1024;
    return (uint64_t)(mb < 64 ? 64 : (mb > 16384 ? 16384 : mb)) << 20;
  }();
  return v;
}

uint64_t batch_bytes_for(uint64_t chunk_len, uint64_t size_hint, bool staged = true) {
  const uint64_t target = staged ? 1ull << 30 : dma_batch_target();
  uint64_t per = std::max<uint64_t>(1, target / chunk_len);
  if (size_hint != UINT64_MAX) {
    const uint64_t n = (size_hint + chunk_len - 1) / chunk_len;
    per = std::max<uint64_t>(1, std::min<uint64_t>(per, size_hint >= (64ull << 20) ? (n + 1) / 2 : n));
  }
  return per * chunk_len;
}

// Host memory the DMA engine can read directly (hipHostMalloc'd or
// registered with bt_sha1_host_register): no staging copy needed.
bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}
// An input is DMA'd in place only when both its ends are pinned (a lock
// around its first bytes alone -- a neighbour's page -- does not make it so).
bool is_pinned_range(const uint8_t *p, uint64_t n) { return n && is_pinned(p) && is_pinned(p + n - 1); }

// Workers of one bt_sha1_chunks_host_devices call (each a host thread with two
// staging lanes of up to 1 GiB pinned + 1 GiB HBM while the call runs).
constexpr int kMaxWorkers = 64;

// Host staging threads for the pipelines' CPU side (memcpy into pinned memory,
// file reads): one core moves ~8 GB/s, PCIe takes ~53.  BT_SHA1_COPY_THREADS
// overrides the default of 8.
int copy_threads() {
  static const int n = [] {
    const char *e = getenv("BT_SHA1_COPY_THREADS");
    const int v = e ? atoi(e) : 8;
    return v < 1 ? 1 : (v > 64 ? 64 : v);
  }();
  return n;
}

// Split [0, n) into page-aligned pieces of at least 16 MiB, one per thread
// (the caller's thread takes the first), and run body(off, len, piece) on each.
// Under a pipeline call's NUMA placement (t_place) every piece runs on a
// helper thread pinned to the GPU node's CPUs (the caller's own affinity is
// left alone); staging pieces (tally) are counted by the node of the CPU
// they started on.
template <class Body>
void parallel_pieces(uint64_t n, Body body, bool tally = false) {
  const uint64_t min_piece = 16ull << 20;
  int t = copy_threads();
  if ((uint64_t)t > n / min_piece) t = (int)std::max<uint64_t>(1, n / min_piece);
  uint64_t piece = (n + t - 1) / t;
  piece = (piece + 4095) & ~4095ull;
  const Placement *pl = t_place;
  std::atomic<int32_t> *counts = tally ? t_piece_nodes : nullptr;
  const bool pin = pl && pl->ncpus > 0;
  auto run = [&, pl, counts, pin](int i) {
    if (pin) (void)pthread_setaffinity_np(pthread_self(), sizeof pl->cpus, &pl->cpus);
    if (counts) {
      const int nd = node_of_cpu(sched_getcpu());
      if (nd >= 0 && nd < BT_SHA1_STATS_NODES) counts[nd].fetch_add(1, std::memory_order_relaxed);
    }
    body((uint64_t)i * piece, std::min<uint64_t>(piece, n - (uint64_t)i * piece), i);
  };
  std::vector<std::thread> th;
  for (int i = pin ? 0 : 1; i < t && (uint64_t)i * piece < n; ++i) th.emplace_back(run, i);
  if (!pin) run(0);
  for (auto &x : th) x.join();
}

void touch_parallel(uint8_t *p, uint64_t n) {
  parallel_pieces(n, [&](uint64_t off, uint64_t len, int) {
    for (uint64_t o = 0; o < len; o += 4096) p[off + o] = 0;
  });
}

void parallel_copy(uint8_t *dst, const uint8_t *src, uint64_t n) {
  if (n < (32ull << 20) && !(t_place && t_place->ncpus > 0)) {
    if (t_piece_nodes) {
      const int nd = node_of_cpu(sched_getcpu());
      if (nd >= 0 && nd < BT_SHA1_STATS_NODES) t_piece_nodes[nd].fetch_add(1, std::memory_order_relaxed);
    }
    memcpy(dst, src, n);
    return;
  }
  parallel_pieces(n, [&](uint64_t off, uint64_t len, int) { memcpy(dst + off, src + off, len); }, true);
}

// Gather one column of `rows` strided rows into a dense buffer with the copy
// threads: dst[r*width ..] = src[r*pitch ..] (width bytes per row).
void parallel_gather(uint8_t *dst, const uint8_t *src, uint64_t rows, uint64_t width, uint64_t pitch) {
  parallel_pieces(
      rows * width,
      [&](uint64_t off, uint64_t len, int) {
        for (uint64_t o = off, end = off + len; o < end;) {
          const uint64_t r = o / width, in = o % width, k = std::min<uint64_t>(width - in, end - o);
          memcpy(dst + o, src + r * pitch + in, k);
          o += k;
        }
      },
      true);
}

// pread `want` bytes at file offset `pos` into dst with several threads.
// Returns the length of the contiguous prefix read (short only at EOF), or -1.
int64_t parallel_pread(int fd, uint8_t *dst, uint64_t want, uint64_t pos) {
  std::vector<int64_t> got(64, 0);
  std::vector<uint64_t> asked(64, 0);
  std::atomic<bool> err{false};
  parallel_pieces(want, [&](uint64_t off, uint64_t len, int i) {
    asked[i] = len;
    uint64_t done = 0;
    while (done < len) {
      const ssize_t r = pread(fd, dst + off + done, (size_t)(len - done), (off_t)(pos + off + done));
      if (r < 0) {
        if (errno == EINTR) continue;
        err = true;
        break;
      }
      if (r == 0) break;  // EOF
      done += (uint64_t)r;
    }
    got[i] = (int64_t)done;
  }, true);
  if (err) return -1;
  int64_t total = 0;
  for (int i = 0; i < 64 && asked[i]; ++i) {
    total += got[i];
    if ((uint64_t)got[i] < asked[i]) break;  // EOF inside piece i
  }
  return total;
}

// Generic double-buffered pipeline over two streams: batch k+1's H2D overlaps
// batch k's hashing, and inside a batch each 128 MiB piece is copied to the
// device as soon as it is staged, so host reads overlap the H2D.
// fill(lane, off, max_bytes, &src, &eof) provides up to max_bytes of the
// image at byte `off` of the lane's batch (staged at lane.h_in + off, or in
// place when the DMA engine can read it) and returns the byte count -- fewer
// than max_bytes at a piece boundary of its own -- setting eof when no input
// follows (a return of 0 is the end too); sink(first_chunk, count, digests)
// receives digests in chunk order.
// BT_SHA1_TRACE=1: per-phase wall times of each pipeline run on stderr.
bool trace_on() {
  static const bool on = [] {
    const char *e = getenv("BT_SHA1_TRACE");
    return e && *e && *e != '0';
  }();
  return on;
}
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

constexpr uint64_t kPage = 4096;  // host page (registration granule)

// Staging -> H2D granule inside a batch: 128 MiB (BT_SHA1_PIECE_MB overrides,
// 16 .. 1024).
uint64_t piece_bytes() {
  static const uint64_t v = [] {
    const char *e = getenv("BT_SHA1_PIECE_MB");
    const long mb = e ? atol(e) : 128;
    return (uint64_t)(mb < 16 ? 16 : (mb > 1024 ? 1024 : mb)) << 20;
  }();
  return v;
}

// Copy order of the two lanes.  "serial": a batch's first H2D waits for the
// previous batch's last one, so one copy runs at a time (hashing still
// overlaps the next copy).  "overlap": a batch's H2D may run beside the
// previous batch's (two DMA engines at once).  Default: serial for direct DMA
// from pinned / registered memory, overlap for the staged lanes.  Measured
// (tools/numa_probe.py 8, profiles/r03/numa_probe.md): an 8 GiB registered
// image on the GPU's socket 50.6 (overlap) / 50.1 (serial) GiB/s, on the other
// socket 42.2 (overlap) / 49.7 (serial) -- two concurrent DMA streams out of
// the other socket's memory lose ~8 GiB/s; the staged lanes (whose pages the
// copy threads place) lose ~1 with serial copies.  BT_SHA1_COPY_ORDER=
// serial|overlap forces one order.
bool serial_copies(bool staged) {
  static const int forced = [] {
    const char *e = getenv("BT_SHA1_COPY_ORDER");
    return e ? (!strcmp(e, "serial") ? 1 : !strcmp(e, "overlap") ? 0 : -1) : -1;
  }();
  return forced >= 0 ? forced == 1 : !staged;
}

// bt_sha1_get_pipeline_stats: the calling thread's last pipeline run.
thread_local bt_sha1_pipeline_stats t_stats;
thread_local bool t_stats_valid = false;

// How a pipeline's input reaches the DMA engine.
enum class Feed {
  kStaged,     // copied (memcpy / pread) into the pinned staging lanes
  kDirect,     // the caller's memory is pinned already: DMA'd in place
  kRegistered  // pageable caller memory page-locked batch by batch (chunks_host_on)
};

// tail.queue(idle_lane, last_copied): called once every batch is queued, with
// the lane that is not carrying the last batch and the event after the last
// batch's copy (NULL when copies may overlap) -- chunks_host_on's column-split
// tail; tail.wait() after the lanes are drained, before any lane buffer is
// resized.  Both return 0 or -1.
template <class Q, class W>
struct TailOps {
  Q queue;
  W wait;
};
template <class Q, class W>
TailOps<Q, W> tail_ops(Q q, W w) {
  return TailOps<Q, W>{q, w};
}
inline auto no_tail() {
  return tail_ops([](Lane &, hipEvent_t) { return 0; }, [] { return 0; });
}

template <class Fill, class Sink, class Tail>
int64_t run_pipeline(DevCtx *c, uint64_t chunk_len, uint64_t size_hint, Feed feed, Fill fill, Sink sink, Tail tail) {
  if (chunk_len == 0 || chunk_len >= (1ull << 32)) {
    set_err("chunk_len must be in [1, 4 GiB)");
    return -1;
  }
  const bool staged = feed == Feed::kStaged;
  const double t_start = now_s();
  double t_fill = 0, t_wait = 0;
  if (ensure_streams(c)) return -1;
  const uint64_t bytes_per = batch_bytes_for(chunk_len, size_hint, staged);
  const uint64_t per = bytes_per / chunk_len;
  double t_alloc = 0;
  // NUMA: staged lanes on the GPU's node, staging threads on its CPUs.
  if (c->numa_node == -2) c->numa_node = gpu_numa_node(c->dev);
  const Placement place = staged ? placement_for(c->numa_node) : Placement{};
  std::atomic<int32_t> piece_nodes[BT_SHA1_STATS_NODES];
  for (auto &x : piece_nodes) x.store(0);
  struct PlaceScope {  // the staging helpers of this thread see the placement for this call only
    const Placement *prev_place;
    std::atomic<int32_t> *prev_nodes;
    PlaceScope(const Placement *p, std::atomic<int32_t> *n) : prev_place(t_place), prev_nodes(t_piece_nodes) {
      t_place = p;
      t_piece_nodes = n;
    }
    ~PlaceScope() {
      t_place = prev_place;
      t_piece_nodes = prev_nodes;
    }
  } place_scope(&place, piece_nodes);
  t_stats_valid = false;
  // Buffers are sized (grow-only, kept across calls) when a lane is first
  // used: an input that fits one batch never pins the second lane's memory.
  auto prepare = [&](Lane &l) -> int {
    const double t0 = now_s();
    if ((staged && l.h_in.ensure(bytes_per, place.node)) || l.d_in.ensure(bytes_per) || l.h_dig.ensure(20 * per) ||
        (feed == Feed::kRegistered && l.h_edge.ensure(2 * kPage)))
      return -1;
    t_alloc += now_s() - t0;
    return 0;
  };
  for (auto &l : c->lane) l.busy = false;
  const size_t kept_cap[2] = {c->lane[0].d_in.cap, c->lane[1].d_in.cap};
  // When a second batch will be needed, size lane 1 on a helper thread while
  // lane 0 is filled and copied: pinning ~1 GiB costs ~0.2-0.5 s per process.
  std::thread pre;
  int pre_rc = 0;
  std::string pre_err;
  if (size_hint > bytes_per) {
    pre = std::thread([&] {
      if (hipSetDevice(c->dev) != hipSuccess) {
        pre_rc = -1;
        pre_err = "hipSetDevice failed on the staging thread";
        return;
      }
      Lane &l = c->lane[1];
      pre_rc = (staged && l.h_in.ensure(bytes_per, place.node)) || l.d_in.ensure(bytes_per) || l.h_dig.ensure(20 * per)
                   ? -1
                   : 0;
      if (pre_rc) pre_err = t_err;
    });
  }
  struct JoinAtExit {  // every return path, including the error ones
    std::thread &t;
    ~JoinAtExit() {
      if (t.joinable()) t.join();
    }
  } join_at_exit{pre};
  auto join_pre = [&]() -> int {
    if (!pre.joinable()) return 0;
    const double t0 = now_s();
    pre.join();
    t_alloc += now_s() - t0;
    if (pre_rc) set_err("%s", pre_err.c_str());
    return pre_rc;
  };
  auto drain = [&](Lane &l) -> int {
    if (!l.busy) return 0;
    const double t0 = now_s();
    BT_CK(hipEventSynchronize(l.ev));
    t_wait += now_s() - t0;
    sink(l.first, l.count, l.h_dig.as<uint8_t>());
    l.busy = false;
    return 0;
  };
  uint64_t next = 0;
  int k = 0;
  for (;;) {
    Lane &l = c->lane[k & 1];
    if ((k == 1 && join_pre()) || drain(l) || prepare(l)) return -1;
    if (k > 0 && serial_copies(staged)) BT_CK(hipStreamWaitEvent(l.s, c->lane[(k + 1) & 1].copied, 0));
    uint64_t got = 0;
    bool eof = false;
    while (got < bytes_per && !eof) {
      // Staged input moves in pieces (host reads overlap the H2D); pinned
      // input goes as one copy per batch -- 128 MiB copies straight from
      // registered memory measured 36.5 GiB/s against 50 for 1 GiB ones.
      const uint64_t want = std::min<uint64_t>(staged ? piece_bytes() : bytes_per, bytes_per - got);
      const uint8_t *src = nullptr;
      const double t0 = now_s();
      const int64_t r = fill(l, got, want, &src, &eof);
      t_fill += now_s() - t0;
      if (r < 0) return -1;
      if (r) {
        const hipError_t ce = hipMemcpyAsync(l.d_in.as<uint8_t>() + got, src, (size_t)r, hipMemcpyHostToDevice, l.s);
        if (ce != hipSuccess) {
          set_err("hipMemcpyAsync of %llu bytes from host %p (batch %d, byte %llu of it) failed: %s",
                  (unsigned long long)r, (const void *)src, k, (unsigned long long)got, hipGetErrorString(ce));
          return -1;
        }
      }
      got += (uint64_t)r;
      if (r == 0) eof = true;
    }
    if (got == 0) break;
    if (serial_copies(staged)) BT_CK(hipEventRecord(l.copied, l.s));
    const uint64_t cnt = (got + chunk_len - 1) / chunk_len;
    if (launch_image(l.d_in.as<uint8_t>(), got, chunk_len, l.h_dig.as<uint8_t>(), l.s)) return -1;
    BT_CK(hipEventRecord(l.ev, l.s));
    l.busy = true;
    l.first = next;
    l.count = cnt;
    next += cnt;
    ++k;
    if (eof) break;
  }
  if (join_pre()) return -1;  // input shorter than the size hint
  if (tail.queue(c->lane[k & 1], k > 0 && serial_copies(staged) ? c->lane[(k + 1) & 1].copied : nullptr)) return -1;
  // Older lane first so digests arrive in order.
  if (drain(c->lane[k & 1]) || drain(c->lane[(k + 1) & 1])) return -1;
  {
    const double t0 = now_s();
    if (tail.wait()) return -1;
    t_wait += now_s() - t0;
  }
  // Direct-DMA batches bigger than a staged batch (BT_SHA1_DMA_BATCH_MB >
  // 1024) are not kept past the call: the lanes keep at most 1 GiB of HBM
  // each, so a process that shares the GPU does not lose more for good.  An
  // oversized lane goes back to what it held before the call (capped at the
  // staged size), so the next staged call finds its kept lane in place.
  if (!staged) {
    const uint64_t keep = batch_bytes_for(chunk_len, UINT64_MAX, true);
    for (int i = 0; i < 2; ++i) {
      DevBuf &d = c->lane[i].d_in;
      if (d.cap <= keep) continue;
      d.release();
      // Every digest has gone through the sink: the kept lane is only a
      // cache, so a failed re-allocation leaves it released (the next
      // call's prepare() grows it again) and the call still succeeds.
      if (kept_cap[i] && d.ensure(std::min<uint64_t>(kept_cap[i], keep))) {
        (void)hipGetLastError();
        t_err.clear();
      }
    }
  }
  const double total = now_s() - t_start;
  bt_sha1_pipeline_stats &s = t_stats;
  memset(&s, 0, sizeof s);
  s.chunks = next;
  s.bytes = 0;
  s.batch_bytes = bytes_per;
  s.batches = (uint32_t)k;
  s.staged = feed == Feed::kStaged ? 1 : feed == Feed::kRegistered ? 2 : 0;
  s.device = c->dev;
  s.copy_threads = copy_threads();
  s.numa_nodes = numa_topo().nodes;
  s.gpu_numa_node = c->numa_node;
  s.numa_policy = place.mode();
  s.total_s = total;
  s.alloc_s = t_alloc;
  s.fill_s = t_fill;
  s.wait_s = t_wait;
  if (staged)
    for (auto &l : c->lane) page_nodes(l.h_in.p, l.h_in.cap, 64, s.lane_pages, BT_SHA1_STATS_NODES);
  for (int i = 0; i < BT_SHA1_STATS_NODES; ++i) s.copy_pieces[i] = piece_nodes[i].load();
  t_stats_valid = true;
  if (trace_on())
    fprintf(stderr, "libbtsha1 pipeline dev %d: %llu chunks, batch %llu B, %s: total %.4f s = alloc %.4f + fill %.4f "
                    "+ wait %.4f + other\n",
            c->dev, (unsigned long long)next, (unsigned long long)bytes_per,
            staged ? "staged" : feed == Feed::kRegistered ? "registered batch by batch" : "direct DMA", total, t_alloc,
            t_fill, t_wait);
  return (int64_t)next;
}

// Pageable input to bt_sha1_chunks_host: page-lock it batch by batch and DMA
// it in place (default), or copy it into the staging lanes
// (BT_SHA1_PAGEABLE=stage).  The staging copy is host memory bandwidth and
// CPU time -- 8 threads moving every byte once more -- so its rate follows
// whatever else the host's cores and memory are doing (profiles/r06: 34-50
// GiB/s on shared hosts); registering a 1 GiB batch's pages costs well under
// its 20 ms DMA and hides behind the previous batch's copy, so the pageable
// path runs at the registered-image rate.  Inputs under kRegisterMin stay
// staged (a few ms of copying at most).
constexpr uint64_t kRegisterMin = 64ull << 20;
// Column-split last batch (chunks_host_on): columns per chunk (8 by default;
// BT_SHA1_COLUMNS overrides, 2..16, 0 or 1 = off), for chunks of at least
// kColumnMinChunk (a chain's latency scales with the chunk) and a split part
// of at least column_min_bytes() (256 MiB; BT_SHA1_COLUMN_MIN_MB overrides:
// below that the columns' copies are shorter than the previous batch's hash,
// which then ends the call anyway).
constexpr uint64_t kColumnMinChunk = 64ull << 10;
uint64_t column_min_bytes() {
  static const uint64_t v = [] {
    const char *e = getenv("BT_SHA1_COLUMN_MIN_MB");
    const long mb = e ? atol(e) : 256;
    return (uint64_t)(mb < 0 ? 0 : mb) << 20;
  }();
  return v;
}
uint32_t columns() {
  static const uint32_t v = [] {
    const char *e = getenv("BT_SHA1_COLUMNS");
    const long x = e ? atol(e) : 8;
    return (uint32_t)(x < 2 ? 0 : (x > (long)kMaxColumns ? kMaxColumns : x));
  }();
  return v;
}
std::atomic<int> g_pageable_feed{-1};  // BT_SHA1_PAGEABLE_REGISTER / _STAGE; -1: not read yet
int pageable_feed() {
  int v = g_pageable_feed.load();
  if (v < 0) {
    const char *e = getenv("BT_SHA1_PAGEABLE");
    const int env = (e && !strcmp(e, "stage")) ? BT_SHA1_PAGEABLE_STAGE : BT_SHA1_PAGEABLE_REGISTER;
    g_pageable_feed.compare_exchange_strong(v, env);
    v = g_pageable_feed.load();
  }
  return v;
}
bool register_pageable() { return pageable_feed() == BT_SHA1_PAGEABLE_REGISTER; }

// own: a worker context of this call (repeated device ids); NULL = the
// device's shared context.
int64_t chunks_host_on(int dev, const uint8_t *h_in, uint64_t total, uint64_t chunk_len, uint8_t *h_dig,
                       DevCtx *own = nullptr) {
  if (chunk_len == 0 || chunk_len >= (1ull << 32)) {  // before any chunk arithmetic
    set_err("chunk_len must be in [1, 4 GiB)");
    return -1;
  }
  KeepDevice keep_dev;
  DevCtx *c = own ? own : ctx_for(dev);
  if (!c) return -1;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(dev) != hipSuccess) {
    set_err("hipSetDevice(%d) failed", dev);
    return -1;
  }
  const bool pinned = is_pinned_range(h_in, total);
  const Feed feed = pinned ? Feed::kDirect
                    : (register_pageable() && total >= kRegisterMin) ? Feed::kRegistered
                                                                      : Feed::kStaged;
  uint64_t off = 0;
  // Registered feed, per batch [b0, b1) of the input: the whole pages inside
  // it, [p0, p1), are page-locked and DMA'd in place; the head [b0, p0) and
  // tail [p1, b1) -- under a page each, shared with the neighbouring batch's
  // pages -- go through the lane's small pinned edge buffer.  Pages that
  // cannot be registered (read-only, registered by the caller elsewhere) are
  // staged through the lane instead.  Every batch is locked before the first
  // copy is queued (pages locked before: ~0.1 ms per 8 GiB; never locked:
  // 14-22 ms per 8 GiB under the ROCm 7.2 runtime, 69-92 ms under the 7.0
  // runtime torch bundles, however the locking is placed -- per batch ahead
  // of its DMA, on a helper thread, or all up front; profiles/r06).
  //
  // Column-split last batch (registered and direct feeds).  A pipeline's last
  // chunks can only be hashed once copied, and a chunk's hash is one serial
  // chain (~6.8 ms per 512 KiB in k_sha1_lat), so an unsplit pipeline ends a
  // chain latency after its last byte crossed PCIe (profiles/r06: 6.8 of the
  // 158 ms an 8 GiB image takes).  The last ~batch of chunks is therefore
  // copied COLUMN by column: columns() 2D copies (rows = the chunks, W =
  // chunk_len / columns() bytes of each; the DMA engine runs them at the 1D
  // rate, tools/copy2d_probe.py) into the idle lane's device buffer, column-
  // major, each hashed by k_sha1_lat's column form (chaining state in HBM) as
  // soon as it has arrived, on a stream of its own, while the next column
  // crosses PCIe.  After the last byte only one column's W/64 blocks remain
  // (~0.9 ms for 512 KiB chunks in 8 columns).  The copies read every byte of
  // their rows, so with the registered feed those rows' pages are locked too
  // -- but never a page reaching past the input (the page holding its end or
  // start may belong to a neighbour: another worker's slice, another call's
  // buffer); the one to three chunks touching such a page, and a short last
  // chunk, are copied into a pinned buffer on the host and hashed from there
  // by the chain kernel on a third stream, beside the columns.
  const uint64_t nchunks = (total + chunk_len - 1) / chunk_len, nfull = total / chunk_len, rem = total % chunk_len;
  struct Split {
    uint64_t t0 = 0, c0 = 0, c1 = 0;  // the split tail: chunks [t0, nchunks); by columns: [c0, c1)
    uint32_t parts = 0, width = 0;    // columns and their width
    bool head = false;                // chunk t0 is a leftover (c0 == t0 + 1)
    void *lock = nullptr;             // registered feed: the columns' locked pages
  } sp;
  const double t_lock0 = now_s();
  {
    uint32_t parts = columns();
    while (parts >= 2 && chunk_len % (64ull * parts)) parts /= 2;
    // about one batch of this feed, never more than a kept lane holds
    // (1 GiB: the idle lane carries the columns, and a staged lane is never
    // shrunk after the call)
    const uint64_t per = std::min<uint64_t>(batch_bytes_for(chunk_len, total, feed == Feed::kStaged),
                                            batch_bytes_for(chunk_len, UINT64_MAX, true)) /
                         chunk_len;
    const uint64_t t0 = nchunks - std::min<uint64_t>(nchunks, per);
    uint64_t c0 = t0, c1 = nfull;
    const uintptr_t base = (uintptr_t)h_in;
    uintptr_t lo = 0, hi = 0;
    if (feed == Feed::kRegistered) {
      const uint64_t bound = ((base + total) & ~(uintptr_t)(kPage - 1)) - base;  // the input's last page boundary
      c1 = std::min<uint64_t>(nfull, bound / chunk_len);  // chunks [0, c1) end at or before it
      if (((base + c0 * chunk_len) & ~(uintptr_t)(kPage - 1)) < base) ++c0;  // t0 == 0, unaligned start
      lo = (base + c0 * chunk_len) & ~(uintptr_t)(kPage - 1);
      hi = (base + c1 * chunk_len + kPage - 1) & ~(uintptr_t)(kPage - 1);
    }
    if (parts >= 2 && chunk_len >= kColumnMinChunk && c1 > c0 + 1 && (c1 - c0) * chunk_len >= column_min_bytes() &&
        !c->h_cdig.ensure(20 * (nchunks - t0 + 3)) && !c->h_cleft.ensure(3 * chunk_len) &&
        !c->d_cstate.ensure(20 * (c1 - c0))) {
      bool ok = true;
      if (feed == Feed::kRegistered) {
        ok = hipHostRegister((void *)lo, (size_t)(hi - lo), hipHostRegisterPortable) == hipSuccess;
        if (ok) {
          sp.lock = (void *)lo;
          if (trace_on())
            fprintf(stderr, "libbtsha1 lock column tail: [%p, %p)\n", (void *)lo, (void *)hi);
        } else {
          (void)hipGetLastError();  // copied with the rest
        }
      }
      if (ok) {
        sp.t0 = t0;
        sp.c0 = c0;
        sp.c1 = c1;
        sp.parts = parts;
        sp.width = (uint32_t)(chunk_len / parts);
        sp.head = c0 > t0;
      }
    }
    t_err.clear();
  }
  const uint64_t dma_total = sp.parts ? sp.t0 * chunk_len : total;  // the part the lane batches carry
  const uint64_t batch = batch_bytes_for(chunk_len, dma_total, false);
  const size_t nbatch = feed == Feed::kRegistered ? (size_t)((dma_total + batch - 1) / batch) : 0;
  std::vector<uint64_t> bp0(nbatch), bp1(nbatch);
  std::vector<char> blocked(nbatch, 0);
  // Locked ranges stay locked until the whole call is done: hipHostUnregister
  // waits for the device's outstanding work, so releasing a batch's pages
  // while the next batch's copy and hash are in flight stalled the pipeline
  // (40.5 GiB/s instead of 50.7 on 8 GiB, profiles/r06).  At the end nothing
  // is in flight and each release is quick; on an error path the streams are
  // drained first.
  std::vector<void *> regs;
  bool split_queued = false;
  struct DrainAtExit {
    DevCtx *c;
    std::vector<void *> &regs;
    bool &queued;
    ~DrainAtExit() {
      if (regs.empty() && !queued) return;
      for (auto &l : c->lane)
        if (l.s) (void)hipStreamSynchronize(l.s);
      for (hipStream_t t : {c->cs, c->xs})
        if (t) (void)hipStreamSynchronize(t);
      for (void *p : regs) (void)hipHostUnregister(p);
    }
  } drain_at_exit{c, regs, split_queued};
  if (sp.lock) regs.push_back(sp.lock);
  double lock_s = now_s() - t_lock0;
  if (nbatch) {
    const double t0 = now_s();
    const uintptr_t base = (uintptr_t)h_in;
    for (size_t k = 0; k < nbatch; ++k) {
      const uint64_t lo = k * batch, hi = std::min<uint64_t>(lo + batch, dma_total);
      bp0[k] = ((base + lo + kPage - 1) & ~(uintptr_t)(kPage - 1)) - base;
      bp1[k] = ((base + hi) & ~(uintptr_t)(kPage - 1)) - base;
      if (bp1[k] <= bp0[k]) {
        bp0[k] = bp1[k] = hi;  // no whole page: the batch (< 2 pages) rides in the edge buffer
        continue;
      }
      if (hipHostRegister((void *)(h_in + bp0[k]), (size_t)(bp1[k] - bp0[k]), hipHostRegisterPortable) == hipSuccess) {
        regs.push_back((void *)(h_in + bp0[k]));
        blocked[k] = 1;
        if (trace_on())
          fprintf(stderr, "libbtsha1 lock batch %zu: [%p, %p)\n", k, (const void *)(h_in + bp0[k]),
                  (const void *)(h_in + bp1[k]));
      } else {
        (void)hipGetLastError();  // that batch is staged
      }
    }
    lock_s += now_s() - t0;
  }
  // The columns land in the lane that is idle once the last batch is queued
  // (its previous batch's hash precedes them on its stream): sized for them
  // up front, never grown while a batch may still read it -- its device
  // buffer, and for the staged feed its staging (on the GPU's node, as the
  // pipeline places it), where the copy threads gather the columns.
  if (sp.parts) {
    const bool staged = feed == Feed::kStaged;
    const uint64_t lane_batch = batch_bytes_for(chunk_len, dma_total, staged);
    const int k_last = dma_total ? (int)((dma_total + lane_batch - 1) / lane_batch) : 0;
    const uint64_t need = std::max<uint64_t>((sp.c1 - sp.c0) * chunk_len, dma_total ? lane_batch : 0);
    Lane &idle = c->lane[k_last & 1];
    if (idle.d_in.ensure(need)) return -1;
    if (staged) {
      if (c->numa_node == -2) c->numa_node = gpu_numa_node(c->dev);
      if (idle.h_in.ensure(need, placement_for(c->numa_node).node)) return -1;
    }
  }
  uint64_t b1 = 0, p0 = 0, p1 = 0;
  bool locked = false;
  auto fill = [&](Lane &l, uint64_t at, uint64_t max, const uint8_t **src, bool *eof) -> int64_t {
    uint64_t n = std::min<uint64_t>(max, dma_total - off);
    if (feed == Feed::kDirect) {
      *src = h_in + off;  // DMA straight from the caller's pinned image
    } else if (feed == Feed::kStaged) {
      parallel_copy(l.h_in.as<uint8_t>() + at, h_in + off, n);
      *src = l.h_in.as<uint8_t>() + at;
    } else {
      if (at == 0) {  // a new batch
        const size_t k = (size_t)(off / batch);
        p0 = bp0[k];
        p1 = bp1[k];
        b1 = std::min<uint64_t>((k + 1) * batch, dma_total);
        locked = blocked[k] != 0;
      }
      uint8_t *edge = l.h_edge.as<uint8_t>();
      if (off < p0) {  // head, or a batch without a whole page
        n = std::min<uint64_t>(n, p0 - off);
        memcpy(edge, h_in + off, n);
        *src = edge;
      } else if (off < p1) {
        n = std::min<uint64_t>(n, p1 - off);
        if (locked) {
          *src = h_in + off;
        } else {
          if (l.h_in.ensure(batch_bytes_for(chunk_len, total, false), -1)) return -1;
          parallel_copy(l.h_in.as<uint8_t>() + at, h_in + off, n);
          *src = l.h_in.as<uint8_t>() + at;
        }
      } else {  // tail
        n = std::min<uint64_t>(n, b1 - off);
        memcpy(edge + kPage, h_in + off, n);
        *src = edge + kPage;
      }
    }
    off += n;
    *eof = off == dma_total;
    return (int64_t)n;
  };

  auto sink = [&](uint64_t first, uint64_t count, const uint8_t *d) { memcpy(h_dig + 20 * first, d, 20 * count); };
  // The split tail: leftovers first (their chain runs beside the columns),
  // then each column's copy on the idle lane's stream and its hash on the
  // column stream once that copy is done.  Digest j of the tail (chunk t0 + j)
  // goes to h_cdig + 20*j; the leftovers' own launch writes theirs after the
  // tail's (h_cdig + 20*(nchunks - t0) ..) and they are moved into place.
  const uint64_t ntail = nchunks - sp.t0, rows = sp.c1 - sp.c0, nleft_full = (sp.head ? 1 : 0) + (nfull - sp.c1);
  double t_gather = 0;  // staged feed: host time gathering the columns
  auto queue_split = [&](Lane &idle, hipEvent_t last_copied) -> int {
    if (!sp.parts) return 0;
    if (!c->cs) {
      BT_CK(hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
      BT_CK(hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking));
      BT_CK(hipEventCreateWithFlags(&c->cdone, hipEventDisableTiming));
      BT_CK(hipEventCreateWithFlags(&c->xdone, hipEventDisableTiming));
    }
    split_queued = true;
    uint8_t *left = c->h_cleft.as<uint8_t>(), *tdig = c->h_cdig.as<uint8_t>();
    if (nleft_full || rem) {
      uint64_t at = 0;
      if (sp.head) {
        memcpy(left, h_in + sp.t0 * chunk_len, chunk_len);
        at = chunk_len;
      }
      memcpy(left + at, h_in + sp.c1 * chunk_len, total - sp.c1 * chunk_len);
      BT_CK(btsha1_launch_chain(left, nullptr, nullptr, chunk_len, chunk_len, nleft_full, tdig + 20 * ntail, c->xs,
                                rem));
    }
    BT_CK(hipEventRecord(c->xdone, c->xs));
    if (last_copied) BT_CK(hipStreamWaitEvent(idle.s, last_copied, 0));
    // Staged feed: the copy threads gather each column into the idle lane's
    // staging (free once its previous batch is done) while the previous
    // column crosses PCIe; pinned / locked input: one strided copy per column.
    const bool staged = feed == Feed::kStaged;
    if (staged && idle.busy) BT_CK(hipEventSynchronize(idle.ev));
    uint8_t *cols = idle.d_in.as<uint8_t>(), *stage = staged ? idle.h_in.as<uint8_t>() : nullptr;
    uint32_t *state = c->d_cstate.as<uint32_t>();
    const uint64_t w = sp.width;
    for (uint32_t j = 0; j < sp.parts; ++j) {
      if (!c->cev[j]) BT_CK(hipEventCreateWithFlags(&c->cev[j], hipEventDisableTiming));
      const uint8_t *src = h_in + sp.c0 * chunk_len + j * w;
      hipError_t ce;
      if (staged) {
        const double g0 = now_s();
        parallel_gather(stage + j * rows * w, src, rows, w, chunk_len);
        t_gather += now_s() - g0;
        ce = hipMemcpyAsync(cols + j * rows * w, stage + j * rows * w, (size_t)(rows * w), hipMemcpyHostToDevice,
                            idle.s);
      } else {
        ce = hipMemcpy2DAsync(cols + j * rows * w, (size_t)w, src, (size_t)chunk_len, (size_t)w, (size_t)rows,
                              hipMemcpyHostToDevice, idle.s);
      }
      if (ce != hipSuccess) {
        set_err("copy of column %u (%llu x %llu bytes, pitch %llu) from host %p failed: %s", j,
                (unsigned long long)rows, (unsigned long long)w, (unsigned long long)chunk_len, (const void *)src,
                hipGetErrorString(ce));
        return -1;
      }
      BT_CK(hipEventRecord(c->cev[j], idle.s));
      BT_CK(hipStreamWaitEvent(c->cs, c->cev[j], 0));
      const int part = j == 0 ? BTSHA1_COLUMN_FIRST : j + 1 == sp.parts ? BTSHA1_COLUMN_LAST : BTSHA1_COLUMN_MIDDLE;
      BT_CK(btsha1_launch_column(cols + j * rows * w, rows, (uint32_t)w, (uint32_t)w, part, state, chunk_len,
                                 tdig + 20 * (sp.c0 - sp.t0), c->cs));
    }
    BT_CK(hipEventRecord(c->cdone, c->cs));
    return 0;
  };
  auto wait_split = [&]() -> int {
    if (!split_queued) return 0;
    BT_CK(hipEventSynchronize(c->cdone));
    BT_CK(hipEventSynchronize(c->xdone));
    return 0;
  };
  int64_t n = run_pipeline(c, chunk_len, dma_total, feed, fill, sink, tail_ops(queue_split, wait_split));
  if (n >= 0 && sp.parts) {  // the tail's digests follow the batches'
    if ((uint64_t)n != sp.t0) {
      set_err("internal: %lld chunks before the split tail, expected %llu", (long long)n,
              (unsigned long long)sp.t0);
      n = -1;
    } else {
      const uint8_t *tdig = c->h_cdig.as<uint8_t>();
      uint8_t *out = h_dig + 20 * sp.t0;
      memcpy(out + 20 * (sp.c0 - sp.t0), tdig + 20 * (sp.c0 - sp.t0), 20 * rows);
      const uint8_t *ld = tdig + 20 * ntail;  // leftovers: [head] [c1, nchunks)
      if (sp.head) {
        memcpy(out, ld, 20);
        ld += 20;
      }
      memcpy(out + 20 * (sp.c1 - sp.t0), ld, 20 * (nchunks - sp.c1));
      n = (int64_t)nchunks;
      if (t_stats_valid) {
        t_stats.chunks = nchunks;
        t_stats.column_chunks = (uint32_t)rows;
        t_stats.fill_s += t_gather;
      }
    }
  }
  if (n >= 0 && t_stats_valid) {
    t_stats.bytes = total;
    page_nodes(h_in, total, 64, t_stats.src_pages, BT_SHA1_STATS_NODES);
  }
  if (n >= 0 && !regs.empty()) {  // every batch is done: release the pages (timed)
    const double t0 = now_s();
    for (void *p : regs)
      if (hipHostUnregister(p) != hipSuccess) (void)hipGetLastError();
    const double dt = now_s() - t0;
    if (t_stats_valid) {
      t_stats.registered_batches = (int32_t)(regs.size() - (sp.lock ? 1 : 0));
      t_stats.register_s = lock_s;
      t_stats.unregister_s = dt;
      t_stats.total_s += lock_s + dt;
    }
    regs.clear();
  }
  split_queued = false;  // waited for by the pipeline
  return n;
}

template <class Sink>
int64_t chunks_file_on(int dev, FILE *fp, uint64_t chunk_len, Sink sink) {
  KeepDevice keep_dev;
  DevCtx *c = ctx_for(dev);
  if (!c) return -1;
  std::lock_guard<std::mutex> g(c->mu);
  if (hipSetDevice(dev) != hipSuccess) {
    set_err("hipSetDevice(%d) failed", dev);
    return -1;
  }
  uint64_t hint = UINT64_MAX;
  struct stat st;
  const off_t pos = ftello(fp);
  const bool regular = fstat(fileno(fp), &st) == 0 && S_ISREG(st.st_mode) && pos >= 0 && st.st_size >= pos;
  if (regular) hint = (uint64_t)(st.st_size - pos);
  uint64_t fpos = regular ? (uint64_t)pos : 0;
  auto fill = [&](Lane &l, uint64_t at, uint64_t max, const uint8_t **src, bool *eof) -> int64_t {
    uint8_t *dst = l.h_in.as<uint8_t>() + at;
    *src = dst;
    if (regular) {
      // Regular file: several threads pread the batch straight into pinned
      // memory at the FILE's logical position; short only at EOF.
      const int64_t got = parallel_pread(fileno(fp), dst, max, fpos);
      if (got < 0) {
        set_err("pread failed: %s", strerror(errno));
        return -1;
      }
      fpos += (uint64_t)got;
      *eof = (uint64_t)got < max;
      return got;
    }
    // Pipe or device: fread to EOF as chunk.c:20 does.
    size_t got = 0;
    while (got < max) {
      size_t r = fread(dst + got, 1, (size_t)(max - got), fp);
      if (r == 0) break;
      got += r;
    }
    if (ferror(fp)) {
      set_err("fread failed");
      return -1;
    }
    *eof = got < max;
    return (int64_t)got;
  };
  uint64_t bytes_in = 0;
  auto counted_fill = [&](Lane &l, uint64_t at, uint64_t max, const uint8_t **src, bool *eof) -> int64_t {
    const int64_t r = fill(l, at, max, src, eof);
    if (r > 0) bytes_in += (uint64_t)r;
    return r;
  };
  const int64_t n = run_pipeline(c, chunk_len, hint, Feed::kStaged, counted_fill, sink, no_tail());
  if (n >= 0 && t_stats_valid) t_stats.bytes = bytes_in;
  if (regular) {
    // Leave the stream where the reference's fread loop leaves it: at EOF,
    // with the end-of-file indicator set.
    if (fseeko(fp, (off_t)fpos, SEEK_SET) == 0) {
      const int ch = fgetc(fp);
      if (ch != EOF) ungetc(ch, fp);
    }
  }
  return n;
}

// Wait for a drop-in call's chain kernel: spin on the completion word it
// stores into pinned memory after its results (a stream wait sleeps and wakes
// late; ~354 such waits per chunk in SHA1Update's packet-sized calls).  The
// stream is polled too, so an error or a kernel that ended without the word
// cannot hang the caller, and after 1 ms the wait blocks on the stream instead
// (long messages do not burn a core; the wake-up latency is then noise).
// BT_SHA1_SYNC=stream always waits on the stream.
bool spin_sync() {
  static const bool on = [] {
    const char *e = getenv("BT_SHA1_SYNC");
    return !(e && !strcmp(e, "stream"));
  }();
  return on;
}

int wait_chain(DevCtx *c, const volatile uint32_t *done, uint32_t seq) {
  if (!spin_sync()) {
    BT_CK(hipStreamSynchronize(c->s));
    return 0;
  }
  const double t0 = now_s();
  for (uint32_t it = 0;; ++it) {
    if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) return 0;
    if ((it & 1023u) == 1023u && now_s() - t0 > 1e-3) {
      BT_CK(hipStreamSynchronize(c->s));
      if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) return 0;
      set_err("chain kernel finished without its completion word");
      return -1;
    }
    if ((it & 63u) == 63u) {
      const hipError_t q = hipStreamQuery(c->s);
      if (q == hipSuccess) {
        if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == seq) return 0;
        set_err("chain kernel finished without its completion word");
        return -1;
      }
      if (q != hipErrorNotReady) {
        set_err("chain kernel: %s", hipGetErrorString(q));
        return -1;
      }
    }
  }
}

uint32_t *done_word(DevCtx *c) { return reinterpret_cast<uint32_t *>(c->h_state.as<uint8_t>() + 32); }

// The reference leaves no copy of the message or of the chaining state behind
// a call: shahash zeroes its context (chunk.c:48) and SHA1Update burns its
// stack frame (sha.c:165-174, 526).  The drop-in's copies live in the
// context's pinned staging, so each call zeroes what it staged there once the
// chain kernel has finished with it (explicit_bzero: not elided as a dead
// store).  The completion word at h_state + 32 is a sequence number, not data.
constexpr size_t kStateBytes = 32;
void wipe_staging(DevCtx *c, size_t msg_bytes) {
  if (msg_bytes) explicit_bzero(c->h_msg.p, std::min(msg_bytes, c->h_msg.cap));
  explicit_bzero(c->h_state.p, kStateBytes);
}

// Single message on the GPU (shahash): copy it into the context's pinned
// staging buffer and launch the chain kernel on it there -- the kernel reads
// the message over PCIe itself (64 blocks per load batch, far ahead of the
// round wave) and writes the digest straight into pinned memory -- so one
// synchronous call is one memcpy, one launch and a wait on the kernel's
// completion word: no H2D or D2H copies (each a queue round trip of its own).
int hash_one(DevCtx *c, const uint8_t *buf, uint32_t len, uint8_t out[20]) {
  if (ensure_streams(c)) return -1;
  if (c->h_msg.ensure((size_t)len + 64) || c->h_state.ensure(64)) return -1;
  if (len) memcpy(c->h_msg.p, buf, len);
  const uint32_t seq = ++c->seq;
  *done_word(c) = seq - 1u;
  const hipError_t e = btsha1_launch_chain_one(c->h_msg.p, len, c->h_state.as<uint8_t>(), c->s, done_word(c), seq);
  if (e != hipSuccess) set_err("chain kernel launch: %s", hipGetErrorString(e));
  const int rc = e != hipSuccess ? -1 : wait_chain(c, done_word(c), seq);
  if (!rc) memcpy(out, c->h_state.p, 20);
  wipe_staging(c, len);
  return rc;
}

// Advance h over `head` (0 or 64 bytes: SHA1Update's completed staging block)
// followed by nblocks whole blocks at host address `blocks`: both go straight
// into pinned memory with the state, the chain kernel reads them from there
// and writes the state back in place (one launch, one wait per call).
int midstate(DevCtx *c, uint32_t h[5], const uint8_t *head, const uint8_t *blocks, uint64_t nblocks) {
  const uint64_t total = nblocks + (head ? 1 : 0);
  if (!total) return 0;
  if (ensure_streams(c)) return -1;
  if (c->h_msg.ensure((size_t)total * 64) || c->h_state.ensure(64)) return -1;
  uint8_t *dst = c->h_msg.as<uint8_t>();
  if (head) memcpy(dst, head, 64);
  if (nblocks) memcpy(dst + (head ? 64 : 0), blocks, (size_t)nblocks * 64);
  memcpy(c->h_state.p, h, 20);
  nblocks = total;
  const uint32_t seq = ++c->seq;
  *done_word(c) = seq - 1u;
  const hipError_t e = btsha1_launch_chain_midstate(c->h_state.as<uint32_t>(), c->h_msg.p, nblocks, c->s,
                                                    done_word(c), seq);
  if (e != hipSuccess) set_err("chain kernel launch: %s", hipGetErrorString(e));
  const int rc = e != hipSuccess ? -1 : wait_chain(c, done_word(c), seq);
  if (!rc) memcpy(h, c->h_state.p, 20);
  wipe_staging(c, (size_t)total * 64);
  return rc;
}

DevCtx *dropin_ctx(const char *who) {
  DevCtx *c = ctx_for(t_dev);
  if (!c) die(who);
  if (hipSetDevice(t_dev) != hipSuccess) {
    set_err("hipSetDevice(%d) failed", t_dev);
    die(who);
  }
  return c;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int bt_sha1_device_count(void) { return device_count(); }

int bt_sha1_set_device(int device) {
  int n = device_count();
  if (device < 0 || device >= n) {
    set_err("device %d out of range (%d visible)", device, n);
    return -1;
  }
  t_dev = device;
  return 0;
}

const char *bt_sha1_last_error(void) { return t_err.c_str(); }

#ifndef BT_SHA1_SRC_ID
#define BT_SHA1_SRC_ID "unknown"
#endif

const char *bt_sha1_build_info(void) {
  static thread_local char info[192];
  const uint64_t lat = btsha1_latency_batch_setting();
  char latbuf[48];
  if (lat == BT_SHA1_LATENCY_AUTO)
    snprintf(latbuf, sizeof latbuf, "auto");
  else
    snprintf(latbuf, sizeof latbuf, "%llu", (unsigned long long)lat);
  snprintf(info, sizeof info, "libbtsha1 gfx950 hip%d.%d ring=%d latency_batch=%s src=%s", HIP_VERSION_MAJOR,
           HIP_VERSION_MINOR, g_variant.load(), latbuf, BT_SHA1_SRC_ID);
  return info;
}

const char *bt_sha1_source_id(void) { return BT_SHA1_SRC_ID; }

int bt_sha1_set_ring_depth(int nbuf) { return bt_sha1_set_variant(nbuf, 1, 0); }

uint64_t bt_sha1_set_latency_batch(uint64_t max_chunks) {
  const uint64_t prev = btsha1_latency_batch_setting();
  btsha1_set_latency_batch(max_chunks);
  return prev;
}

uint64_t bt_sha1_set_chain_batch(uint64_t max_messages) {
  const uint64_t prev = btsha1_chain_batch_setting();
  btsha1_set_chain_batch(max_messages);
  return prev;
}

const char *bt_sha1_kernel_name(uint64_t n_chunks) {
  if (device_count() <= 0) {
    set_err("no HIP device visible");
    return nullptr;
  }
  return btsha1_fixed_kernel_name(n_chunks, g_variant.load());
}

int bt_sha1_clock_probe(const void *d_in, uint64_t n, uint64_t chunk_len, uint64_t pitch, uint8_t *d_digests,
                        uint64_t *d_stamps, void *stream) {
  if (n == 0) return 0;
  if (!d_in || !d_digests || !d_stamps) {
    set_err("null pointer");
    return -1;
  }
  if (!fast_layout(d_in, chunk_len, pitch, d_digests)) {
    set_err("clock probe needs the hot kernel's layout");
    return -1;
  }
  int dev = 0;
  BT_CK(hipGetDevice(&dev));
  if (!ctx_for(dev)) return -1;
  BT_CK(btsha1_launch_fixed_stamped(d_in, n, (uint32_t)pitch, (uint32_t)chunk_len, d_digests, d_stamps,
                                    pick_stream(stream), g_variant.load()));
  return 0;
}

int64_t bt_sha1_wallclock_khz(void) {
  int dev = 0, khz = 0;
  BT_CK(hipGetDevice(&dev));
  BT_CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  return khz;
}

int bt_sha1_debug_barrier_stats(uint64_t out[3], int reset) {
  if (!out) {
    set_err("null pointer");
    return -1;
  }
  const hipError_t e = btsha1_debug_barrier_stats(out, reset);
  if (e == hipErrorNotSupported) {
    set_err("barrier tallies exist only in the -DBT_SHA1_DEBUG_BARRIERS build (make dbgbar)");
    return -1;
  }
  BT_CK(e);
  return 0;
}

int64_t bt_sha1_debug_dropin_residue(int device) {
  DevCtx *c = nullptr;
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    if (device < 0) {
      set_err("device %d out of range", device);
      return -1;
    }
    if (device < (int)g_ctx.size()) c = g_ctx[device].get();
  }
  if (!c) return 0;  // no drop-in call has run on this device: nothing staged
  std::lock_guard<std::mutex> g(c->mu);
  int64_t nz = 0;
  const uint8_t *m = c->h_msg.as<uint8_t>();
  for (size_t i = 0; m && i < c->h_msg.cap; ++i) nz += m[i] != 0;
  const uint8_t *st = c->h_state.as<uint8_t>();
  for (size_t i = 0; st && i < kStateBytes; ++i) nz += st[i] != 0;
  return nz;
}

int bt_sha1_set_variant(int nbuf, int lines, int nt) {
  const int code = nbuf * 100 + lines * 10 + (nt ? 1 : 0);
  if (!btsha1_fixed_variant_ok(code)) {
    if (btsha1_experiments_build())
      set_err("no hot-kernel variant ring=%d lines=%d nt=%d", nbuf, lines, nt);
    else
      set_err("no hot-kernel variant ring=%d lines=%d nt=%d in the product library: it carries only the default "
              "(3, 1, 0); the rejected variants are in build_variants/experiments/libbtsha1.so (make experiments)",
              nbuf, lines, nt);
    return -1;
  }
  g_variant.store(code);
  return 0;
}

int bt_sha1_chunks_dev(const void *d_in, uint64_t n, uint64_t chunk_len, uint64_t pitch, uint8_t *d_digests,
                       void *stream) {
  if (n && (!d_in || !d_digests)) {
    set_err("null pointer");
    return -1;
  }
  if (n > 1 && pitch < chunk_len) {
    set_err("pitch < chunk_len");
    return -1;
  }
  if (n == 1 && pitch < chunk_len) pitch = (chunk_len + 15) & ~15ull;
  int dev = 0;
  BT_CK(hipGetDevice(&dev));
  DevCtx *c = ctx_for(dev);
  if (!c) return -1;
  hipStream_t st = pick_stream(stream);
  return launch_chunks(d_in, n, chunk_len, pitch, d_digests, st);
}

int bt_sha1_verify_dev(const void *d_in, uint64_t n, uint64_t chunk_len, uint64_t pitch, const uint8_t *d_expected,
                       uint8_t *d_ok, uint8_t *d_digests, void *stream) {
  if (n == 0) return 0;
  if (!d_in || !d_expected || !d_ok) {
    set_err("null pointer");
    return -1;
  }
  if (!fast_layout(d_in, chunk_len, pitch, d_digests)) {
    set_err("verify needs a 16-byte aligned layout with 64*pitch + 4096 <= 4 GiB");
    return -1;
  }
  int dev = 0;
  BT_CK(hipGetDevice(&dev));
  DevCtx *c = ctx_for(dev);
  if (!c) return -1;
  hipStream_t st = pick_stream(stream);
  BT_CK(btsha1_launch_fixed(d_in, n, (uint32_t)pitch, (uint32_t)chunk_len, d_digests, d_expected, d_ok, st,
                            g_variant.load()));
  return 0;
}

int bt_sha1_ragged_dev(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens, uint64_t n,
                       uint8_t *d_digests, void *stream) {
  if (n == 0) return 0;
  if (!d_base || !d_offsets || !d_lens || !d_digests) {
    set_err("null pointer");
    return -1;
  }
  int dev = 0;
  BT_CK(hipGetDevice(&dev));
  DevCtx *c = ctx_for(dev);
  if (!c) return -1;
  hipStream_t st = pick_stream(stream);
  BT_CK(btsha1_launch_ragged(d_base, d_offsets, d_lens, 0, 0, n, d_digests, st));
  return 0;
}

int bt_sha1_fill_synthetic(void *d_buf, uint64_t nbytes, uint64_t first_word, uint64_t seed, void *stream) {
  if (nbytes && (!d_buf || ((uintptr_t)d_buf & 15))) {
    set_err("fill needs a non-null 16-byte aligned buffer");
    return -1;
  }
  int dev = 0;
  BT_CK(hipGetDevice(&dev));
  DevCtx *c = ctx_for(dev);
  if (!c) return -1;
  hipStream_t st = pick_stream(stream);
  BT_CK(btsha1_launch_fill(d_buf, nbytes, first_word, seed, st));
  return 0;
}

int bt_sha1_host_register(void *h_ptr, uint64_t len) {
  if (!h_ptr || !len) {
    set_err("null pointer or zero length");
    return -1;
  }
  if (!ctx_for(t_dev)) return -1;
  BT_CK(hipHostRegister(h_ptr, (size_t)len, hipHostRegisterPortable));
  return 0;
}

int bt_sha1_host_unregister(void *h_ptr) {
  BT_CK(hipHostUnregister(h_ptr));
  return 0;
}

int bt_sha1_lookup_dev(const uint8_t *d_table, uint64_t n_table, const uint8_t *d_queries, uint64_t n_queries,
                       int64_t *d_index, void *stream) {
  if (n_queries == 0) return 0;
  if ((n_table && !d_table) || !d_queries || !d_index || ((uintptr_t)d_table & 3) || ((uintptr_t)d_queries & 3)) {
    set_err("lookup needs non-null, 4-byte aligned digest arrays");
    return -1;
  }
  if (n_table >= (1ull << 31)) {
    set_err("lookup table too large");
    return -1;
  }
  int dev = 0;
  BT_CK(hipGetDevice(&dev));
  DevCtx *c = ctx_for(dev);
  if (!c) return -1;
  hipStream_t st = pick_stream(stream);
  uint32_t cap = 1024;
  while (cap < 2 * n_table) cap <<= 1;  // load factor <= 1/2
  void *slots = nullptr;
  BT_CK(hipMallocAsync(&slots, (size_t)cap * 4, st));
  BT_CK(btsha1_launch_lookup(d_table, n_table, d_queries, n_queries, (uint32_t *)slots, cap, d_index, st));
  BT_CK(hipFreeAsync(slots, st));
  return 0;
}

int64_t bt_sha1_chunks_host(const void *h_in, uint64_t total_len, uint64_t chunk_len, uint8_t *h_digests) {
  if (total_len && (!h_in || !h_digests)) {
    set_err("null pointer");
    return -1;
  }
  if (total_len == 0) return 0;
  return chunks_host_on(t_dev, (const uint8_t *)h_in, total_len, chunk_len, h_digests);
}

int64_t bt_sha1_chunks_host_devices(const void *h_in, uint64_t total_len, uint64_t chunk_len, uint8_t *h_digests,
                                    const int *devs, int nworkers) {
  if (chunk_len == 0 || chunk_len >= (1ull << 32)) {
    set_err("chunk_len must be in [1, 4 GiB)");
    return -1;
  }
  if (nworkers <= 0 || !devs) {
    set_err("empty device list");
    return -1;
  }
  if (nworkers > kMaxWorkers) {
    set_err("%d workers: at most %d (one host thread and two staging lanes each)", nworkers, kMaxWorkers);
    return -1;
  }
  if (total_len == 0) return 0;
  if (!h_in || !h_digests) {
    set_err("null pointer");
    return -1;
  }
  const int avail = device_count();
  if (avail <= 0) {
    set_err("no HIP device visible");
    return -1;
  }
  for (int g = 0; g < nworkers; ++g)
    if (devs[g] < 0 || devs[g] >= avail) {
      set_err("device %d out of range (%d visible)", devs[g], avail);
      return -1;
    }
  const uint64_t n = (total_len + chunk_len - 1) / chunk_len;
  // Contiguous block split of the chunk index: worker g gets
  // [g*n/G, (g+1)*n/G) -- possibly empty when G > n; only the globally last
  // chunk can be short.  One host thread per worker; a device listed k times
  // gets k independent contexts (streams + staging lanes), so the split,
  // staging and ordered gather run exactly as on k distinct GPUs.  The first
  // use of a device takes its shared context; the repeats get contexts of
  // their own that are released (buffers, streams) before the call returns.
  std::vector<int64_t> rc(nworkers, 0);
  std::vector<std::string> errs(nworkers);
  std::vector<std::unique_ptr<DevCtx>> own(nworkers);
  for (int g = 0; g < nworkers; ++g)
    for (int h = 0; h < g; ++h)
      if (devs[h] == devs[g]) {
        own[g] = std::make_unique<DevCtx>();
        own[g]->dev = devs[g];
        break;
      }
  struct ReleaseAtExit {
    std::vector<std::unique_ptr<DevCtx>> &v;
    ~ReleaseAtExit() {
      for (auto &c : v) release_ctx(c.get());
    }
  } release_at_exit{own};
  std::vector<std::thread> th;
  for (int g = 0; g < nworkers; ++g) {
    th.emplace_back([&, g] {
      const uint64_t lo = n * g / nworkers, hi = n * (g + 1) / nworkers;
      if (lo == hi) return;
      const uint64_t off = lo * chunk_len;
      const uint64_t bytes = std::min<uint64_t>(hi * chunk_len, total_len) - off;
      rc[g] = chunks_host_on(devs[g], (const uint8_t *)h_in + off, bytes, chunk_len, h_digests + 20 * lo, own[g].get());
      if (rc[g] >= 0 && (uint64_t)rc[g] != hi - lo) {
        rc[g] = -1;
        t_err = "short digest count";
      }
      errs[g] = t_err;
    });
  }
  for (auto &t : th) t.join();
  for (int g = 0; g < nworkers; ++g)
    if (rc[g] < 0) {
      t_err = "worker " + std::to_string(g) + " (device " + std::to_string(devs[g]) + "): " + errs[g];
      return -1;
    }
  return (int64_t)n;
}

int64_t bt_sha1_chunks_host_multi(const void *h_in, uint64_t total_len, uint64_t chunk_len, uint8_t *h_digests,
                                  int ndev) {
  const int avail = device_count();
  if (avail <= 0) {
    set_err("no HIP device visible");
    return -1;
  }
  if (ndev <= 0 || ndev > avail) ndev = avail;
  std::vector<int> devs(ndev);
  for (int g = 0; g < ndev; ++g) devs[g] = g;
  return bt_sha1_chunks_host_devices(h_in, total_len, chunk_len, h_digests, devs.data(), ndev);
}

int bt_sha1_set_pageable_feed(int feed) {
  if (feed != BT_SHA1_PAGEABLE_REGISTER && feed != BT_SHA1_PAGEABLE_STAGE) {
    set_err("pageable feed %d: BT_SHA1_PAGEABLE_REGISTER (0) or BT_SHA1_PAGEABLE_STAGE (1)", feed);
    return -1;
  }
  const int prev = pageable_feed();
  g_pageable_feed.store(feed);
  return prev;
}

int bt_sha1_get_pipeline_stats(bt_sha1_pipeline_stats *out) {
  if (!out) {
    set_err("null pointer");
    return -1;
  }
  if (!t_stats_valid) {
    set_err("no host pipeline has run on this thread");
    return -1;
  }
  *out = t_stats;
  return 0;
}

int64_t bt_sha1_chunks_file(void *fp, uint64_t chunk_len, uint8_t *h_digests, uint64_t max_chunks) {
  if (!fp || !h_digests) {
    set_err("null pointer");
    return -1;
  }
  bool overflow = false;
  int64_t n = chunks_file_on(t_dev, (FILE *)fp, chunk_len, [&](uint64_t first, uint64_t count, const uint8_t *d) {
    for (uint64_t i = 0; i < count; ++i) {
      if (first + i >= max_chunks) {
        overflow = true;
        return;
      }
      memcpy(h_digests + 20 * (first + i), d + 20 * i, 20);
    }
  });
  if (n >= 0 && overflow) {
    set_err("file has more than max_chunks chunks");
    return -1;
  }
  return n;
}

// ---- drop-in: chunk.h --------------------------------------------------------

// chunk.c:13-25.  Same contract: reads fp to EOF in BT_CHUNK_SIZE pieces,
// digest i -> chunk_hashes[i] (caller-sized, as make_chunks.c:32-45 does).
int make_chunks(FILE *fp, uint8_t **chunk_hashes) {
  if (!fp || !chunk_hashes) {
    set_err("null pointer");
    return -1;
  }
  int64_t n = chunks_file_on(t_dev, fp, BT_CHUNK_SIZE, [&](uint64_t first, uint64_t count, const uint8_t *d) {
    for (uint64_t i = 0; i < count; ++i) memcpy(chunk_hashes[first + i], d + 20 * i, 20);
  });
  if (n < 0) {
    fprintf(stderr, "make_chunks: %s\n", t_err.c_str());
    return -1;
  }
  return (int)n;
}

// chunk.c:33-49 (int length, like the reference).
void shahash(uint8_t *str, int len, uint8_t *hash) {
  if (len < 0) {
    set_err("negative length %d", len);
    die("shahash");
  }
  KeepDevice keep_dev;
  DevCtx *c = dropin_ctx("shahash");
  std::lock_guard<std::mutex> g(c->mu);
  if (hash_one(c, str, (uint32_t)len, hash)) die("shahash");
}

// chunk.c:55-61: "%.2x" per byte, NUL-terminated.
void binary2hex(uint8_t *buf, int len, char *hex) {
  static const char dig[] = "0123456789abcdef";
  for (int i = 0; i < len; ++i) {
    hex[2 * i] = dig[buf[i] >> 4];
    hex[2 * i + 1] = dig[buf[i] & 15];
  }
  hex[len < 0 ? 0 : 2 * len] = 0;
}

// chunk.c:66-83: toupper, '0'..'9' -> 0..9, otherwise ch - ('A' - 10); no
// validation (kept bug-compatible: garbage in, garbage out).
static inline uint8_t hexval(char ch) {
  if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
  return (uint8_t)(ch <= '9' ? ch - '0' : ch - ('A' - 10));
}
void hex2binary(char *hex, int len, uint8_t *buf) {
  for (int i = 0; i < len; i += 2) buf[i / 2] = (uint8_t)((hexval(hex[i]) << 4) | hexval(hex[i + 1]));
}

// ---- drop-in: sha.h ------------------------------------------------------------

void SHA1Init(SHA1Context *sc) {  // sha.c:149-163
  sc->totalLength = 0;
  sc->hash[0] = 0x67452301u;
  sc->hash[1] = 0xefcdab89u;
  sc->hash[2] = 0x98badcfeu;
  sc->hash[3] = 0x10325476u;
  sc->hash[4] = 0xc3d2e1f0u;
  sc->bufferLength = 0;
}

// sha.c:453-527: bytes top up the 64-byte staging block; every completed
// block (the staged one plus all whole blocks of `data`) is compressed in one
// GPU call; the remainder is staged.  totalLength counts bits like sha.c:511.
void SHA1Update(SHA1Context *sc, const void *vdata, uint32_t len) {
  if (!len) return;
  const uint8_t *p = (const uint8_t *)vdata;
  sc->totalLength += (uint64_t)len * 8u;
  uint32_t take = 0;
  if (sc->bufferLength) {
    take = std::min<uint32_t>(64u - sc->bufferLength, len);
    memcpy(sc->buffer.bytes + sc->bufferLength, p, take);
    sc->bufferLength += take;
    p += take;
    len -= take;
    if (sc->bufferLength < 64u) return;
  }
  const uint64_t nfull = len / 64u;
  const bool staged_full = sc->bufferLength == 64u;
  if (staged_full || nfull) {
    KeepDevice keep_dev;
    DevCtx *c = dropin_ctx("SHA1Update");
    std::lock_guard<std::mutex> g(c->mu);
    if (midstate(c, sc->hash, staged_full ? sc->buffer.bytes : nullptr, p, nfull)) die("SHA1Update");
    sc->bufferLength = 0;
  }
  const uint32_t rest = len - (uint32_t)(64u * nfull);
  if (rest) {
    memcpy(sc->buffer.bytes, p + 64u * nfull, rest);
    sc->bufferLength = rest;
  }
}

// sha.c:529-558: 0x80, zeros to 56 mod 64, 64-bit big-endian bit count; the
// last one or two blocks are compressed on the GPU; digest big-endian.
void SHA1Final(SHA1Context *sc, uint8_t hash[SHA1_HASH_SIZE]) {
  const uint32_t bl = sc->bufferLength;
  uint32_t npad = 120u - bl;
  if (npad > 64u) npad -= 64u;
  uint8_t blk[128];
  memset(blk, 0, sizeof blk);
  memcpy(blk, sc->buffer.bytes, bl);
  blk[bl] = 0x80;
  const uint64_t bits = sc->totalLength;
  const uint32_t end = bl + npad + 8u;  // 64 or 128
  for (int i = 0; i < 8; ++i) blk[end - 8 + i] = (uint8_t)(bits >> (56 - 8 * i));
  KeepDevice keep_dev;
  DevCtx *c = dropin_ctx("SHA1Final");
  {
    std::lock_guard<std::mutex> g(c->mu);
    if (midstate(c, sc->hash, nullptr, blk, end / 64u)) die("SHA1Final");
  }
  explicit_bzero(blk, sizeof blk);  // the message tail (sha.c:165-174's burnStack)
  sc->totalLength += (uint64_t)(npad + 8u) * 8u;
  sc->bufferLength = 0;
  if (hash)
    for (int i = 0; i < SHA1_HASH_WORDS; ++i) {
      hash[4 * i] = (uint8_t)(sc->hash[i] >> 24);
      hash[4 * i + 1] = (uint8_t)(sc->hash[i] >> 16);
      hash[4 * i + 2] = (uint8_t)(sc->hash[i] >> 8);
      hash[4 * i + 3] = (uint8_t)sc->hash[i];
    }
}

}  // extern "C"

// ===========================================================================
// Batched asynchronous verifier (util.c:304-337 without the synchronous hash).
// ===========================================================================
// A ring of `nstreams` batches of `batch` pinned chunk slots.  Slots are handed
// out in ring order and may be committed (or released) in any order -- a peer
// assembles up to max_conn chunks at once (util.c:250-277).  A batch launches
// (one H2D of its slots, one hot-kernel launch with the fused verify epilogue)
// once it is closed -- every slot handed out, or flushed -- and each of its
// handed-out slots has been committed or released.
struct VBatch {
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;
  // column-split batches (v_launch): the columns' hashes run on hs, each after
  // its copy's event on s; the chunks' chaining state between columns
  hipStream_t hs = nullptr;
  hipEvent_t cev[kMaxColumns] = {};
  uint32_t *d_state = nullptr;
  StageBuf slots;  // the received chunks: written by the caller, read by the H2D copy
  uint8_t *h_in = nullptr, *h_exp = nullptr, *h_ok = nullptr, *h_dig = nullptr;
  uint8_t *d_in = nullptr;
  std::vector<uint64_t> tags;
  std::vector<uint8_t> state;  // per slot: 0 free, 1 handed out, 2 committed, 3 released
  uint32_t reserved = 0, settled = 0;
  bool closed = false, inflight = false;
};

struct bt_sha1_verifier {
  int dev = 0;
  uint32_t chunk_len = 0, batch = 0;
  std::vector<VBatch> b;
  uint32_t fill = 0;             // batch handing out slots
  std::deque<uint32_t> order;    // batches in flight, oldest first
  std::deque<bt_sha1_verdict> done;
  int64_t queued = 0;            // committed, verdict not yet returned
};

namespace {

int v_harvest(bt_sha1_verifier *v, VBatch &b) {
  BT_CK(hipEventSynchronize(b.ev));
  for (uint32_t i = 0; i < b.reserved; ++i) {
    if (b.state[i] != 2) continue;  // released slots produce no verdict
    bt_sha1_verdict r;
    r.tag = b.tags[i];
    r.ok = b.h_ok[i] ? 1 : 0;
    memcpy(r.digest, b.h_dig + 20 * i, 20);
    v->done.push_back(r);
  }
  std::fill(b.state.begin(), b.state.end(), 0);
  b.reserved = b.settled = 0;
  b.closed = b.inflight = false;
  return 0;
}

// Columns a batch of `rows` chunks is split into (0: one copy, one launch):
// as the host pipelines' tail (chunks_host_on), a batch of at least
// column_min_bytes() of chunks of at least 64 KiB is copied in columns and
// each column hashed as soon as it has arrived, so its verdicts come one
// column's hash (~0.9 ms), not one whole chunk's (~6.7 ms), after its last
// byte crossed PCIe.
uint32_t v_columns(uint64_t chunk_len, uint64_t rows) {
  uint32_t parts = columns();
  while (parts >= 2 && chunk_len % (64ull * parts)) parts /= 2;
  return parts >= 2 && chunk_len >= kColumnMinChunk && rows >= 2 && rows * chunk_len >= column_min_bytes() ? parts
                                                                                                            : 0;
}

int v_launch_columns(bt_sha1_verifier *v, VBatch &b, uint32_t parts) {
  const uint64_t cl = v->chunk_len, rows = b.reserved, w = cl / parts;
  if (!b.hs) BT_CK(hipStreamCreateWithFlags(&b.hs, hipStreamNonBlocking));
  if (!b.d_state) BT_CK(hipMalloc((void **)&b.d_state, 20 * (size_t)v->batch));
  for (uint32_t j = 0; j < parts; ++j) {
    if (!b.cev[j]) BT_CK(hipEventCreateWithFlags(&b.cev[j], hipEventDisableTiming));
    BT_CK(hipMemcpy2DAsync(b.d_in + j * rows * w, (size_t)w, b.h_in + j * w, (size_t)cl, (size_t)w, (size_t)rows,
                           hipMemcpyHostToDevice, b.s));
    BT_CK(hipEventRecord(b.cev[j], b.s));
    BT_CK(hipStreamWaitEvent(b.hs, b.cev[j], 0));
    const bool last = j + 1 == parts;
    BT_CK(btsha1_launch_column(b.d_in + j * rows * w, rows, (uint32_t)w, (uint32_t)w,
                               j == 0 ? BTSHA1_COLUMN_FIRST : last ? BTSHA1_COLUMN_LAST : BTSHA1_COLUMN_MIDDLE,
                               b.d_state, cl, last ? b.h_dig : nullptr, b.hs, last ? b.h_exp : nullptr,
                               last ? b.h_ok : nullptr));
  }
  BT_CK(hipEventRecord(b.ev, b.hs));
  return 0;
}

int v_launch(bt_sha1_verifier *v, uint32_t idx) {
  VBatch &b = v->b[idx];
  if (b.reserved == 0) {  // closed while empty: nothing to do
    b.closed = false;
    return 0;
  }
  if (const uint32_t parts = v_columns(v->chunk_len, b.reserved)) {
    if (v_launch_columns(v, b, parts)) {  // leave nothing of the batch in flight behind the error
      if (b.s) (void)hipStreamSynchronize(b.s);
      if (b.hs) (void)hipStreamSynchronize(b.hs);
      return -1;
    }
    b.inflight = true;
    v->order.push_back(idx);
    return 0;
  }
  const size_t bytes = (size_t)b.reserved * v->chunk_len;
  BT_CK(hipMemcpyAsync(b.d_in, b.h_in, bytes, hipMemcpyHostToDevice, b.s));
  // Expected hashes are read, verdicts and digests written, by the kernel in
  // pinned host memory: the chunk bytes are the only copy (see run_pipeline).
  BT_CK(btsha1_launch_fixed(b.d_in, b.reserved, v->chunk_len, v->chunk_len, b.h_dig, b.h_exp, b.h_ok, b.s,
                            g_variant.load()));
  BT_CK(hipEventRecord(b.ev, b.s));
  b.inflight = true;
  v->order.push_back(idx);
  return 0;
}

int v_maybe_launch(bt_sha1_verifier *v, uint32_t idx) {
  VBatch &b = v->b[idx];
  if (b.closed && !b.inflight && b.settled == b.reserved) return v_launch(v, idx);
  return 0;
}

// The filling batch is closed: move the fill pointer on, waiting for the next
// batch of the ring if it is still in flight.
int v_advance(bt_sha1_verifier *v) {
  const uint32_t nxt = (v->fill + 1) % (uint32_t)v->b.size();
  VBatch &n = v->b[nxt];
  if (n.inflight) {  // ring wrapped: harvest up to and including it
    while (!v->order.empty()) {
      const uint32_t o = v->order.front();
      v->order.pop_front();
      if (v_harvest(v, v->b[o])) return -1;
      if (o == nxt) break;
    }
  } else if (n.closed) {
    set_err("verifier: every batch holds slots that were handed out but never committed");
    return -1;
  }
  v->fill = nxt;
  return 0;
}

// Slot pointer -> (batch, index); -1 if it is not a handed-out slot.
int v_locate(bt_sha1_verifier *v, const uint8_t *slot, uint32_t *bi, uint32_t *si) {
  for (uint32_t k = 0; k < v->b.size(); ++k) {
    VBatch &b = v->b[k];
    if (slot >= b.h_in && slot < b.h_in + (size_t)v->batch * v->chunk_len) {
      const size_t off = (size_t)(slot - b.h_in);
      if (off % v->chunk_len || b.state[off / v->chunk_len] != 1) break;
      *bi = k;
      *si = (uint32_t)(off / v->chunk_len);
      return 0;
    }
  }
  set_err("verifier: pointer is not an outstanding slot");
  return -1;
}

}  // namespace

extern "C" {

bt_sha1_verifier *bt_sha1_verifier_create(int device, uint32_t chunk_len, uint32_t batch, uint32_t nstreams) {
  if (chunk_len == 0 || (chunk_len & 15) || chunk_len > (32u << 20) || batch == 0) {
    set_err("verifier: chunk_len must be a 16-byte multiple <= 32 MiB and batch > 0");
    return nullptr;
  }
  DevCtx *c = ctx_for(device);
  if (!c) return nullptr;
  KeepDevice keep_dev;
  if (hipSetDevice(device) != hipSuccess) {
    set_err("hipSetDevice(%d) failed", device);
    return nullptr;
  }
  // The receive slots are written by the caller's receive path and read by
  // the DMA engine: on the GPU's NUMA node, like the pipelines' lanes.
  int node = -1;
  {
    std::lock_guard<std::mutex> g(c->mu);
    if (c->numa_node == -2) c->numa_node = gpu_numa_node(device);
    node = placement_for(c->numa_node).node;
  }
  auto *v = new bt_sha1_verifier;
  v->dev = device;
  v->chunk_len = chunk_len;
  v->batch = batch;
  v->b.resize(std::max<uint32_t>(nstreams, 2));
  const size_t bytes = (size_t)batch * chunk_len;
  t_err.clear();
  for (auto &b : v->b) {
    b.tags.resize(batch);
    b.state.assign(batch, 0);
    if (hipStreamCreateWithFlags(&b.s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess ||
        b.slots.ensure(bytes, node) != 0 ||
        hipHostMalloc((void **)&b.h_exp, 20 * (size_t)batch, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&b.h_ok, batch, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void **)&b.h_dig, 20 * (size_t)batch, hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void **)&b.d_in, bytes) != hipSuccess) {
      if (t_err.empty()) set_err("verifier: allocation failed");
      bt_sha1_verifier_destroy(v);
      return nullptr;
    }
    b.h_in = b.slots.as<uint8_t>();
  }
  return v;
}

void bt_sha1_verifier_destroy(bt_sha1_verifier *v) {
  if (!v) return;
  KeepDevice keep_dev;
  (void)hipSetDevice(v->dev);
  for (auto &b : v->b) {
    if (b.s) (void)hipStreamSynchronize(b.s);
    if (b.hs) (void)hipStreamSynchronize(b.hs);
    if (b.ev) (void)hipEventDestroy(b.ev);
    for (hipEvent_t e : b.cev)
      if (e) (void)hipEventDestroy(e);
    if (b.s) (void)hipStreamDestroy(b.s);
    if (b.hs) (void)hipStreamDestroy(b.hs);
    if (b.d_state) (void)hipFree(b.d_state);
    b.slots.release();
    if (b.h_exp) (void)hipHostFree(b.h_exp);
    if (b.h_ok) (void)hipHostFree(b.h_ok);
    if (b.h_dig) (void)hipHostFree(b.h_dig);
    if (b.d_in) (void)hipFree(b.d_in);
  }
  delete v;
}

uint8_t *bt_sha1_verifier_slot(bt_sha1_verifier *v) {
  if (!v) return nullptr;
  KeepDevice keep_dev;
  if (hipSetDevice(v->dev) != hipSuccess) return nullptr;
  if (v->b[v->fill].closed && v_advance(v)) return nullptr;
  VBatch &b = v->b[v->fill];
  const uint32_t j = b.reserved++;
  b.state[j] = 1;
  if (b.reserved == v->batch) b.closed = true;  // launches when its last slot settles
  return b.h_in + (size_t)j * v->chunk_len;
}

int bt_sha1_verifier_commit(bt_sha1_verifier *v, uint8_t *slot, uint32_t len, const uint8_t expected[20],
                            uint64_t tag) {
  if (!v || !slot || !expected) {
    set_err("null pointer");
    return -1;
  }
  if (len != v->chunk_len) {
    set_err("verifier: chunk of %u bytes, verifier built for %u", len, v->chunk_len);
    return -1;
  }
  KeepDevice keep_dev;
  if (hipSetDevice(v->dev) != hipSuccess) return -1;
  uint32_t bi, si;
  if (v_locate(v, slot, &bi, &si)) return -1;
  VBatch &b = v->b[bi];
  memcpy(b.h_exp + 20 * (size_t)si, expected, 20);
  b.tags[si] = tag;
  b.state[si] = 2;
  ++b.settled;
  ++v->queued;
  return v_maybe_launch(v, bi);
}

int bt_sha1_verifier_release(bt_sha1_verifier *v, uint8_t *slot) {
  if (!v || !slot) {
    set_err("null pointer");
    return -1;
  }
  KeepDevice keep_dev;
  if (hipSetDevice(v->dev) != hipSuccess) return -1;
  uint32_t bi, si;
  if (v_locate(v, slot, &bi, &si)) return -1;
  VBatch &b = v->b[bi];
  memset(b.h_exp + 20 * (size_t)si, 0, 20);
  b.state[si] = 3;
  ++b.settled;
  return v_maybe_launch(v, bi);
}

int bt_sha1_verifier_submit(bt_sha1_verifier *v, const void *h_chunk, uint32_t len, const uint8_t expected[20],
                            uint64_t tag) {
  if (!v || !h_chunk) {
    set_err("null pointer");
    return -1;
  }
  if (len != v->chunk_len) {
    set_err("verifier: chunk of %u bytes, verifier built for %u", len, v->chunk_len);
    return -1;
  }
  uint8_t *slot = bt_sha1_verifier_slot(v);
  if (!slot) return -1;
  memcpy(slot, h_chunk, len);
  return bt_sha1_verifier_commit(v, slot, len, expected, tag);
}

int bt_sha1_verifier_flush(bt_sha1_verifier *v) {
  if (!v) return -1;
  KeepDevice keep_dev;
  if (hipSetDevice(v->dev) != hipSuccess) return -1;
  VBatch &b = v->b[v->fill];
  if (b.reserved == 0 || b.closed) return 0;
  b.closed = true;
  return v_maybe_launch(v, v->fill);
}

static int v_take(bt_sha1_verifier *v, bt_sha1_verdict *out, int max) {
  int n = 0;
  while (n < max && !v->done.empty()) {
    out[n++] = v->done.front();
    v->done.pop_front();
  }
  v->queued -= n;
  return n;
}

int bt_sha1_verifier_poll(bt_sha1_verifier *v, bt_sha1_verdict *out, int max) {
  if (!v) return -1;
  KeepDevice keep_dev;
  if (hipSetDevice(v->dev) != hipSuccess) return -1;
  while (!v->order.empty()) {
    VBatch &b = v->b[v->order.front()];
    hipError_t q = hipEventQuery(b.ev);
    if (q == hipErrorNotReady) break;
    if (q != hipSuccess) {
      set_err("verifier: %s", hipGetErrorString(q));
      return -1;
    }
    v->order.pop_front();
    if (v_harvest(v, b)) return -1;
  }
  return v_take(v, out, max);
}

int bt_sha1_verifier_drain(bt_sha1_verifier *v, bt_sha1_verdict *out, int max) {
  if (!v) return -1;
  if (bt_sha1_verifier_flush(v)) return -1;
  while (!v->order.empty()) {
    const uint32_t o = v->order.front();
    v->order.pop_front();
    if (v_harvest(v, v->b[o])) return -1;
  }
  return v_take(v, out, max);
}

int64_t bt_sha1_verifier_pending(bt_sha1_verifier *v) { return v ? v->queued : -1; }

}  // extern "C"
