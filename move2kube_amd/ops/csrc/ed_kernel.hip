// Batched weighted edit distance (Wagner-Fischer with ins=1, del=1, sub=2) and
// fused closest-match search on MI355X (gfx950).
//
// Used by the fuzzy matcher behind common.GetClosestMatchingString
// (reference internal/common/utils.go:377-401), which the CF container-types
// collector (internal/collector/cfcontainertypescollector.go:110-124) runs for
// every (buildpack name x builder buildpack) pair.  On a CF foundation export
// this is a |names| x |buildpacks| all-pairs problem.
//
// With substitution cost == insertion + deletion the weighted distance is
// exactly  |a| + |b| - 2 * LCS(a, b),  so each pair reduces to Hyyro's
// bit-parallel LCS: one 64-bit word holds the DP column for a query of up to 64
// bytes, and every character of the option costs one LDS lookup + 4 integer ops.
//
// Layout (CDNA4-first; tuned from rocprofv3 PMC, see profiles/):
//  * Byte remap.  The host assigns every byte value that occurs a dense code,
//    most frequent option byte first, code 0 = padding, and (when <= 63
//    symbols occur) stores code*4 - the byte offset into the u32 mask table -
//    so turning a character into an LDS address is one VALU op.  M[0] = 0,
//    so a padding code leaves the LCS column unchanged: no per-character
//    length checks.
//  * Width.  Queries of <= 32 bytes run a 32-bit LCS column (u32 table,
//    `ds_read_b32`, one VALU op per and/add/sub/or): per character ~5 VALU ops
//    instead of ~11 for the 64-bit column.  PMC of v2 showed the kernel at
//    ~1 VALU wave-instruction per CU-cycle, i.e. VALU-bound, so this is the
//    lever that matters.
//  * Options are sorted by length and cut into panels of 512 (256 threads x 2
//    options each: two independent dependency chains per lane hide the
//    LDS-lookup -> VALU latency).  A panel is stored as 16-byte blocks
//    [block][slot]: one `global_load_dwordx4` gives a lane its next 16
//    characters (1 KiB per wave instruction), and the next block is prefetched
//    while the current one is consumed (v1 waited on one byte load per char).
//  * blockIdx.y = query; the query's 256-entry mask table (2 KiB) is staged in
//    LDS once per workgroup.  blockIdx.x walks panels, remapped so consecutive
//    panels of one query land on the same XCD (blockIdx % 8 picks the XCD).
//  * ed_matrix kernel: distances go to a query-major [nB][nA] matrix (Python
//    returns the transposed view, so no host transpose).
//  * ed_closest kernel: the argmin is fused into the producer - key =
//    (dist << 32 | original_index) is min-reduced across the wave with
//    shuffles, across the 4 waves in LDS, then one 64-bit atomicMin per
//    workgroup, so only nB (index, dist) pairs leave the GPU.  Ties resolve to
//    the lowest original index, matching the reference's strict "<" scan.
//  * queries are launched in slabs of <= 65535 rows (gridDim.y limit).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <numeric>
#include <thread>
#include <vector>

#define THREADS 256
#define OPT_PER_THREAD 2
#define SLOTS (THREADS * OPT_PER_THREAD)
#define MAX_Y 65535

typedef unsigned long long u64;

namespace {

__device__ __forceinline__ int remap_panel(int bx, int n) {
  if (n % 8 != 0) return bx;
  const int per = n / 8;
  return (bx % 8) * per + (bx / 8);
}

// One 32-bit word = 4 coded characters.  Byte i holds either the code (SCALED=0)
// or code*4 (SCALED=1, a ready-made byte offset into the u32 table; the u64
// table offset is twice that), so extracting a character is one VALU op.
template <typename W, bool SCALED>
__device__ __forceinline__ void step4(uint32_t w, const W *M, W &V) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t c = (w >> (8 * i)) & 0xffu;
    const uint32_t off = SCALED ? c * (uint32_t)(sizeof(W) / 4) : c * (uint32_t)sizeof(W);
    const W m = *reinterpret_cast<const W *>(reinterpret_cast<const char *>(M) + off);
    const W U = V & m;
    V = (V + U) | (V - U);
  }
}

// LCS columns of this lane's OPT_PER_THREAD options in panel p.
template <typename W, bool SCALED>
__device__ __forceinline__ void panel_lcs(const uint4 *__restrict__ panel, int blocks, const W *M,
                                          W (&V)[OPT_PER_THREAD]) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int u = 0; u < OPT_PER_THREAD; u++) V[u] = ~(W)0;
  if (blocks == 0) return;
  uint4 cur[OPT_PER_THREAD], nxt[OPT_PER_THREAD];
#pragma unroll
  for (int u = 0; u < OPT_PER_THREAD; u++) cur[u] = panel[u * THREADS + lane];
  for (int b = 0; b < blocks; b++) {
    if (b + 1 < blocks) {
#pragma unroll
      for (int u = 0; u < OPT_PER_THREAD; u++) nxt[u] = panel[(size_t)(b + 1) * SLOTS + u * THREADS + lane];
    }
    // interleave the two independent chains word by word
    step4<W, SCALED>(cur[0].x, M, V[0]);
    step4<W, SCALED>(cur[1].x, M, V[1]);
    step4<W, SCALED>(cur[0].y, M, V[0]);
    step4<W, SCALED>(cur[1].y, M, V[1]);
    step4<W, SCALED>(cur[0].z, M, V[0]);
    step4<W, SCALED>(cur[1].z, M, V[1]);
    step4<W, SCALED>(cur[0].w, M, V[0]);
    step4<W, SCALED>(cur[1].w, M, V[1]);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) cur[u] = nxt[u];
  }
}

// Distances of this lane's options in panel p to the query whose masks are in
// LDS; queries of <= 32 bytes run the 32-bit column (half the VALU work).
template <bool SCALED>
__device__ __forceinline__ void panel_dists(const uint4 *__restrict__ panel, int blocks, const uint32_t *M32,
                                            const u64 *M64, int lb, int (&lcs)[OPT_PER_THREAD]) {
  if (lb <= 32) {
    uint32_t V[OPT_PER_THREAD];
    panel_lcs<uint32_t, SCALED>(panel, blocks, M32, V);
    const uint32_t mask = (lb >= 32) ? ~0u : ((1u << lb) - 1u);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) lcs[u] = __popc(~V[u] & mask);
  } else {
    u64 V[OPT_PER_THREAD];
    panel_lcs<u64, SCALED>(panel, blocks, M64, V);
    const u64 mask = (lb >= 64) ? ~0ULL : ((1ULL << lb) - 1ULL);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) lcs[u] = __popcll(~V[u] & mask);
  }
}

}  // namespace

template <bool SCALED>
__global__ __launch_bounds__(THREADS) void ed_matrix_kernel(const uint4 *__restrict__ panels,
                                                            const int64_t *__restrict__ panelOff,
                                                            const int *__restrict__ panelBlocks,
                                                            const int *__restrict__ lenSorted,
                                                            const int *__restrict__ perm, const u64 *__restrict__ qmask,
                                                            const int *__restrict__ lenB, int nA, int nPanels, int q0,
                                                            int *__restrict__ outT) {
  __shared__ u64 M64[256];
  __shared__ uint32_t M32[256];
  const int q = q0 + blockIdx.y;
  for (int c = threadIdx.x; c < 256; c += THREADS) {
    const u64 m = qmask[(size_t)q * 256 + c];
    M64[c] = m;
    M32[c] = (uint32_t)m;
  }
  __syncthreads();
  const int lb = lenB[q];
  for (int p = remap_panel(blockIdx.x, gridDim.x); p < nPanels; p += gridDim.x) {
    int lcs[OPT_PER_THREAD];
    panel_dists<SCALED>(panels + panelOff[p], panelBlocks[p], M32, M64, lb, lcs);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) {
      const int s = p * SLOTS + u * THREADS + threadIdx.x;
      const int o = perm[s];
      if (o >= 0) outT[(size_t)q * nA + o] = lenSorted[s] + lb - 2 * lcs[u];
    }
  }
}

template <bool SCALED>
__global__ __launch_bounds__(THREADS) void ed_closest_kernel(const uint4 *__restrict__ panels,
                                                             const int64_t *__restrict__ panelOff,
                                                             const int *__restrict__ panelBlocks,
                                                             const int *__restrict__ lenSorted,
                                                             const int *__restrict__ perm,
                                                             const u64 *__restrict__ qmask, const int *__restrict__ lenB,
                                                             int nPanels, int q0, u64 *__restrict__ best) {
  __shared__ u64 M64[256];
  __shared__ uint32_t M32[256];
  __shared__ u64 red[THREADS / 64];
  const int q = q0 + blockIdx.y;
  for (int c = threadIdx.x; c < 256; c += THREADS) {
    const u64 m = qmask[(size_t)q * 256 + c];
    M64[c] = m;
    M32[c] = (uint32_t)m;
  }
  __syncthreads();
  const int lb = lenB[q];
  u64 key = ~0ULL;
  for (int p = remap_panel(blockIdx.x, gridDim.x); p < nPanels; p += gridDim.x) {
    int lcs[OPT_PER_THREAD];
    panel_dists<SCALED>(panels + panelOff[p], panelBlocks[p], M32, M64, lb, lcs);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) {
      const int s = p * SLOTS + u * THREADS + threadIdx.x;
      const int o = perm[s];
      if (o >= 0) {
        const int d = lenSorted[s] + lb - 2 * lcs[u];
        const u64 k = ((u64)(unsigned)d << 32) | (unsigned)o;
        key = k < key ? k : key;
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const u64 o = __shfl_xor(key, off, 64);
    key = o < key ? o : key;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = key;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 k = red[0];
    for (int w = 1; w < THREADS / 64; w++) k = red[w] < k ? red[w] : k;
    if (k != ~0ULL) atomicMin(&best[q], k);
  }
}

// ---------------------------------------------------------------------------
// Host side.  One request = code map + length sort + panel fill, written
// straight into a pinned staging buffer that is laid out exactly like the
// device buffer, then ONE async H2D copy, the kernels and the D2H of the
// results on one stream.  Staging/device buffers and the stream live in a
// grow-only per-process arena (no hipMalloc/hipFree/hipHostMalloc per call;
// hipFree would also serialise the device).  The fill runs on host threads.
// ---------------------------------------------------------------------------
namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int host_threads() {
  unsigned h = std::thread::hardware_concurrency();
  int t = h ? (int)h : 4;
  if (const char *e = getenv("M2K_ED_THREADS")) t = atoi(e);
  return std::max(1, std::min(t, 32));
}

// f(lo, hi) over [0, n) in nt contiguous chunks
template <class F>
void par_for(int64_t n, int nt, int64_t grain, F f) {
  if (n <= 0) return;
  if (nt <= 1 || n < 2 * grain) {
    f(0, n);
    return;
  }
  nt = (int)std::min<int64_t>(nt, (n + grain - 1) / grain);
  std::vector<std::thread> pool;
  const int64_t chunk = (n + nt - 1) / nt;
  for (int t = 1; t < nt; t++) {
    const int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) pool.emplace_back(f, lo, hi);
  }
  f(0, std::min(n, chunk));
  for (auto &th : pool) th.join();
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Layout {
  int nA = 0, nB = 0, nPanels = 0, scaled = 0;
  int64_t totalU4 = 0;
  size_t oPanels = 0, oPanelOff = 0, oPanelBlocks = 0, oLenSorted = 0, oPerm = 0, oLenB = 0, oM = 0;
  size_t h2dBytes = 0, oBest = 0, bytes = 0;
};

struct Arena {
  std::mutex mu;
  char *host = nullptr;  // pinned staging, same layout as dev
  char *dev = nullptr;
  size_t cap = 0;
  int *out = nullptr;  // ed_matrix output
  size_t outCap = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  double last[4] = {0, 0, 0, 0};  // prep, h2d, kernel, d2h (ms)

  int ensure(size_t bytes) {
    if (!stream) {
      if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return -4;
      for (auto &e : ev)
        if (hipEventCreate(&e) != hipSuccess) return -4;
    }
    if (bytes <= cap) return 0;
    const size_t want = std::max(bytes, cap + cap / 2);
    if (host) (void)hipHostFree(host);
    if (dev) (void)hipFree(dev);
    host = dev = nullptr;
    cap = 0;
    if (hipHostMalloc(reinterpret_cast<void **>(&host), want, hipHostMallocDefault) != hipSuccess) return -4;
    if (hipMalloc(reinterpret_cast<void **>(&dev), want) != hipSuccess) return -4;
    cap = want;
    return 0;
  }
  int ensure_out(size_t bytes) {
    if (bytes <= outCap) return 0;
    if (out) (void)hipFree(out);
    out = nullptr;
    outCap = 0;
    if (hipMalloc(reinterpret_cast<void **>(&out), bytes) != hipSuccess) return -4;
    outCap = bytes;
    return 0;
  }
};

// Process lifetime on purpose: destroying HIP objects from a static destructor
// races the runtime's own teardown.
Arena &arena() {
  static Arena *a = new Arena();
  return *a;
}

// Dense codes ranked by option-byte frequency; 0 is reserved for padding.
// Returns false when all 256 byte values occur (no free code for padding).
bool build_code_map(const uint8_t *opts, int64_t nOptBytes, const uint8_t *qs, int64_t nQBytes, int nt,
                    uint8_t code[256], int *nsym) {
  std::vector<std::array<int64_t, 256>> part(std::max(1, nt));
  for (auto &p : part) p.fill(0);
  std::atomic<int> slot{0};
  par_for(nOptBytes, nt, 1 << 20, [&](int64_t lo, int64_t hi) {
    auto &f = part[slot.fetch_add(1)];
    for (int64_t i = lo; i < hi; i++) f[opts[i]]++;
  });
  int64_t freq[256] = {0};
  bool seen[256] = {false};
  for (auto &p : part)
    for (int b = 0; b < 256; b++) freq[b] += p[b];
  for (int b = 0; b < 256; b++) seen[b] = freq[b] > 0;
  for (int64_t i = 0; i < nQBytes; i++) seen[qs[i]] = true;
  int order[256];
  int n = 0;
  for (int b = 0; b < 256; b++)
    if (seen[b]) order[n++] = b;
  if (n > 255) return false;
  std::stable_sort(order, order + n, [&](int x, int y) { return freq[x] > freq[y]; });
  memset(code, 0, 256);
  for (int i = 0; i < n; i++) code[order[i]] = (uint8_t)(i + 1);
  *nsym = n;
  return true;
}

// Everything up to (not including) the H2D copy.  Returns 0 or an error code.
int prepare(const uint8_t *opts, const int64_t *offA, int nA, const uint8_t *qs, const int64_t *offB, int nB,
            Arena &ar, Layout &L) {
  for (int j = 0; j < nB; j++) {
    const int64_t len = offB[j + 1] - offB[j];
    if (len < 0 || len > 64) return -2;
  }
  const int nt = host_threads();
  uint8_t code[256];
  int nsym = 0;
  if (!build_code_map(opts, offA[nA], qs, offB[nB], nt, code, &nsym)) return -8;
  L.nA = nA;
  L.nB = nB;
  L.scaled = nsym <= 63;
  uint8_t stored[256];
  for (int b = 0; b < 256; b++) stored[b] = L.scaled ? (uint8_t)(code[b] * 4) : code[b];

  // stable counting sort of the options by length
  int maxLen = 0;
  for (int i = 0; i < nA; i++) maxLen = std::max(maxLen, (int)(offA[i + 1] - offA[i]));
  std::vector<int> order(nA);
  if (maxLen <= (1 << 20)) {
    std::vector<int> start(maxLen + 2, 0);
    for (int i = 0; i < nA; i++) start[(int)(offA[i + 1] - offA[i]) + 1]++;
    for (int l = 0; l <= maxLen; l++) start[l + 1] += start[l];
    for (int i = 0; i < nA; i++) order[start[(int)(offA[i + 1] - offA[i])]++] = i;
  } else {
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int x, int y) { return (offA[x + 1] - offA[x]) < (offA[y + 1] - offA[y]); });
  }
  L.nPanels = (nA + SLOTS - 1) / SLOTS;
  std::vector<int> blocks(L.nPanels);
  std::vector<int64_t> poff(L.nPanels + 1);
  int64_t total = 0;
  for (int p = 0; p < L.nPanels; p++) {
    const int last = std::min(nA, (p + 1) * SLOTS) - 1;  // sorted: the panel's longest option
    const int o = order[last];
    blocks[p] = (int)((offA[o + 1] - offA[o] + 15) / 16);
    poff[p] = total;
    total += (int64_t)blocks[p] * SLOTS;
  }
  poff[L.nPanels] = total;
  L.totalU4 = total;

  size_t o = 0;
  L.oPanels = o;
  o = align256(o + sizeof(uint4) * (size_t)std::max<int64_t>(total, 1));
  L.oPanelOff = o;
  o = align256(o + sizeof(int64_t) * (size_t)(L.nPanels + 1));
  L.oPanelBlocks = o;
  o = align256(o + sizeof(int) * (size_t)L.nPanels);
  L.oLenSorted = o;
  o = align256(o + sizeof(int) * (size_t)L.nPanels * SLOTS);
  L.oPerm = o;
  o = align256(o + sizeof(int) * (size_t)L.nPanels * SLOTS);
  L.oLenB = o;
  o = align256(o + sizeof(int) * (size_t)nB);
  L.oM = o;
  o = align256(o + sizeof(u64) * (size_t)nB * 256);
  L.h2dBytes = o;
  L.oBest = o;
  o = align256(o + sizeof(u64) * (size_t)nB);
  L.bytes = o;
  if (int rc = ar.ensure(L.bytes)) return rc;

  char *h = ar.host;
  memcpy(h + L.oPanelOff, poff.data(), sizeof(int64_t) * poff.size());
  memcpy(h + L.oPanelBlocks, blocks.data(), sizeof(int) * blocks.size());
  int *lenSorted = reinterpret_cast<int *>(h + L.oLenSorted);
  int *perm = reinterpret_cast<int *>(h + L.oPerm);
  uint4 *panels = reinterpret_cast<uint4 *>(h + L.oPanels);
  par_for(L.nPanels, nt, 4, [&](int64_t plo, int64_t phi) {
    for (int64_t p = plo; p < phi; p++) {
      uint8_t *base = reinterpret_cast<uint8_t *>(panels + poff[p]);
      memset(base, 0, sizeof(uint4) * (size_t)blocks[p] * SLOTS);
      for (int s = 0; s < SLOTS; s++) {
        const int64_t k = p * SLOTS + s;
        if (k >= nA) {
          perm[k] = -1;
          lenSorted[k] = 0;
          continue;
        }
        const int opt = order[k];
        const uint8_t *src = opts + offA[opt];
        const int len = (int)(offA[opt + 1] - offA[opt]);
        perm[k] = opt;
        lenSorted[k] = len;
        for (int b = 0; b * 16 < len; b++) {
          uint8_t *dst = base + ((size_t)b * SLOTS + s) * 16;
          const int n = std::min(16, len - b * 16);
          for (int t = 0; t < n; t++) dst[t] = stored[src[b * 16 + t]];
        }
      }
    }
  });
  int *lenB = reinterpret_cast<int *>(h + L.oLenB);
  u64 *M = reinterpret_cast<u64 *>(h + L.oM);
  par_for(nB, nt, 256, [&](int64_t lo, int64_t hi) {
    for (int64_t j = lo; j < hi; j++) {
      const int len = (int)(offB[j + 1] - offB[j]);
      lenB[j] = len;
      u64 *mj = M + (size_t)j * 256;
      memset(mj, 0, sizeof(u64) * 256);
      for (int k = 0; k < len; k++) mj[code[qs[offB[j] + k]]] |= (1ULL << k);
    }
  });
  return 0;
}

int grid_x(int nPanels, int nB) {
  // >> 256 CUs worth of workgroups in total; x a multiple of 8 for the XCD remap
  int x = nPanels;
  const int want = (nB >= 2048) ? 8 : (nB >= 256 ? 64 : 1024);
  if (x > want) x = want;
  if (x >= 8) x = (x / 8) * 8;
  return x < 1 ? 1 : x;
}

struct DevPtrs {
  const uint4 *panels;
  const int64_t *panelOff;
  const int *panelBlocks, *lenSorted, *perm, *lenB;
  const u64 *M;
  u64 *best;
};

DevPtrs dev_ptrs(const Arena &ar, const Layout &L) {
  char *d = ar.dev;
  return {reinterpret_cast<const uint4 *>(d + L.oPanels), reinterpret_cast<const int64_t *>(d + L.oPanelOff),
          reinterpret_cast<const int *>(d + L.oPanelBlocks), reinterpret_cast<const int *>(d + L.oLenSorted),
          reinterpret_cast<const int *>(d + L.oPerm),        reinterpret_cast<const int *>(d + L.oLenB),
          reinterpret_cast<const u64 *>(d + L.oM),            reinterpret_cast<u64 *>(d + L.oBest)};
}

void record_times(Arena &ar, double prep) {
  float a = 0, b = 0, c = 0;
  (void)hipEventElapsedTime(&a, ar.ev[0], ar.ev[1]);
  (void)hipEventElapsedTime(&b, ar.ev[1], ar.ev[2]);
  (void)hipEventElapsedTime(&c, ar.ev[2], ar.ev[3]);
  ar.last[0] = prep;
  ar.last[1] = a;
  ar.last[2] = b;
  ar.last[3] = c;
  if (getenv("M2K_ED_PROFILE"))
    fprintf(stderr, "[m2k_ed] prep %.3f ms  h2d %.3f ms  kernel %.3f ms  d2h %.3f ms\n", prep, a, b, c);
}

}  // namespace

extern "C" {

// Full distance matrix, query-major: outT[j * nA + i] = dist(opts[i], queries[j]).
// Strings are packed back to back with (n+1) int64 offsets.  Queries must be <= 64 bytes.
// Returns 0 on success, negative on error.
int m2k_ed_matrix(const uint8_t *opts, const int64_t *offA, int nA, const uint8_t *qs, const int64_t *offB, int nB,
                  int32_t *outT) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -1;
  if (nA <= 0 || nB <= 0) return 0;
  Arena &ar = arena();
  std::lock_guard<std::mutex> lock(ar.mu);
  const double t0 = now_ms();
  Layout L;
  int rc = prepare(opts, offA, nA, qs, offB, nB, ar, L);
  if (rc) return rc;
  if ((rc = ar.ensure_out(sizeof(int) * (size_t)nA * nB))) return rc;
  const double prep = now_ms() - t0;
  const DevPtrs d = dev_ptrs(ar, L);
  hipStream_t s = ar.stream;
  (void)hipEventRecord(ar.ev[0], s);
  if (hipMemcpyAsync(ar.dev, ar.host, L.h2dBytes, hipMemcpyHostToDevice, s) != hipSuccess) return -7;
  (void)hipEventRecord(ar.ev[1], s);
  const int gx = grid_x(L.nPanels, nB);
  for (int q0 = 0; q0 < nB && rc == 0; q0 += MAX_Y) {
    const int rows = (nB - q0) < MAX_Y ? (nB - q0) : MAX_Y;
    if (L.scaled)
      hipLaunchKernelGGL(ed_matrix_kernel<true>, dim3(gx, rows), dim3(THREADS), 0, s, d.panels, d.panelOff,
                         d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, nA, L.nPanels, q0, ar.out);
    else
      hipLaunchKernelGGL(ed_matrix_kernel<false>, dim3(gx, rows), dim3(THREADS), 0, s, d.panels, d.panelOff,
                         d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, nA, L.nPanels, q0, ar.out);
    if (hipGetLastError() != hipSuccess) rc = -5;
  }
  (void)hipEventRecord(ar.ev[2], s);
  if (rc == 0 && hipMemcpyAsync(outT, ar.out, sizeof(int) * (size_t)nA * nB, hipMemcpyDeviceToHost, s) != hipSuccess)
    rc = -7;
  (void)hipEventRecord(ar.ev[3], s);
  if (hipStreamSynchronize(s) != hipSuccess && rc == 0) rc = -6;
  if (rc == 0) record_times(ar, prep);
  return rc;
}

// Closest option per query: bestIdx[j] = first i minimising dist(opts[i], queries[j]),
// bestDist[j] = that distance (-1/-1 when there are no options).
int m2k_ed_closest(const uint8_t *opts, const int64_t *offA, int nA, const uint8_t *qs, const int64_t *offB, int nB,
                   int32_t *bestIdx, int32_t *bestDist) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -1;
  if (nB <= 0) return 0;
  if (nA <= 0) {
    for (int j = 0; j < nB; j++) bestIdx[j] = -1, bestDist[j] = -1;
    return 0;
  }
  Arena &ar = arena();
  std::lock_guard<std::mutex> lock(ar.mu);
  const double t0 = now_ms();
  Layout L;
  int rc = prepare(opts, offA, nA, qs, offB, nB, ar, L);
  if (rc) return rc;
  const double prep = now_ms() - t0;
  const DevPtrs d = dev_ptrs(ar, L);
  hipStream_t s = ar.stream;
  (void)hipEventRecord(ar.ev[0], s);
  if (hipMemcpyAsync(ar.dev, ar.host, L.h2dBytes, hipMemcpyHostToDevice, s) != hipSuccess) return -7;
  if (hipMemsetAsync(d.best, 0xff, sizeof(u64) * nB, s) != hipSuccess) return -4;
  (void)hipEventRecord(ar.ev[1], s);
  const int gx = grid_x(L.nPanels, nB);
  for (int q0 = 0; q0 < nB && rc == 0; q0 += MAX_Y) {
    const int rows = (nB - q0) < MAX_Y ? (nB - q0) : MAX_Y;
    if (L.scaled)
      hipLaunchKernelGGL(ed_closest_kernel<true>, dim3(gx, rows), dim3(THREADS), 0, s, d.panels, d.panelOff,
                         d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, L.nPanels, q0, d.best);
    else
      hipLaunchKernelGGL(ed_closest_kernel<false>, dim3(gx, rows), dim3(THREADS), 0, s, d.panels, d.panelOff,
                         d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, L.nPanels, q0, d.best);
    if (hipGetLastError() != hipSuccess) rc = -5;
  }
  (void)hipEventRecord(ar.ev[2], s);
  u64 *hBest = reinterpret_cast<u64 *>(ar.host + L.oBest);
  if (rc == 0 && hipMemcpyAsync(hBest, d.best, sizeof(u64) * nB, hipMemcpyDeviceToHost, s) != hipSuccess) rc = -7;
  (void)hipEventRecord(ar.ev[3], s);
  if (hipStreamSynchronize(s) != hipSuccess && rc == 0) rc = -6;
  if (rc == 0) {
    for (int j = 0; j < nB; j++) {
      bestIdx[j] = (int32_t)(hBest[j] & 0xffffffffULL);
      bestDist[j] = (int32_t)(hBest[j] >> 32);
    }
    record_times(ar, prep);
  }
  return rc;
}

// prep / H2D / kernel / D2H milliseconds of the last successful call
void m2k_ed_last_timings(double *out4) {
  Arena &ar = arena();
  std::lock_guard<std::mutex> lock(ar.mu);
  for (int i = 0; i < 4; i++) out4[i] = ar.last[i];
}

int m2k_gpu_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char *m2k_gpu_arch() {
  static char name[256];
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) != hipSuccess) return "";
  strncpy(name, p.gcnArchName, sizeof(name) - 1);
  return name;
}
}
