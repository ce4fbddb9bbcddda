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
#include <numeric>
#include <vector>

#define THREADS 256
#define OPT_PER_THREAD 2
#define SLOTS (THREADS * OPT_PER_THREAD)
#define MAX_Y 65535

typedef unsigned long long u64;

namespace {

struct Prepared {
  std::vector<uint4> data;        // panels: [block][slot] of 16 coded chars
  std::vector<int64_t> panelOff;  // uint4 offset of each panel
  std::vector<int> panelBlocks;   // 16-char blocks in each panel
  std::vector<int> perm;          // sorted position -> original option index (-1 = padding slot)
  std::vector<int> lenSorted;     // option length in sorted order
  std::vector<u64> M;             // [nB][256] match masks indexed by code
  std::vector<int> lenB;
  int nPanels = 0;
  int scaled = 0;  // panel bytes hold code*4 (the byte offset into a u32 table) when <= 63 symbols
};

// Dense codes ranked by option-byte frequency; 0 is reserved for padding.
// Returns false when all 256 byte values occur (no free code for padding).
// *nsym = number of symbols in use (codes 1..nsym).
bool build_code_map(const uint8_t *opts, int64_t nOptBytes, const uint8_t *qs, int64_t nQBytes, uint8_t code[256],
                    int *nsym) {
  int64_t freq[256] = {0};
  bool seen[256] = {false};
  for (int64_t i = 0; i < nOptBytes; i++) freq[opts[i]]++, seen[opts[i]] = true;
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

int prepare(const uint8_t *opts, const int64_t *offA, int nA, const uint8_t *qs, const int64_t *offB, int nB,
            Prepared &P) {
  for (int j = 0; j < nB; j++) {
    const int64_t len = offB[j + 1] - offB[j];
    if (len < 0 || len > 64) return -2;
  }
  uint8_t code[256];
  int nsym = 0;
  if (!build_code_map(opts, offA[nA], qs, offB[nB], code, &nsym)) return -8;
  P.scaled = nsym <= 63;
  uint8_t stored[256];
  for (int b = 0; b < 256; b++) stored[b] = P.scaled ? (uint8_t)(code[b] * 4) : code[b];

  P.M.assign((size_t)nB * 256, 0ULL);
  P.lenB.resize(nB);
  for (int j = 0; j < nB; j++) {
    const int len = (int)(offB[j + 1] - offB[j]);
    P.lenB[j] = len;
    for (int k = 0; k < len; k++) P.M[(size_t)j * 256 + code[qs[offB[j] + k]]] |= (1ULL << k);
  }

  std::vector<int> order(nA);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(),
                   [&](int x, int y) { return (offA[x + 1] - offA[x]) < (offA[y + 1] - offA[y]); });
  P.nPanels = (nA + SLOTS - 1) / SLOTS;
  P.perm.assign((size_t)P.nPanels * SLOTS, -1);
  P.lenSorted.assign((size_t)P.nPanels * SLOTS, 0);
  P.panelOff.resize(P.nPanels + 1);
  P.panelBlocks.resize(P.nPanels);
  int64_t total = 0;
  for (int p = 0; p < P.nPanels; p++) {
    int ml = 0;
    for (int s = 0; s < SLOTS && p * SLOTS + s < nA; s++) {
      const int o = order[p * SLOTS + s];
      const int len = (int)(offA[o + 1] - offA[o]);
      P.perm[p * SLOTS + s] = o;
      P.lenSorted[p * SLOTS + s] = len;
      ml = len > ml ? len : ml;
    }
    P.panelBlocks[p] = (ml + 15) / 16;
    P.panelOff[p] = total;
    total += (int64_t)P.panelBlocks[p] * SLOTS;
  }
  P.panelOff[P.nPanels] = total;
  P.data.assign((size_t)(total > 0 ? total : 1), make_uint4(0, 0, 0, 0));
  for (int p = 0; p < P.nPanels; p++) {
    uint8_t *base = reinterpret_cast<uint8_t *>(P.data.data() + P.panelOff[p]);
    for (int s = 0; s < SLOTS && p * SLOTS + s < nA; s++) {
      const int o = P.perm[p * SLOTS + s];
      const uint8_t *src = opts + offA[o];
      const int len = P.lenSorted[p * SLOTS + s];
      for (int k = 0; k < len; k++) base[((size_t)(k / 16) * SLOTS + s) * 16 + (k % 16)] = stored[src[k]];
    }
  }
  return 0;
}

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

namespace {

struct Dev {
  uint4 *panels = nullptr;
  int64_t *panelOff = nullptr;
  int *panelBlocks = nullptr, *lenSorted = nullptr, *perm = nullptr, *lenB = nullptr;
  u64 *M = nullptr;
  ~Dev() {
    (void)hipFree(panels);
    (void)hipFree(panelOff);
    (void)hipFree(panelBlocks);
    (void)hipFree(lenSorted);
    (void)hipFree(perm);
    (void)hipFree(lenB);
    (void)hipFree(M);
  }
};

template <class T>
bool up(T **dst, const std::vector<T> &src) {
  const size_t bytes = sizeof(T) * (src.empty() ? 1 : src.size());
  if (hipMalloc(dst, bytes) != hipSuccess) return false;
  return src.empty() || hipMemcpy(*dst, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice) == hipSuccess;
}

int upload(const Prepared &P, Dev &d) {
  if (!up(&d.panels, P.data) || !up(&d.panelOff, P.panelOff) || !up(&d.panelBlocks, P.panelBlocks) ||
      !up(&d.lenSorted, P.lenSorted) || !up(&d.perm, P.perm) || !up(&d.lenB, P.lenB) || !up(&d.M, P.M))
    return -4;
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
  Prepared P;
  int rc = prepare(opts, offA, nA, qs, offB, nB, P);
  if (rc) return rc;
  Dev d;
  int *dOut = nullptr;
  rc = upload(P, d);
  if (rc == 0 && hipMalloc(&dOut, sizeof(int) * (size_t)nA * nB) != hipSuccess) rc = -4;
  if (rc == 0) {
    const int gx = grid_x(P.nPanels, nB);
    for (int q0 = 0; q0 < nB && rc == 0; q0 += MAX_Y) {
      const int rows = (nB - q0) < MAX_Y ? (nB - q0) : MAX_Y;
      if (P.scaled)
        hipLaunchKernelGGL(ed_matrix_kernel<true>, dim3(gx, rows), dim3(THREADS), 0, 0, d.panels, d.panelOff,
                           d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, nA, P.nPanels, q0, dOut);
      else
        hipLaunchKernelGGL(ed_matrix_kernel<false>, dim3(gx, rows), dim3(THREADS), 0, 0, d.panels, d.panelOff,
                           d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, nA, P.nPanels, q0, dOut);
      if (hipGetLastError() != hipSuccess) rc = -5;
    }
    if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = -6;
    if (rc == 0 && hipMemcpy(outT, dOut, sizeof(int) * (size_t)nA * nB, hipMemcpyDeviceToHost) != hipSuccess) rc = -7;
  }
  (void)hipFree(dOut);
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
  Prepared P;
  int rc = prepare(opts, offA, nA, qs, offB, nB, P);
  if (rc) return rc;
  Dev d;
  u64 *dBest = nullptr;
  rc = upload(P, d);
  if (rc == 0 && hipMalloc(&dBest, sizeof(u64) * nB) != hipSuccess) rc = -4;
  if (rc == 0 && hipMemset(dBest, 0xff, sizeof(u64) * nB) != hipSuccess) rc = -4;
  if (rc == 0) {
    const int gx = grid_x(P.nPanels, nB);
    for (int q0 = 0; q0 < nB && rc == 0; q0 += MAX_Y) {
      const int rows = (nB - q0) < MAX_Y ? (nB - q0) : MAX_Y;
      if (P.scaled)
        hipLaunchKernelGGL(ed_closest_kernel<true>, dim3(gx, rows), dim3(THREADS), 0, 0, d.panels, d.panelOff,
                           d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, P.nPanels, q0, dBest);
      else
        hipLaunchKernelGGL(ed_closest_kernel<false>, dim3(gx, rows), dim3(THREADS), 0, 0, d.panels, d.panelOff,
                           d.panelBlocks, d.lenSorted, d.perm, d.M, d.lenB, P.nPanels, q0, dBest);
      if (hipGetLastError() != hipSuccess) rc = -5;
    }
    if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = -6;
    if (rc == 0) {
      std::vector<u64> h(nB);
      if (hipMemcpy(h.data(), dBest, sizeof(u64) * nB, hipMemcpyDeviceToHost) != hipSuccess) rc = -7;
      for (int j = 0; j < nB && rc == 0; j++) {
        bestIdx[j] = (int32_t)(h[j] & 0xffffffffULL);
        bestDist[j] = (int32_t)(h[j] >> 32);
      }
    }
  }
  (void)hipFree(dBest);
  return rc;
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
