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
// Layout (CDNA4-first):
//  * Options are sorted by length on the host and cut into panels of 256 (one
//    workgroup = 4 wave64s).  A panel is stored transposed [panelMaxLen][256]:
//    the k-th character load of a wave is one coalesced 64-byte read, lanes of
//    a wave have near-equal lengths (no divergence), and padding is bounded by
//    the length spread inside a panel instead of by the global maximum.
//  * blockIdx.y = query; the query's 256-entry match-mask table (2 KiB) is
//    staged once into LDS and shared by the 4 waves.
//  * blockIdx.x walks panels, remapped so consecutive panels of one query land
//    on the same XCD (blockIdx % 8 selects the XCD under round-robin dispatch),
//    keeping that query's slice of the option panels in one L2.
//  * ed_matrix kernel: results go to a query-major [nB][nA] matrix (Python
//    returns the transposed view, so no host transpose).
//  * ed_closest kernel: the argmin over options is fused into the producer -
//    key = (dist << 32 | original_index) is min-reduced across the wave with
//    cross-lane shuffles, then across the 4 waves in LDS, then with one 64-bit
//    atomicMin per workgroup - so only nB (index, dist) pairs ever leave the
//    GPU.  Ties resolve to the lowest original index, matching the
//    reference's strict "<" scan.
//  * queries are launched in slabs of <= 65535 rows (gridDim.y limit).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <vector>

#define THREADS 256
#define MAX_Y 65535

namespace {

struct Panels {
  std::vector<uint8_t> data;      // concatenated transposed panels
  std::vector<int64_t> panelOff;  // byte offset of each panel in data
  std::vector<int> panelLen;      // max option length of each panel
  std::vector<int> perm;          // sorted position -> original option index
  std::vector<int> lenSorted;     // option length in sorted order
};

void build_panels(const uint8_t *opts, const int64_t *offA, int nA, Panels &P) {
  P.perm.resize(nA);
  std::iota(P.perm.begin(), P.perm.end(), 0);
  std::stable_sort(P.perm.begin(), P.perm.end(),
                   [&](int x, int y) { return (offA[x + 1] - offA[x]) < (offA[y + 1] - offA[y]); });
  const int nPanels = (nA + THREADS - 1) / THREADS;
  P.panelOff.resize(nPanels + 1);
  P.panelLen.resize(nPanels);
  P.lenSorted.assign((size_t)nPanels * THREADS, 0);
  int64_t total = 0;
  for (int p = 0; p < nPanels; p++) {
    int ml = 0;
    for (int l = 0; l < THREADS; l++) {
      const int s = p * THREADS + l;
      if (s >= nA) break;
      const int o = P.perm[s];
      const int len = (int)(offA[o + 1] - offA[o]);
      P.lenSorted[s] = len;
      ml = len > ml ? len : ml;
    }
    P.panelLen[p] = ml;
    P.panelOff[p] = total;
    total += (int64_t)ml * THREADS;
  }
  P.panelOff[nPanels] = total;
  P.data.assign((size_t)(total > 0 ? total : 1), 0);
  for (int p = 0; p < nPanels; p++) {
    uint8_t *base = P.data.data() + P.panelOff[p];
    for (int l = 0; l < THREADS; l++) {
      const int s = p * THREADS + l;
      if (s >= nA) break;
      const uint8_t *src = opts + offA[P.perm[s]];
      const int len = P.lenSorted[s];
      for (int k = 0; k < len; k++) base[(size_t)k * THREADS + l] = src[k];
    }
  }
}

int build_masks(const uint8_t *qs, const int64_t *offB, int nB, std::vector<unsigned long long> &M,
                std::vector<int> &lenB) {
  M.assign((size_t)nB * 256, 0ULL);
  lenB.resize(nB);
  for (int j = 0; j < nB; j++) {
    const int len = (int)(offB[j + 1] - offB[j]);
    if (len < 0 || len > 64) return -2;
    lenB[j] = len;
    for (int k = 0; k < len; k++) M[(size_t)j * 256 + qs[offB[j] + k]] |= (1ULL << k);
  }
  return 0;
}

__device__ __forceinline__ int remap_panel(int bx, int n) {
  if (n % 8 != 0) return bx;
  const int per = n / 8;
  return (bx % 8) * per + (bx / 8);
}

__device__ __forceinline__ int lcs_dist(const uint8_t *__restrict__ col, int len, const unsigned long long *M, int lb,
                                        unsigned long long mask) {
  unsigned long long V = ~0ULL;
  for (int k = 0; k < len; k++) {
    const unsigned long long U = V & M[col[(size_t)k * THREADS]];
    V = (V + U) | (V - U);
  }
  return len + lb - 2 * __popcll(~V & mask);
}

}  // namespace

__global__ __launch_bounds__(THREADS) void ed_matrix_kernel(const uint8_t *__restrict__ panels,
                                                            const int64_t *__restrict__ panelOff,
                                                            const int *__restrict__ lenSorted,
                                                            const int *__restrict__ perm,
                                                            const unsigned long long *__restrict__ qmask,
                                                            const int *__restrict__ lenB, int nA, int nPanels, int q0,
                                                            int *__restrict__ outT) {
  __shared__ unsigned long long M[256];
  const int q = q0 + blockIdx.y;
  for (int c = threadIdx.x; c < 256; c += THREADS) M[c] = qmask[(size_t)q * 256 + c];
  __syncthreads();
  const int lb = lenB[q];
  const unsigned long long mask = (lb >= 64) ? ~0ULL : ((1ULL << lb) - 1ULL);
  for (int p = remap_panel(blockIdx.x, gridDim.x); p < nPanels; p += gridDim.x) {
    const int s = p * THREADS + threadIdx.x;
    if (s < nA) {
      const int d = lcs_dist(panels + panelOff[p] + threadIdx.x, lenSorted[s], M, lb, mask);
      outT[(size_t)q * nA + perm[s]] = d;
    }
  }
}

__global__ __launch_bounds__(THREADS) void ed_closest_kernel(const uint8_t *__restrict__ panels,
                                                             const int64_t *__restrict__ panelOff,
                                                             const int *__restrict__ lenSorted,
                                                             const int *__restrict__ perm,
                                                             const unsigned long long *__restrict__ qmask,
                                                             const int *__restrict__ lenB, int nA, int nPanels, int q0,
                                                             unsigned long long *__restrict__ best) {
  __shared__ unsigned long long M[256];
  __shared__ unsigned long long red[THREADS / 64];
  const int q = q0 + blockIdx.y;
  for (int c = threadIdx.x; c < 256; c += THREADS) M[c] = qmask[(size_t)q * 256 + c];
  __syncthreads();
  const int lb = lenB[q];
  const unsigned long long mask = (lb >= 64) ? ~0ULL : ((1ULL << lb) - 1ULL);
  unsigned long long key = ~0ULL;
  for (int p = remap_panel(blockIdx.x, gridDim.x); p < nPanels; p += gridDim.x) {
    const int s = p * THREADS + threadIdx.x;
    if (s < nA) {
      const int d = lcs_dist(panels + panelOff[p] + threadIdx.x, lenSorted[s], M, lb, mask);
      const unsigned long long k = ((unsigned long long)(unsigned)d << 32) | (unsigned)perm[s];
      key = k < key ? k : key;
    }
  }
  // wave64 min-reduction
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(key, off, 64);
    key = o < key ? o : key;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64] = key;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < THREADS / 64; w++) k = red[w] < k ? red[w] : k;
    if (k != ~0ULL) atomicMin(&best[q], k);
  }
}

namespace {

struct Dev {
  uint8_t *panels = nullptr;
  int64_t *panelOff = nullptr;
  int *lenSorted = nullptr, *perm = nullptr, *lenB = nullptr;
  unsigned long long *M = nullptr;
  ~Dev() {
    (void)hipFree(panels);
    (void)hipFree(panelOff);
    (void)hipFree(lenSorted);
    (void)hipFree(perm);
    (void)hipFree(lenB);
    (void)hipFree(M);
  }
};

int upload(const Panels &P, const std::vector<unsigned long long> &M, const std::vector<int> &lenB, Dev &d) {
  const size_t nPanels = P.panelLen.size();
  if (hipMalloc(&d.panels, P.data.size()) != hipSuccess ||
      hipMalloc(&d.panelOff, sizeof(int64_t) * (nPanels + 1)) != hipSuccess ||
      hipMalloc(&d.lenSorted, sizeof(int) * P.lenSorted.size()) != hipSuccess ||
      hipMalloc(&d.perm, sizeof(int) * P.perm.size()) != hipSuccess ||
      hipMalloc(&d.lenB, sizeof(int) * lenB.size()) != hipSuccess ||
      hipMalloc(&d.M, sizeof(unsigned long long) * M.size()) != hipSuccess)
    return -4;
  if (hipMemcpy(d.panels, P.data.data(), P.data.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d.panelOff, P.panelOff.data(), sizeof(int64_t) * (nPanels + 1), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d.lenSorted, P.lenSorted.data(), sizeof(int) * P.lenSorted.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d.perm, P.perm.data(), sizeof(int) * P.perm.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d.lenB, lenB.data(), sizeof(int) * lenB.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(d.M, M.data(), sizeof(unsigned long long) * M.size(), hipMemcpyHostToDevice) != hipSuccess)
    return -4;
  return 0;
}

int grid_x(int nPanels, int nB) {
  // >> 256 CUs worth of workgroups in total, x a multiple of 8 for the XCD remap
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
  std::vector<unsigned long long> M;
  std::vector<int> lenB;
  int rc = build_masks(qs, offB, nB, M, lenB);
  if (rc) return rc;
  Panels P;
  build_panels(opts, offA, nA, P);
  const int nPanels = (int)P.panelLen.size();
  Dev d;
  int *dOut = nullptr;
  rc = upload(P, M, lenB, d);
  if (rc == 0 && hipMalloc(&dOut, sizeof(int) * (size_t)nA * nB) != hipSuccess) rc = -4;
  if (rc == 0) {
    const int gx = grid_x(nPanels, nB);
    for (int q0 = 0; q0 < nB && rc == 0; q0 += MAX_Y) {
      const int rows = (nB - q0) < MAX_Y ? (nB - q0) : MAX_Y;
      hipLaunchKernelGGL(ed_matrix_kernel, dim3(gx, rows), dim3(THREADS), 0, 0, d.panels, d.panelOff, d.lenSorted,
                         d.perm, d.M, d.lenB, nA, nPanels, q0, dOut);
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
  std::vector<unsigned long long> M;
  std::vector<int> lenB;
  int rc = build_masks(qs, offB, nB, M, lenB);
  if (rc) return rc;
  Panels P;
  build_panels(opts, offA, nA, P);
  const int nPanels = (int)P.panelLen.size();
  Dev d;
  unsigned long long *dBest = nullptr;
  rc = upload(P, M, lenB, d);
  if (rc == 0 && hipMalloc(&dBest, sizeof(unsigned long long) * nB) != hipSuccess) rc = -4;
  if (rc == 0 && hipMemset(dBest, 0xff, sizeof(unsigned long long) * nB) != hipSuccess) rc = -4;
  if (rc == 0) {
    const int gx = grid_x(nPanels, nB);
    for (int q0 = 0; q0 < nB && rc == 0; q0 += MAX_Y) {
      const int rows = (nB - q0) < MAX_Y ? (nB - q0) : MAX_Y;
      hipLaunchKernelGGL(ed_closest_kernel, dim3(gx, rows), dim3(THREADS), 0, 0, d.panels, d.panelOff, d.lenSorted,
                         d.perm, d.M, d.lenB, nA, nPanels, q0, dBest);
      if (hipGetLastError() != hipSuccess) rc = -5;
    }
    if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = -6;
    if (rc == 0) {
      std::vector<unsigned long long> h(nB);
      if (hipMemcpy(h.data(), dBest, sizeof(unsigned long long) * nB, hipMemcpyDeviceToHost) != hipSuccess) rc = -7;
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
