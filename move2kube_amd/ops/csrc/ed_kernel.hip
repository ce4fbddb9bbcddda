// Batched weighted edit distance (Wagner-Fischer with ins=1, del=1, sub=2) on
// MI355X (gfx950).
//
// Used by the fuzzy matcher behind common.GetClosestMatchingString
// (reference internal/common/utils.go:377-401), which the CF container-types
// collector (internal/collector/cfcontainertypescollector.go:110-124) runs for
// every (buildpack name x builder buildpack) pair.  On a CF foundation export
// this is a |apps| x |buildpacks| all-pairs problem.
//
// With substitution cost == insertion + deletion the weighted distance is
// exactly  |a| + |b| - 2 * LCS(a, b),  so each pair reduces to Hyyro's
// bit-parallel LCS: one 64-bit word holds the DP column for a query of up to 64
// bytes, and every character of the option costs one LDS lookup + 4 integer ops.
//
// Layout (CDNA4-first):
//  * blockIdx.y = query; the query's 256-entry match-mask table (2 KiB) is
//    staged once into LDS and shared by the 4 wave64s of the workgroup.
//  * lanes walk options; options are stored transposed [maxLen][nOpts] so the
//    k-th character load of a wave is one coalesced 64-byte read.
//  * blockIdx.x is remapped so consecutive option chunks of one query land on
//    the same XCD (blockIdx % 8 selects the XCD under round-robin dispatch),
//    keeping that query's slice of the option matrix in one L2.
//  * results are written query-major ([nB][nA], one coalesced store per wave)
//    and transposed on the host; queries are launched in slabs of <= 65535
//    rows so gridDim.y stays within the hardware limit.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#define THREADS 256

__global__ __launch_bounds__(THREADS) void lcs_dist_kernel(const uint8_t *__restrict__ optsT, const int *__restrict__ lenA,
                                                          const unsigned long long *__restrict__ qmask,
                                                          const int *__restrict__ lenB, int nA, int q0,
                                                          int *__restrict__ outT) {
  __shared__ unsigned long long M[256];
  const int q = q0 + blockIdx.y;
  for (int c = threadIdx.x; c < 256; c += THREADS) M[c] = qmask[(size_t)q * 256 + c];
  __syncthreads();

  // XCD-aware chunk remap: 8 XCDs, round-robin workgroup placement.
  const int nchunks = gridDim.x;
  int bx = blockIdx.x;
  if (nchunks % 8 == 0) {
    const int per = nchunks / 8;
    bx = (bx % 8) * per + (bx / 8);
  }

  const int lb = lenB[q];
  const unsigned long long mask = (lb >= 64) ? ~0ULL : ((1ULL << lb) - 1ULL);
  for (int a = bx * THREADS + threadIdx.x; a < nA; a += nchunks * THREADS) {
    const int la = lenA[a];
    unsigned long long V = ~0ULL;
    for (int k = 0; k < la; k++) {
      const uint8_t ch = optsT[(size_t)k * nA + a];
      const unsigned long long U = V & M[ch];
      V = (V + U) | (V - U);
    }
    const int lcs = __popcll(~V & mask);
    outT[(size_t)q * nA + a] = la + lb - 2 * lcs;  // [query][option]: coalesced across lanes
  }
}

extern "C" {

// Returns 0 on success, negative on error (no device, launch failure...).
// opts: nA strings packed back to back, lens in lenA; queries likewise (each <= 64 bytes).
int m2k_ed_batch(const uint8_t *opts, const int *lenA, int nA, const uint8_t *queries, const int *lenB, int nB,
                 int *out) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return -1;
  if (nA <= 0 || nB <= 0) return 0;
  int maxLen = 1;
  size_t off = 0;
  for (int i = 0; i < nA; i++) maxLen = lenA[i] > maxLen ? lenA[i] : maxLen;
  for (int j = 0; j < nB; j++)
    if (lenB[j] > 64 || lenB[j] < 0) return -2;

  // host staging: transpose options, build per-query match masks
  uint8_t *hT = (uint8_t *)calloc((size_t)maxLen * nA, 1);
  unsigned long long *hM = (unsigned long long *)calloc((size_t)nB * 256, sizeof(unsigned long long));
  if (!hT || !hM) {
    free(hT);
    free(hM);
    return -3;
  }
  for (int i = 0; i < nA; i++) {
    for (int k = 0; k < lenA[i]; k++) hT[(size_t)k * nA + i] = opts[off + k];
    off += lenA[i];
  }
  off = 0;
  for (int j = 0; j < nB; j++) {
    for (int k = 0; k < lenB[j]; k++) hM[(size_t)j * 256 + queries[off + k]] |= (1ULL << k);
    off += lenB[j];
  }

  uint8_t *dT = nullptr;
  int *dLA = nullptr, *dLB = nullptr, *dOut = nullptr;
  unsigned long long *dM = nullptr;
  int rc = 0;
  if (hipMalloc(&dT, (size_t)maxLen * nA) != hipSuccess || hipMalloc(&dLA, sizeof(int) * nA) != hipSuccess ||
      hipMalloc(&dLB, sizeof(int) * nB) != hipSuccess || hipMalloc(&dM, sizeof(unsigned long long) * 256 * nB) != hipSuccess ||
      hipMalloc(&dOut, sizeof(int) * (size_t)nA * nB) != hipSuccess) {
    rc = -4;
  }
  if (rc == 0) {
    (void)hipMemcpy(dT, hT, (size_t)maxLen * nA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dLA, lenA, sizeof(int) * nA, hipMemcpyHostToDevice);
    (void)hipMemcpy(dLB, lenB, sizeof(int) * nB, hipMemcpyHostToDevice);
    (void)hipMemcpy(dM, hM, sizeof(unsigned long long) * 256 * nB, hipMemcpyHostToDevice);
    int chunks = (nA + THREADS - 1) / THREADS;
    if (chunks > 1024) chunks = 1024;
    if (chunks >= 8) chunks = (chunks / 8) * 8;  // multiple of 8 enables the XCD remap
    for (int q0 = 0; q0 < nB && rc == 0; q0 += 65535) {
      const int rows = (nB - q0) < 65535 ? (nB - q0) : 65535;
      dim3 grid(chunks, rows);
      hipLaunchKernelGGL(lcs_dist_kernel, grid, dim3(THREADS), 0, 0, dT, dLA, dM, dLB, nA, q0, dOut);
      if (hipGetLastError() != hipSuccess) rc = -5;
    }
    if (rc == 0 && hipDeviceSynchronize() != hipSuccess) rc = -6;
    if (rc == 0) {
      int *hOut = (int *)malloc(sizeof(int) * (size_t)nA * nB);
      if (!hOut) {
        rc = -3;
      } else {
        (void)hipMemcpy(hOut, dOut, sizeof(int) * (size_t)nA * nB, hipMemcpyDeviceToHost);
        for (int j = 0; j < nB; j++)
          for (int i = 0; i < nA; i++) out[(size_t)i * nB + j] = hOut[(size_t)j * nA + i];
        free(hOut);
      }
    }
  }
  (void)hipFree(dT);
  (void)hipFree(dLA);
  (void)hipFree(dLB);
  (void)hipFree(dM);
  (void)hipFree(dOut);
  free(hT);
  free(hM);
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
