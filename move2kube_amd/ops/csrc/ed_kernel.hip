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
// bit-parallel LCS over a DP column of |query| <= 64 bits.
//
// Layout (CDNA4-first; every step below was kept or dropped on rocprofv3
// numbers, see profiles/r01_ed_kernel*):
//  * Byte remap.  The host assigns every byte value that occurs a dense code,
//    most frequent option byte first, code 0 = padding, and (<= 63 symbols)
//    stores code*4 so the LDS byte address of a character is one VALU op.
//    Masks of code 0 are 0, so padding leaves a column unchanged: no
//    per-character length checks.
//  * Query tiles.  Queries are sorted by length and grouped so one pass over
//    the option characters serves several queries: 8 queries <= 16 bytes
//    (two per 32-bit word, v_pk_add_u16 keeps the halves independent),
//    4 <= 32 bytes (one per word) or 2 <= 64 bytes (one u64 each).
//    blockIdx.y = tile; its 4 KiB of masks are staged in LDS as two u64
//    sub-tables, so a character costs two conflict-free ds_read_b64
//    (banked mod 64 over 32-lane groups) whatever the tile kind.
//  * LCS step.  U = V & M; V' = (V + U) | (V & ~M)  (V - U never borrows
//    because U is a subset of V) = and + add + one v_bitop3_b32 per word.
//  * Options are sorted by length and cut into panels of 512 (256 threads x 2
//    options each: two independent chains per lane).  A panel is stored as
//    16-byte blocks [block][slot]: one global_load_dwordx4 gives a lane its
//    next 16 characters, and the next block is prefetched while the current
//    one is consumed.  blockIdx.x walks panels, remapped XCD-aware
//    (consecutive panels of one tile on one XCD's L2).
//  * ed_closest fuses the argmin: key = (dist << 32 | original index), min
//    over the wave by shuffles, over the 4 waves in LDS, then one 64-bit
//    atomicMin per query per workgroup, so only (index, dist) pairs leave
//    the GPU.  Ties resolve to the lowest index, like the reference's scan.
//  * ed_matrix writes a query-major [nB][nA] matrix (Python returns the
//    transposed view); it is bound by the scattered int32 stores and, end to
//    end, by the device-to-host copy of the matrix itself.
//  * Tiles are launched in slabs of <= 65535 (gridDim.y limit).

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

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// Tile kinds: how many queries share one pass over the option characters.
//   K16: 8 queries <= 16 bytes, two per 32-bit word (v_pk_add_u16/v_pk_sub_u16
//        keep the halves independent, exactly two 16-bit LCS columns)
//   K32: 4 queries <= 32 bytes, one per 32-bit word
//   K64: 2 queries <= 64 bytes, one per 64-bit word
enum { K16 = 0, K32 = 1, K64 = 2 };
template <int KIND> struct TileT;
template <> struct TileT<K16> { typedef uint32_t W; enum { NW = 4, NQ = 8 }; };
template <> struct TileT<K32> { typedef uint32_t W; enum { NW = 4, NQ = 4 }; };
template <> struct TileT<K64> { typedef u64 W; enum { NW = 2, NQ = 2 }; };

// One LCS step of a column word against its match mask.  Hyyro's
// V' = (V + U) | (V - U) with U = V & M; U's bits are a subset of V's, so
// V - U borrows nowhere and equals V & ~M:  V' = (V + U) | (V & ~M) - an and,
// an add and one 3-input v_bitop3_b32 per 32-bit word (v2 spent ~4.4 ops).
// f(A, V, M) = A | (V & ~M) as one v_bitop3_b32 (truth table 0xF4, operand
// bits indexing it as A*4 + V*2 + M); spelled out because the compiler emits
// v_bfi + v_or for the 64-bit halves.
__device__ __forceinline__ uint32_t or_andn(uint32_t a, uint32_t v, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(a, v, m, 0xF4);
}

template <int KIND>
__device__ __forceinline__ void lcs_step(typename TileT<KIND>::W &V, typename TileT<KIND>::W m) {
  typedef typename TileT<KIND>::W W;
  const W U = V & m;
  if constexpr (KIND == K16) {
    const uint32_t A = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, V) + __builtin_bit_cast(u16x2, U));
    V = or_andn(A, V, m);
  } else if constexpr (KIND == K32) {
    V = or_andn(V + U, V, m);
  } else {
    const W A = V + U;
    V = ((W)or_andn((uint32_t)(A >> 32), (uint32_t)(V >> 32), (uint32_t)(m >> 32)) << 32) |
        or_andn((uint32_t)A, (uint32_t)V, (uint32_t)m);
  }
}

// Four coded characters of one option against every word of the tile.
//
// LDS layout (4 KiB per tile): two sub-tables of 256 u64 entries, sub-table h
// at byte 2048*h.  K16/K32: entry c of sub-table h = words 2h (low half) and
// 2h+1 (high half) of the code's masks; K64: entry c of sub-table h = query h.
// Each character costs two `ds_read_b64` (bank = (addr/4) mod 64 over 32-lane
// groups, so the <= 32 most frequent codes never conflict; 2 LDS cycles each).
// The second address goes through an empty asm so the compiler cannot fuse
// the pair into `ds_read2st64_b64` - that form banks mod 32 in 16-lane groups
// and cost 8 cycles + ~7 conflict cycles per instruction in PMC (v5).
template <int KIND, bool SCALED>
__device__ __forceinline__ void step4(uint32_t w, const char *T, typename TileT<KIND>::W (&V)[TileT<KIND>::NW]) {
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t c = (w >> (8 * i)) & 0xffu;
    const uint32_t off = SCALED ? c * 2u : c * 8u;  // byte offset of entry c in a u64 table
    uint32_t off1 = off + 2048u;
    __asm__ volatile("" : "+v"(off1));
    const u64 m0 = *reinterpret_cast<const u64 *>(T + off);
    const u64 m1 = *reinterpret_cast<const u64 *>(T + off1);
    if constexpr (KIND == K64) {
      lcs_step<KIND>(V[0], m0);
      lcs_step<KIND>(V[1], m1);
    } else {
      lcs_step<KIND>(V[0], (uint32_t)m0);
      lcs_step<KIND>(V[1], (uint32_t)(m0 >> 32));
      lcs_step<KIND>(V[2], (uint32_t)m1);
      lcs_step<KIND>(V[3], (uint32_t)(m1 >> 32));
    }
  }
}

// LCS columns of this lane's OPT_PER_THREAD options in one panel against the tile.
template <int KIND, bool SCALED>
__device__ __forceinline__ void panel_lcs(const uint4 *__restrict__ panel, int blocks, const char *T,
                                          typename TileT<KIND>::W (&V)[OPT_PER_THREAD][TileT<KIND>::NW]) {
  typedef typename TileT<KIND>::W W;
  const int lane = threadIdx.x;
#pragma unroll
  for (int u = 0; u < OPT_PER_THREAD; u++)
#pragma unroll
    for (int k = 0; k < TileT<KIND>::NW; k++) V[u][k] = ~(W)0;
  if (blocks == 0) return;
  uint4 cur[OPT_PER_THREAD], nxt[OPT_PER_THREAD];
#pragma unroll
  for (int u = 0; u < OPT_PER_THREAD; u++) cur[u] = panel[u * THREADS + lane];
  for (int b = 0; b < blocks; b++) {
    if (b + 1 < blocks) {
#pragma unroll
      for (int u = 0; u < OPT_PER_THREAD; u++) nxt[u] = panel[(size_t)(b + 1) * SLOTS + u * THREADS + lane];
    }
    // the two options' chains interleave word by word
    step4<KIND, SCALED>(cur[0].x, T, V[0]);
    step4<KIND, SCALED>(cur[1].x, T, V[1]);
    step4<KIND, SCALED>(cur[0].y, T, V[0]);
    step4<KIND, SCALED>(cur[1].y, T, V[1]);
    step4<KIND, SCALED>(cur[0].z, T, V[0]);
    step4<KIND, SCALED>(cur[1].z, T, V[1]);
    step4<KIND, SCALED>(cur[0].w, T, V[0]);
    step4<KIND, SCALED>(cur[1].w, T, V[1]);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) cur[u] = nxt[u];
  }
}

// LCS length of tile query j from the final column words.
template <int KIND>
__device__ __forceinline__ int query_lcs(const typename TileT<KIND>::W (&V)[TileT<KIND>::NW], int j, int len) {
  if constexpr (KIND == K16) {
    const uint32_t bits = (~V[j >> 1] >> (16 * (j & 1))) & ((1u << len) - 1u);  // len <= 16
    return __popc(bits);
  } else if constexpr (KIND == K32) {
    const uint32_t mask = len >= 32 ? ~0u : ((1u << len) - 1u);
    return __popc(~V[j] & mask);
  } else {
    const u64 mask = len >= 64 ? ~0ULL : ((1ULL << len) - 1ULL);
    return __popcll(~V[j] & mask);
  }
}

// Stage the tile's mask tables (4 KiB) in LDS.
__device__ __forceinline__ void load_tile(const uint4 *__restrict__ tileM, int tile, uint4 *T) {
  const uint4 *src = tileM + (size_t)tile * 256;
  for (int i = threadIdx.x; i < 256; i += THREADS) T[i] = src[i];
  __syncthreads();
}

}  // namespace

// Tile metadata: tileQ[t][8] = query index (-1 = empty), tileLen[t][8] = its length.
template <int KIND, bool SCALED>
__global__ __launch_bounds__(THREADS) void ed_matrix_kernel(
    const uint4 *__restrict__ panels, const int64_t *__restrict__ panelOff, const int *__restrict__ panelBlocks,
    const int *__restrict__ lenSorted, const int *__restrict__ perm, const uint4 *__restrict__ tileM,
    const int *__restrict__ tileQ, const int *__restrict__ tileLen, int nA, int nPanels, int tile0,
    int *__restrict__ outT) {
  typedef TileT<KIND> TT;
  __shared__ uint4 T[256];
  const int tile = tile0 + blockIdx.y;
  load_tile(tileM, tile, T);
  int qid[TT::NQ], qlen[TT::NQ];
#pragma unroll
  for (int j = 0; j < TT::NQ; j++) qid[j] = tileQ[tile * 8 + j], qlen[j] = tileLen[tile * 8 + j];
  for (int p = remap_panel(blockIdx.x, gridDim.x); p < nPanels; p += gridDim.x) {
    typename TT::W V[OPT_PER_THREAD][TT::NW];
    panel_lcs<KIND, SCALED>(panels + panelOff[p], panelBlocks[p], reinterpret_cast<const char *>(T), V);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) {
      const int s = p * SLOTS + u * THREADS + threadIdx.x;
      const int o = perm[s];
      if (o < 0) continue;
      const int la = lenSorted[s];
#pragma unroll
      for (int j = 0; j < TT::NQ; j++)
        if (qid[j] >= 0) outT[(size_t)qid[j] * nA + o] = la + qlen[j] - 2 * query_lcs<KIND>(V[u], j, qlen[j]);
    }
  }
}

template <int KIND, bool SCALED>
__global__ __launch_bounds__(THREADS) void ed_closest_kernel(
    const uint4 *__restrict__ panels, const int64_t *__restrict__ panelOff, const int *__restrict__ panelBlocks,
    const int *__restrict__ lenSorted, const int *__restrict__ perm, const uint4 *__restrict__ tileM,
    const int *__restrict__ tileQ, const int *__restrict__ tileLen, int nPanels, int tile0, u64 *__restrict__ best) {
  typedef TileT<KIND> TT;
  __shared__ uint4 T[256];
  __shared__ u64 red[THREADS / 64][TT::NQ];
  const int tile = tile0 + blockIdx.y;
  load_tile(tileM, tile, T);
  int qid[TT::NQ], qlen[TT::NQ];
  u64 key[TT::NQ];
#pragma unroll
  for (int j = 0; j < TT::NQ; j++) qid[j] = tileQ[tile * 8 + j], qlen[j] = tileLen[tile * 8 + j], key[j] = ~0ULL;
  for (int p = remap_panel(blockIdx.x, gridDim.x); p < nPanels; p += gridDim.x) {
    typename TT::W V[OPT_PER_THREAD][TT::NW];
    panel_lcs<KIND, SCALED>(panels + panelOff[p], panelBlocks[p], reinterpret_cast<const char *>(T), V);
#pragma unroll
    for (int u = 0; u < OPT_PER_THREAD; u++) {
      const int s = p * SLOTS + u * THREADS + threadIdx.x;
      const int o = perm[s];
      if (o < 0) continue;
      const int la = lenSorted[s];
#pragma unroll
      for (int j = 0; j < TT::NQ; j++) {
        const int d = la + qlen[j] - 2 * query_lcs<KIND>(V[u], j, qlen[j]);
        const u64 k = ((u64)(unsigned)d << 32) | (unsigned)o;
        key[j] = k < key[j] ? k : key[j];
      }
    }
  }
  // argmin per query: wave shuffles, then the 4 waves through LDS, one atomic each
#pragma unroll
  for (int j = 0; j < TT::NQ; j++) {
    u64 k = key[j];
    for (int off = 32; off > 0; off >>= 1) {
      const u64 o = __shfl_xor(k, off, 64);
      k = o < k ? o : k;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x / 64][j] = k;
  }
  __syncthreads();
  if (threadIdx.x < TT::NQ) {
    const int j = threadIdx.x;
    const int q = tileQ[tile * 8 + j];  // (not qid[j]: a dynamic index would spill the array)
    u64 k = red[0][j];
    for (int w = 1; w < THREADS / 64; w++) k = red[w][j] < k ? red[w][j] : k;
    if (q >= 0 && k != ~0ULL) atomicMin(&best[q], k);
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
  int nTiles = 0, kindStart[3] = {0, 0, 0}, kindCount[3] = {0, 0, 0};
  int64_t totalU4 = 0;
  size_t oPanels = 0, oPanelOff = 0, oPanelBlocks = 0, oLenSorted = 0, oPerm = 0;
  size_t oTileM = 0, oTileQ = 0, oTileLen = 0;
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

  // Query tiles, by length class: 8 x <=16 B (16-bit halves), 4 x <=32 B, 2 x <=64 B.
  std::vector<int> qorder(nB);
  {
    int start[66] = {0};
    for (int j = 0; j < nB; j++) start[(int)(offB[j + 1] - offB[j]) + 1]++;
    for (int l = 0; l <= 64; l++) start[l + 1] += start[l];
    for (int j = 0; j < nB; j++) qorder[start[(int)(offB[j + 1] - offB[j])]++] = j;
  }
  std::vector<int> tileQ, tileLen;
  int kindOfPrev = -1, fill = 0;
  for (int r = 0; r < nB; r++) {
    const int j = qorder[r];
    const int len = (int)(offB[j + 1] - offB[j]);
    const int kind = len <= 16 ? K16 : (len <= 32 ? K32 : K64);
    const int cap = 8 >> kind;
    if (kind != kindOfPrev || fill == cap) {
      if (kind != kindOfPrev) L.kindStart[kind] = (int)(tileQ.size() / 8);
      tileQ.insert(tileQ.end(), 8, -1);
      tileLen.insert(tileLen.end(), 8, 0);
      L.kindCount[kind]++;
      kindOfPrev = kind;
      fill = 0;
    }
    tileQ[tileQ.size() - 8 + fill] = j;
    tileLen[tileLen.size() - 8 + fill] = len;
    fill++;
  }
  L.nTiles = (int)(tileQ.size() / 8);

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
  L.oTileQ = o;
  o = align256(o + sizeof(int) * (size_t)L.nTiles * 8);
  L.oTileLen = o;
  o = align256(o + sizeof(int) * (size_t)L.nTiles * 8);
  L.oTileM = o;
  o = align256(o + (size_t)4096 * L.nTiles);
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
  memcpy(h + L.oTileQ, tileQ.data(), sizeof(int) * tileQ.size());
  memcpy(h + L.oTileLen, tileLen.data(), sizeof(int) * tileLen.size());
  char *tm = h + L.oTileM;
  par_for(L.nTiles, nt, 32, [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; t++) {
      char *T = tm + (size_t)t * 4096;
      memset(T, 0, 4096);
      const int kind = t >= L.kindStart[K64] && L.kindCount[K64] && t < L.kindStart[K64] + L.kindCount[K64]
                           ? K64
                           : (t >= L.kindStart[K32] && L.kindCount[K32] && t < L.kindStart[K32] + L.kindCount[K32]
                                  ? K32
                                  : K16);
      for (int slot = 0; slot < (8 >> kind); slot++) {
        const int j = tileQ[t * 8 + slot];
        if (j < 0) continue;
        const int len = tileLen[t * 8 + slot];
        for (int k = 0; k < len; k++) {
          const int c = code[qs[offB[j] + k]];
          // word = the 32-bit column word holding this query; sub-table word/2, half word%2
          u64 *T64 = reinterpret_cast<u64 *>(T);
          if (kind == K64) {
            T64[slot * 256 + c] |= 1ULL << k;
          } else {
            const int word = kind == K32 ? slot : (slot >> 1);
            const int bit = kind == K32 ? k : k + 16 * (slot & 1);
            T64[(word >> 1) * 256 + c] |= (u64)(1u << bit) << (32 * (word & 1));
          }
        }
      }
    }
  });
  return 0;
}

int grid_x(int nPanels, int tiles) {
  // ~4k workgroups per launch: ~2 rounds of the 256 CUs x 7 resident 256-thread
  // groups, each walking enough panels to amortise staging its 4 KiB tile table
  // and the per-query reductions (16k tiny groups measured 3x slower for K16).
  // x is a multiple of 8 for the XCD remap.
  static const int target = getenv("M2K_ED_WGS") ? std::max(1, atoi(getenv("M2K_ED_WGS"))) : 4096;
  int want = (target + tiles - 1) / tiles;
  want = std::max(8, std::min(want, 1024));
  int x = std::min(nPanels, want);
  if (x >= 8) x = (x / 8) * 8;
  return x < 1 ? 1 : x;
}

struct DevPtrs {
  const uint4 *panels;
  const int64_t *panelOff;
  const int *panelBlocks, *lenSorted, *perm, *tileQ, *tileLen;
  const uint4 *tileM;
  u64 *best;
};

DevPtrs dev_ptrs(const Arena &ar, const Layout &L) {
  char *d = ar.dev;
  return {reinterpret_cast<const uint4 *>(d + L.oPanels), reinterpret_cast<const int64_t *>(d + L.oPanelOff),
          reinterpret_cast<const int *>(d + L.oPanelBlocks), reinterpret_cast<const int *>(d + L.oLenSorted),
          reinterpret_cast<const int *>(d + L.oPerm),        reinterpret_cast<const int *>(d + L.oTileQ),
          reinterpret_cast<const int *>(d + L.oTileLen),     reinterpret_cast<const uint4 *>(d + L.oTileM),
          reinterpret_cast<u64 *>(d + L.oBest)};
}

template <int KIND, bool SCALED>
int launch_kind(const Layout &L, const DevPtrs &d, int nA, int *out, hipStream_t s) {
  const int count = L.kindCount[KIND];
  if (count == 0) return 0;
  const int gx = grid_x(L.nPanels, count);
  for (int t = 0; t < count; t += MAX_Y) {
    const int rows = std::min(MAX_Y, count - t);
    const int tile0 = L.kindStart[KIND] + t;
    if (out)
      hipLaunchKernelGGL((ed_matrix_kernel<KIND, SCALED>), dim3(gx, rows), dim3(THREADS), 0, s, d.panels, d.panelOff,
                         d.panelBlocks, d.lenSorted, d.perm, d.tileM, d.tileQ, d.tileLen, nA, L.nPanels, tile0, out);
    else
      hipLaunchKernelGGL((ed_closest_kernel<KIND, SCALED>), dim3(gx, rows), dim3(THREADS), 0, s, d.panels,
                         d.panelOff, d.panelBlocks, d.lenSorted, d.perm, d.tileM, d.tileQ, d.tileLen, L.nPanels, tile0,
                         d.best);
    if (hipGetLastError() != hipSuccess) return -5;
  }
  return 0;
}

template <bool SCALED>
int launch_all(const Layout &L, const DevPtrs &d, int nA, int *out, hipStream_t s) {
  int rc = launch_kind<K16, SCALED>(L, d, nA, out, s);
  if (rc == 0) rc = launch_kind<K32, SCALED>(L, d, nA, out, s);
  if (rc == 0) rc = launch_kind<K64, SCALED>(L, d, nA, out, s);
  return rc;
}

int launch_matrix(const Layout &L, const DevPtrs &d, int nA, int *out, hipStream_t s) {
  return L.scaled ? launch_all<true>(L, d, nA, out, s) : launch_all<false>(L, d, nA, out, s);
}

int launch_closest(const Layout &L, const DevPtrs &d, hipStream_t s) {
  return L.scaled ? launch_all<true>(L, d, 0, nullptr, s) : launch_all<false>(L, d, 0, nullptr, s);
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
  rc = launch_matrix(L, d, nA, ar.out, s);
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
  rc = launch_closest(L, d, s);
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
