// sme_sort.hip -- the shuffle sort of the index job: (term, posting) pairs
// ordered by term id, stable, so the postings of a term keep the docno order
// the aggregation emitted them in (the reducer's docno sort,
// TermKGramDocIndexer.java:168-213; key order TermDF.compareTo,
// TermDF.java:64-70 = term id order, ids being String.compareTo ranks).
//
// LSD radix sort over the term id, <= 11-bit digits (2 passes for the 21-bit
// ids of c2).  Each pass is reduce-then-scan, no inter-block waiting:
//   k_rs_count   one 8192-item tile per 512-thread block: LDS digit
//                histogram, written tile-major (coalesced)
//   k_rs_colsum  per (digit, tile group) sums, up to 1024 groups (c2's 45 k
//                tiles x 2048 digits are 372 MB, which 256 groups of 178 tiles
//                read at 1.3 TB/s); an exclusive scan over them in digit-major
//                order (one block, or device-wide when long); k_rs_colscan turns
//                the tile counts into each (tile, digit)'s global output offset
//   k_rs_scatter each wave ranks its 1024 contiguous items with ballot peer
//                masks and running per-wave digit counters in LDS (stable);
//                the block scans those counters (digits, then waves) into the
//                tile's digit-sorted order, stages keys and then values in
//                LDS in that order, and writes them out as contiguous runs
//                per digit (offset(tile, digit) + slot - digit's first slot).
// The last pass writes the sorted keys and unpacks the packed values
// ((docno - dmin) * F + tf) straight into the CSR's docno / tf arrays.
#include <hip/hip_runtime.h>

#include "sme_internal.hpp"

namespace sme {
namespace {

#ifndef SME_RSNT
#define SME_RSNT 512
#endif
constexpr int kRsNT = SME_RSNT;             // threads per block (8 waves: two blocks per CU overlap their phases)
constexpr int kRsWaves = kRsNT / 64;
constexpr int kRsIPL = 16;                  // items per lane
constexpr int kRsTile = kRsNT * kRsIPL;     // items per tile
constexpr int kRsWaveItems = 64 * kRsIPL;   // 1024 contiguous items per wave
constexpr int kRsMaxBits = 11;
constexpr int kRsMaxBins = 1 << kRsMaxBits;
constexpr int kRsBPT = kRsMaxBins / kRsNT;  // digits per thread in the scatter's tile scan
constexpr int kRsGroups = 1024;             // most tile groups of the column scan
constexpr int kRsScanSums = 1024;           // device scan of the (digit, group) sums: its tile sums

// Tile groups of the column scan: at least 4 tiles a group, so the one-block
// scan over (digit, group) sums stays short for small sorts; a multiple of 16
// (the scan's granule; groups past the last tile sum to 0).
struct RsGroups {
  int64_t tpg;
  int G;
};
static RsGroups rs_groups(int64_t ntiles) {
  const int64_t tpg = std::max<int64_t>(4, (ntiles + kRsGroups - 1) / kRsGroups);
  const int64_t g = (ntiles + tpg - 1) / tpg;
  return RsGroups{tpg, (int)((g + 15) / 16 * 16)};
}

// Gather mode (first pass after the single-pass aggregation): pair x of the
// docno order lives in the region of the record i holding it,
// reg[i] + (x - xoff[i]) (xoff = exclusive scan of the records' pair counts);
// crec[c] = the record holding pair 1024 c, so a wave's walk over its 1024
// items starts there and advances a record at a time.
struct Gather {
  const int64_t *reg, *xoff, *crec;
  int64_t nrec;
};
__device__ __forceinline__ void gather_start(const Gather &g, int64_t x, int64_t &rec, int64_t &nx, int64_t &dl) {
  rec = g.crec[x >> 10];
  nx = g.xoff[rec + 1];
  dl = g.reg[rec] - g.xoff[rec];
}
__device__ __forceinline__ int64_t gather_pos(const Gather &g, int64_t x, int64_t &rec, int64_t &nx, int64_t &dl) {
  while (x >= nx) {
    rec++;
    nx = g.xoff[rec + 1];
    dl = g.reg[rec] - g.xoff[rec];
  }
  return x + dl;
}
// A wave's 1024 items span a few records: lane j loads record rec0 + j's pair
// start and region delta into LDS once, so the per-item walk reads LDS and the
// item loads are not held behind dependent global loads (vmcnt is in order).
// Walks past kGRec records fall back to the global walk.
constexpr int kGRec = 48;  // (LDS: two 512-thread scatter blocks per CU)
__device__ __forceinline__ int64_t gather_table(const Gather &g, int64_t x0, int lane, int64_t *gx, int64_t *gdl) {
  const int64_t rec0 = g.crec[x0 >> 10];
  const int64_t r = rec0 + lane;
  if (lane < kGRec) {
    gx[lane] = r <= g.nrec ? g.xoff[r] : INT64_MAX;
    gdl[lane] = r < g.nrec ? g.reg[r] - g.xoff[r] : 0;
  }
  if (lane == 0) gx[kGRec] = rec0 + kGRec <= g.nrec ? g.xoff[rec0 + kGRec] : INT64_MAX;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return rec0;
}
__device__ __forceinline__ int64_t gather_at(const Gather &g, int64_t x, int &j, const int64_t *gx, const int64_t *gdl,
                                             int64_t rec0) {
  while (j < kGRec - 1 && x >= gx[j + 1]) j++;
  if (x < gx[j + 1]) return x + gdl[j];
  int64_t rec = rec0 + kGRec - 1, nx = g.xoff[rec + 1], dl = g.reg[rec] - g.xoff[rec];
  return gather_pos(g, x, rec, nx, dl);
}
__global__ void k_rs_chunk_rec(const int64_t *__restrict__ xoff, int64_t nrec, int64_t P, int64_t *__restrict__ crec) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; (c << 10) < P; c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = c << 10;
    int64_t lo = 0, hi = nrec;  // last record i with xoff[i] <= x
    while (hi - lo > 1) {
      const int64_t m = (lo + hi) >> 1;
      if (xoff[m] <= x) lo = m;
      else hi = m;
    }
    crec[c] = lo;
  }
}

__global__ __launch_bounds__(kRsNT) void k_rs_count(const uint32_t *__restrict__ key, int64_t P, int shift,
                                                    int nbins, uint32_t *__restrict__ counts, Gather g) {
  __shared__ uint32_t h[kRsMaxBins];
  const int tid = threadIdx.x;
  for (int b = tid; b < nbins; b += kRsNT) h[b] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kRsTile;
  const uint32_t mask = (uint32_t)nbins - 1u;
  const int64_t n = min((int64_t)kRsTile, P - t0);
  if (g.reg != nullptr) {
    __shared__ int64_t gx_all[kRsWaves][kGRec + 1], gdl_all[kRsWaves][kGRec];
    const int lane = tid & 63, w = tid >> 6;
    const int64_t wb = t0 + (int64_t)w * kRsWaveItems;
    if (wb < P) {
      const int64_t rec0 = gather_table(g, wb, lane, gx_all[w], gdl_all[w]);
      int j = 0;
      uint32_t kk[kRsIPL];
#pragma unroll
      for (int s = 0; s < kRsIPL; s++) {
        const int64_t x = wb + s * 64 + lane;
        kk[s] = x < P ? key[gather_at(g, x, j, gx_all[w], gdl_all[w], rec0)] : 0u;
      }
#pragma unroll
      for (int s = 0; s < kRsIPL; s++)
        if (wb + s * 64 + lane < P) atomicAdd(&h[(kk[s] >> shift) & mask], 1u);
    }
  } else if (n == kRsTile) {
    const uint4 *k4 = reinterpret_cast<const uint4 *>(key + t0);
#pragma unroll
    for (int i = 0; i < kRsIPL / 4; i++) {
      const uint4 v = k4[i * kRsNT + tid];
      atomicAdd(&h[(v.x >> shift) & mask], 1u);
      atomicAdd(&h[(v.y >> shift) & mask], 1u);
      atomicAdd(&h[(v.z >> shift) & mask], 1u);
      atomicAdd(&h[(v.w >> shift) & mask], 1u);
    }
  } else {
    for (int64_t i = tid; i < n; i += kRsNT) atomicAdd(&h[(key[t0 + i] >> shift) & mask], 1u);
  }
  __syncthreads();
  for (int b = tid; b < nbins; b += kRsNT) counts[(int64_t)blockIdx.x * nbins + b] = h[b];
}

// gsum[b * G + g] = sum of counts[t][b] over the tiles t of group g
__global__ __launch_bounds__(kRsNT) void k_rs_colsum(const uint32_t *__restrict__ counts, int64_t ntiles, int nbins,
                                                     int64_t tpg, int G, uint32_t *__restrict__ gsum) {
  const int g = blockIdx.x;
  const int64_t ta = (int64_t)g * tpg, tb = min(ntiles, ta + tpg);
  for (int b = threadIdx.x; b < nbins; b += kRsNT) {
    uint32_t s = 0;
    for (int64_t t = ta; t < tb; t++) s += counts[t * nbins + b];
    gsum[(int64_t)b * G + g] = s;
  }
}

// in-place exclusive scan of n u32 (one block; n a multiple of 16): rounds
// of 8192, 16 contiguous elements per thread (four 16-byte loads); the next
// round's loads are issued before this round's barriers (latency-bound kernel)
__global__ __launch_bounds__(kRsNT) void k_rs_scan(uint32_t *__restrict__ a, int n) {
  __shared__ uint32_t ws[kRsWaves];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint32_t carry = 0;
  uint4 x[4];
  auto load = [&](int r0, uint4 *y) {
    const int i0 = r0 + 16 * tid;
#pragma unroll
    for (int c = 0; c < 4; c++) y[c] = i0 < n ? reinterpret_cast<const uint4 *>(a + i0)[c] : make_uint4(0, 0, 0, 0);
  };
  load(0, x);
  for (int r0 = 0; r0 < n; r0 += 16 * kRsNT) {
    const int i0 = r0 + 16 * tid;
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) s += x[c].x + x[c].y + x[c].z + x[c].w;
    uint32_t incl = s;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    uint4 xn[4];
    load(r0 + 16 * kRsNT, xn);
    __syncthreads();
    uint32_t wb = carry, tot = 0;
    for (int j = 0; j < kRsWaves; j++) {
      const uint32_t t = ws[j];
      if (j < w) wb += t;
      tot += t;
    }
    uint32_t run = wb + incl - s;
    if (i0 < n) {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        uint4 y;
        y.x = run;
        run += x[c].x;
        y.y = run;
        run += x[c].y;
        y.z = run;
        run += x[c].z;
        y.w = run;
        run += x[c].w;
        reinterpret_cast<uint4 *>(a + i0)[c] = y;
      }
    }
    carry += tot;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; c++) x[c] = xn[c];
  }
}

// counts[t][b] <- global offset of digit b's items of tile t
__global__ __launch_bounds__(kRsNT) void k_rs_colscan(uint32_t *__restrict__ counts, int64_t ntiles, int nbins,
                                                      int64_t tpg, int G, const uint32_t *__restrict__ gsum) {
  const int g = blockIdx.x;
  const int64_t ta = (int64_t)g * tpg, tb = min(ntiles, ta + tpg);
  for (int b = threadIdx.x; b < nbins; b += kRsNT) {
    uint32_t run = gsum[(int64_t)b * G + g];
    for (int64_t t = ta; t < tb; t++) {
      const uint32_t c = counts[t * nbins + b];
      counts[t * nbins + b] = run;
      run += c;
    }
  }
}

template <bool LAST>
__global__ __launch_bounds__(kRsNT) void k_rs_scatter(const uint32_t *__restrict__ key, const uint32_t *__restrict__ val,
                                                      int64_t P, int shift, int nbits,
                                                      const uint32_t *__restrict__ offs, uint32_t *__restrict__ okey,
                                                      uint32_t *__restrict__ oval, int32_t *__restrict__ odocno,
                                                      int32_t *__restrict__ otf, int64_t dmin, uint32_t F,
                                                      Gather g, const double *__restrict__ lut, double idf,
                                                      double *__restrict__ ow, const uint2 *__restrict__ xw) {
  // wc: per-wave running digit counts, then each (wave, digit)'s first slot in
  // the tile sorted by digit; gd: global offset - tile slot of each digit
  __shared__ uint16_t wc[kRsWaves * kRsMaxBins];
  __shared__ uint32_t gd[kRsMaxBins];
  __shared__ uint32_t stage[kRsTile];
  __shared__ uint32_t ws[kRsWaves];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nbins = 1 << nbits;
  const uint32_t mask = (uint32_t)nbins - 1u;
  // XCD-aware tile order: blocks are dealt round-robin to the 8 XCDs, so XCD x
  // gets the contiguous tile range [x * per, (x + 1) * per).  Neighbouring
  // tiles write neighbouring pieces of every digit's run at about the same
  // time, and those partial lines meet in one L2 instead of reaching HBM as
  // partial writes from different XCDs.
  const int64_t per = (int64_t)(gridDim.x >> 3);
  const int64_t tile = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const int64_t t0 = tile * kRsTile;
  if (t0 >= P) return;
  const int n = (int)min((int64_t)kRsTile, P - t0);
  for (int i = tid; i < kRsWaves * kRsMaxBins / 2; i += kRsNT) reinterpret_cast<uint32_t *>(wc)[i] = 0u;
  __syncthreads();
  uint16_t *mine = wc + w * kRsMaxBins;
  const int wb = w * kRsWaveItems;  // this wave's items: tile slots [wb, wb + 1024)
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t k[kRsIPL], v[kRsIPL], pos[kRsIPL];
  if (g.reg != nullptr) {
    __shared__ int64_t gx_all[kRsWaves][kGRec + 1], gdl_all[kRsWaves][kGRec];
    int64_t rec0 = 0;
    if (wb < n) rec0 = gather_table(g, t0 + wb, lane, gx_all[w], gdl_all[w]);
    int j = 0;
#pragma unroll
    for (int s = 0; s < kRsIPL; s++) {
      const int i = wb + s * 64 + lane;
      k[s] = 0u;
      v[s] = 0u;
      if (i < n) {
        const int64_t p = gather_at(g, t0 + i, j, gx_all[w], gdl_all[w], rec0);
        k[s] = key[p];
        v[s] = val[p];
      }
    }
  } else {
#pragma unroll
    for (int s = 0; s < kRsIPL; s++) {
      const int i = wb + s * 64 + lane;
      const bool ok = i < n;
      k[s] = ok ? key[t0 + i] : 0u;
      v[s] = ok ? val[t0 + i] : 0u;
    }
  }
  // 1. stable rank of every item among its wave's items of the same digit
#pragma unroll
  for (int s = 0; s < kRsIPL; s++) {
    const bool ok = wb + s * 64 + lane < n;
    const uint32_t d = (k[s] >> shift) & mask;
    uint64_t peers = (uint64_t)__ballot(ok);
    for (int b = 0; b < nbits; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = (uint64_t)__ballot(bit);
      peers &= bit ? m : ~m;
    }
    uint32_t r = 0;
    if (ok) {
      const uint32_t c = mine[d];
      r = c + (uint32_t)__popcll(peers & lt);
      if ((peers & lt) == 0) mine[d] = (uint16_t)(c + (uint32_t)__popcll(peers));
    }
    pos[s] = r;
  }
  __syncthreads();
  // 2. tile slot of each (wave, digit): digits in order, waves in order
  {
    const int b0 = kRsBPT * tid;  // this thread's digits b0 .. b0 + kRsBPT - 1
    uint32_t tc[kRsBPT];
    uint32_t s2 = 0;
#pragma unroll
    for (int q = 0; q < kRsBPT; q++) {
      tc[q] = 0;
      if (b0 + q < nbins) {
#pragma unroll
        for (int x = 0; x < kRsWaves; x++) tc[q] += wc[x * kRsMaxBins + b0 + q];
      }
      s2 += tc[q];
    }
    uint32_t incl = s2;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t ex = incl - s2;
    for (int j = 0; j < w; j++) ex += ws[j];
#pragma unroll
    for (int q = 0; q < kRsBPT; q++) {
      if (b0 + q < nbins) {
        uint32_t r = ex;
        gd[b0 + q] = offs[tile * nbins + b0 + q] - r;
#pragma unroll
        for (int x = 0; x < kRsWaves; x++) {
          const uint32_t c = wc[x * kRsMaxBins + b0 + q];
          wc[x * kRsMaxBins + b0 + q] = (uint16_t)r;
          r += c;
        }
      }
      ex += tc[q];
    }
  }
  __syncthreads();
  // 3. keys through LDS in digit order, then coalesced runs to their digits
#pragma unroll
  for (int s = 0; s < kRsIPL; s++) {
    if (wb + s * 64 + lane >= n) continue;
    pos[s] += mine[(k[s] >> shift) & mask];
    stage[pos[s]] = k[s];
  }
  __syncthreads();
  uint32_t dst[kRsIPL];
#pragma unroll
  for (int j = 0; j < kRsIPL; j++) {
    const int p = j * kRsNT + tid;
    if (p < n) {
      const uint32_t kk = stage[p];
      dst[j] = gd[(kk >> shift) & mask] + (uint32_t)p;
      if (LAST && xw) {  // K6b: word kk's docid shift and merged id
        const uint2 x = xw[kk];
        dst[j] += x.x;
        okey[dst[j]] = x.y;
      } else {
        okey[dst[j]] = kk;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int s = 0; s < kRsIPL; s++)
    if (wb + s * 64 + lane < n) stage[pos[s]] = v[s];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRsIPL; j++) {
    const int p = j * kRsNT + tid;
    if (p < n) {
      const uint32_t vv = stage[p];
      if (LAST) {
        odocno[dst[j]] = (int32_t)((int64_t)(vv / F) + dmin);
        otf[dst[j]] = (int32_t)(vv % F);
        // the TF-IDF weight pass fused in for one idf for every term (reference
        // mode, T1/T2): w = (1 + ln tf) * log10(N / 1), fp64, no contraction
        if (ow) ow[dst[j]] = __dmul_rn(lut[vv % F], idf);
      } else {
        oval[dst[j]] = vv;
      }
    }
  }
}

// Generic stable (key, u32 value) pass for the build's other sorts (vocabulary
// words, docid words): the same reduce-then-scan structure, plain coalesced
// loads, 32- or 64-bit keys staged through LDS as 32-bit halves.
template <typename K>
__global__ __launch_bounds__(kRsNT) void k_kv_count(const K *__restrict__ key, int64_t n, int shift, int nbins,
                                                    uint32_t *__restrict__ counts) {
  __shared__ uint32_t h[kRsMaxBins];
  const int tid = threadIdx.x;
  for (int b = tid; b < nbins; b += kRsNT) h[b] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kRsTile;
  const int m = (int)min((int64_t)kRsTile, n - t0);
  const uint32_t mask = (uint32_t)nbins - 1u;
  for (int i = tid; i < m; i += kRsNT) atomicAdd(&h[(uint32_t)(key[t0 + i] >> shift) & mask], 1u);
  __syncthreads();
  for (int b = tid; b < nbins; b += kRsNT) counts[(int64_t)blockIdx.x * nbins + b] = h[b];
}

template <typename K, bool KEYS>
__global__ __launch_bounds__(kRsNT) void k_kv_scatter(const K *__restrict__ key, const uint32_t *__restrict__ val,
                                                      int64_t n_all, int shift, int nbits,
                                                      const uint32_t *__restrict__ offs, K *__restrict__ okey,
                                                      uint32_t *__restrict__ oval) {
  __shared__ uint16_t wc[kRsWaves * kRsMaxBins];
  __shared__ uint32_t gd[kRsMaxBins];
  __shared__ uint32_t stage[kRsTile];
  __shared__ uint32_t ws[kRsWaves];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nbins = 1 << nbits;
  const uint32_t mask = (uint32_t)nbins - 1u;
  const int64_t per = (int64_t)(gridDim.x >> 3);  // XCD-aware tile order, as k_rs_scatter
  const int64_t tile = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  const int64_t t0 = tile * kRsTile;
  if (t0 >= n_all) return;
  const int n = (int)min((int64_t)kRsTile, n_all - t0);
  for (int i = tid; i < kRsWaves * kRsMaxBins / 2; i += kRsNT) reinterpret_cast<uint32_t *>(wc)[i] = 0u;
  __syncthreads();
  uint16_t *mine = wc + w * kRsMaxBins;
  const int wb = w * kRsWaveItems;
  const uint64_t lt = (1ull << lane) - 1ull;
  K k[kRsIPL];
  uint32_t v[kRsIPL], pos[kRsIPL];
#pragma unroll
  for (int s = 0; s < kRsIPL; s++) {
    const int i = wb + s * 64 + lane;
    const bool ok = i < n;
    k[s] = ok ? key[t0 + i] : (K)0;
    v[s] = ok ? val[t0 + i] : 0u;
  }
#pragma unroll
  for (int s = 0; s < kRsIPL; s++) {
    const bool ok = wb + s * 64 + lane < n;
    const uint32_t d = (uint32_t)(k[s] >> shift) & mask;
    uint64_t peers = (uint64_t)__ballot(ok);
    for (int b = 0; b < nbits; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = (uint64_t)__ballot(bit);
      peers &= bit ? m : ~m;
    }
    uint32_t r = 0;
    if (ok) {
      const uint32_t c = mine[d];
      r = c + (uint32_t)__popcll(peers & lt);
      if ((peers & lt) == 0) mine[d] = (uint16_t)(c + (uint32_t)__popcll(peers));
    }
    pos[s] = r;
  }
  __syncthreads();
  {
    const int b0 = kRsBPT * tid;
    uint32_t tc[kRsBPT];
    uint32_t s2 = 0;
#pragma unroll
    for (int q = 0; q < kRsBPT; q++) {
      tc[q] = 0;
      if (b0 + q < nbins) {
#pragma unroll
        for (int x = 0; x < kRsWaves; x++) tc[q] += wc[x * kRsMaxBins + b0 + q];
      }
      s2 += tc[q];
    }
    uint32_t incl = s2;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) ws[w] = incl;
    __syncthreads();
    uint32_t ex = incl - s2;
    for (int j = 0; j < w; j++) ex += ws[j];
#pragma unroll
    for (int q = 0; q < kRsBPT; q++) {
      if (b0 + q < nbins) {
        uint32_t r = ex;
        gd[b0 + q] = offs[tile * nbins + b0 + q] - r;
#pragma unroll
        for (int x = 0; x < kRsWaves; x++) {
          const uint32_t c = wc[x * kRsMaxBins + b0 + q];
          wc[x * kRsMaxBins + b0 + q] = (uint16_t)r;
          r += c;
        }
      }
      ex += tc[q];
    }
  }
  __syncthreads();
  // each slot's digit through LDS first (its output offset), then the key's
  // 32-bit halves and the values, each staged in digit order and written out
#pragma unroll
  for (int s = 0; s < kRsIPL; s++) {
    if (wb + s * 64 + lane >= n) continue;
    pos[s] += mine[(uint32_t)(k[s] >> shift) & mask];
    stage[pos[s]] = (uint32_t)(k[s] >> shift) & mask;
  }
  __syncthreads();
  uint32_t dst[kRsIPL];
#pragma unroll
  for (int j = 0; j < kRsIPL; j++) {
    const int p = j * kRsNT + tid;
    if (p < n) dst[j] = gd[stage[p]] + (uint32_t)p;
  }
  constexpr int kHalves = KEYS ? (int)(sizeof(K) / 4) : 0;
#pragma unroll
  for (int hf = 0; hf <= kHalves; hf++) {
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kRsIPL; s++)
      if (wb + s * 64 + lane < n) stage[pos[s]] = hf < kHalves ? (uint32_t)((uint64_t)k[s] >> (32 * hf)) : v[s];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRsIPL; j++) {
      const int p = j * kRsNT + tid;
      if (p < n) {
        if (hf < kHalves) reinterpret_cast<uint32_t *>(okey + dst[j])[hf] = stage[p];
        else oval[dst[j]] = stage[p];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Device-wide exclusive scan (reduce-then-scan, no inter-block waiting): one
// 4096-item tile per 256-thread block.  k_sc_sums: each tile's sum (coalesced
// loads, a wave reduction); k_sc_carry: one block scans the tile sums in place
// (rounds of 4096, a running carry); k_sc_apply: each tile staged in LDS, each
// thread scans 16 contiguous items, the block scans the thread totals, and the
// results go out with the tile's carry.  in == out is allowed.
constexpr int kScNT = 256, kScIPT = 16, kScTile = kScNT * kScIPT;

template <typename T>
__device__ __forceinline__ T sc_block_excl(T v, T *ws, T *total) {  // 256 threads
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) ws[w] = incl;
  __syncthreads();
  T base = 0, tot = 0;
  for (int j = 0; j < kScNT / 64; j++) {
    if (j < w) base += ws[j];
    tot += ws[j];
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

template <typename T>
__global__ __launch_bounds__(kScNT) void k_sc_sums(const T *__restrict__ in, int64_t n, T *__restrict__ sums) {
  __shared__ T ws[kScNT / 64];
  const int64_t t0 = (int64_t)blockIdx.x * kScTile;
  T s = 0;
#pragma unroll
  for (int j = 0; j < kScIPT; j++) {
    const int64_t i = t0 + j * kScNT + threadIdx.x;
    if (i < n) s += in[i];
  }
  T tot;
  (void)sc_block_excl<T>(s, ws, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

template <typename T>
__global__ __launch_bounds__(kScNT) void k_sc_carry(T *__restrict__ a, int64_t n) {
  __shared__ T ws[kScNT / 64];
  T carry = 0;
  for (int64_t r0 = 0; r0 < n; r0 += kScTile) {
    const int64_t i0 = r0 + (int64_t)threadIdx.x * kScIPT;
    T x[kScIPT], s = 0;
#pragma unroll
    for (int j = 0; j < kScIPT; j++) {
      x[j] = i0 + j < n ? a[i0 + j] : (T)0;
      s += x[j];
    }
    T tot;
    T run = carry + sc_block_excl<T>(s, ws, &tot);
#pragma unroll
    for (int j = 0; j < kScIPT; j++) {
      if (i0 + j < n) a[i0 + j] = run;
      run += x[j];
    }
    carry += tot;
  }
}

template <typename T>
__global__ __launch_bounds__(kScNT) void k_sc_apply(const T *in, T *out, int64_t n, const T *__restrict__ carry) {
  // one pad slot every 16 items: thread t's 16 contiguous items start at bank 17 t
  __shared__ T st[kScTile + kScTile / 16];
  __shared__ T ws[kScNT / 64];
  auto P = [](int i) { return i + (i >> 4); };
  const int64_t t0 = (int64_t)blockIdx.x * kScTile;
#pragma unroll
  for (int j = 0; j < kScIPT; j++) {
    const int64_t i = t0 + j * kScNT + threadIdx.x;
    st[P(j * kScNT + threadIdx.x)] = i < n ? in[i] : (T)0;
  }
  __syncthreads();
  T x[kScIPT], s = 0;
#pragma unroll
  for (int j = 0; j < kScIPT; j++) {
    x[j] = st[P(threadIdx.x * kScIPT + j)];
    s += x[j];
  }
  T tot;
  T run = carry[blockIdx.x] + sc_block_excl<T>(s, ws, &tot);
#pragma unroll
  for (int j = 0; j < kScIPT; j++) {
    st[P(threadIdx.x * kScIPT + j)] = run;
    run += x[j];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kScIPT; j++) {
    const int64_t i = t0 + j * kScNT + threadIdx.x;
    if (i < n) out[i] = st[P(j * kScNT + threadIdx.x)];
  }
}

// compaction: out[k] = i for the k-th i in [0, n) with flag[i] != 0 (ascending),
// *count = the number of them; pos = exclusive scan of the flags (as int64)
__global__ void k_flags_i64(const uint8_t *__restrict__ f, int64_t n, int64_t *__restrict__ v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = f[i] ? 1 : 0;
}
__global__ void k_select_scatter(const uint8_t *__restrict__ f, const int64_t *__restrict__ pos, int64_t n,
                                 int32_t *__restrict__ out, int32_t *__restrict__ count) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (f[i]) out[pos[i]] = (int32_t)i;
    if (i == n - 1) *count = (int32_t)(pos[i] + (f[i] ? 1 : 0));
  }
}

// exclusive scan of the n (digit, group) sums in place: one block when short,
// else the device-wide reduce-then-scan (sums: kRsScanSums u32 of scratch)
void rs_scan(uint32_t *gsum, int64_t n, uint32_t *sums, hipStream_t st) {
  if (n <= 16 * 4 * kRsNT) {
    hipLaunchKernelGGL(k_rs_scan, dim3(1), dim3(kRsNT), 0, st, gsum, (int)n);
    return;
  }
  const int64_t nt = (n + kScTile - 1) / kScTile;
  hipLaunchKernelGGL(k_sc_sums<uint32_t>, dim3((unsigned)nt), dim3(kScNT), 0, st, gsum, n, sums);
  hipLaunchKernelGGL(k_sc_carry<uint32_t>, dim3(1), dim3(kScNT), 0, st, sums, nt);
  hipLaunchKernelGGL(k_sc_apply<uint32_t>, dim3((unsigned)nt), dim3(kScNT), 0, st, gsum, gsum, n, sums);
}

}  // namespace

// Stable sort of P (key, packed value) pairs by the low `bits` bits of key.
// k0/v0 hold the input; k1/v1 are a second buffer pair of the same size.  The
// sorted keys end in k0 or k1 (returned); the values are unpacked into docno /
// tf.  counts: ceil(P / 16384) * 2048 + 2048 * 256 u32 of scratch.
uint32_t *term_sort(uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, int64_t nrec, const int64_t *reg,
                    const int64_t *xoff, int64_t P, int bits, int64_t dmin, uint32_t F, int32_t *docno, int32_t *tf,
                    uint32_t *counts, hipStream_t st, const double *lut, double idf, double *w, int maxbits,
                    const uint2 *xw, int64_t Pout) {
  if (P <= 0) return k0;
  if (P > 0xFFFFFFFFll) throw Error(SME_ELIMIT, "term sort of more than 2^32 pairs");
  bits = std::max(bits, 1);
  maxbits = std::min(std::max(maxbits, 1), kRsMaxBits);
  const int npass = (bits + maxbits - 1) / maxbits;
  const int64_t ntiles = (P + kRsTile - 1) / kRsTile;
  const RsGroups rg = rs_groups(ntiles);
  const int64_t tpg = rg.tpg;
  const int G = rg.G;
  uint32_t *gsum = counts + ntiles * kRsMaxBins;
  Gather g0{nullptr, nullptr, nullptr, 0};
  if (reg != nullptr) {
    int64_t *crec = reinterpret_cast<int64_t *>(gsum + kRsMaxBins * kRsGroups + kRsScanSums);
    const int64_t nch = (P + 1023) >> 10;
    hipLaunchKernelGGL(k_rs_chunk_rec, dim3((unsigned)std::min<int64_t>((nch + 255) / 256, 4096)), dim3(256), 0, st,
                       xoff, nrec, P, crec);
    g0 = Gather{reg, xoff, crec, nrec};
  }
  int shift = 0;
  for (int p = 0; p < npass; p++) {
    const Gather g = p == 0 ? g0 : Gather{nullptr, nullptr, nullptr, 0};
#ifdef SME_RS_LOFIRST  // (experiment: the narrower digit first)
    const int nb = (bits - shift) / (npass - p);
#else
    const int nb = (bits - shift + (npass - p) - 1) / (npass - p);  // near-equal digits
#endif
    const int nbins = 1 << nb;
    const bool last = p == npass - 1;
    hipLaunchKernelGGL(k_rs_count, dim3((unsigned)ntiles), dim3(kRsNT), 0, st, k0, P, shift, nbins, counts, g);
    hipLaunchKernelGGL(k_rs_colsum, dim3(G), dim3(kRsNT), 0, st, counts, ntiles, nbins, tpg, G, gsum);
    rs_scan(gsum, (int64_t)nbins * G, gsum + kRsMaxBins * kRsGroups, st);
    hipLaunchKernelGGL(k_rs_colscan, dim3(G), dim3(kRsNT), 0, st, counts, ntiles, nbins, tpg, G, gsum);
    const unsigned sgrid = (unsigned)(8 * ((ntiles + 7) / 8));  // see the XCD tile order in k_rs_scatter
    if (last && xw)  // K6b: the docid pairs' slots stay keyed 0xFFFFFFFF (k_term_offsets<true> skips them)
      SME_HIP(hipMemsetAsync(k1, 0xFF, (size_t)Pout * sizeof(uint32_t), st));
    if (last)
      hipLaunchKernelGGL(k_rs_scatter<true>, dim3(sgrid), dim3(kRsNT), 0, st, k0, v0, P, shift, nb, counts,
                         k1, nullptr, docno, tf, dmin, F, g, lut, idf, w, xw);
    else
      hipLaunchKernelGGL(k_rs_scatter<false>, dim3(sgrid), dim3(kRsNT), 0, st, k0, v0, P, shift, nb,
                         counts, k1, v1, nullptr, nullptr, dmin, F, g, nullptr, 0.0, nullptr, nullptr);
    SME_CHECK_LAUNCH();
    std::swap(k0, k1);
    std::swap(v0, v1);
    shift += nb;
  }
  return k0;
}

size_t term_sort_scratch(int64_t P) {
  const int64_t ntiles = (std::max<int64_t>(P, 1) + kRsTile - 1) / kRsTile;
  return (size_t)(ntiles * kRsMaxBins + (int64_t)kRsMaxBins * kRsGroups + kRsScanSums) * sizeof(uint32_t) +
         (size_t)(((std::max<int64_t>(P, 1) + 1023) >> 10) + 1) * sizeof(int64_t);
}
// Stable sort of n (key, u32 value) pairs by the low `bits` bits of the key
// (11-bit digits).  k0/v0 hold the input, k1/v1 are second buffers of the same
// size; returns the buffer holding the sorted values (v0 or v1).  The sorted
// keys are in the matching key buffer (k0 or k1) when keys_out, else the last
// pass does not write them.  scratch: kv_sort_scratch(n) bytes.
template <typename K>
uint32_t *kv_sort(K *k0, uint32_t *v0, K *k1, uint32_t *v1, int64_t n, int bits, uint32_t *scratch, hipStream_t st,
                  bool keys_out) {
  if (n <= 1) return v0;
  if (n > 0xFFFFFFFFll) throw Error(SME_ELIMIT, "sort of more than 2^32 pairs");
  bits = std::min(std::max(bits, 1), (int)(8 * sizeof(K)));
  const int npass = (bits + kRsMaxBits - 1) / kRsMaxBits;
  const int64_t ntiles = (n + kRsTile - 1) / kRsTile;
  const RsGroups rg = rs_groups(ntiles);
  const int64_t tpg = rg.tpg;
  const int G = rg.G;
  uint32_t *counts = scratch, *gsum = scratch + ntiles * kRsMaxBins;
  int shift = 0;
  for (int p = 0; p < npass; p++) {
    const int nb = (bits - shift + (npass - p) - 1) / (npass - p);
    const int nbins = 1 << nb;
    hipLaunchKernelGGL(k_kv_count<K>, dim3((unsigned)ntiles), dim3(kRsNT), 0, st, k0, n, shift, nbins, counts);
    hipLaunchKernelGGL(k_rs_colsum, dim3(G), dim3(kRsNT), 0, st, counts, ntiles, nbins, tpg, G, gsum);
    rs_scan(gsum, (int64_t)nbins * G, gsum + kRsMaxBins * kRsGroups, st);
    hipLaunchKernelGGL(k_rs_colscan, dim3(G), dim3(kRsNT), 0, st, counts, ntiles, nbins, tpg, G, gsum);
    const unsigned sgrid = (unsigned)(8 * ((ntiles + 7) / 8));
    if (p == npass - 1 && !keys_out)
      hipLaunchKernelGGL((k_kv_scatter<K, false>), dim3(sgrid), dim3(kRsNT), 0, st, k0, v0, n, shift, nb, counts,
                         k1, v1);
    else
      hipLaunchKernelGGL((k_kv_scatter<K, true>), dim3(sgrid), dim3(kRsNT), 0, st, k0, v0, n, shift, nb, counts, k1,
                         v1);
    SME_CHECK_LAUNCH();
    std::swap(k0, k1);
    std::swap(v0, v1);
    shift += nb;
  }
  return v0;
}
template uint32_t *kv_sort<uint64_t>(uint64_t *, uint32_t *, uint64_t *, uint32_t *, int64_t, int, uint32_t *,
                                     hipStream_t, bool);
template uint32_t *kv_sort<uint32_t>(uint32_t *, uint32_t *, uint32_t *, uint32_t *, int64_t, int, uint32_t *,
                                     hipStream_t, bool);

namespace {
__global__ void k_sp_iota(uint32_t *a, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}
__global__ void k_sp_gather64(const uint64_t *__restrict__ v, const uint32_t *__restrict__ idx, int64_t n,
                              uint64_t *__restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = v[idx[i]];
}
template <typename T>
__global__ void k_max_zero(T *m) {
  *m = 0;
}
__device__ __forceinline__ void atomic_max_t(int32_t *p, int32_t v) { atomicMax(p, v); }
__device__ __forceinline__ void atomic_max_t(int64_t *p, int64_t v) {
  atomicMax(reinterpret_cast<unsigned long long *>(p), (unsigned long long)v);  // values are >= 0
}
template <typename T>
__global__ void k_max_reduce(const T *__restrict__ in, int64_t n, T *m) {
  T x = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x = in[i] > x ? in[i] : x;
  for (int o = 32; o > 0; o >>= 1) {
    const T y = __shfl_xor(x, o, 64);
    x = y > x ? y : x;
  }
  if ((threadIdx.x & 63) == 0 && x > 0) atomic_max_t(m, x);
}
__global__ void k_run_heads(const uint64_t *__restrict__ k, int64_t n, int64_t *__restrict__ f) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= n; i += (int64_t)gridDim.x * blockDim.x)
    f[i] = (i < n && (i == 0 || k[i] != k[i - 1])) ? 1 : 0;
}
// run r = pos[i + 1] - 1 of item i (pos: exclusive scan of the head flags); sums
// by integer atomics (order-free)
__global__ void k_run_sums(const uint64_t *__restrict__ k, const int32_t *__restrict__ v, int64_t n,
                           const int64_t *__restrict__ f, const int64_t *__restrict__ pos, uint64_t *__restrict__ uk,
                           int32_t *__restrict__ sums, int64_t *d_runs) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = pos[i] + f[i] - 1;
    if (f[i]) uk[r] = k[i];
    atomicAdd(&sums[r], v[i]);
    if (i == n - 1) *d_runs = r + 1;
  }
}
unsigned sp_grid(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)); }
}  // namespace

template <typename K>
void sort_pairs(K *keys_in, K *keys_out, uint32_t *vals_in, uint32_t *vals_out, int64_t n, int bits, DevBuf &radix,
                hipStream_t st) {
  if (n <= 0) return;
  uint32_t *scr = radix.as<uint32_t>(kv_sort_scratch(n) / sizeof(uint32_t) + 1);
  if (kv_sort<K>(keys_in, vals_in, keys_out, vals_out, n, bits, scr, st, true) == vals_in) {
    SME_HIP(hipMemcpyAsync(keys_out, keys_in, (size_t)n * sizeof(K), hipMemcpyDeviceToDevice, st));
    SME_HIP(hipMemcpyAsync(vals_out, vals_in, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
  }
}
template void sort_pairs<uint64_t>(uint64_t *, uint64_t *, uint32_t *, uint32_t *, int64_t, int, DevBuf &,
                                   hipStream_t);
template void sort_pairs<uint32_t>(uint32_t *, uint32_t *, uint32_t *, uint32_t *, int64_t, int, DevBuf &,
                                   hipStream_t);
template <typename K>
void sort_pairs_v64(K *keys_in, K *keys_out, const uint64_t *vals_in, uint64_t *vals_out, int64_t n, int bits,
                    DevBuf &ia, DevBuf &ib, DevBuf &radix, hipStream_t st) {
  if (n <= 0) return;
  uint32_t *a = ia.as<uint32_t>((size_t)n + 1), *b = ib.as<uint32_t>((size_t)n + 1);
  hipLaunchKernelGGL(k_sp_iota, dim3(sp_grid(n)), dim3(256), 0, st, a, n);
  sort_pairs<K>(keys_in, keys_out, a, b, n, bits, radix, st);
  if (vals_in) hipLaunchKernelGGL(k_sp_gather64, dim3(sp_grid(n)), dim3(256), 0, st, vals_in, b, n, vals_out);
  SME_CHECK_LAUNCH();
}
template void sort_pairs_v64<uint64_t>(uint64_t *, uint64_t *, const uint64_t *, uint64_t *, int64_t, int, DevBuf &,
                                       DevBuf &, DevBuf &, hipStream_t);
template void sort_pairs_v64<uint32_t>(uint32_t *, uint32_t *, const uint64_t *, uint64_t *, int64_t, int, DevBuf &,
                                       DevBuf &, DevBuf &, hipStream_t);
template <typename T>
void reduce_max(const T *in, int64_t n, T *d_max, hipStream_t st) {
  hipLaunchKernelGGL(k_max_zero<T>, dim3(1), dim3(1), 0, st, d_max);
  if (n > 0) hipLaunchKernelGGL(k_max_reduce<T>, dim3(std::min(sp_grid(n), 2048u)), dim3(256), 0, st, in, n, d_max);
  SME_CHECK_LAUNCH();
}
template void reduce_max<int32_t>(const int32_t *, int64_t, int32_t *, hipStream_t);
template void reduce_max<int64_t>(const int64_t *, int64_t, int64_t *, hipStream_t);
void reduce_by_key_sum(const uint64_t *keys, const int32_t *vals, int64_t n, uint64_t *ukeys, int32_t *sums,
                       int64_t *d_runs, DevBuf &flags, DevBuf &pos, DevBuf &scan, hipStream_t st) {
  if (n <= 0) {
    SME_HIP(hipMemsetAsync(d_runs, 0, sizeof(int64_t), st));
    return;
  }
  int64_t *f = flags.as<int64_t>((size_t)n + 1), *p = pos.as<int64_t>((size_t)n + 1);
  hipLaunchKernelGGL(k_run_heads, dim3(sp_grid(n + 1)), dim3(256), 0, st, keys, n, f);
  excl_scan(f, p, n + 1, scan, st);
  SME_HIP(hipMemsetAsync(sums, 0, (size_t)n * sizeof(int32_t), st));
  hipLaunchKernelGGL(k_run_sums, dim3(sp_grid(n)), dim3(256), 0, st, keys, vals, n, f, p, ukeys, sums, d_runs);
  SME_CHECK_LAUNCH();
}

template <typename T>
void excl_scan(const T *in, T *out, int64_t n, DevBuf &scratch, hipStream_t st) {
  if (n <= 0) return;
  const int64_t nt = (n + kScTile - 1) / kScTile;
  T *sums = scratch.as<T>((size_t)nt + 1);
  hipLaunchKernelGGL(k_sc_sums<T>, dim3((unsigned)nt), dim3(kScNT), 0, st, in, n, sums);
  hipLaunchKernelGGL(k_sc_carry<T>, dim3(1), dim3(kScNT), 0, st, sums, nt);
  hipLaunchKernelGGL(k_sc_apply<T>, dim3((unsigned)nt), dim3(kScNT), 0, st, in, out, n, (const T *)sums);
  SME_CHECK_LAUNCH();
}
template void excl_scan<int64_t>(const int64_t *, int64_t *, int64_t, DevBuf &, hipStream_t);
template void excl_scan<int32_t>(const int32_t *, int32_t *, int64_t, DevBuf &, hipStream_t);
template void excl_scan<uint32_t>(const uint32_t *, uint32_t *, int64_t, DevBuf &, hipStream_t);

void select_flagged(const uint8_t *flag, int64_t n, int32_t *out, int32_t *d_count, DevBuf &s1, DevBuf &s2,
                    hipStream_t st) {
  if (n <= 0) {
    SME_HIP(hipMemsetAsync(d_count, 0, sizeof(int32_t), st));
    return;
  }
  int64_t *pos = s1.as<int64_t>((size_t)n);
  const unsigned g = (unsigned)std::min<int64_t>((n + 255) / 256, 16384);
  hipLaunchKernelGGL(k_flags_i64, dim3(g), dim3(256), 0, st, flag, n, pos);
  excl_scan<int64_t>(pos, pos, n, s2, st);
  hipLaunchKernelGGL(k_select_scatter, dim3(g), dim3(256), 0, st, flag, pos, n, out, d_count);
  SME_CHECK_LAUNCH();
}

size_t kv_sort_scratch(int64_t n) {
  const int64_t ntiles = (std::max<int64_t>(n, 1) + kRsTile - 1) / kRsTile;
  return (size_t)(ntiles * kRsMaxBins + (int64_t)kRsMaxBins * kRsGroups + kRsScanSums) * sizeof(uint32_t);
}
}  // namespace sme
