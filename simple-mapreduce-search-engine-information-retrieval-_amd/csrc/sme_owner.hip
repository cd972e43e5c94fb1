// sme_owner.hip -- the owner-side steps of the multi-GPU query path
// that dist.py used to do with torch sorts:
//
//   merge rows   dist.merge_topk_owner: per query this rank owns, the W shards'
//                top-k lists (W x k candidates, any order) -> the best k in
//                (score desc, tie word asc, docno asc) order.  The tie word is 0
//                under SME_TIE_DOCNO and the first-encounter rank under
//                SME_TIE_REFERENCE (sme_query_topk_tie), a property of the
//                document and the query alone, so the merged rows equal the
//                single index's (IntDocVectorsForwardIndex.java:215-222).
//   shared keys  dist.docno_duplicates: (key, source rank) rows received by the
//                key's owner -> how many distinct keys arrive from two or more
//                ranks (a docid in two shards is ONE posting with summed tf in
//                the reference's single reducer, TermKGramDocIndexer.java:202-210)
#include "sme_common.hpp"
#include "sme_internal.hpp"

#include <algorithm>
#include <cmath>

namespace sme {
namespace {

constexpr int kMrNT = 256;
constexpr uint64_t kMrPad = ~0ull;  // key of an empty slot / a padding entry (docno -1)
constexpr uint64_t kShEmpty = ~0ull;
constexpr uint32_t kShNone = 0xFFFFFFFFu;

__device__ __forceinline__ bool mr_better(double as, uint64_t ak, double bs, uint64_t bk) {
  return as > bs || (as == bs && ak < bk);
}

// One workgroup per row: the row's m candidates in chunks of C - k, each chunk
// bitonic-sorted in LDS together with the best k of the chunks before it.  A
// candidate's key is tie << 32 | (docno ^ 2^31) (docno order as signed int32:
// docids missing from the mapping have negative docnos, T14); docno -1 pads.
__global__ __launch_bounds__(kMrNT) void k_merge_rows(const double *s, const int32_t *d, const uint32_t *t, int64_t rows,
                                                       int m, int k, int C, int32_t *od, double *os, uint32_t *ot) {
  extern __shared__ __align__(16) unsigned char mr_smem[];
  double *ls = reinterpret_cast<double *>(mr_smem);
  uint64_t *lk = reinterpret_cast<uint64_t *>(mr_smem + (size_t)C * sizeof(double));
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    int nb = 0;  // entries kept from the chunks so far: [0, nb), sorted
    for (int c0 = 0; c0 < m || (m == 0 && c0 == 0); c0 += C - k) {
      const int cn = min(m - c0, C - k);
      const int n = nb + max(cn, 0);
      int n2 = 2;
      while (n2 < n) n2 <<= 1;
      for (int i = threadIdx.x; i < n2 - nb; i += kMrNT) {
        double sc = -INFINITY;
        uint64_t key = kMrPad;
        if (i < cn) {
          const int64_t src = r * (int64_t)m + c0 + i;
          const int32_t dd = d[src];
          if (dd != -1) {
            sc = s[src];
            key = ((uint64_t)(t ? t[src] : 0u) << 32) | ((uint32_t)dd ^ 0x80000000u);
          }
        }
        ls[nb + i] = sc;
        lk[nb + i] = key;
      }
      __syncthreads();
      for (int size = 2; size <= n2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int i = threadIdx.x; i < (n2 >> 1); i += kMrNT) {
            const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1)), hi = lo + stride;
            const double a = ls[lo], b = ls[hi];
            const uint64_t ka = lk[lo], kb = lk[hi];
            const bool sw = (lo & size) == 0 ? mr_better(b, kb, a, ka) : mr_better(a, ka, b, kb);
            if (sw) {
              ls[lo] = b;
              ls[hi] = a;
              lk[lo] = kb;
              lk[hi] = ka;
            }
          }
          __syncthreads();
        }
      nb = min(k, n);
      if (m == 0) break;
    }
    for (int i = threadIdx.x; i < k; i += kMrNT) {
      const int64_t o = r * (int64_t)k + i;
      const bool real = i < nb && !(lk[i] == kMrPad && ls[i] == -INFINITY);
      od[o] = real ? (int32_t)((uint32_t)lk[i] ^ 0x80000000u) : -1;
      os[o] = real ? ls[i] : 0.0;
      if (ot) ot[o] = real ? (uint32_t)(lk[i] >> 32) : 0xFFFFFFFFu;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint64_t sh_mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// rows[2i] = key (never ~0), rows[2i + 1] = source rank.  Per key slot: the first
// source seen; a second, different source flags the slot once (one count per key)
__global__ void k_shared_insert(const uint64_t *rows, int64_t n, uint64_t *keys, uint32_t *first, uint32_t *flag,
                                uint64_t mask, unsigned long long *cnt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = rows[2 * i];
    const uint32_t src = (uint32_t)rows[2 * i + 1];
    if (key == kShEmpty) {  // (the caller's keys are zero-extended 32-bit values: never)
      atomicAdd(cnt + 1, 1ull);
      continue;
    }
    uint64_t h = sh_mix(key) & mask;
    for (;;) {
      const unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long *>(keys + h),
                                               (unsigned long long)kShEmpty, (unsigned long long)key);
      if (old == kShEmpty || old == key) break;
      h = (h + 1) & mask;
    }
    const uint32_t f = atomicCAS(first + h, kShNone, src);
    if (f != kShNone && f != src && atomicExch(flag + h, 1u) == 0u) atomicAdd(cnt, 1ull);
  }
}

unsigned grid_of(int64_t n, int64_t per, int64_t cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, cap));
}

}  // namespace

void merge_rows(const double *s, const int32_t *d, const uint32_t *t, int64_t rows, int m, int k, int32_t *od,
                double *os, uint32_t *ot, hipStream_t st) {
  if (k < 1 || m < 0 || rows < 0) throw Error(SME_EINVAL, "merge_rows: bad shape");
  if (k > 2048) throw Error(SME_ELIMIT, "merge_rows: k > 2048");
  if (rows == 0) return;
  // LDS: C (score, key) pairs, C - k >= k new candidates per chunk
  const int C = k <= 512 ? 1024 : k <= 1024 ? 2048 : 4096;
  const size_t lds = (size_t)C * (sizeof(double) + sizeof(uint64_t));
  hipLaunchKernelGGL(k_merge_rows, dim3(grid_of(rows, 1, 65536)), dim3(kMrNT), lds, st, s, d, t, rows, m, k, C, od, os,
                     ot);
  SME_CHECK_LAUNCH();
}

int64_t count_shared_keys(sme_ctx *cx, const uint64_t *rows, int64_t n, hipStream_t st) {
  if (n <= 0) return 0;
  uint64_t cap = 1024;
  while (cap < 2 * (uint64_t)n) cap <<= 1;
  uint64_t *keys = cx->ws[125].as<uint64_t>(cap);
  uint32_t *first = reinterpret_cast<uint32_t *>(cx->ws[126].as<uint64_t>(cap));  // first | flag
  uint32_t *flag = first + cap;
  unsigned long long *cnt = reinterpret_cast<unsigned long long *>(cx->ws[127].as<uint64_t>(2));
  SME_HIP(hipMemsetAsync(keys, 0xFF, cap * sizeof(uint64_t), st));
  SME_HIP(hipMemsetAsync(first, 0xFF, cap * sizeof(uint32_t), st));
  SME_HIP(hipMemsetAsync(flag, 0, cap * sizeof(uint32_t), st));
  SME_HIP(hipMemsetAsync(cnt, 0, 2 * sizeof(uint64_t), st));
  hipLaunchKernelGGL(k_shared_insert, dim3(grid_of(n, 256, 16384)), dim3(256), 0, st, rows, n, keys, first, flag,
                     cap - 1, cnt);
  SME_CHECK_LAUNCH();
  unsigned long long h[2] = {0, 0};
  SME_HIP(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (h[1]) throw Error(SME_EINVAL, "count_shared_keys: a key equal to the empty marker");
  return (int64_t)h[0];
}

}  // namespace sme
