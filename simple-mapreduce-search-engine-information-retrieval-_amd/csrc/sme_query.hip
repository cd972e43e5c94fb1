// sme_query.hip -- batched rank() (IntDocVectorsForwardIndex.rank, C/sa/edu/kaust/fwindex/
// IntDocVectorsForwardIndex.java:192-223), query-string tokenization
// (GalagoTokenizer.processContent on the REPL line, :292-295) and term lookup
// (getValue's forward-index lookup, :148-184).
//
// Scoring semantics: for each query token in order (unknown ones skipped,
// duplicates twice), for each posting of that term, score[d] += w where
// w = (1 + ln tf) * idf, evaluated as __dmul_rn(lut[tf], idf[term]) -- the same
// fp64 product the build's weight pass (k_weights) stores, recomputed here
// from 8-byte (docno, tf) postings.  A document's score is therefore the
// left-to-right fp64 sum of its weights in query-token order, exactly as the
// JVM accumulates `score.score += ...`.  Output order: score desc, docno asc
// (north-star tie-break; equals the reference's stable Collections.sort for
// single-term queries).
//
// Two kernels: k_query_imp (tiled, impact-gated; queries of <= 64 terms, any
// k <= 448), described below, and k_query (streaming; one 256-lane workgroup
// per query with fp64 LDS accumulators over 4096-document tiles; per-lane
// register lists for k <= 32, one LDS candidate list per workgroup above), which
// takes batches holding a longer query.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <functional>

#include "sme_internal.hpp"
#include "sme_text.hpp"

namespace sme {

constexpr int kQNT = 256;
constexpr int kTile = 4096;
constexpr int kQPer = 4;  // postings per lane per step
constexpr int kMaxQTerms = 128;      // register-list streaming kernel
constexpr int kMaxQTermsList = 1024; // LDS-list streaming kernel
constexpr int kLutLds = 256;  // 1 + ln(tf) for tf < 256 from LDS, the rare rest from HBM

// Result order: score desc, then a 64-bit key asc.  key = tie << 32 | (docno
// with its sign bit flipped, so docnos compare as signed ints); tie = 0 for the
// north-star order (docno asc) and ref_tie() for the reference's (SME_TIE_REFERENCE):
// rank() appends candidates to `scores` in first-encounter order -- query token
// order, each term's postings in reduce order (tf desc, docno asc) -- and
// Collections.sort is stable and only ever asks compareTo <= 0 / > 0, i.e.
// b.score <= a.score / b.score > a.score, so equal scores keep that order
// (IntDocVectorsForwardIndex.java:195-215,363-365; tools/t5_divergence.py).
__device__ __forceinline__ bool better(double as, uint64_t ak, double bs, uint64_t bk) {
  return as > bs || (as == bs && ak < bk);
}
__device__ __forceinline__ uint64_t doc_key(uint32_t tie, int32_t d) {
  return ((uint64_t)tie << 32) | ((uint32_t)d ^ 0x80000000u);
}
__device__ __forceinline__ int32_t key_doc(uint64_t k) { return (int32_t)((uint32_t)k ^ 0x80000000u); }
// first-encounter rank of a document first met at query token j with tf f: the
// token index above tb bits of (2^tb - 1 - tf).  tb = 24 for batches of queries of
// <= 256 terms, 22 for longer ones (<= 1024 terms); the host checks max_tf < 2^tb.
// (`reftie` in the kernels' arguments is tb, 0 for the north-star order.)
__device__ __forceinline__ uint32_t ref_tie(int j, int f, int tb) {
  return ((uint32_t)j << tb) | (((1u << tb) - 1u) - (uint32_t)f);
}
constexpr uint64_t kNoKey = ~0ull;

// insert (s, d) into the descending register list ts/td (fully unrolled: no
// dynamic register indexing)
template <int K>
__device__ __forceinline__ void topk_insert(double (&ts)[K], uint64_t (&td)[K], double s, uint64_t d) {
  if (!better(s, d, ts[K - 1], td[K - 1])) return;
  bool done = false;
#pragma unroll
  for (int i = K - 1; i >= 1; i--) {
    if (!done) {
      if (better(s, d, ts[i - 1], td[i - 1])) {
        ts[i] = ts[i - 1];
        td[i] = td[i - 1];
      } else {
        ts[i] = s;
        td[i] = d;
        done = true;
      }
    }
  }
  if (!done) {
    ts[0] = s;
    td[0] = d;
  }
}

// 64-bit value of lane l (l wave-uniform) as a scalar
__device__ __forceinline__ int64_t rl64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// merge the per-lane lists: k rounds of block arg-max over list heads; thread 0
// writes query q's k results (docno -1 / score 0 padding)
template <int KMAX>
__device__ __forceinline__ void emit_topk(double (&ts)[KMAX], uint64_t (&td)[KMAX], int k, int q, int32_t *out_d,
                                          double *out_s, uint32_t *out_t, double *red_s, uint64_t *red_d,
                                          int32_t *red_t) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int r = 0; r < k; r++) {
    double bs = ts[0];
    uint64_t bd = td[0];
    int32_t bt = tid;
    for (int o = 32; o > 0; o >>= 1) {
      double os = __shfl_xor(bs, o, 64);
      uint64_t od = __shfl_xor(bd, o, 64);
      int32_t ot = __shfl_xor(bt, o, 64);
      if (better(os, od, bs, bd)) {
        bs = os;
        bd = od;
        bt = ot;
      }
    }
    if (lane == 0) {
      red_s[wave] = bs;
      red_d[wave] = bd;
      red_t[wave] = bt;
    }
    __syncthreads();
    bs = red_s[0];
    bd = red_d[0];
    bt = red_t[0];
    for (int x = 1; x < kQNT / 64; x++)
      if (better(red_s[x], red_d[x], bs, bd)) {
        bs = red_s[x];
        bd = red_d[x];
        bt = red_t[x];
      }
    if (tid == bt) {  // pop the head: shift the winner's list left
#pragma unroll
      for (int j = 0; j < KMAX - 1; j++) {
        ts[j] = ts[j + 1];
        td[j] = td[j + 1];
      }
      ts[KMAX - 1] = -INFINITY;
      td[KMAX - 1] = kNoKey;
    }
    if (tid == 0) {
      const bool valid = bs != -INFINITY;
      out_d[(int64_t)q * k + r] = valid ? key_doc(bd) : -1;
      out_s[(int64_t)q * k + r] = valid ? bs : 0.0;
      if (out_t) out_t[(int64_t)q * k + r] = valid ? (uint32_t)(bd >> 32) : 0xFFFFFFFFu;
    }
    __syncthreads();
  }
}

// k > 32 on the streaming kernel: one candidate list per workgroup in LDS instead
// of per-lane register lists. A tile's documents join it when they beat the
// list's k-th best (score, key) so far; when the next kQNT might not fit, the
// list is sorted (bitonic, best first) and cut to its k best, whose last entry
// becomes the entry bar. Exact: a document below the k-th best of a subset
// cannot be in the top k.
constexpr int kListCap = 2048;

// bitonic sort of l_s / l_k [0, kListCap), best first; entries >= n padded (all threads)
__device__ void list_sort(double *l_s, uint64_t *l_k, int n) {
  const int tid = threadIdx.x;
  for (int i = n + tid; i < kListCap; i += kQNT) {
    l_s[i] = -INFINITY;
    l_k[i] = kNoKey;
  }
  __syncthreads();
  for (int size = 2; size <= kListCap; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < kListCap / 2; t += kQNT) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;
        const double a = l_s[i], b = l_s[j];
        const uint64_t ka = l_k[i], kb = l_k[j];
        const bool swap = (i & size) == 0 ? better(b, kb, a, ka) : better(a, ka, b, kb);
        if (swap) {
          l_s[i] = b;
          l_s[j] = a;
          l_k[i] = kb;
          l_k[j] = ka;
        }
      }
      __syncthreads();
    }
}

template <int KMAX, bool LIST>
__global__ __launch_bounds__(kQNT) void k_query(const int64_t *__restrict__ off, const int32_t *__restrict__ docno,
                                                const int32_t *__restrict__ tf, const double *__restrict__ lut,
                                                int max_tf, const double *__restrict__ idf, int64_t V,
                                                const int32_t *__restrict__ terms, const int64_t *__restrict__ qoff,
                                                int nq, int k, int32_t *out_d, double *out_s, uint32_t *out_t,
                                                int reftie, int *err) {
  __shared__ double acc[kTile];
  __shared__ uint32_t first[kTile];  // SME_TIE_REFERENCE: ref_tie of the document's first token
  __shared__ double s_lut[kLutLds];
  constexpr int QT = LIST ? kMaxQTermsList : kMaxQTerms;
  __shared__ int64_t cur[QT], endp[QT];
  __shared__ double tidf[QT];
  __shared__ int32_t s_next;
  __shared__ unsigned long long s_stop;
  __shared__ double red_s[kQNT / 64];
  __shared__ uint64_t red_d[kQNT / 64];
  __shared__ int32_t red_t[kQNT / 64];
  __shared__ double l_s[LIST ? kListCap : 1];  // LIST: the candidate list
  __shared__ uint64_t l_k[LIST ? kListCap : 1];
  __shared__ int l_n;
  __shared__ double l_ths;
  __shared__ uint64_t l_thk;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int j = tid; j < kTile; j += kQNT) acc[j] = -1.0;  // untouched (weights are >= 0)
  for (int j = tid; j < kLutLds; j += kQNT) s_lut[j] = j <= max_tf ? lut[j] : 0.0;
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int64_t q0 = qoff[q];
    int nt = (int)(qoff[q + 1] - q0);
    if (nt > QT) {
      if (tid == 0) atomicOr(err, 1);
      nt = QT;
    }
    if (tid == 0) {
      s_next = 0x7FFFFFFF;
      l_n = 0;
      l_ths = -INFINITY;
      l_thk = kNoKey;
    }
    __syncthreads();
    for (int i = tid; i < nt; i += kQNT) {
      const int32_t t0 = terms[q0 + i];
      const int32_t t = t0 < V ? t0 : -1;  // out-of-range ids are skipped like unknown ones
      const int64_t b = t >= 0 ? off[t] : 0, e = t >= 0 ? off[t + 1] : 0;
      cur[i] = b;
      endp[i] = e;
      tidf[i] = t >= 0 ? idf[t] : 0.0;
      if (b < e) atomicMin(&s_next, docno[b]);
    }
    double ts[KMAX];
    uint64_t td[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; j++) {
      ts[j] = -INFINITY;
      td[j] = kNoKey;
    }
    __syncthreads();
    while (s_next != 0x7FFFFFFF) {  // uniform: read after a barrier
      const int32_t lo = s_next;
      const int64_t hi = (int64_t)lo + kTile;
      __syncthreads();
      if (tid == 0) s_next = 0x7FFFFFFF;
      for (int i = 0; i < nt; i++) {
        const int64_t c = cur[i], e = endp[i];
        if (c >= e) continue;  // uniform
        const double w_idf = tidf[i];
        if (tid == 0) s_stop = (unsigned long long)e;
        __syncthreads();
        // Each lane walks its stride of the term's postings until the first docno
        // >= hi; the smallest stop over lanes is the term's first posting beyond
        // the tile, and the docno there is that term's next docno.
        int64_t p = c + tid;
        int32_t dstop = 0x7FFFFFFF;
        for (;;) {
          int32_t dv[kQPer], fv[kQPer];
#pragma unroll
          for (int u = 0; u < kQPer; u++) {
            const int64_t pu = p + (int64_t)u * kQNT;
            dv[u] = pu < e ? docno[pu] : 0x7FFFFFFF;
            fv[u] = pu < e ? tf[pu] : 0;
          }
          bool stop = false;
#pragma unroll
          for (int u = 0; u < kQPer; u++) {
            if (stop) continue;
            if ((int64_t)dv[u] >= hi || p + (int64_t)u * kQNT >= e) {
              stop = true;
              p += (int64_t)u * kQNT;
              dstop = p < e ? dv[u] : 0x7FFFFFFF;
              continue;
            }
            const int d = dv[u] - lo;
            const double l = fv[u] < kLutLds ? s_lut[fv[u]] : lut[fv[u]];
            const double w = __dmul_rn(l, w_idf);
            const double v = acc[d];
            acc[d] = v < 0.0 ? w : __dadd_rn(v, w);
            if (reftie && v < 0.0) first[d] = ref_tie(i, fv[u], reftie);  // terms run in token order
          }
          if (stop) break;
          p += (int64_t)kQPer * kQNT;
        }
        // wave minima first: one LDS atomic per wave, not per lane
        unsigned long long pm = (unsigned long long)p;
        int32_t dm = dstop;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const unsigned long long po = __shfl_xor(pm, o, 64);
          const int32_t dd = __shfl_xor(dm, o, 64);
          pm = po < pm ? po : pm;
          dm = dd < dm ? dd : dm;
        }
        if (lane == 0) {
          atomicMin(&s_stop, pm);
          if (dm != 0x7FFFFFFF) atomicMin(&s_next, dm);
        }
        __syncthreads();  // also orders this term's adds before the next term's
        if (tid == 0) cur[i] = (int64_t)s_stop;
      }
      __syncthreads();
      if constexpr (LIST) {
        for (int j0 = 0; j0 < kTile; j0 += kQNT) {  // uniform (l_n read after a barrier)
          if (l_n + kQNT > kListCap) {
            const int n = l_n;
            list_sort(l_s, l_k, n);
            if (tid == 0) {
              l_n = min(n, k);
              if (n >= k) {
                l_ths = l_s[k - 1];
                l_thk = l_k[k - 1];
              }
            }
            __syncthreads();
          }
          const int j = j0 + tid;
          const double sc = acc[j];
          if (sc >= 0.0) {
            acc[j] = -1.0;
            const uint64_t key = doc_key(reftie ? first[j] : 0u, lo + j);
            if (better(sc, key, l_ths, l_thk)) {
              const int p = atomicAdd(&l_n, 1);
              l_s[p] = sc;
              l_k[p] = key;
            }
          }
          __syncthreads();
        }
      } else {
        for (int j = tid; j < kTile; j += kQNT) {
          const double sc = acc[j];
          if (sc < 0.0) continue;
          acc[j] = -1.0;
          topk_insert<KMAX>(ts, td, sc, doc_key(reftie ? first[j] : 0u, lo + j));
        }
        __syncthreads();
      }
    }
    if constexpr (LIST) {
      const int n = l_n;
      list_sort(l_s, l_k, n);
      for (int r = tid; r < k; r += kQNT) {
        const bool valid = r < n;
        out_d[(int64_t)q * k + r] = valid ? key_doc(l_k[r]) : -1;
        out_s[(int64_t)q * k + r] = valid ? l_s[r] : 0.0;
        if (out_t) out_t[(int64_t)q * k + r] = valid ? (uint32_t)(l_k[r] >> 32) : 0xFFFFFFFFu;
      }
      __syncthreads();  // the list is read before the next query resets it
    } else {
      emit_topk<KMAX>(ts, td, k, q, out_d, out_s, out_t, red_s, red_d, red_t);
    }
  }
}


// ---------------------------------------------------------------------------
// Block-max pruned scoring (default path), k_query_bm.
//
// The docno axis is cut into tiles of kQT = 1024 documents from the index's
// smallest docno, each tile into 64 blocks of 16 documents (lane l of a wave
// owns block l).  Two structures bound what a document can score:
//
//  * index-resident HEAVY rows (prepare_queries, built once per index, tf-based
//    so they survive sme_index_reweight): for every term whose postings cover
//    >= 1/div of the docno span (the Zipf head) and whose tf never exceeds 255,
//    its tf byte of every document (0 where absent), the largest tf of every
//    16-document block (bm16) and of every tile (bm1k);
//  * per batch, for every DISTINCT batch term: a skip table (its first posting
//    in every tile) and an impact table q(tf) = floor(w(tf) * alpha) + 1,
//    w(tf) = lut[tf] * idf the exact fp64 weight, alpha = 253.5 / (largest
//    weight of any batch term), so 1 <= q <= 254 where the term occurs.
//
// q is monotone in tf, so the impact of a block's (tile's) largest tf bounds
// every document in it, and for a "sparse" term (no heavy row) the impact of
// its largest tf (the first posting of the reduce-order CSR) bounds every
// posting.  A(d) = sum_j q_j(tf_j(d)) > alpha * R(d) (R the real sum of d's
// weights), so a document whose fp64 score can reach the current k-th best
// score th has A(d) >= gate = floor(alpha * th * (1 - 2^-40)) + 1 (the factor
// absorbs every rounding of S(d) vs R(d) and of the product).
//
// One wave per query:
//  1. seed: tile upper bounds UB(x) = sum_heavy q(bm1k) + sum_sparse [postings
//     in x] * q(maxtf) of every tile; the best `nseed` tiles are scored first,
//     so th (and the gate) start near their final values;
//  2. sweep: tiles in docno order, skipped when UB(x) < gate; a visited tile
//     gets block bounds (heavy bm16 + the block's largest exact sparse sum; the
//     sparse terms' postings of the tile are added into LDS), blocks below the
//     gate are dropped, the rest get exact per-document A(d) (heavy tf bytes
//     through the LDS impact tables), and documents with A(d) >= gate are
//     scored exactly: the left-to-right fp64 sum of lut[tf] * idf over the
//     query's terms in token order, bit-identical to the reference's
//     `score += (1 + Math.log(tf)) * idf` (IntDocVectorsForwardIndex.java:197-213).
// Candidates that beat th go to a per-wave LDS buffer of C entries; when it
// fills, a bitonic sort (score desc, docno asc) keeps the best k and raises th.
// The order tiles are visited in does not matter: `better` compares (score,
// docno) completely, and th / the gate only ever rise.
// ---------------------------------------------------------------------------
constexpr int kQB = 10;
constexpr int kQT = 1 << kQB;   // documents per tile
constexpr int kQBlk = kQT / 64;  // documents per block (one lane per block)
constexpr int kIMaxTerms = 64;   // lane j holds query term j
constexpr int kHSlots = 16;      // heavy terms per query with an LDS impact table (more: posting path)
constexpr int kSRows = 4;        // LDS tf rows per tile for sparse terms (more: binary search)
constexpr int kMaxSeed = 8;
static_assert(kQBlk == 16, "one uint4 of tf bytes per lane and heavy term");

__device__ __forceinline__ uint32_t impact(double l, double widf, double alpha) {
  return (uint32_t)floor(__dmul_rn(__dmul_rn(l, widf), alpha)) + 1u;
}
__device__ __forceinline__ double rld(double v, int l) { return __longlong_as_double(rl64(__double_as_longlong(v), l)); }
__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t max_u8x4(uint32_t w) {
  return max(max(w & 0xFFu, (w >> 8) & 0xFFu), max((w >> 16) & 0xFFu, w >> 24));
}

// ---- index-resident heavy rows (prepare_queries) ----------------------------
__global__ void k_heavy_flags(const int64_t *off, const int32_t *tf_o, int64_t V, int64_t span, int64_t div,
                              int32_t *flag) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t df = off[t + 1] - off[t];
    flag[t] = (div > 0 && df > 0 && df * div >= span && tf_o[off[t]] <= 255) ? 1 : 0;
  }
}
__global__ void k_heavy_rows(const int32_t *flag, const int32_t *scan, int64_t V, int64_t cap, const int64_t *off,
                             int32_t *hrow_of, int32_t *hterm, int64_t *hdf) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = scan[t];
    if (flag[t] && r < cap) {
      hrow_of[t] = r;
      hterm[r] = (int32_t)t;
      hdf[r] = off[t + 1] - off[t];
    } else {
      hrow_of[t] = -1;
    }
  }
}
// tf byte of every heavy posting at docno - dmin of its row, over the heavy
// rows' postings as one flat list (chunks of kSkipChunk) so a head term's
// million postings spread over the whole chip
constexpr int kSkipChunk = 2048;
__global__ __launch_bounds__(256) void k_heavy_fill(const int64_t *hpre, int64_t H, const int32_t *hterm,
                                                    const int64_t *off, const int32_t *docno, const int32_t *tf,
                                                    int64_t dmin, int64_t stride, uint8_t *tfrow) {
  const int64_t total = hpre[H];
  for (int64_t x0 = (int64_t)blockIdx.x * kSkipChunk; x0 < total; x0 += (int64_t)gridDim.x * kSkipChunk) {
    const int64_t x1 = x0 + kSkipChunk < total ? x0 + kSkipChunk : total;
    int64_t lo = 0, hi = H;  // row of x0: hpre[lo] <= x0 < hpre[hi]
    while (hi - lo > 1) {
      const int64_t m = (lo + hi) >> 1;
      if (hpre[m] <= x0) lo = m;
      else hi = m;
    }
    int64_t row = lo, rb = hpre[row], re = hpre[row + 1], b = off[hterm[row]];
    for (int64_t x = x0 + threadIdx.x; x < x1; x += blockDim.x) {
      while (x >= re) {
        row++;
        rb = re;
        re = hpre[row + 1];
        b = off[hterm[row]];
      }
      const int64_t p = b + (x - rb);
      tfrow[row * stride + ((int64_t)docno[p] - dmin)] = (uint8_t)tf[p];
    }
  }
}
// bm1k[i] = largest of the 64 block maxima of tile i
__global__ void k_heavy_bm1k(const uint4 *bm16, int64_t n, uint8_t *bm1k) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint4 v = bm16[4 * i + c];
      m = max(m, max(max(max_u8x4(v.x), max_u8x4(v.y)), max(max_u8x4(v.z), max_u8x4(v.w))));
    }
    bm1k[i] = (uint8_t)m;
  }
}

// ---- per-batch tables --------------------------------------------------------
__global__ void k_mark_terms(const int32_t *terms, int64_t n, int64_t V, int32_t *mark) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t t = terms[i];
    if (t >= 0 && t < V) mark[t] = 1;
  }
}
// distinct marked terms -> rows (row = exclusive scan of mark), their df
__global__ void k_term_rows(const int32_t *mark, const int32_t *row_of, int64_t V, const int64_t *off,
                            int32_t *term_of_row, int64_t *rdf) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x)
    if (mark[t]) {
      term_of_row[row_of[t]] = (int32_t)t;
      rdf[row_of[t]] = off[t + 1] - off[t];
    }
}
// df of the rows the window skip table needs (sparse terms); heavy rows 0, and
// the last entry 0 (the exclusive scan's total)
__global__ void k_sparse_rdf(const int32_t *term_of_row, const int64_t *rdf, const int32_t *hrow_of, int64_t nrows,
                             int64_t *rdfw) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= nrows; r += (int64_t)gridDim.x * blockDim.x)
    rdfw[r] = r == nrows ? 0 : (hrow_of[term_of_row[r]] >= 0 ? 0 : rdf[r]);
}
__global__ void k_max_qlen(const int64_t *qoff, int nq, int *mx) {
  int m = 0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x)
    m = max(m, (int)(qoff[q + 1] - qoff[q]));
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(mx, m);
}
// sk[row * (T + 1) + j] = first posting (term-relative) with tile >= j.  The
// table starts as "infinity" with sk[row][T] = df; every posting that opens a
// tile writes its index there (a change point), and a backward min-scan per
// row fills the gaps (k_skip_suffix).
__global__ __launch_bounds__(256) void k_skip_fill(const int64_t *rpre, int64_t nrows, const int32_t *term_of_row,
                                                   const int64_t *off, const int32_t *docno, int64_t dmin, int64_t T,
                                                   int32_t *sk) {
  const int64_t total = rpre[nrows];
  for (int64_t x0 = (int64_t)blockIdx.x * kSkipChunk; x0 < total; x0 += (int64_t)gridDim.x * kSkipChunk) {
    const int64_t x1 = x0 + kSkipChunk < total ? x0 + kSkipChunk : total;
    int64_t lo = 0, hi = nrows;  // row of x0: rpre[lo] <= x0 < rpre[hi] (same in every thread)
    while (hi - lo > 1) {
      const int64_t m = (lo + hi) >> 1;
      if (rpre[m] <= x0) lo = m;
      else hi = m;
    }
    int64_t row = lo, rb = rpre[row], re = rpre[row + 1], b = off[term_of_row[row]];
    for (int64_t x = x0 + threadIdx.x; x < x1; x += blockDim.x) {
      while (x >= re) {  // the chunk crosses into later rows
        row++;
        rb = re;
        re = rpre[row + 1];
        b = off[term_of_row[row]];
      }
      const int64_t i = x - rb, n = re - rb;
      int32_t *r = sk + row * (T + 1);
      const int64_t j = ((int64_t)docno[b + i] - dmin) >> kQB;
      const int64_t jp = i == 0 ? -1 : (((int64_t)docno[b + i - 1] - dmin) >> kQB);
      if (jp < j) r[j] = (int32_t)i;
      if (i == n - 1) r[T] = (int32_t)n;
    }
  }
}
// one wave per row: suffix minimum from j = T down to 0, 64 entries at a time
__global__ __launch_bounds__(256) void k_skip_suffix(int64_t nrows, int64_t T, int32_t *sk) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < nrows; r += nw) {
    int32_t *row = sk + r * (T + 1);
    int32_t carry = 0x7FFFFFFF;
    for (int64_t j1 = T + 1; j1 > 0; j1 -= 64) {
      const int64_t j = j1 - 1 - lane;  // lane 0 = highest index of the chunk
      int32_t v = j >= 0 ? row[j] : 0x7FFFFFFF;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t u = __shfl_up(v, o, 64);
        if (lane >= o) v = min(v, u);
      }
      v = min(v, carry);
      if (j >= 0) row[j] = v;
      carry = __shfl(v, 63, 64);
    }
  }
}
// window-granular skip table, transposed: skt[w * nrows + row] = first posting of
// the row's term in window w (4 tiles) or later.  Every query of a k_query_win
// workgroup reads window x's entries, so they sit together (L2-resident).
__global__ void k_skip_win(const int32_t *sk, int64_t nrows, int64_t T, int64_t nwin, int32_t *skt) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nrows * (nwin + 1);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = i / nrows, row = i - w * nrows;
    skt[i] = sk[row * (T + 1) + (w << 2)];
  }
}
// rows with df = 0 (possible only for empty terms) never get a posting: all zeros
__global__ void k_skip_zero_rows(const int64_t *rdf, int64_t nrows, int64_t T, int32_t *sk) {
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x)
    if (rdf[r] == 0)
      for (int64_t j = threadIdx.x; j <= T; j += blockDim.x) sk[r * (T + 1) + j] = 0;
}
// largest weight of any batch term (its max tf is the first posting of the
// reduce-order CSR, tf desc), as bits (non-negative doubles order like them)
__global__ void k_row_wmax(const int32_t *term_of_row, const int64_t *rdf, int64_t nrows, const int64_t *off,
                           const int32_t *tf_o, const double *lut, const double *idf, unsigned long long *wmax_bits) {
  unsigned long long wm = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    if (rdf[r] > 0) {
      const int32_t t = term_of_row[r];
      const unsigned long long wb =
          (unsigned long long)__double_as_longlong(__dmul_rn(lut[tf_o[off[t]]], idf[t]));
      wm = wb > wm ? wb : wm;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(wm, o, 64);
    wm = u > wm ? u : wm;
  }
  // one atomic per block, and only when it can raise the maximum (single-address
  // atomics serialise: one per wave took ~0.2 ms on c2's 2 M terms)
  __shared__ unsigned long long s_wm[4];
  if ((threadIdx.x & 63) == 0) s_wm[threadIdx.x >> 6] = wm;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); i++) wm = s_wm[i] > wm ? s_wm[i] : wm;
    if (wm && wm > __hip_atomic_load(wmax_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(wmax_bits, wm);
  }
}
// impact table of every batch row: q(tf) for tf < 256 (0 for tf = 0; tf above
// the index's largest tf never occurs)
__global__ void k_row_qlut(const int32_t *term_of_row, int64_t nrows, const double *lut, int max_tf,
                           const double *idf, const unsigned long long *wmax_bits, uint8_t *qlut) {
  const double wmax = __longlong_as_double((long long)*wmax_bits);
  const double alpha = wmax > 0.0 ? 253.5 / wmax : 1.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nrows * 256;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int f = (int)(i & 255);
    const int32_t t = term_of_row[i >> 8];
    qlut[i] = (uint8_t)(f == 0 ? 0u : f <= max_tf ? impact(lut[f], idf[t], alpha) : 255u);
  }
}

// Query order for cache sharing: queries sorted by their heaviest term (largest
// df, then smaller id) and second heaviest, so concurrent waves on one XCD read
// the same rows / posting ranges.
__global__ void k_query_keys(const int32_t *terms, const int64_t *qoff, int nq, const int64_t *off, int64_t V,
                             int tb, uint64_t *keys, int32_t *idx) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
    int64_t d1 = -1, d2 = -1;
    uint32_t t1 = 0xFFFFFFFFu, t2 = 0xFFFFFFFFu;
    for (int64_t i = qoff[q]; i < qoff[q + 1]; i++) {
      const int32_t t = terms[i];
      if (t < 0 || t >= V) continue;
      const int64_t d = off[t + 1] - off[t];
      if (d > d1 || (d == d1 && (uint32_t)t < t1)) {
        d2 = d1;
        t2 = t1;
        d1 = d;
        t1 = (uint32_t)t;
      } else if ((uint32_t)t != t1 && (d > d2 || (d == d2 && (uint32_t)t < t2))) {
        d2 = d;
        t2 = (uint32_t)t;
      }
    }
    // (heaviest, second heaviest) term ids in tb bits each (no term: V, last)
    keys[q] = ((uint64_t)min<uint64_t>(t1, (uint64_t)V) << tb) | min<uint64_t>(t2, (uint64_t)V);
    idx[q] = q;
  }
}

// Bitonic sort of n (power of two) entries of one wave's LDS buffer, best
// first (score desc, docno asc).  The workgroup is one wave, so the barriers
// only order the LDS traffic.
__device__ __forceinline__ void wave_sort(double *s, uint64_t *d, int n) {
  const int lane = threadIdx.x;
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (n >> 1); i += 64) {
        const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1)), hi = lo + stride;
        const double as = s[lo], bs = s[hi];
        const uint64_t ad = d[lo], bd = d[hi];
        const bool sw = (lo & size) == 0 ? better(bs, bd, as, ad) : better(as, ad, bs, bd);
        if (sw) {
          s[lo] = bs;
          d[lo] = bd;
          s[hi] = as;
          d[hi] = ad;
        }
      }
      __syncthreads();
    }
}

struct QBmArgs {
  const int64_t *off;     // postings per term (docno-sorted CSR; also the reduce-order CSR's offsets)
  const int32_t *docno;   // docno-ascending postings
  const int32_t *tf;
  const int32_t *tf_o;    // reduce order: tf_o[off[t]] is term t's largest tf
  const double *lut;      // 1 + ln(tf)
  const double *idf;
  int64_t V;
  const int32_t *row_of;  // term -> batch row
  const int32_t *sk;      // skip table [rows][T + 1]
  const uint8_t *qlut;    // impact tables [rows][256]
  const int32_t *hrow_of;  // term -> heavy row or -1 (nullptr: no heavy rows)
  const uint8_t *tfrow;   // [H][T * kQT]
  const uint8_t *bm16;    // [H][T * 64]
  const uint8_t *bm1k;    // [H][T]
  int64_t dmin, T;
  const int32_t *terms;
  const int64_t *qoff;
  const int32_t *qorder;
  int nq, k, nseed;
  int reftie;             // SME_TIE_REFERENCE order: ref_tie's tf bits (0: docno order)
  int32_t *out_d;
  double *out_s;
  uint32_t *out_t;        // optional: tie word of every result (multi-shard merges)
  const unsigned long long *wmax_bits;
  unsigned long long *stats;  // SME_EXPERIMENTS builds only (else nullptr)
};

template <int C>
__global__ __launch_bounds__(64) void k_query_bm(QBmArgs a) {
  __shared__ uint8_t s_qlut[kHSlots * 256];  // impact tables of the query's heavy terms
  __shared__ uint32_t lacc[kQT];             // sparse terms' impact sums of the tile's documents
  __shared__ uint8_t trow[kSRows * kQT];     // tf bytes of the tile for the first kSRows sparse terms
  __shared__ double bs[C];
  __shared__ uint64_t bd[C];  // doc_key of every buffered candidate
  __shared__ uint32_t s_big;  // sparse slots whose term has a tf > 255 in the tile
  const int lane = threadIdx.x;
  const double wmax = __longlong_as_double((long long)*a.wmax_bits);
  const double alpha = wmax > 0.0 ? 253.5 / wmax : 1.0;
  const int64_t T = a.T, span = T << kQB;
  // queries in `qorder` (heaviest terms first) are dealt in 8 contiguous slices,
  // slice x to the blocks b with b % 8 == x, which share an XCD and its L2
  const int slice = (a.nq + 7) >> 3;
  for (int qi = blockIdx.x; qi < 8 * slice; qi += gridDim.x) {
    const int pos = (qi & 7) * slice + (qi >> 3);
    if (pos >= a.nq) continue;
    const int q = a.qorder ? a.qorder[pos] : pos;
    const int64_t q0 = a.qoff[q];
    const int nt = (int)(a.qoff[q + 1] - q0);  // <= kIMaxTerms (host checked)
    // lane j < nt holds token j: postings base, df, idf, batch row, heavy row,
    // impact of its largest tf
    int64_t mb = 0;
    int32_t mdf = 0, brow = 0, hr = -1;
    double midf = 0.0;
    uint32_t qmx = 0;
    if (lane < nt) {
      const int32_t t = a.terms[q0 + lane];
      if (t >= 0 && t < a.V) {  // unknown (-1) and out-of-range ids are skipped
        mb = a.off[t];
        mdf = (int32_t)(a.off[t + 1] - mb);
        midf = a.idf[t];
        brow = a.row_of[t];
        if (mdf > 0) {
          if (a.hrow_of) hr = a.hrow_of[t];
          const int32_t mt = a.tf_o[mb];
          qmx = mt <= 255 ? a.qlut[(int64_t)brow * 256 + mt] : impact(a.lut[mt], midf, alpha);
        }
      }
    }
    // heavy terms: the first kHSlots tokens with a heavy row (slot = rank); the
    // rest, and every term without one, are "sparse" (postings + skip table)
    const uint64_t hcand = (uint64_t)__ballot(hr >= 0);
    const uint32_t hslot = lane_prefix(hcand);
    const bool ish = hr >= 0 && hslot < (uint32_t)kHSlots;
    const uint64_t hm = (uint64_t)__ballot(ish);
    const uint64_t sm = (uint64_t)__ballot(lane < nt && mdf > 0 && !ish);
    const int32_t *mrow = a.sk + (int64_t)brow * (T + 1);
    const int64_t h1k = ish ? (int64_t)hr * T : 0, h16 = ish ? (int64_t)hr * (T << 6) : 0,
                  htf = ish ? (int64_t)hr * span : 0;
    for (uint64_t m = hm; m; m &= m - 1) {
      const int j = (int)__builtin_ctzll(m);
      const int s = __popcll(hm & ((1ull << j) - 1));
      const int r = __builtin_amdgcn_readlane(brow, j);
      reinterpret_cast<uint32_t *>(s_qlut)[s * 64 + lane] =
          reinterpret_cast<const uint32_t *>(a.qlut + (int64_t)r * 256)[lane];
    }
    __syncthreads();

    int cnt = 0;  // buffer fill (wave-uniform)
    bool th_ok = false;
    double th_s = 0.0;
    uint64_t th_d = 0;
    uint32_t gate = 1;  // touched documents only until k of them are held
    uint32_t st_tiles = 0, st_blocks = 0, st_cand = 0, st_comp = 0;
    // sort the buffer, keep the best k, raise th and the gate
    auto compact = [&]() {
      st_comp++;
      int n2 = 2;
      while (n2 < cnt) n2 <<= 1;
      for (int i = cnt + lane; i < n2; i += 64) {
        bs[i] = -INFINITY;
        bd[i] = kNoKey;
      }
      __syncthreads();
      wave_sort(bs, bd, n2);
      cnt = min(cnt, a.k);
      if (cnt >= a.k) {
        th_ok = true;
        th_s = bs[a.k - 1];
        th_d = bd[a.k - 1];
        const double g = floor(__dmul_rn(__dmul_rn(th_s, alpha), 1.0 - 0x1p-40));
        gate = g >= 0.0 ? (uint32_t)g + 1u : 1u;
      }
    };
    // upper bound of tile x (any lane, x < T): heavy tile maxima + sparse maxima
    auto tile_ub = [&](int64_t x) -> uint32_t {
      uint32_t u = 0;
      for (uint64_t m = hm; m; m &= m - 1) {
        const int j = (int)__builtin_ctzll(m);
        const int s = __popcll(hm & ((1ull << j) - 1));
        u += s_qlut[(s << 8) + a.bm1k[rl64(h1k, j) + x]];
      }
      for (uint64_t m = sm; m; m &= m - 1) {
        const int j = (int)__builtin_ctzll(m);
        const int32_t *row = a.sk + (int64_t)__builtin_amdgcn_readlane(brow, j) * (T + 1);
        if (row[x] < row[x + 1]) u += (uint32_t)__builtin_amdgcn_readlane((int)qmx, j);
      }
      return u;
    };
    // score tile x (wave-uniform)
    auto tile = [&](int64_t x) {
      st_tiles++;
      const int64_t dbase = a.dmin + (x << kQB);
      int32_t mc = 0, me = 0;  // this lane's sparse term: postings in the tile (term-relative)
      if ((sm >> lane) & 1) {
        mc = mrow[x];
        me = mrow[x + 1];
      }
      const uint64_t spm = (uint64_t)__ballot(me > mc);
      // block bounds from the heavy rows
      uint32_t hub = 0;
      for (uint64_t m = hm; m; m &= m - 1) {
        const int j = (int)__builtin_ctzll(m);
        const int s = __popcll(hm & ((1ull << j) - 1));
        hub += s_qlut[(s << 8) + a.bm16[rl64(h16, j) + (x << 6) + lane]];
      }
      const uint32_t sub = wave_sum_u32(((spm >> lane) & 1) ? qmx : 0u);
      if (wave_max_u32(hub) + sub < gate) return;
      uint32_t A[kQBlk];
#pragma unroll
      for (int i = 0; i < kQBlk; i++) A[i] = 0;
      uint64_t rmask = spm;  // the first kSRows sparse terms with postings own an LDS tf row (slot = rank)
#pragma unroll
      for (int s = 0; s < kSRows; s++) rmask &= rmask - 1;
      rmask = spm & ~rmask;
      uint32_t bigs = 0;
      uint32_t smax = 0;
      if (spm) {
        uint4 *la = reinterpret_cast<uint4 *>(lacc + kQBlk * lane);
#pragma unroll
        for (int c = 0; c < kQBlk / 4; c++) la[c] = make_uint4(0, 0, 0, 0);
        for (int s = 0; s < __popcll(rmask); s++)
          *reinterpret_cast<uint4 *>(trow + (s << kQB) + kQBlk * lane) = make_uint4(0, 0, 0, 0);
        if (lane == 0) s_big = 0;
        __syncthreads();
        // the tile's postings of all sparse terms as one list, 256 per step:
        // entry e belongs to the last term j of spm with pre_j <= e
        const int32_t cj = ((spm >> lane) & 1) ? me - mc : 0;
        const int32_t incl = wave_incl_sum(cj), prej = incl - cj;
        const int32_t total = __builtin_amdgcn_readlane(incl, 63);
        const int64_t plo = mb + mc;
        for (int32_t e0 = 0; e0 < total; e0 += 256) {
          const int nu = min(4, (total - e0 + 63) >> 6);  // 64-entry chunks in this step (wave-uniform)
          int32_t dv[4], fv[4], sv[4], rv[4];
          double wv[4];
#pragma unroll
          for (int u = 0; u < 4; u++) {
            dv[u] = 0;
            fv[u] = 0;
            wv[u] = 0.0;
            sv[u] = kSRows;
            rv[u] = 0;
            if (u < nu) {
              const int32_t e = e0 + 64 * u + lane;
              int64_t pb = 0;
              double wj = 0.0;
              int sj = kSRows, rj = 0;
              for (uint64_t m = spm; m; m &= m - 1) {
                const int j = (int)__builtin_ctzll(m);
                const int32_t pj = __builtin_amdgcn_readlane(prej, j);
                if (e >= pj) {
                  pb = rl64(plo, j) - pj;
                  wj = rld(midf, j);
                  rj = __builtin_amdgcn_readlane(brow, j);
                  sj = ((rmask >> j) & 1) ? __popcll(spm & ((1ull << j) - 1)) : kSRows;
                }
              }
              if (e < total) {
                dv[u] = a.docno[pb + e];
                fv[u] = a.tf[pb + e];
              }
              wv[u] = wj;
              sv[u] = sj;
              rv[u] = rj;
            }
          }
#pragma unroll
          for (int u = 0; u < 4; u++) {
            if (fv[u] == 0) continue;
            const int r = (int)((int64_t)dv[u] - dbase);
            if (sv[u] < kSRows) {
              trow[(sv[u] << kQB) + r] = (uint8_t)(fv[u] > 255 ? 0 : fv[u]);
              if (fv[u] > 255) atomicOr(&s_big, 1u << sv[u]);
            }
            const uint32_t qv =
                fv[u] <= 255 ? (uint32_t)a.qlut[(int64_t)rv[u] * 256 + fv[u]] : impact(a.lut[fv[u]], wv[u], alpha);
            atomicAdd(&lacc[r], qv);
          }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kQBlk / 4; c++) {
          const uint4 v = la[c];
          A[4 * c] = v.x;
          A[4 * c + 1] = v.y;
          A[4 * c + 2] = v.z;
          A[4 * c + 3] = v.w;
          smax = max(smax, max(max(v.x, v.y), max(v.z, v.w)));
        }
        bigs = s_big;
      }
      const bool pass = hub + smax >= gate;
      if (__ballot(pass) == 0) return;
      st_blocks++;
      uint32_t cm = 0;  // candidate documents of this lane's block
      if (pass) {
        for (uint64_t m = hm; m; m &= m - 1) {
          const int j = (int)__builtin_ctzll(m);
          const int s = __popcll(hm & ((1ull << j) - 1));
          const uint4 v = *reinterpret_cast<const uint4 *>(a.tfrow + rl64(htf, j) + (x << kQB) + kQBlk * lane);
          const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int i = 0; i < kQBlk; i++) A[i] += s_qlut[(s << 8) + ((w4[i >> 2] >> ((i & 3) << 3)) & 0xFFu)];
        }
#pragma unroll
        for (int i = 0; i < kQBlk; i++)
          if (A[i] >= gate) cm |= 1u << i;
      }
      if (a.stats) st_cand += (uint32_t)__popc(cm);
      const uint64_t amask = hm | spm;  // terms that can contribute, in token order
      for (;;) {
        const bool have = cm != 0;
        if (__ballot(have) == 0) break;  // wave-uniform
        double S = 0.0;
        uint64_t key = kNoKey;
        bool keep = false;
        if (have) {
          const int b = (int)__builtin_ctz(cm);
          cm &= cm - 1;
          const int r = kQBlk * lane + b;
          const int32_t d = (int32_t)(dbase + r);
          uint32_t tie = 0xFFFFFFFFu;  // first contributing token (reference order)
          // exact score: query-token order, fp64, as rank() accumulates it
          for (uint64_t m = amask; m; m &= m - 1) {
            const int j = (int)__builtin_ctzll(m);
            int f = 0;
            if ((hm >> j) & 1) {
              f = a.tfrow[rl64(htf, j) + (x << kQB) + r];
            } else {
              const int sl = ((rmask >> j) & 1) ? __popcll(spm & ((1ull << j) - 1)) : kSRows;
              if (sl < kSRows && !((bigs >> sl) & 1)) {
                f = trow[(sl << kQB) + r];
              } else {
                const int64_t base = rl64(mb, j);
                int64_t lo = base + __builtin_amdgcn_readlane(mc, j);
                const int64_t e = base + __builtin_amdgcn_readlane(me, j);
                int64_t hi = e;
                while (lo < hi) {
                  const int64_t mid = (lo + hi) >> 1;
                  if (a.docno[mid] < d) lo = mid + 1;
                  else hi = mid;
                }
                if (lo < e && a.docno[lo] == d) f = a.tf[lo];
              }
            }
            if (f != 0) {
              S = __dadd_rn(S, __dmul_rn(a.lut[f], rld(midf, j)));
              if (tie == 0xFFFFFFFFu) tie = ref_tie(j, f, a.reftie);
            }
          }
          key = doc_key(a.reftie ? tie : 0u, d);
          keep = !th_ok || better(S, key, th_s, th_d);
        }
        const uint64_t km = (uint64_t)__ballot(keep);
        if (keep) {
          const int p = cnt + (int)lane_prefix(km);
          bs[p] = S;
          bd[p] = key;
        }
        cnt += __popcll(km);
        if (cnt > C - 64) compact();
      }
    };

    if (nt > 0 && (hm | sm)) {
      // 1. seed tiles: the best tile bound of every lane's column, then the
      //    nseed best of those
      int64_t seed[kMaxSeed];
      int ns = 0;
      if (a.nseed > 0) {
        uint32_t bu = 0;
        int64_t bx = -1;
        for (int64_t x0 = 0; x0 < T; x0 += 64) {
          const int64_t x = x0 + lane;
          const uint32_t u = x < T ? tile_ub(x) : 0u;
          if (u > bu) {
            bu = u;
            bx = x;
          }
        }
        for (; ns < a.nseed && ns < kMaxSeed; ns++) {
          const uint32_t top = wave_max_u32(bu);
          if (top == 0) break;
          const uint64_t wm = (uint64_t)__ballot(bu == top);
          const int wl = (int)__builtin_ctzll(wm);
          seed[ns] = rl64(bx, wl);
          if (lane == wl) bu = 0;
        }
        for (int s = 0; s < ns; s++) tile(seed[s]);
      }
      // 2. sweep in docno order
      for (int64_t x0 = 0; x0 < T; x0 += 64) {
        const int64_t x = x0 + lane;
        uint32_t u = 0;
        if (x < T) {
          bool seeded = false;
          for (int s = 0; s < ns; s++) seeded |= seed[s] == x;
          if (!seeded) u = tile_ub(x);
        }
        uint64_t vm = (uint64_t)__ballot(u >= gate && u > 0);
        while (vm) {
          const int j = (int)__builtin_ctzll(vm);
          vm &= vm - 1;
          if ((uint32_t)__builtin_amdgcn_readlane((int)u, j) >= gate) tile(x0 + j);
        }
      }
    }
    __syncthreads();
    compact();
    if (a.stats) {
      uint32_t c = st_cand;
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0) {
        atomicAdd(a.stats + 0, (unsigned long long)st_tiles);
        atomicAdd(a.stats + 1, (unsigned long long)st_blocks);
        atomicAdd(a.stats + 2, (unsigned long long)c);
        atomicAdd(a.stats + 3, (unsigned long long)st_comp);
      }
    }
    for (int r = lane; r < a.k; r += 64) {
      a.out_d[(int64_t)q * a.k + r] = r < cnt ? key_doc(bd[r]) : -1;
      a.out_s[(int64_t)q * a.k + r] = r < cnt ? bs[r] : 0.0;
      if (a.out_t) a.out_t[(int64_t)q * a.k + r] = r < cnt ? (uint32_t)(bd[r] >> 32) : 0xFFFFFFFFu;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t qhash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ void qwave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
// Window-major scoring (default path): k_query_seed -> k_query_win -> k_query_final.
//
// 1. Seed (one wave per query): a lower bound th0 of the query's k-th best
//    score.  Every term's first M postings in REDUCE order (its highest tf, the
//    documents most likely to rank) are scored over a SUBSET of the query's
//    terms -- the heavy terms (tf from the index-resident tf rows) and the term
//    itself -- in query-token order.  fp64 addition is monotone and every weight
//    is >= 0, so this partial sum S'(d) <= S(d) bit for bit, and the k-th best
//    S' over distinct documents is <= the k-th best S.  Fewer than k distinct
//    seeds (every term's df < k): th0 = -1, every touched document qualifies.
// 2. Windows (one wave per (query, 4096-document window)): workgroup b takes
//    window x and a slice of the query batch, with the 8 XCDs on 8 different
//    windows and every slice of a window on one XCD, so each window's heavy
//    rows are fetched into that XCD's L2 once and read there by every query of
//    the batch.  A(d) = sum of the term impacts q_j(tf) (index-resident impact
//    rows for heavy terms: four bytes per dword split into packed u16 pairs by
//    two v_perm; sparse terms' postings of the window added into LDS) is > alpha
//    * R(d), so S(d) >= th0 implies A(d) >= gate(th0) (the gate of k_query_bm).
//    Documents over the gate are scored exactly (left-to-right fp64 sum in
//    token order, as rank() accumulates) and those with S >= th0 appended to the
//    query's candidate list.  The threshold is static, so windows and queries
//    are independent: no cross-window state, no rising-gate sweep.
// 3. Final (one wave per query): sort the candidates (score desc, key asc), emit
//    the best k.  A query with more candidates than the list holds (deep exact
//    ties at th0) goes to k_query_bm, which sweeps it with a rising gate.
// ---------------------------------------------------------------------------
constexpr int kWinB = 12;
constexpr int kWin = 1 << kWinB;     // documents per window (4 tiles of 1024)
constexpr int kWDL = kWin / 64;      // documents per lane (64)
constexpr int kWNT = 256;            // 4 waves per workgroup, each on its own query
constexpr int kSList = 256;          // a window's sparse postings kept in LDS for exact tf lookups
constexpr int kSeedSlots = 1024;     // seed documents per query (LDS hash)
constexpr int kCandMax = 2048;       // largest candidate list per query (final kernel LDS)
constexpr int kWinRounds = 3;        // window passes before an overflowing query goes to k_query_bm
constexpr int kCList = 128;          // documents over the gate listed per round of exact scoring
#ifndef SME_QRAISE_SMALL
#define SME_QRAISE_SMALL 512
#endif
constexpr int kRaiseSmall = SME_QRAISE_SMALL;  // k_query_raise / k_query_final: lists sorted by the small-LDS instance
constexpr int kWinLut = 128;         // k_query_win: 1 + ln(tf) for tf < 128 from LDS
static_assert(kWDL == 64, "one lane owns 64 documents: four uint4 impact loads per heavy term");

__device__ __forceinline__ uint32_t gate_of(double th0, double alpha) {
  if (!(th0 > 0.0)) return 1u;
  const double g = floor(__dmul_rn(__dmul_rn(th0, alpha), 1.0 - 0x1p-40));
  return g >= 0.0 ? (uint32_t)g + 1u : 1u;
}

// the window pass's per-query gates, computed once per launch from the current
// thresholds (the kernel then holds one scalar per query instead of the fp64
// threshold, and loads th0 / thk only for its candidates)
__global__ void k_gates(const double *th0, int n, double alpha, uint32_t *gate) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) gate[q] = gate_of(th0[q], alpha);
}

// Per-batch query tables for the window path: one 32-byte record per query
// term (postings base, df, batch row, heavy row, idf) and one per position of
// the query order (query, first term, term count), so a wave reaches a query's
// terms in two independent loads instead of four dependent ones.
struct QDesc {
  int64_t mb;
  int32_t mdf, brow, hr, pad;
  double idf;
};
struct QPos {
  int64_t q0;
  int32_t q, nt;
};
static_assert(sizeof(QDesc) == 32 && sizeof(QPos) == 16, "record sizes");
// Window-granular skip table of the k_query_win path, built directly (no tile
// table, no transpose): skt[w * nrows + row] = first posting (term-relative) of
// the row's term in window w or later; skt[nwin * nrows + row] = df.  Change
// points (k_skipw_fill_rm), then a suffix minimum per row over the windows
// (k_skipw_suffix_tr). One wave per row: a chunk walk over a batch's many short
// sparse rows made every thread advance row by row through dependent offset loads.
// Row-major variant (R[row * (nwin + 1) + w]): a row's change points land in its
// own contiguous run instead of one cache line per window of the window-major
// table, and k_skipw_suffix_tr turns R into skt through LDS tiles with coalesced
// reads and writes (the window-major fill's scattered 4-byte stores bound it)
__global__ __launch_bounds__(256) void k_skipw_fill_rm(const int64_t *rdf, int64_t nrows, const int32_t *term_of_row,
                                                       const int64_t *off, const int32_t *docno, int64_t dmin,
                                                       int64_t nwin, int32_t *R) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < nrows; row += nw) {
    const int64_t n = rdf[row];
    if (n == 0) continue;  // (wave-uniform) heavy rows and absent terms
    const int64_t b = off[term_of_row[row]];
    int32_t *rr = R + row * (nwin + 1);
    for (int64_t i = lane; i < n; i += 64) {
      const int64_t j = ((int64_t)docno[b + i] - dmin) >> kWinB;
      const int64_t jp = i == 0 ? -1 : (((int64_t)docno[b + i - 1] - dmin) >> kWinB);
      if (jp < j) rr[j] = (int32_t)i;
      if (i == n - 1) rr[nwin] = (int32_t)n;
    }
  }
}
// 64 rows per workgroup, windows in 64-wide chunks from the last: chunk rows
// loaded along R's rows, a suffix minimum per row (thread t walks row t, the
// carry from the chunk to its right in a register), then written along skt's
// window rows; rows with df = 0 are all zeros
__global__ __launch_bounds__(256) void k_skipw_suffix_tr(const int64_t *rdf, int64_t nrows, int64_t nwin,
                                                         const int32_t *R, int32_t *skt) {
  __shared__ int32_t tile[64][65];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t NW1 = nwin + 1;
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < nrows; r0 += (int64_t)gridDim.x * 64) {  // block-uniform
    const bool empty = tid < 64 && (r0 + tid >= nrows || rdf[r0 + tid] == 0);
    int32_t carry = 0x7FFFFFFF;
    for (int64_t w0 = ((NW1 - 1) >> 6) << 6; w0 >= 0; w0 -= 64) {
      for (int rr = wv; rr < 64; rr += 4) {
        const int64_t row = r0 + rr, w = w0 + lane;
        tile[rr][lane] = (row < nrows && w < NW1) ? R[row * NW1 + w] : 0x7FFFFFFF;
      }
      __syncthreads();
      if (tid < 64) {
        for (int c = 63; c >= 0; c--) {
          carry = min(carry, tile[tid][c]);
          tile[tid][c] = empty ? 0 : carry;
        }
      }
      __syncthreads();
      for (int ww = wv; ww < 64; ww += 4) {
        const int64_t w = w0 + ww, row = r0 + lane;
        if (w < NW1 && row < nrows) skt[w * nrows + row] = tile[lane][ww];
      }
      __syncthreads();
    }
  }
}

__global__ void k_query_desc(const int32_t *terms, int64_t n, int64_t V, const int64_t *off, const double *idf,
                             const int32_t *row_of, const int32_t *hrow_of, QDesc *out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t t = terms[i];
    QDesc d{0, 0, 0, -1, 0, 0.0};
    if (t >= 0 && t < V) {
      d.mb = off[t];
      d.mdf = (int32_t)(off[t + 1] - d.mb);
      d.brow = row_of[t];
      d.hr = (hrow_of && d.mdf > 0) ? hrow_of[t] : -1;
      d.idf = idf[t];
    }
    out[i] = d;
  }
}
__global__ void k_query_pos(const int32_t *qorder, const int64_t *qoff, int nq, int64_t tbase, QPos *out) {
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < nq; p += gridDim.x * blockDim.x) {
    const int q = qorder ? qorder[p] : p;
    out[p] = QPos{qoff[q] - tbase, q, (int32_t)(qoff[q + 1] - qoff[q])};
  }
}
// Streamed records: every window pass reads the whole batch's once, with no
// reuse inside the pass, so the per-lane term records are loaded non-temporally
// (they do not evict the window's index rows from L2); the wave-uniform position
// records and thresholds go through the scalar cache (ld_uni below).
typedef uint32_t qu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ QDesc ld_desc_nt(const QDesc *d, int64_t q0, int nt, int lane) {
  if (lane < nt) {
    // (q0 is wave-uniform: scalar base + 32-bit lane offset, no per-lane 64-bit address)
    uint32_t lo = (uint32_t)lane << 5;
    asm volatile("" : "+v"(lo));  // (keeps the compiler from hoisting d + 32 lane into a 64-bit register pair)
    const qu32x4 *p = reinterpret_cast<const qu32x4 *>(reinterpret_cast<const char *>(d + q0) + lo);
    const qu32x4 u = __builtin_nontemporal_load(p), v = __builtin_nontemporal_load(p + 1);
    QDesc r;
    r.mb = (int64_t)(((uint64_t)u.y << 32) | u.x);
    r.mdf = (int32_t)u.z;
    r.brow = (int32_t)u.w;
    r.hr = (int32_t)v.x;
    r.pad = (int32_t)v.y;
    r.idf = __longlong_as_double((long long)(((uint64_t)v.w << 32) | v.z));
    return r;
  }
  return QDesc{0, 0, 0, -1, 0, 0.0};
}
// a wave-uniform pointer pinned to SGPRs (opaque to reassociation, so a load at
// p + 32-bit lane offset uses the scalar-base address mode: no 64-bit VALU math)
typedef const __attribute__((address_space(1))) uint8_t gbyte;
__device__ __forceinline__ gbyte *uni_ptr(const uint8_t *p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<gbyte *>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t ld_g4(gbyte *base, uint32_t off) {
  return *reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(base + off);
}
__device__ __forceinline__ uint4 ld_g16(gbyte *base, uint32_t off) {
  const qu32x4 v = *reinterpret_cast<const __attribute__((address_space(1))) qu32x4 *>(base + off);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// wave-uniform records through the scalar cache (read-only here: written by
// earlier launches), so the pipelined next-query records hold no VGPRs
template <typename T>
__device__ __forceinline__ T ld_uni(const T *p) {
  return *reinterpret_cast<const __attribute__((address_space(4))) T *>(reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ QPos ld_pos_uni(const QPos *p) {
  const qu32x4 u = ld_uni(reinterpret_cast<const qu32x4 *>(p));
  return QPos{(int64_t)(((uint64_t)u.y << 32) | u.x), (int32_t)u.z, (int32_t)u.w};
}
__device__ __forceinline__ QDesc ld_desc(const QDesc *d, int64_t q0, int nt, int lane) {
  if (lane < nt) return d[q0 + lane];
  return QDesc{0, 0, 0, -1, 0, 0.0};
}

// Bitonic sort of n (power of two) doubles of one wave's LDS array, descending.
__device__ __forceinline__ void wave_sort_desc(double *s, int n) {
  const int lane = threadIdx.x & 63;
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (n >> 1); i += 64) {
        const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1)), hi = lo + stride;
        const double a = s[lo], b = s[hi];
        if ((lo & size) == 0 ? b > a : a > b) {
          s[lo] = b;
          s[hi] = a;
        }
      }
      __syncthreads();
    }
}

struct QSeedArgs {
  const QDesc *desc;
  const int64_t *qoff;
  const int32_t *docno_o, *tf_o;  // reduce order: tf desc, docno asc
  const double *lut;
  const uint8_t *tfrow;           // [H][hstride] tf bytes at docno - dmin
  int64_t hstride, dmin;
  int64_t tbase;                  // desc[i] describes term d_terms[tbase + i]
  int nq, k, M;
  double *th0;
  uint64_t *thk;  // key part of the threshold: kNoKey (every key passes at th0)
};

__global__ __launch_bounds__(64) void k_query_seed(QSeedArgs a) {
  __shared__ int32_t hk[kSeedSlots];             // docno (INT32_MIN empty: never a docno)
  // best S' per seed as float bits rounded DOWN (non-negative floats order as u32):
  // th0 only has to bound the k-th best score from below, and 4-byte entries leave
  // the wave 8 KB of LDS (twice the workgroups per CU of 8-byte ones)
  __shared__ unsigned int hs[kSeedSlots];
  __shared__ int s_n;
  const int lane = threadIdx.x;
  for (int q = blockIdx.x; q < a.nq; q += gridDim.x) {
    const int64_t q0 = a.qoff[q];
    const int nt = (int)(a.qoff[q + 1] - q0);
    const QDesc D = ld_desc(a.desc, q0 - a.tbase, nt, lane);
    const uint64_t am = (uint64_t)__ballot(D.mdf > 0);
    const uint64_t hm = (uint64_t)__ballot(D.hr >= 0);
    for (int i = lane; i < kSeedSlots; i += 64) {
      hk[i] = INT32_MIN;
      hs[i] = 0u;
    }
    if (lane == 0) s_n = 0;
    __syncthreads();
    // seeds per term: M, so that every term's seeds fit the table at load <= 1/2
    const int na = __popcll(am);
    const int M = na > 0 ? min(a.M, (kSeedSlots / 2) / na) : 0;
    for (uint64_t mj = am; mj; mj &= mj - 1) {
      const int j = (int)__builtin_ctzll(mj);
      const int64_t b = rl64(D.mb, j);
      const int32_t n = min(M, __builtin_amdgcn_readlane(D.mdf, j));
      for (int32_t i0 = 0; i0 < n; i0 += 64) {
        const int32_t i = i0 + lane;
        if (i >= n) continue;
        const int32_t d = a.docno_o[b + i], fj = a.tf_o[b + i];
        double S = 0.0;
        for (uint64_t m = am; m; m &= m - 1) {
          const int x = (int)__builtin_ctzll(m);
          int f = 0;
          if (x == j) f = fj;
          else if ((hm >> x) & 1)
            f = a.tfrow[(int64_t)__builtin_amdgcn_readlane(D.hr, x) * a.hstride + ((int64_t)d - a.dmin)];
          if (f != 0) S = __dadd_rn(S, __dmul_rn(a.lut[f], rld(D.idf, x)));
        }
        uint32_t h = qhash32((uint32_t)d) & (kSeedSlots - 1);
        for (;;) {
          const int32_t old = atomicCAS(&hk[h], INT32_MIN, d);
          if (old == INT32_MIN || old == d) break;
          h = (h + 1) & (kSeedSlots - 1);
        }
        atomicMax(&hs[h], (unsigned int)__float_as_uint(__double2float_rd(S)));
      }
    }
    __syncthreads();
    // k-th largest S' over the distinct seeds: compact the used slots' scores
    // (read into registers first, then written over the table), sort, pick
    double v[kSeedSlots / 64];
#pragma unroll
    for (int u = 0; u < kSeedSlots / 64; u++) {
      const int i = u * 64 + lane;
      v[u] = hk[i] != INT32_MIN ? (double)__uint_as_float(hs[i]) : -1.0;
    }
    __syncthreads();
    double th = -1.0;
    int nused = 0;
#pragma unroll
    for (int u = 0; u < kSeedSlots / 64; u++) nused += __popcll((uint64_t)__ballot(v[u] >= 0.0));
    if (a.k <= 32 && nused >= a.k) {
      // small k: the k-th largest by k rounds of wave max + removal of one
      // instance (duplicates count, as in the sorted list), all in registers
      for (int r = 0; r < a.k; r++) {
        double m = v[0];
#pragma unroll
        for (int u = 1; u < kSeedSlots / 64; u++) m = v[u] > m ? v[u] : m;
        double M = m;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const double y = __shfl_xor(M, o, 64);
          M = y > M ? y : M;
        }
        const uint64_t has = (uint64_t)__ballot(m == M);
        if (lane == (int)__builtin_ctzll(has)) {
          bool done = false;
#pragma unroll
          for (int u = 0; u < kSeedSlots / 64; u++)
            if (!done && v[u] == M) {
              v[u] = -2.0;
              done = true;
            }
        }
        th = M;
      }
      if (lane == 0) {
        a.th0[q] = th;
        a.thk[q] = kNoKey;
      }
      continue;  // (no LDS use after the last barrier: the next query's clear follows a barrier)
    }
    double *ss = reinterpret_cast<double *>(hs);
#pragma unroll
    for (int u = 0; u < kSeedSlots / 64; u++)
      if (v[u] >= 0.0) ss[atomicAdd(&s_n, 1)] = v[u];
    __syncthreads();
    const int n = s_n;
    if (n >= a.k) {
      int n2 = 2;
      while (n2 < n) n2 <<= 1;
      for (int i = n + lane; i < n2; i += 64) ss[i] = -INFINITY;
      __syncthreads();
      wave_sort_desc(ss, n2);
      th = ss[a.k - 1];
    }
    if (lane == 0) {
      a.th0[q] = th;
      a.thk[q] = kNoKey;
    }
    __syncthreads();
  }
}

struct QWinArgs {
  const QDesc *desc;
  const QPos *qpos;
  const int32_t *docno, *tf;   // docno-order CSR
  const uint32_t *spk;         // sparse posting words of the docno-order CSR (prepare_queries)
  const double *lut;
  int max_tf;
  const int32_t *skt;          // window skip table, transposed [nwin + 1][nrows]
  int64_t nrows;
  const uint8_t *qlut;         // impact tables [rows][256]
  const uint8_t *imp, *tfrow;  // [H][hstride] impact / tf bytes
  const uint8_t *sbq;          // [H][hstride / 4] impact bound of every 4-document sub-block
  int64_t hstride, dmin, T, nwin;
  const int32_t *wlist;        // windows of this launch (nullptr: 0 .. nwin - 1), nw of them
  int64_t nw;
  int nq, nslices, reftie, cap;
  double alpha;
  const double *th0;           // per query threshold: keep (S, key) not worse than (th0, thk)
  const uint64_t *thk;
  const uint32_t *gate;        // per query gate_of(th0): the impact sum a document must reach (k_gates)
  unsigned int *ccnt;          // candidates per query
  double *cs;                  // [nq][cap] scores
  uint64_t *ck;                // [nq][cap] doc keys
  unsigned long long *stats;   // SME_EXPERIMENTS builds only (else nullptr)
  int exper;                   // SME_EXPERIMENTS timing switches (0 in the product)
};

// waves per SIMD the register allocation targets (16 KB of LDS per workgroup
// allows eight): with two heavy terms' impact loads in flight per passing block
// (SME_QIMPG), the uniform records in SGPRs and the biased block accumulators the
// kernel fits 64 VGPRs without spilling (c3: 31.2 ms at five waves / four loads,
// 28.3 at six, 23.7 at eight with the scans and posting words of round 5)
#ifndef SME_QWIN_WAVES
#define SME_QWIN_WAVES 8
#endif
#ifndef SME_QIMPG
#define SME_QIMPG 2
#endif
#ifndef SME_QFB
#define SME_QFB 4
#endif
// heavy sub-block bound rows (uint4 per lane) in flight per step of the first level
#ifndef SME_QSBG
#define SME_QSBG 2
#endif
// SME_QW_KARG (default 1): the pair loop reads its pointer arguments from the
// kernarg segment where it uses them (SGPR spills into VGPR lanes 106 -> 36 reads;
// c3 20.64 -> 20.21 ms, c5 1 M top-100 1782 -> 1741 ms, digests unchanged)
#ifndef SME_QW_KARG
#define SME_QW_KARG 1
#endif
#ifndef SME_QWIN_SPARSE_NT
#define SME_QWIN_SPARSE_NT 0
#endif
// the experiment build's counters and timing switches; constants in the product
// (so the product kernel holds no registers or branches for them)
#ifdef SME_EXPERIMENTS
#define QW_STATS a.stats
#define QW_EXPER a.exper
#else
#define QW_STATS ((unsigned long long *)nullptr)
#define QW_EXPER 0
#endif
__global__ __launch_bounds__(kWNT, SME_QWIN_WAVES) void k_query_win(QWinArgs a) {
  // LDS: 2.8 KB per wave + the LUT = 12 KB per workgroup, so LDS does not bound
  // the occupancy (a per-document sparse accumulator, 8 KB per wave, held it at
  // four workgroups per CU): the window's sparse postings are summed per
  // 16-document block for the bounds, and a passing block's documents take
  // their sparse impacts from the listed postings
  // per block: sparse postings << 16 | their impact sum (<= 256 x 254 < 2^16), and
  // the first two postings inline ((r & 15) | q << 4), so a passing block reads its
  // documents' sparse impacts without searching the list
  // (16-byte aligned: read as uint4, and bent / slist hold 32-byte slots)
  __shared__ alignas(16) uint32_t bsum_all[kWNT / 64][kWin / 16];
  __shared__ alignas(16) uint16_t bent_all[kWNT / 64][2 * (kWin / 16)];
  __shared__ alignas(16) uint32_t slist_all[kWNT / 64][kSList];  // the window's sparse postings: r | q << 12 | tf << 20
  __shared__ uint16_t blist_all[kWNT / 64][kWin / 16];  // sub-blocks over the gate (chunks of 256)
  __shared__ uint16_t clist_all[kWNT / 64][kCList];     // documents over the gate
  __shared__ double s_lut[kWinLut];                    // 1 + ln(tf) for tf < 128
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t *bsum = bsum_all[wv], *slist = slist_all[wv];
  uint16_t *bent = bent_all[wv];
  uint16_t *blist = blist_all[wv], *clist = clist_all[wv];
  for (int i = threadIdx.x; i < kWinLut; i += kWNT) s_lut[i] = i <= a.max_tf ? a.lut[i] : 0.0;
  __syncthreads();
  // workgroup -> (window, query slice): the 8 XCDs (b % 8) on 8 windows, every
  // slice of one window on one XCD
  const int64_t G = 8 * (int64_t)a.nslices;
  const int64_t b = blockIdx.x, w = b % G;
  const int64_t xi = (b / G) * 8 + (w & 7);
  if (xi >= a.nw) return;
  const int64_t x = a.wlist ? a.wlist[xi] : xi;
  const int s = (int)(w >> 3);
  const int p_lo = (int)((int64_t)a.nq * s / a.nslices), p_hi = (int)((int64_t)a.nq * (s + 1) / a.nslices);
  const int64_t wbase = a.dmin + (x << kWinB);  // first docno of the window
  int pos = p_lo + wv;
  if (pos >= p_hi) return;
#pragma unroll
  for (int m = 0; m < 4; m++) bsum[m * 64 + lane] = 0;
  // software pipeline over this wave's queries: the next query's position
  // record, term records, threshold and skip entries load while this one runs
  QPos P = ld_pos_uni(a.qpos + pos);
  QDesc D = ld_desc_nt(a.desc, P.q0, P.nt, lane);
  uint32_t gate = ld_uni(a.gate + P.q);
  int32_t mc = 0, me = 0;
  if (D.mdf > 0 && D.hr < 0) {
    mc = a.skt[x * a.nrows + D.brow];
    me = a.skt[(x + 1) * a.nrows + D.brow];
  }
  QPos NP{0, 0, 0};  // next query's position record, loaded a pair ahead
  if (pos + kWNT / 64 < p_hi) NP = ld_pos_uni(a.qpos + pos + kWNT / 64);
  for (;;) {
#if SME_QW_KARG
    // the arguments re-read from the kernarg segment through a pointer the
    // compiler cannot hoist: loop-invariant pointers then live only where they
    // are used instead of in SGPRs spilled to VGPR lanes across the whole loop
    const __attribute__((address_space(4))) QWinArgs *ka =
        (const __attribute__((address_space(4))) QWinArgs *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
#define QA (*ka)
#else
#define QA a
#endif
    const int npos = pos + kWNT / 64;
    const bool hasn = npos < p_hi;
    // the next query's term records and gate, and the position record after it
    QDesc ND{0, 0, 0, -1, 0, 0.0};
    uint32_t ngate = 0;
    QPos NNP{0, 0, 0};
    if (hasn) {
      ND = ld_desc_nt(QA.desc, NP.q0, NP.nt, lane);
      ngate = ld_uni(QA.gate + NP.q);
      if (npos + kWNT / 64 < p_hi) NNP = ld_pos_uni(QA.qpos + npos + kWNT / 64);
    }
#ifdef SME_EXPERIMENTS  // timing switches: 4 = no sparse terms, 8 = no heavy terms
    const uint64_t hm = (QW_EXPER & 8) ? 0ull : (uint64_t)__ballot(D.hr >= 0);
    const uint64_t sm = (QW_EXPER & 4) ? 0ull : (uint64_t)__ballot(D.mdf > 0 && D.hr < 0);
#else
    const uint64_t hm = (uint64_t)__ballot(D.hr >= 0);
    const uint64_t sm = (uint64_t)__ballot(D.mdf > 0 && D.hr < 0);
#endif
    // every u16 accumulator below starts at 2^15 - gate, so a bound or an A(d)
    // reaching the gate is its bit 15 (A(d) < 2^14 and gate <= 2^14 + 1 leave no
    // carry between halves; a gate past 2^15 - 1 takes no bias, and nothing
    // reaches bit 15)
    const uint32_t bias = gate > 0x7FFFu ? 0u : 0x8000u - gate;
    const uint32_t bias2 = bias | (bias << 16);
    // heavy terms' sub-block maxima: one uint4 per term = the impact bounds of the
    // 16 four-document sub-blocks of this lane's 64 documents (index-resident sbq
    // rows), two loads in flight; sb[i] holds sub-blocks 2i (low u16) and 2i + 1
    uint32_t sb[8];
#pragma unroll
    for (int i = 0; i < 8; i++) sb[i] = bias2;
    {
      const int64_t soff = (x << (kWinB - 2)) + 16 * lane;
      const int64_t hstr4 = QA.hstride >> 2;
      for (uint64_t mh = hm; mh;) {
        uint4 v[SME_QSBG];
#pragma unroll
        for (int g = 0; g < SME_QSBG; g++) {
          v[g] = make_uint4(0, 0, 0, 0);
          if (mh) {
            const int j = (int)__builtin_ctzll(mh);
            mh &= mh - 1;
            v[g] = *reinterpret_cast<const uint4 *>(QA.sbq + (int64_t)__builtin_amdgcn_readlane(D.hr, j) * hstr4 + soff);
          }
        }
#pragma unroll
        for (int g = 0; g < SME_QSBG; g++) {
          const uint32_t w4[4] = {v[g].x, v[g].y, v[g].z, v[g].w};
#pragma unroll
          for (int u = 0; u < 4; u++) {
            sb[2 * u] += __builtin_amdgcn_perm(0u, w4[u], 0x0C010C00u);
            sb[2 * u + 1] += __builtin_amdgcn_perm(0u, w4[u], 0x0C030C02u);
          }
        }
      }
    }
    // sparse terms: the window's postings into LDS -- impact sums per block, and
    // the (document, impact, tf) list (per term docno-ascending) for the exact
    // sums of passing blocks and the candidates' tf lookups
    const int32_t cj = ((sm >> lane) & 1) ? me - mc : 0;
    const int32_t incl = wave_incl_sum(cj), prej = incl - cj;
    const int32_t total = __builtin_amdgcn_readlane(incl, 63);
    const bool listed = total <= kSList;  // else the block sum bounds every document of the block
    // a block holds at most 16 postings per sparse term: with more than 16 sparse
    // terms an unlisted window's block may hold > 258 postings, whose 16-bit impact
    // sum can wrap -- such blocks pass the bounds (their documents' exact sums
    // decide, below)
    const bool wide_nl = !listed && __popcll(sm) > 16;
    if (total > 0) {
      const int64_t plo = D.mb + mc;
      for (int32_t e0 = 0; e0 < total; e0 += 64) {
        const int32_t e = e0 + lane;
        int64_t pb = 0;
        for (uint64_t m = sm; m; m &= m - 1) {
          const int j = (int)__builtin_ctzll(m);
          const int32_t pj = __builtin_amdgcn_readlane(prej, j);
          if (e >= pj) pb = rl64(plo, j) - pj;
        }
        if (e < total) {
          // the posting's word: its place in the window, q(tf) and tf, as the list keeps them
#if SME_QWIN_SPARSE_NT  // the window's sparse postings without L2 allocation (kept for the heavy rows)
          const uint32_t pw = __builtin_nontemporal_load(QA.spk + pb + e);
#else
          const uint32_t pw = QA.spk[pb + e];
#endif
          const int r = (int)(pw & 0xFFFu);
          const uint32_t qv = (pw >> 12) & 0xFFu;
          const uint32_t c = atomicAdd(&bsum[r >> 4], (1u << 16) | qv) >> 16;
          if (listed) {
            slist[e] = pw;
            if (c < 2) bent[2 * (r >> 4) + c] = (uint16_t)((r & 15) | (qv << 4));
          }
        }
      }
      qwave_sync();
    }
    // the next query's skip entries (its records arrived during the sparse pass)
    int32_t nmc = 0, nme = 0;
    if (ND.mdf > 0 && ND.hr < 0) {
      nmc = QA.skt[x * QA.nrows + ND.brow];
      nme = QA.skt[(x + 1) * QA.nrows + ND.brow];
    }
    // sub-blocks over the gate: heavy maxima + their block's sparse impact sum
    if (total > 0) {
      // + the block's sparse impact sum (>= the sparse sum of any of its documents;
      // clamped: any sum >= 2^14 passes every gate, A(d) <= 64 x 254 < 2^14)
      int li = lane;
      asm volatile("" : "+v"(li));  // (an address recomputed here, not a hoisted register that spills)
      const uint4 b4 = reinterpret_cast<const uint4 *>(bsum)[li];
      const uint32_t bws[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int m = 0; m < 4; m++) {
        const uint32_t c = wide_nl ? (bws[m] ? 0x4000u : 0u) : min(bws[m] & 0xFFFFu, 0x4000u);
        sb[2 * m] += c | (c << 16);
        sb[2 * m + 1] += c | (c << 16);
      }
    }
    uint32_t smk = 0;  // bit i: sub-block 16 lane + i reaches the gate
    {
      uint32_t hi = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) hi |= (sb[i] & 0x80008000u) >> (15 - 2 * i);
      smk = (hi & 0x5555u) | ((hi >> 15) & 0xAAAAu);
    }
    const int32_t sl = __popc(smk);
    const int32_t sincl = wave_incl_sum(sl);
    const int32_t nsub = __builtin_amdgcn_readlane(sincl, 63);
    if (QW_STATS && lane == 0) {
      atomicAdd(QW_STATS + 0, 1ull);
      atomicAdd(QW_STATS + 1, (unsigned long long)total);
      atomicAdd(QW_STATS + 2, (unsigned long long)nsub);
      atomicAdd(QW_STATS + 3, (unsigned long long)__popcll(hm));
    }
    if (nsub > 0 && !(QW_EXPER & 1)) {
      const uint64_t amask = hm | sm;
      const bool unl = !listed && total > 0;  // (wave-uniform)
      // slots: the first 64 blocks holding a passing sub-block, 32 bytes each, the
      // first 32 in slist, the rest in bent
      uint32_t *const slot0 = slist, *const slot32 = reinterpret_cast<uint32_t *>(bent);
      auto slot_of = [&](int i) { return i < 32 ? slot0 + 8 * i : slot32 + 8 * (i - 32); };
      if (unl) {
        // a window whose sparse postings are too many to list: its first 64 blocks
        // with a passing sub-block take slots (bit 31 | slot over their block sums:
        // the bounds are done), and a second pass over the postings sums each slot's
        // documents exactly into a u16 table in the list's LDS, which this pair
        // leaves unused
        uint32_t bm = 0;
#pragma unroll
        for (int m = 0; m < 4; m++) bm |= ((smk >> (4 * m)) & 0xFu) ? (1u << m) : 0u;
        const int32_t bl = __popc(bm);
        const int32_t bincl = wave_incl_sum(bl);
        const int32_t nblk = __builtin_amdgcn_readlane(bincl, 63);
        qwave_sync();
        {
          int32_t o = bincl - bl;
          for (uint32_t m = bm; m; m &= m - 1, o++)
            if (o < 64) clist[o] = (uint16_t)(4 * lane + __builtin_ctz(m));
        }
        qwave_sync();
        if (lane < nblk) bsum[clist[lane]] = 0x80000000u | (uint32_t)lane;
        uint32_t *my = slot_of(lane);
        *reinterpret_cast<uint4 *>(my) = make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4 *>(my + 4) = make_uint4(0, 0, 0, 0);
        qwave_sync();
        const int64_t plo = D.mb + mc;
        for (int32_t e0 = 0; e0 < total; e0 += 64) {
          const int32_t e = e0 + lane;
          int64_t pb = 0;
          for (uint64_t m = sm; m; m &= m - 1) {
            const int j = (int)__builtin_ctzll(m);
            const int32_t pj = __builtin_amdgcn_readlane(prej, j);
            if (e >= pj) pb = rl64(plo, j) - pj;
          }
          if (e < total) {
            const uint32_t pw = QA.spk[pb + e];
            const int r = (int)(pw & 0xFFFu);
            const uint32_t sw = bsum[r >> 4];
            if (sw >> 31) {
              uint32_t *t = slot_of((int)(sw & 0xFFu));
              atomicAdd(t + ((r & 15) >> 1), ((pw >> 12) & 0xFFu) << ((r & 1) << 4));  // A(d) < 2^14: no carry
            }
          }
        }
        qwave_sync();
      }
      // one passing sub-block per lane: exact A(d) of its 4 documents (one impact
      // dword per heavy term + its sparse impacts), then the candidates.  The
      // sub-blocks are listed in chunks of 256 (blist)
      for (int32_t s0 = 0; s0 < nsub; s0 += kWin / 16) {
        const int32_t sn = min(nsub - s0, kWin / 16);
        qwave_sync();
        {
          int32_t o = sincl - sl - s0;
          for (uint32_t m = smk; m; m &= m - 1, o++)
            if (o >= 0 && o < sn) blist[o] = (uint16_t)(16 * lane + __builtin_ctz(m));
        }
        qwave_sync();
        for (int32_t e0 = 0; e0 < sn; e0 += 64) {
          const bool hs = e0 + lane < sn;
          const int sid = hs ? (int)blist[e0 + lane] : 0;  // sub-block in the window
          const int bk = sid >> 2, sj = sid & 3;
          const int r0 = sid << 2;  // its first document in the window
          uint32_t acc0 = bias2, acc1 = bias2;  // documents r0, r0 + 1 | r0 + 2, r0 + 3
          if (hs && total > 0) {
            const uint32_t bw = bsum[bk];
            if (unl) {
              if (bw >> 31) {  // its block's slot: exact sums
                const uint32_t *my = slot_of((int)(bw & 0xFFu)) + 2 * sj;
                acc0 += my[0];
                acc1 += my[1];
              } else {  // past 64 blocks: the block's sum bounds each document
                const uint32_t bsc = wide_nl ? 0x4000u : min(bw & 0xFFFFu, 0x4000u);
                acc0 += bsc | (bsc << 16);
                acc1 += bsc | (bsc << 16);
              }
            } else {
              const uint32_t bs = bw & 0xFFFFu, bn = bw >> 16;
              if (bs != 0 && bn <= 2) {  // the block's inline entries in this sub-block
                for (uint32_t k2 = 0; k2 < bn; k2++) {
                  const uint32_t ent = bent[2 * bk + k2];
                  const int dr = (int)(ent & 15u) - (sj << 2);
                  const uint32_t add = (ent >> 4) << ((dr & 1) << 4);
                  acc0 += (dr == 0 || dr == 1) ? add : 0u;
                  acc1 += (dr == 2 || dr == 3) ? add : 0u;
                }
              } else if (bs != 0) {
                // per sparse term, its listed entries from the first with r >= r0 while r < r0 + 4
                for (uint64_t m = sm; m; m &= m - 1) {
                  const int j = (int)__builtin_ctzll(m);
                  int lo = __builtin_amdgcn_readlane(prej, j);
                  const int hi0 = lo + __builtin_amdgcn_readlane(cj, j);
                  int hi = hi0;
                  while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if ((int)(slist[mid] & 0xFFFu) < r0) lo = mid + 1;
                    else hi = mid;
                  }
                  for (; lo < hi0; lo++) {
                    const uint32_t ent = slist[lo];
                    const int dr = (int)(ent & 0xFFFu) - r0;
                    if (dr >= 4) break;
                    const uint32_t add = ((ent >> 12) & 0xFFu) << ((dr & 1) << 4);
                    acc0 += dr < 2 ? add : 0u;
                    acc1 += dr < 2 ? 0u : add;
                  }
                }
              }
            }
          }
          {  // heavy impacts: one dword (four documents) per term, four loads in flight
            const int64_t io = (x << kWinB) + r0;
            for (uint64_t mh = hm; mh;) {
              uint32_t wq[4];
#pragma unroll
              for (int g = 0; g < 4; g++) {
                wq[g] = 0;
                if (mh) {
                  const int j = (int)__builtin_ctzll(mh);
                  mh &= mh - 1;
                  if (hs)
                    wq[g] = *reinterpret_cast<const uint32_t *>(
                        QA.imp + (int64_t)__builtin_amdgcn_readlane(D.hr, j) * QA.hstride + io);
                }
              }
#pragma unroll
              for (int g = 0; g < 4; g++) {
                acc0 += __builtin_amdgcn_perm(0u, wq[g], 0x0C010C00u);
                acc1 += __builtin_amdgcn_perm(0u, wq[g], 0x0C030C02u);
              }
            }
          }
          // documents of the sub-block over the gate (bit 15 of each biased half)
          const uint32_t cm = hs ? (((acc0 >> 15) & 1u) | ((acc0 >> 30) & 2u) | ((acc1 >> 13) & 4u) | ((acc1 >> 28) & 8u))
                                 : 0u;
          // candidates listed in LDS, scored one per lane
          const int32_t cl = __popc(cm);
          const int32_t cincl = wave_incl_sum(cl);
          const int32_t ncand = (QW_EXPER & 2) ? 0 : __builtin_amdgcn_readlane(cincl, 63);
          if (QW_STATS && lane == 0) atomicAdd(QW_STATS + 4, (unsigned long long)ncand);
          // the threshold itself (score, key) only where documents reached the gate
          const double th0 = ncand > 0 ? ld_uni(QA.th0 + P.q) : 0.0;
          const uint64_t thk = ncand > 0 ? ld_uni(QA.thk + P.q) : kNoKey;
          for (int32_t k0 = 0; k0 < ncand; k0 += kCList) {
            const int32_t kn = min(ncand - k0, kCList);
            qwave_sync();
            {
              int32_t o = cincl - cl - k0;
              for (uint32_t m = cm; m; m &= m - 1, o++)
                if (o >= 0 && o < kn) clist[o] = (uint16_t)(r0 + __builtin_ctz(m));
            }
            qwave_sync();
            for (int32_t c0 = 0; c0 < kn; c0 += 64) {
              double S = 0.0;
              uint64_t key = kNoKey;
              bool keep = false;
              if (c0 + lane < kn) {
                const int r = (int)clist[c0 + lane];
                const int32_t d = (int32_t)(wbase + r);
                uint32_t tie = 0xFFFFFFFFu;
                // the first 8 heavy terms' tf bytes first, their loads in flight
                // together (the ordered sum below would wait on each in turn)
                uint64_t hb8 = 0;
                {
                  uint64_t mh = hm;
                  uint32_t fb[8];
#pragma unroll
                  for (int c = 0; c < SME_QFB; c++) {
                    fb[c] = 0;
                    if (mh) {
                      const int j = (int)__builtin_ctzll(mh);
                      mh &= mh - 1;
                      fb[c] = QA.tfrow[(int64_t)__builtin_amdgcn_readlane(D.hr, j) * QA.hstride + (x << kWinB) + r];
                    }
                  }
#pragma unroll
                  for (int c = 0; c < SME_QFB; c++) hb8 |= (uint64_t)fb[c] << (8 * c);
                }
                int hseen = 0;
                for (uint64_t m = amask; m; m &= m - 1) {
                  const int j = (int)__builtin_ctzll(m);
                  int f = 0;
                  if ((hm >> j) & 1) {
                    if (hseen < SME_QFB) {
                      f = (int)(hb8 & 0xFFu);
                      hb8 >>= 8;
                    } else {
                      f = QA.tfrow[(int64_t)__builtin_amdgcn_readlane(D.hr, j) * QA.hstride + (x << kWinB) + r];
                    }
                    hseen++;
                  } else if (listed) {
                    const int lo0 = __builtin_amdgcn_readlane(prej, j), hi0 = lo0 + __builtin_amdgcn_readlane(cj, j);
                    int lo = lo0, hi = hi0;
                    while (lo < hi) {  // the term's entries are docno-ascending
                      const int mid = (lo + hi) >> 1;
                      if ((int)(slist[mid] & 0xFFFu) < r) lo = mid + 1;
                      else hi = mid;
                    }
                    if (lo < hi0 && (int)(slist[lo] & 0xFFFu) == r) {
                      f = (int)(slist[lo] >> 20);
                      if (f == 0xFFF) f = -1;  // tf >= 4095: read it from the postings
                    }
                  } else {
                    f = -1;
                  }
                  if (f < 0) {  // global binary search over the term's postings in the window
                    const int64_t base = rl64(D.mb, j);
                    int64_t lo = base + __builtin_amdgcn_readlane(mc, j);
                    const int64_t e = base + __builtin_amdgcn_readlane(me, j);
                    int64_t hi = e;
                    while (lo < hi) {
                      const int64_t mid = (lo + hi) >> 1;
                      if (QA.docno[mid] < d) lo = mid + 1;
                      else hi = mid;
                    }
                    f = (lo < e && QA.docno[lo] == d) ? QA.tf[lo] : 0;
                  }
                  if (f != 0) {
                    S = __dadd_rn(S, __dmul_rn(f < kWinLut ? s_lut[f] : QA.lut[f], rld(D.idf, j)));
                    if (tie == 0xFFFFFFFFu) tie = ref_tie(j, f, QA.reftie);
                  }
                }
                key = doc_key(QA.reftie ? tie : 0u, d);
                keep = S > th0 || (S == th0 && key <= thk);  // th0 < 0 (no seed): every touched document
              }
              const uint64_t km = (uint64_t)__ballot(keep);
              if (QW_STATS && lane == 0) atomicAdd(QW_STATS + 5, (unsigned long long)__popcll(km));
              if (km) {
                unsigned int base = 0;
                if (lane == 0) base = atomicAdd(&QA.ccnt[P.q], (unsigned int)__popcll(km));
                base = (unsigned int)__shfl((int)base, 0, 64);
                if (keep) {
                  const unsigned int idx = base + lane_prefix(km);
                  if (idx < (unsigned int)QA.cap) {
                    QA.cs[(int64_t)P.q * QA.cap + idx] = S;
                    QA.ck[(int64_t)P.q * QA.cap + idx] = key;
                  }
                }
              }
            }
          }
        }
      }
    }
    if (!hasn) break;
    if (total > 0) {  // clear the block sums this pair wrote
#pragma unroll
      for (int m = 0; m < 4; m++) bsum[m * 64 + lane] = 0;
    }
    qwave_sync();  // this wave's LDS is rewritten for the next query
    pos = npos;
    P = NP;
    NP = NNP;
    D = ND;
    gate = ngate;
    mc = nmc;
    me = nme;
#undef QA
  }
}

struct QFinalArgs {
  const int32_t *qlist;       // queries of this round (nullptr: 0 .. n-1)
  int n, k, cap;
  const unsigned int *ccnt;
  const unsigned int *oflag;  // lists that overflowed in an earlier stage (k_query_raise)
  const double *cs;
  const uint64_t *ck;
  int32_t *out_d;
  double *out_s;
  uint32_t *out_t;
  double *th_s;               // overflowed queries: raised threshold for the next round
  uint64_t *th_k;
  int32_t *ovf;               // queries whose list overflowed
  unsigned int *novf;
  const unsigned int *nlist;  // qlist's length on the device (nullptr: n)
  int32_t *defer;             // lists longer than this instance's LDS sort -> a bigger one (nullptr: none)
  unsigned int *ndefer;
};

// Per query: sort the candidates (score desc, key asc) and emit the best k.  A
// list that overflowed holds `cap` arbitrary candidates -- real documents with
// exact scores -- so the k-th best of them, B, is a valid bound: every document
// of the true top k is at least as good as B.  It becomes the query's threshold
// (score and key) for the next round, which keeps only documents not worse
// than B (deep exact ties at the score are cut by key).
template <int CM>
__global__ __launch_bounds__(64) void k_query_final(QFinalArgs a) {
  __shared__ double bs[CM];
  __shared__ uint64_t bk[CM];
  const int lane = threadIdx.x;
  const int nitems = a.nlist ? (int)*a.nlist : a.n;
  for (int i = blockIdx.x; i < nitems; i += gridDim.x) {
    const int q = a.qlist ? a.qlist[i] : i;
    const unsigned int c = a.ccnt[q];
    const bool over = c > (unsigned int)a.cap || a.oflag[q] != 0u;
    if (over && a.cap < a.k) {  // too few to bound anything: straight to the fallback
      if (lane == 0) a.ovf[atomicAdd(a.novf, 1u)] = q;
      continue;
    }
    const int n = min((int)c, a.cap);
    int n2 = 2;
    while (n2 < n) n2 <<= 1;
    if (n2 > CM) {  // (a.defer is set whenever a list can outgrow CM)
      if (lane == 0) a.defer[atomicAdd(a.ndefer, 1u)] = q;
      continue;
    }
    for (int j = lane; j < n2; j += 64) {
      bs[j] = j < n ? a.cs[(int64_t)q * a.cap + j] : -INFINITY;
      bk[j] = j < n ? a.ck[(int64_t)q * a.cap + j] : kNoKey;
    }
    __syncthreads();
    wave_sort(bs, bk, n2);
    if (over) {
      if (lane == 0) {
        a.th_s[q] = bs[a.k - 1];
        a.th_k[q] = bk[a.k - 1];
        a.ovf[atomicAdd(a.novf, 1u)] = q;
      }
    } else {
      for (int r = lane; r < a.k; r += 64) {
        a.out_d[(int64_t)q * a.k + r] = r < n ? key_doc(bk[r]) : -1;
        a.out_s[(int64_t)q * a.k + r] = r < n ? bs[r] : 0.0;
        if (a.out_t) a.out_t[(int64_t)q * a.k + r] = r < n ? (uint32_t)(bk[r] >> 32) : 0xFFFFFFFFu;
      }
    }
    __syncthreads();
  }
}
// Between window stages: every query's k-th best candidate so far (stored
// entries, all real documents with exact scores) bounds its k-th best score
// from below; if it beats the threshold it replaces it, so the later stages
// keep far fewer documents.  A list that overflowed lost candidates: its cap
// stored entries still bound the threshold, it is compacted like the others
// and flagged, so the final pass sends the query to another round (with the
// threshold the later stages raised further).
// Two instances: a small-LDS one over every query (many workgroups per CU) that
// hands lists longer than its CM to `defer`, and a large-LDS one over that list.
template <int CM>
__global__ __launch_bounds__(64) void k_query_raise(int nq, int k, int cap, unsigned int *ccnt, unsigned int *oflag,
                                                    double *cs, uint64_t *ck, double *th_s, uint64_t *th_k,
                                                    const int32_t *qlist, const unsigned int *nlist, int32_t *defer,
                                                    unsigned int *ndefer) {
  __shared__ double bs[CM];
  __shared__ uint64_t bk[CM];
  const int lane = threadIdx.x;
  const int nitems = qlist ? (int)*nlist : nq;
  for (int i = blockIdx.x; i < nitems; i += gridDim.x) {
    const int q = qlist ? qlist[i] : i;
    const unsigned int c = ccnt[q];
    const bool over = c > (unsigned int)cap;
    const int n = over ? cap : (int)c;
    if (n < k) continue;  // too few to bound (cap >= k here)
    int n2 = 2;
    while (n2 < n) n2 <<= 1;
    if (n2 > CM) {  // (defer is set whenever a list can outgrow CM)
      if (lane == 0) defer[atomicAdd(ndefer, 1u)] = q;
      continue;
    }
    for (int j = lane; j < n2; j += 64) {
      bs[j] = j < n ? cs[(int64_t)q * cap + j] : -INFINITY;
      bk[j] = j < n ? ck[(int64_t)q * cap + j] : kNoKey;
    }
    __syncthreads();
    wave_sort(bs, bk, n2);
    // the list keeps only its best k (nothing worse than its k-th best can be in
    // the top k), so later windows append into free room
    const bool up = better(bs[k - 1], bk[k - 1], th_s[q], th_k[q]);
    for (int r = lane; r < k; r += 64) {
      cs[(int64_t)q * cap + r] = bs[r];
      ck[(int64_t)q * cap + r] = bk[r];
    }
    if (lane == 0) {
      ccnt[q] = (unsigned int)k;
      if (over) oflag[q] = 1u;
      if (up) {
        th_s[q] = bs[k - 1];
        th_k[q] = bk[k - 1];
      }
    }
    __syncthreads();
  }
}
__global__ void k_reset_cnt(const int32_t *qlist, int n, unsigned int *ccnt, unsigned int *oflag) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    ccnt[qlist[i]] = 0;
    oflag[qlist[i]] = 0;
  }
}

// impact rows q(tf) = floor(lut[tf] * idf * alpha) + 1 (0 for tf = 0), 16-document
// tf maxima (bm16) and 4-document impact maxima (sbq) in one pass over the tf rows: thread = one 16-byte block of 16 documents (the
// three used to re-read the tf and impact rows in separate passes)
__global__ __launch_bounds__(256) void k_heavy_imp3(const uint8_t *tfrow, const int32_t *hterm, int64_t H,
                                                    int64_t stride, const double *lut, int max_tf, const double *idf,
                                                    double alpha, uint8_t *imp, uint8_t *bm16, uint32_t *sbq) {
  __shared__ uint8_t ql[256];
  const int64_t chunks = stride >> 12;  // 4096-byte chunks per row
  for (int64_t c = blockIdx.x; c < H * chunks; c += gridDim.x) {
    const int64_t row = c / chunks;
    const double wi = idf[hterm[row]];
    __syncthreads();
    const int f = threadIdx.x;
    ql[f] = (uint8_t)(f == 0 ? 0u : f <= max_tf ? impact(lut[f], wi, alpha) : 255u);
    __syncthreads();
    const int64_t i = c * 256 + threadIdx.x;  // flat 16-document block
    const uint4 v = reinterpret_cast<const uint4 *>(tfrow)[i];
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; u++)
      o[u] = (uint32_t)ql[w4[u] & 0xFF] | ((uint32_t)ql[(w4[u] >> 8) & 0xFF] << 8) |
             ((uint32_t)ql[(w4[u] >> 16) & 0xFF] << 16) | ((uint32_t)ql[w4[u] >> 24] << 24);
    reinterpret_cast<uint4 *>(imp)[i] = make_uint4(o[0], o[1], o[2], o[3]);
    bm16[i] = (uint8_t)max(max(max_u8x4(v.x), max_u8x4(v.y)), max(max_u8x4(v.z), max_u8x4(v.w)));
    sbq[i] = max_u8x4(o[0]) | (max_u8x4(o[1]) << 8) | (max_u8x4(o[2]) << 16) | (max_u8x4(o[3]) << 24);
  }
}
// SME_HEAVY_FUSED (default 1): the heavy rows in one pass -- a block per (row,
// run of kHvWpb 4096-document windows) finds the run's postings (two 64-ary lower
// bounds), scatters them into zeroed LDS rows (four loads per thread in flight)
// and writes each window's tf bytes, impact bytes, 16-document tf maxima and
// 4-document impact maxima densely from them (no row memset, no byte-scatter into
// HBM, no second pass reading the tf rows back)
#ifndef SME_HEAVY_FUSED
#define SME_HEAVY_FUSED 1
#endif
constexpr int kHvWpb = 8;  // windows per block: 32 KB of LDS rows
// 64-ary lower bound (one wave): first p in [lo, hi) with docno[p] >= target
__device__ __forceinline__ int64_t wave_lower_bound(const int32_t *docno, int64_t lo, int64_t hi, int64_t target,
                                                    int lane) {
  while (lo < hi) {
    const int64_t step = (hi - lo + 63) / 64, pos = lo + lane * step;
    const uint64_t m = (uint64_t)__ballot(pos < hi && (int64_t)docno[pos] < target);
    const int k = __popcll(m);
    if (k == 0) {
      hi = lo;
    } else {
      const int64_t nhi = min(hi, lo + k * step);
      lo = lo + (k - 1) * step + 1;
      hi = nhi;
    }
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_heavy_build(const int32_t *hterm, int64_t H, const int64_t *off,
                                                     const int32_t *docno, const int32_t *tf, int64_t dmin,
                                                     int64_t stride, const double *lut, int max_tf, const double *idf,
                                                     double alpha, uint8_t *tfrow, uint8_t *imp, uint8_t *bm16,
                                                     uint32_t *sbq) {
  __shared__ uint8_t ql[256];
  __shared__ alignas(16) uint8_t buf[kHvWpb * kWin];
  __shared__ int64_t s_cur[2];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t chunks = stride >> kWinB, nbr = (chunks + kHvWpb - 1) / kHvWpb;
  for (int64_t bi = blockIdx.x; bi < H * nbr; bi += gridDim.x) {
    const int64_t row = bi / nbr, c0 = (bi % nbr) * kHvWpb, c1 = min(chunks, c0 + kHvWpb);
    const int64_t t = hterm[row], b = off[t], e = off[t + 1];
    const int64_t wbase = dmin + (c0 << kWinB);
    const double wi = idf[t];
    __syncthreads();  // the previous run's LDS reads are done
    ql[tid] = (uint8_t)(tid == 0 ? 0u : tid <= max_tf ? impact(lut[tid], wi, alpha) : 255u);
    for (int64_t c = c0; c < c1; c++) reinterpret_cast<uint4 *>(buf)[((c - c0) << 8) + tid] = make_uint4(0, 0, 0, 0);
    // the run's postings: [lower bound of its first docno, lower bound past its last window)
    if (wv < 2) {
      const int64_t p = wave_lower_bound(docno, b, e, wv == 0 ? wbase : dmin + (c1 << kWinB), lane);
      if (lane == 0) s_cur[wv] = p;
    }
    __syncthreads();
    const int64_t p0 = s_cur[0], p1 = s_cur[1];
    // scatter into the LDS rows, four postings per thread in flight
    for (int64_t i0 = p0 + tid; i0 < p1; i0 += 4 * 256) {
      int32_t d[4], f[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int64_t i = i0 + u * 256;
        d[u] = i < p1 ? docno[i] : 0;
        f[u] = i < p1 ? tf[i] : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (f[u] >= 0) buf[(int64_t)d[u] - wbase] = (uint8_t)f[u];
    }
    __syncthreads();
    for (int64_t c = c0; c < c1; c++) {
      const uint4 v = reinterpret_cast<const uint4 *>(buf)[((c - c0) << 8) + tid];
      const int64_t fi = row * (stride >> 4) + (c << 8) + tid;  // flat 16-document block
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
#pragma unroll
      for (int u = 0; u < 4; u++)
        o[u] = (uint32_t)ql[w4[u] & 0xFF] | ((uint32_t)ql[(w4[u] >> 8) & 0xFF] << 8) |
               ((uint32_t)ql[(w4[u] >> 16) & 0xFF] << 16) | ((uint32_t)ql[w4[u] >> 24] << 24);
      reinterpret_cast<uint4 *>(tfrow)[fi] = v;
      reinterpret_cast<uint4 *>(imp)[fi] = make_uint4(o[0], o[1], o[2], o[3]);
      bm16[fi] = (uint8_t)max(max(max_u8x4(v.x), max_u8x4(v.y)), max(max_u8x4(v.z), max_u8x4(v.w)));
      sbq[fi] = max_u8x4(o[0]) | (max_u8x4(o[1]) << 8) | (max_u8x4(o[2]) << 16) | (max_u8x4(o[3]) << 24);
    }
  }
}

// k_query_win's sparse posting words (index-resident, like the impact rows):
// (docno - dmin) mod 4096 = the posting's place in its 4096-document window, its
// impact q(tf) at the index's scale and its tf (4095 = "4095 or more"), so the
// window pass loads one word per posting and does no arithmetic on it.  One
// wave per term; terms with a heavy row are skipped (the window pass reads rows).
#ifndef SME_SPK_LANES
#define SME_SPK_LANES 1
#endif
__device__ __forceinline__ uint32_t sparse_word(int32_t dn, int32_t f, const double *lut, double wi, double alpha,
                                                int64_t dmin) {
  return (uint32_t)(((int64_t)dn - dmin) & (kWin - 1)) | (impact(lut[f], wi, alpha) << 12) |
         ((uint32_t)min(f, 0xFFF) << 20);
}
#if SME_SPK_LANES
// 64 terms per wave step, one per lane: a term of <= kSpkSmall postings is packed
// by its own lane (most terms: the Zipf tail and the df-1 docid terms); longer
// ones are listed (one atomic per wave) for k_sparse_pack_big, a wave per term
// over the whole grid (a wave per term for every term spent a wave step and four
// dependent loads on each one-posting term; the listed terms packed by the wave
// that met them clustered c5's word terms on a few waves)
constexpr int kSpkSmall = 16;
__global__ __launch_bounds__(256) void k_sparse_pack(const int64_t *off, int64_t V, const int32_t *hrow_of,
                                                     const int32_t *docno, const int32_t *tf, const double *lut,
                                                     const double *idf, double alpha, int64_t dmin, uint32_t *spk,
                                                     int32_t *big_list, unsigned int *nbig) {
  const int lane = threadIdx.x & 63;
  const int64_t nwv = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t0 = (blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6)) * 64; t0 < V; t0 += nwv * 64) {
    const int64_t t = t0 + lane;
    int64_t b = 0, e = 0;
    double wi = 0.0;
    if (t < V && !(hrow_of && hrow_of[t] >= 0)) {
      b = off[t];
      e = off[t + 1];
      wi = idf[t];
    }
    if (e - b <= kSpkSmall) {
      for (int64_t i = b; i < e; i++) spk[i] = sparse_word(docno[i], tf[i], lut, wi, alpha, dmin);
    }
    const uint64_t bm = (uint64_t)__ballot(e - b > kSpkSmall);
    if (bm) {
      unsigned int base = 0;
      if (lane == 0) base = atomicAdd(nbig, (unsigned int)__popcll(bm));
      base = (unsigned int)__shfl((int)base, 0, 64);
      if ((bm >> lane) & 1ull) big_list[base + __popcll(bm & ((1ull << lane) - 1ull))] = (int32_t)t;
    }
  }
}
__global__ __launch_bounds__(256) void k_sparse_pack_big(const int64_t *off, const int32_t *docno, const int32_t *tf,
                                                         const double *lut, const double *idf, double alpha,
                                                         int64_t dmin, uint32_t *spk, const int32_t *big_list,
                                                         const unsigned int *nbig) {
  const int lane = threadIdx.x & 63;
  const int64_t nwv = (int64_t)gridDim.x * (blockDim.x >> 6), n = (int64_t)*nbig;
  for (int64_t w = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); w < n; w += nwv) {
    const int64_t t = big_list[w];
    const int64_t b = off[t], e = off[t + 1];
    const double wi = idf[t];
    for (int64_t i = b + lane; i < e; i += 64) spk[i] = sparse_word(docno[i], tf[i], lut, wi, alpha, dmin);
  }
}
#else
__global__ __launch_bounds__(256) void k_sparse_pack(const int64_t *off, int64_t V, const int32_t *hrow_of,
                                                     const int32_t *docno, const int32_t *tf, const double *lut,
                                                     const double *idf, double alpha, int64_t dmin, uint32_t *spk) {
  const int lane = threadIdx.x & 63;
  const int64_t nwv = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); t < V; t += nwv) {
    if (hrow_of && hrow_of[t] >= 0) continue;  // (wave-uniform)
    const int64_t b = off[t], e = off[t + 1];
    const double wi = idf[t];
    for (int64_t i = b + lane; i < e; i += 64) spk[i] = sparse_word(docno[i], tf[i], lut, wi, alpha, dmin);
  }
}
#endif

// largest weight of any term (its max tf is the first posting of the
// reduce-order CSR): the index's impact scale alpha = 253.5 / wmax
__global__ __launch_bounds__(256) void k_index_wmax(const int64_t *off, int64_t V, const int32_t *tf_o, const double *lut,
                             const double *idf, unsigned long long *wmax_bits) {
  unsigned long long wm = 0;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    if (off[t + 1] > off[t]) {
      const unsigned long long wb =
          (unsigned long long)__double_as_longlong(__dmul_rn(lut[tf_o[off[t]]], idf[t]));
      wm = wb > wm ? wb : wm;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(wm, o, 64);
    wm = u > wm ? u : wm;
  }
  // one atomic per block, and only when it can raise the maximum (single-address
  // atomics serialise: one per wave took ~0.2 ms on c2's 2 M terms)
  __shared__ unsigned long long s_wm[4];
  if ((threadIdx.x & 63) == 0) s_wm[threadIdx.x >> 6] = wm;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); i++) wm = s_wm[i] > wm ? s_wm[i] : wm;
    if (wm && wm > __hip_atomic_load(wmax_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(wmax_bits, wm);
  }
}

// Index-resident query structures, built once per index and heavy threshold:
// the heavy terms' tf rows with their 16 / 1024-document maxima (k_query_bm),
// the index's impact scale alpha = 253.5 / (largest weight of any term) and the
// heavy terms' impact rows q(tf) at that scale (k_query_win).  The impact rows
// and alpha depend on idf: sme_index_reweight drops them (q_ready).
void prepare_queries(sme_index *ix, hipStream_t st) {
  sme_ctx *cx = ix->ctx;
  const int64_t div = cx->opt_heavy_div;
  if (ix->q_ready && ix->q_div == div) return;
  hipEvent_t e0, e1;
  SME_HIP(hipEventCreate(&e0));
  SME_HIP(hipEventCreate(&e1));
  SME_HIP(hipEventRecord(e0, st));
  ix->q_H = 0;
  // tiles of 1024 documents, a multiple of 4 (k_query_win's 4096-document windows)
  ix->q_T = (ix->V > 0 && ix->P > 0 && ix->dmax >= ix->dmin) ? ((((ix->dmax - ix->dmin) >> kQB) + 1 + 3) & ~int64_t(3))
                                                             : 0;
  const int64_t V = ix->V, T = ix->q_T;
  ix->q_alpha = 1.0;
  if (V > 0 && ix->P > 0) {
    unsigned long long *wb = reinterpret_cast<unsigned long long *>(cx->ws[35].as<uint64_t>(1));
    SME_HIP(hipMemsetAsync(wb, 0, sizeof(uint64_t), st));
    hipLaunchKernelGGL(k_index_wmax, dim3((unsigned)std::min<int64_t>((V + 255) / 256, 4096)), dim3(256), 0, st,
                       (const int64_t *)ix->d_off.p, V, (const int32_t *)ix->d_tf_o.p, (const double *)ix->d_lut.p,
                       (const double *)ix->d_idf.p, wb);
    SME_CHECK_LAUNCH();
    unsigned long long h = 0;
    SME_HIP(hipMemcpyAsync(&h, wb, sizeof h, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    ix->q_wmax_bits = h;
    const double wmax = __builtin_bit_cast(double, h);
    ix->q_alpha = wmax > 0.0 ? 253.5 / wmax : 1.0;
  }
  if (T > 0 && div > 0) {
    auto &W = cx->ws;
    const int64_t *off = (const int64_t *)ix->d_off.p;
    const int64_t span = ix->dmax - ix->dmin + 1, stride = T << kQB;
    int32_t *flag = W[36].as<int32_t>(V + 1), *scan = W[37].as<int32_t>(V + 1);
    SME_HIP(hipMemsetAsync(flag + V, 0, sizeof(int32_t), st));
    const unsigned gV = (unsigned)std::min<int64_t>((V + 255) / 256, 8192);
    hipLaunchKernelGGL(k_heavy_flags, dim3(gV), dim3(256), 0, st, off, (const int32_t *)ix->d_tf_o.p, V, span, div,
                       flag);
    size_t tbb = 0;
    excl_scan(flag, scan, (int64_t)(V + 1), cx->ws[23], st);
    int32_t nh = 0;
    SME_HIP(hipMemcpyAsync(&nh, scan + V, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    // memory budget for the rows: a quarter of the device's free memory, at most
    // 64 GB (a heavy term without a row reaches the window pass as a long sparse
    // list; the c4 shard's ~2,300 heavy terms need ~33 GB of rows).  Free memory
    // includes the blocks the context's pool holds for reuse (a closed index's
    // rows among them) and this index's own row buffer: hipMemGetInfo counts
    // neither, so a second index on the same context got fewer rows than the first
    // (the c4 shard's 100 k batch: 100 -> 373 ms)
    size_t fr = 0, tot = 0;
    SME_HIP(hipMemGetInfo(&fr, &tot));
    const double avail = (double)fr + (double)cx->pool.idle() + (double)ix->d_heavy.cap;
    const double per_row = 2.0 * (double)stride + (double)(T << 6) + (double)T + (double)(T << 8);
    const int64_t cap = (int64_t)(std::min<double>(avail / 4.0, 64e9) / per_row);
    const int64_t H = std::min<int64_t>(nh, cap);
    int32_t *hrow_of = ix->d_hrow_of.as<int32_t>(V);
    int32_t *hterm = W[38].as<int32_t>(H + 1);
    int64_t *hdf = W[39].as<int64_t>(H + 1), *hpre = W[40].as<int64_t>(H + 1);
    hipLaunchKernelGGL(k_heavy_rows, dim3(gV), dim3(256), 0, st, flag, scan, V, H, off, hrow_of, hterm, hdf);
    SME_CHECK_LAUNCH();
    if (H > 0) {
      SME_HIP(hipMemsetAsync(hdf + H, 0, sizeof(int64_t), st));
      excl_scan(hdf, hpre, (int64_t)(H + 1), cx->ws[23], st);
      uint8_t *buf = ix->d_heavy.as<uint8_t>((size_t)H * (size_t)per_row + 128);
      uint8_t *tfrow = buf, *imp = buf + H * stride, *bm16 = imp + H * stride, *bm1k = bm16 + H * (T << 6);
      uint8_t *sbq = bm1k + H * T + 64 - ((H * T) & 15);  // 16-byte aligned
      const int64_t n16 = H * (T << 6), n1k = H * T;
#if SME_HEAVY_FUSED
      hipLaunchKernelGGL(k_heavy_build, dim3((unsigned)std::min<int64_t>(H * (((stride >> kWinB) + kHvWpb - 1) / kHvWpb), 1 << 16)),
                         dim3(256), 0, st, hterm, H, off, (const int32_t *)ix->d_docno_d.p,
                         (const int32_t *)ix->d_tf_d.p, ix->dmin, stride, (const double *)ix->d_lut.p, ix->max_tf,
                         (const double *)ix->d_idf.p, ix->q_alpha, tfrow, imp, bm16, reinterpret_cast<uint32_t *>(sbq));
#else
      SME_HIP(hipMemsetAsync(tfrow, 0, (size_t)(H * stride), st));
      hipLaunchKernelGGL(k_heavy_fill, dim3(16384), dim3(256), 0, st, hpre, H, hterm, off,
                         (const int32_t *)ix->d_docno_d.p, (const int32_t *)ix->d_tf_d.p, ix->dmin, stride, tfrow);
      hipLaunchKernelGGL(k_heavy_imp3, dim3((unsigned)std::min<int64_t>(H * (stride >> 12), 1 << 16)), dim3(256), 0, st,
                         tfrow, hterm, H, stride, (const double *)ix->d_lut.p, ix->max_tf,
                         (const double *)ix->d_idf.p, ix->q_alpha, imp, bm16, reinterpret_cast<uint32_t *>(sbq));
#endif
      hipLaunchKernelGGL(k_heavy_bm1k, dim3((unsigned)std::min<int64_t>((n1k + 255) / 256, 1 << 16)), dim3(256), 0,
                         st, (const uint4 *)bm16, n1k, bm1k);
      SME_CHECK_LAUNCH();
      ix->q_imp = imp;
      ix->q_sbq = sbq;
      ix->q_tfrow = tfrow;
      ix->q_bm16 = bm16;
      ix->q_bm1k = bm1k;
    }
    ix->q_H = H;
  }
  // sparse posting words for the window pass, if 4 B per posting fits a quarter
  // of the free memory (else query_topk takes the block-max path)
  ix->q_spk = nullptr;
  if (T > 0 && ix->P > 0) {
    size_t fr = 0, tot = 0;
    SME_HIP(hipMemGetInfo(&fr, &tot));
    const size_t need = (size_t)ix->P * sizeof(uint32_t);
    if (ix->d_spk.cap >= need || need <= (fr + cx->pool.idle()) / 4) {
      uint32_t *spk = ix->d_spk.as<uint32_t>((size_t)ix->P);
      const int32_t *hro = ix->q_H > 0 ? (const int32_t *)ix->d_hrow_of.p : nullptr;
#if SME_SPK_LANES
      // (stream-ordered after the heavy-row kernels: their flag / scan slots are free)
      int32_t *big_list = cx->ws[37].as<int32_t>(V + 1);
      unsigned int *nbig = reinterpret_cast<unsigned int *>(cx->ws[35].as<uint64_t>(1));
      SME_HIP(hipMemsetAsync(nbig, 0, sizeof(unsigned int), st));
      hipLaunchKernelGGL(k_sparse_pack, dim3((unsigned)std::min<int64_t>((V + 255) / 256, 65536)), dim3(256), 0, st,
                         (const int64_t *)ix->d_off.p, V, hro, (const int32_t *)ix->d_docno_d.p,
                         (const int32_t *)ix->d_tf_d.p, (const double *)ix->d_lut.p, (const double *)ix->d_idf.p,
                         ix->q_alpha, ix->dmin, spk, big_list, nbig);
      hipLaunchKernelGGL(k_sparse_pack_big, dim3(16384), dim3(256), 0, st, (const int64_t *)ix->d_off.p,
                         (const int32_t *)ix->d_docno_d.p, (const int32_t *)ix->d_tf_d.p, (const double *)ix->d_lut.p,
                         (const double *)ix->d_idf.p, ix->q_alpha, ix->dmin, spk, (const int32_t *)big_list,
                         (const unsigned int *)nbig);
#else
      hipLaunchKernelGGL(k_sparse_pack, dim3((unsigned)std::min<int64_t>((V + 3) / 4, 65536)), dim3(256), 0, st,
                         (const int64_t *)ix->d_off.p, V, hro, (const int32_t *)ix->d_docno_d.p,
                         (const int32_t *)ix->d_tf_d.p, (const double *)ix->d_lut.p, (const double *)ix->d_idf.p,
                         ix->q_alpha, ix->dmin, spk);
#endif
      SME_CHECK_LAUNCH();
      ix->q_spk = spk;
    }
  }
  SME_HIP(hipEventRecord(e1, st));
  SME_HIP(hipEventSynchronize(e1));
  float ms = 0;
  SME_HIP(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  ix->q_prep_ms = ms;
  ix->q_div = div;
  ix->q_ready = true;
}

// rows of a sub-batch's results back into the batch's output rows
__global__ void k_scatter_rows(const int32_t *qlist, int n, int k, const int32_t *sd, const double *ss,
                               const uint32_t *st_, int32_t *d, double *s, uint32_t *t) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (int64_t)n * k;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = qlist[i / k], j = i % k;
    d[q * k + j] = sd[i];
    s[q * k + j] = ss[i];
    if (t) t[q * k + j] = st_[i];
  }
}

namespace {
struct QTimes {  // the per-call query timings of the context, summed over sub-batches
  float ms = 0, prep = 0, seed = 0, fin = 0, tot = 0;
  int64_t ovf = 0, fb = 0;
  void add(const sme_ctx *cx) {
    ms += cx->last_query_ms;
    prep += cx->last_query_prep_ms;
    seed += cx->last_query_seed_ms;
    fin += cx->last_query_final_ms;
    tot += cx->last_query_total_ms;
    ovf += cx->last_query_overflow;
    fb += cx->last_query_fallback;
  }
  void store(sme_ctx *cx) const {
    cx->last_query_ms = ms;
    cx->last_query_prep_ms = prep;
    cx->last_query_seed_ms = seed;
    cx->last_query_final_ms = fin;
    cx->last_query_total_ms = tot;
    cx->last_query_overflow = ovf;
    cx->last_query_fallback = fb;
  }
};
}  // namespace

// Queries `qlist` (device, n entries: rows of this batch) as their own compact
// batch, results scattered back into the batch's output rows.  The rare path
// for queries whose candidate lists still overflow after the window rounds
// when the batch's tile table does not fit in HBM: the subset's distinct terms
// are few, so its own tables fit (a single query of <= 64 terms always does).
static void query_subset(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, const int32_t *h_qlist,
                         int n, int k, int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie,
                         hipStream_t st, int tie_bits);

void query_topk(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, int k, int32_t *d_out_docno,
                double *d_out_score, uint32_t *d_out_tie, hipStream_t st, int tie_bits) {
  if (k < 1) throw Error(SME_EINVAL, "k must be >= 1");
  // k <= 448 on the window / block-max kernels; larger k up to 1792 on the streaming
  // kernel's LDS candidate list
  if (k > kListCap - kQNT) throw Error(SME_ELIMIT, "top-k with k > 1792");
  if (nq <= 0) return;
  sme_ctx *cx = ix->ctx;
  if (cx->cfg.tiebreak == SME_TIE_JAVA7) {  // the whole list and Java 7's TimSort (sme_timsort.hip)
    query_topk_java7(ix, d_terms, d_qoff, nq, k, d_out_docno, d_out_score, d_out_tie, st);
    return;
  }
  auto &W = cx->ws;
  int *err = W[63].as<int>(4);
  unsigned long long *wmax = reinterpret_cast<unsigned long long *>(err + 2);
  SME_HIP(hipMemsetAsync(err, 0, 4 * sizeof(int), st));
  int h_mx = 0;  // the batch's longest query (terms)
  // reference tie order: ref_tie keys hold the token index above tb tf bits, 24
  // for queries of <= 256 terms, 22 for longer ones (the top-level batch decides
  // and its nested calls inherit it, so doc shards answering one batch build the
  // same keys whatever the splits each shard's memory makes)
  int reftie = 0;
  if (cx->cfg.tiebreak == SME_TIE_REFERENCE) {
    if (tie_bits > 0) {
      reftie = tie_bits;
    } else {
      hipLaunchKernelGGL(k_max_qlen, dim3(std::min((nq + 255) / 256, 1024)), dim3(256), 0, st, d_qoff, nq, err + 1);
      SME_HIP(hipMemcpyAsync(&h_mx, err + 1, sizeof(int), hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
      reftie = h_mx > 256 ? 22 : 24;
    }
    if ((int64_t)ix->max_tf >= (int64_t(1) << reftie))
      throw Error(SME_ELIMIT, reftie == 24 ? "reference tie order with a term frequency >= 2^24"
                                           : "reference tie order, a query of > 256 terms and a term frequency >= 2^22");
  }
  const int64_t *off = (const int64_t *)ix->d_off.p;
  const int32_t *dn = (const int32_t *)ix->d_docno_d.p;
  const int32_t *tf = (const int32_t *)ix->d_tf_d.p;
  const double *lut = (const double *)ix->d_lut.p;
  const double *idf = (const double *)ix->d_idf.p;
  const int64_t V = ix->V;
  // the block-max path unless a query is longer than kIMaxTerms or the batch's
  // skip table would be unreasonably large; option query_kernel = 1 forces the
  // streaming kernel (tests run both)
  bool tiled = V > 0 && ix->P > 0 && ix->dmax >= ix->dmin && cx->opt_query_kernel != 1 && k <= 448;
  if (tiled) prepare_queries(ix, st);  // once per index (timed separately: q_prep_ms)
  hipEvent_t ep;
  SME_HIP(hipEventCreate(&ep));
  SME_HIP(hipEventRecord(ep, st));
  const int64_t T = tiled ? ix->q_T : 0;
  const int32_t *row_of = nullptr, *sk = nullptr;
  const uint8_t *qlut = nullptr;
  int64_t nrows_b = 0;      // distinct batch terms (rows of the skip / impact tables)
  int32_t *skt = nullptr;   // k_query_win: window skip table, transposed
  std::function<void()> build_sk;  // the tile skip table `sk` (k_query_bm), built on demand on the window path
  bool list_kernel = false;  // the streaming kernel with the LDS candidate list ran
  if (tiled) {
    hipLaunchKernelGGL(k_max_qlen, dim3(std::min((nq + 255) / 256, 1024)), dim3(256), 0, st, d_qoff, nq, err + 1);
    SME_HIP(hipMemcpyAsync(&h_mx, err + 1, sizeof(int), hipMemcpyDeviceToHost, st));
    int64_t nterm = 0, tbase = 0;  // the batch's terms are d_terms[tbase, nterm) (a sub-batch: tbase > 0)
    SME_HIP(hipMemcpyAsync(&nterm, d_qoff + nq, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(&tbase, d_qoff, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    tiled = h_mx <= kIMaxTerms;
    if (tiled) {
      // distinct batch terms -> rows of the skip and impact tables
      int32_t *mark = W[55].as<int32_t>(V + 1), *rowo = W[56].as<int32_t>(V + 1);
      SME_HIP(hipMemsetAsync(mark, 0, (V + 1) * sizeof(int32_t), st));
      if (nterm > tbase)
        hipLaunchKernelGGL(k_mark_terms, dim3((unsigned)std::min<int64_t>((nterm - tbase + 255) / 256, 8192)), dim3(256),
                           0, st, d_terms + tbase, nterm - tbase, V, mark);
      size_t tbb = 0;
      excl_scan(mark, rowo, (int64_t)(V + 1), cx->ws[23], st);
      int32_t nrows32 = 0;
      SME_HIP(hipMemcpyAsync(&nrows32, rowo + V, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
      const int64_t nrows = nrows32;
      nrows_b = nrows;
      // per-batch table budget: a quarter of the free HBM (plus the table
      // buffer this context already holds); a batch over it is split by query
      // range (each half has fewer distinct terms), so every batch of queries
      // of <= 64 terms is answered on this path
      size_t fr = 0, tot = 0;
      SME_HIP(hipMemGetInfo(&fr, &tot));
      const bool winp = cx->opt_query_kernel == 0 && ix->q_spk;
      // (the window path holds two tables of this size: the row-major change
      // points W[29] and the window-major skip table W[31])
      const double need = (double)nrows * (double)((winp ? (T >> 2) : T) + 1) * 4.0 * (winp ? 2.0 : 1.0);
      const double budget = cx->opt_query_budget > 0
                                ? (double)cx->opt_query_budget
                                : (double)fr / 4.0 + (winp ? (double)W[31].cap + (double)W[29].cap : (double)W[60].cap);
      if (need > budget && nq > 1) {
        SME_HIP(hipEventDestroy(ep));
        QTimes acc;
        const int h = nq / 2;
        query_topk(ix, d_terms, d_qoff, h, k, d_out_docno, d_out_score, d_out_tie, st, reftie);
        acc.add(cx);
        query_topk(ix, d_terms, d_qoff + h, nq - h, k, d_out_docno + (int64_t)h * k, d_out_score + (int64_t)h * k,
                   d_out_tie ? d_out_tie + (int64_t)h * k : nullptr, st, reftie);
        acc.add(cx);
        acc.store(cx);
        cx->last_query_split = true;
        return;
      }
      {  // (a single query's tables are always built: <= 64 rows)
        row_of = rowo;
        // impact scale: the index's (prepare_queries), shared by every batch
        SME_HIP(hipMemcpyAsync(wmax, &ix->q_wmax_bits, sizeof(uint64_t), hipMemcpyHostToDevice, st));
        if (!winp) qlut = W[44].as<uint8_t>(std::max<int64_t>(nrows, 1) * 256);
        if (nrows > 0) {
          int32_t *tor = W[57].as<int32_t>(nrows + 1);
          int64_t *rdf = W[58].as<int64_t>(nrows + 1), *rpre = W[59].as<int64_t>(nrows + 1);
          const unsigned gV = (unsigned)std::min<int64_t>((V + 255) / 256, 8192);
          hipLaunchKernelGGL(k_term_rows, dim3(gV), dim3(256), 0, st, mark, rowo, V, off, tor, rdf);
          SME_HIP(hipMemsetAsync(rdf + nrows, 0, sizeof(int64_t), st));
          excl_scan(rdf, rpre, (int64_t)(nrows + 1), cx->ws[23], st);
          // tile skip table and impact tables (k_query_bm); the window path
          // builds its window table directly (its postings carry their impacts)
          // and these only if a query falls back
          build_sk = [=, &W, &sk, &qlut]() {
            uint8_t *ql = W[44].as<uint8_t>(nrows * 256);
            qlut = ql;
            hipLaunchKernelGGL(k_row_qlut, dim3((unsigned)std::min<int64_t>(nrows, 16384)), dim3(256), 0, st, tor,
                               nrows, lut, ix->max_tf, idf, (const unsigned long long *)wmax, ql);
            int32_t *skw = W[60].as<int32_t>(std::max<int64_t>(nrows, 1) * (T + 1));  // allocated on first use
            sk = skw;
            SME_HIP(hipMemsetAsync(skw, 0x7F, (size_t)nrows * (T + 1) * sizeof(int32_t), st));
            hipLaunchKernelGGL(k_skip_zero_rows, dim3((unsigned)std::min<int64_t>(nrows, 4096)), dim3(256), 0, st,
                               rdf, nrows, T, skw);
            hipLaunchKernelGGL(k_skip_fill, dim3(16384), dim3(256), 0, st, rpre, nrows, tor, off, dn, ix->dmin, T,
                               skw);
            hipLaunchKernelGGL(k_skip_suffix, dim3((unsigned)std::min<int64_t>((nrows + 3) / 4, 16384)), dim3(256),
                               0, st, nrows, T, skw);
            SME_CHECK_LAUNCH();
          };
          if (winp) {
            const int64_t nwin = T >> 2, ne = nrows * (nwin + 1);
            skt = W[31].as<int32_t>(ne);
            int32_t *rm = W[29].as<int32_t>(ne);  // row-major change points (prep only)
            SME_HIP(hipMemsetAsync(rm, 0x7F, (size_t)ne * sizeof(int32_t), st));
            // only the sparse rows: k_query_win reads heavy terms from their impact
            // rows, never their skip entries (and heavy terms hold most postings)
            const int32_t *hro = ix->q_H > 0 ? (const int32_t *)ix->d_hrow_of.p : nullptr;
            int64_t *rdfw = rdf;
            if (hro) {
              rdfw = W[12].as<int64_t>(nrows + 1);
              hipLaunchKernelGGL(k_sparse_rdf, dim3((unsigned)std::min<int64_t>((nrows + 255) / 256, 16384)), dim3(256),
                                 0, st, tor, rdf, hro, nrows, rdfw);
            }
            hipLaunchKernelGGL(k_skipw_fill_rm, dim3((unsigned)std::min<int64_t>((nrows + 3) / 4, 65536)),
                               dim3(256), 0, st, rdfw, nrows, tor, off, dn, ix->dmin, nwin, rm);
            hipLaunchKernelGGL(k_skipw_suffix_tr, dim3((unsigned)std::min<int64_t>((nrows + 63) / 64, 16384)),
                               dim3(256), 0, st, rdfw, nrows, nwin, rm, skt);
          } else {
            build_sk();
          }
          SME_CHECK_LAUNCH();
        }
        if (!sk && !winp) {  // no valid term in the batch: an empty (all 'none') table row for k_query_bm
          int32_t *skw = W[60].as<int32_t>(T + 1);
          SME_HIP(hipMemsetAsync(skw, 0x7F, (size_t)(T + 1) * sizeof(int32_t), st));
          sk = skw;
        }
      }
    }
  }
  const int32_t *qord = nullptr;
  if (tiled && cx->opt_query_order) {
    // heaviest-term query order
    uint64_t *qk = W[46].as<uint64_t>(2 * (size_t)nq);
    int32_t *qi = W[45].as<int32_t>(2 * (size_t)nq);
    int tb = 1;
    while (tb < 32 && (1ll << tb) <= V) tb++;  // ids 0 .. V (V = no term)
    hipLaunchKernelGGL(k_query_keys, dim3(std::min((nq + 255) / 256, 4096)), dim3(256), 0, st, d_terms, d_qoff, nq, off,
                       V, tb, qk, qi);
    uint32_t *rscr = W[35].as<uint32_t>(kv_sort_scratch(nq) / sizeof(uint32_t) + 1);
    qord = reinterpret_cast<const int32_t *>(kv_sort<uint64_t>(qk, reinterpret_cast<uint32_t *>(qi), qk + nq,
                                                               reinterpret_cast<uint32_t *>(qi + nq), nq, 2 * tb, rscr,
                                                               st));
  }
  // events on the launch stream bracket the scoring kernel (bench.py roofline)
  hipEvent_t e0, e1, e2, e3;
  for (hipEvent_t *e : {&e0, &e1, &e2, &e3}) SME_HIP(hipEventCreate(e));
  SME_HIP(hipEventRecord(e0, st));
  unsigned long long *qstats = nullptr;
#ifdef SME_EXPERIMENTS
  const char *eq = getenv("SME_QSTATS");
  if (eq && atoi(eq)) {
    qstats = reinterpret_cast<unsigned long long *>(W[47].as<uint64_t>(8));
    SME_HIP(hipMemsetAsync(qstats, 0, 8 * sizeof(uint64_t), st));
  }
#endif
  QBmArgs qa{};
  if (tiled) {
    qa.off = off;
    qa.docno = dn;
    qa.tf = tf;
    qa.tf_o = (const int32_t *)ix->d_tf_o.p;
    qa.lut = lut;
    qa.idf = idf;
    qa.V = V;
    qa.row_of = row_of;
    qa.sk = sk;
    qa.qlut = qlut;
    qa.hrow_of = ix->q_H > 0 ? (const int32_t *)ix->d_hrow_of.p : nullptr;
    qa.tfrow = ix->q_tfrow;
    qa.bm16 = ix->q_bm16;
    qa.bm1k = ix->q_bm1k;
    qa.dmin = ix->dmin;
    qa.T = T;
    qa.terms = d_terms;
    qa.qoff = d_qoff;
    qa.qorder = qord;
    qa.nq = nq;
    qa.k = k;
    qa.nseed = (int)std::max<int64_t>(0, std::min<int64_t>(cx->opt_seed_tiles, kMaxSeed));
    qa.reftie = reftie;
    qa.out_d = d_out_docno;
    qa.out_s = d_out_score;
    qa.out_t = d_out_tie;
    qa.wmax_bits = (const unsigned long long *)wmax;
    qa.stats = qstats;
  }
  auto launch_bm = [&](const QBmArgs &x) {
    const unsigned wgrid = (unsigned)std::min<int64_t>(8 * (((int64_t)x.nq + 7) / 8), 1 << 30);
    if (k <= 64)
      hipLaunchKernelGGL(k_query_bm<128>, dim3(wgrid), dim3(64), 0, st, x);
    else if (k <= 192)
      hipLaunchKernelGGL(k_query_bm<256>, dim3(wgrid), dim3(64), 0, st, x);
    else
      hipLaunchKernelGGL(k_query_bm<512>, dim3(wgrid), dim3(64), 0, st, x);
  };
  const bool win = tiled && cx->opt_query_kernel == 0 && ix->q_spk;
  int64_t n_ovf = 0;
  bool subset_ran = false;  // the overflow fallback answered queries as nested compact batches
  QTimes sub_times;
  if (win) {
    // per-batch records: term descriptors (batch term order), position records (query order)
    // the batch's terms are d_terms[tbase, nterm): a sub-batch of a split keeps
    // absolute offsets, so descriptors cover only its own terms and every record
    // indexes them relative to tbase (QPos.q0, QSeedArgs.tbase)
    int64_t nterm = 0, tbase = 0;
    SME_HIP(hipMemcpyAsync(&nterm, d_qoff + nq, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(&tbase, d_qoff, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    const int64_t nbt = nterm - tbase;
    QDesc *qdesc = reinterpret_cast<QDesc *>(W[34].as<uint4>(2 * (size_t)std::max<int64_t>(nbt, 1)));
    QPos *qpos = reinterpret_cast<QPos *>(W[33].as<uint4>((size_t)nq));
    if (nbt > 0)
      hipLaunchKernelGGL(k_query_desc, dim3((unsigned)std::min<int64_t>((nbt + 255) / 256, 8192)), dim3(256), 0, st,
                         d_terms + tbase, nbt, V, off, idf, row_of, qa.hrow_of, qdesc);
    hipLaunchKernelGGL(k_query_pos, dim3((unsigned)std::min((nq + 255) / 256, 8192)), dim3(256), 0, st, qord, d_qoff,
                       nq, tbase, qpos);
    SME_CHECK_LAUNCH();
    SME_HIP(hipEventRecord(e0, st));
    // 1. seed thresholds
    double *th0 = W[41].as<double>(nq);
    uint64_t *thk = W[32].as<uint64_t>(nq);
    QSeedArgs sa;
    sa.desc = qdesc;
    sa.qoff = d_qoff;
    sa.docno_o = (const int32_t *)ix->d_docno_o.p;
    sa.tf_o = (const int32_t *)ix->d_tf_o.p;
    sa.lut = lut;
    sa.tfrow = ix->q_tfrow;
    sa.hstride = T << kQB;
    sa.dmin = ix->dmin;
    sa.tbase = tbase;
    sa.nq = nq;
    sa.k = k;
    sa.M = (int)std::min<int64_t>(std::max<int64_t>(cx->opt_seed_m, cx->opt_seed_m > 0 ? 2 * (int64_t)k : 0),
                                  kSeedSlots / 2);
    sa.th0 = th0;
    sa.thk = thk;
    hipLaunchKernelGGL(k_query_seed, dim3((unsigned)std::min(nq, 1 << 16)), dim3(64), 0, st, sa);
    SME_CHECK_LAUNCH();
    SME_HIP(hipEventRecord(e1, st));
    // 2. windows x query slices; 3. per-query selection.  Overflowed lists run
    // again with the raised threshold (at most kWinRounds rounds), the rest -> k_query_bm
    // candidate list per query: the option, at least 16 k for large k (deep
    // exact ties at the k-th score), at most kCandMax
    const int cap = (int)std::min<int64_t>(std::max<int64_t>(cx->opt_cand_cap, cx->opt_cand_cap >= 1024 ? 16 * (int64_t)k : 0),
                                           kCandMax);
    unsigned int *ccnt = W[42].as<unsigned int>(2 * (size_t)nq + 4);
    unsigned int *ndefer = ccnt + 2 * (size_t)nq + 2;  // count of `defer`
    double *cs = W[43].as<double>((size_t)nq * cap);
    uint64_t *ckk = W[61].as<uint64_t>((size_t)nq * cap);
    int32_t *ovf = W[62].as<int32_t>(3 * (size_t)nq + 4);
    int32_t *defer = ovf + 2 * (size_t)nq + 2;  // long lists of a raise / final pass

    unsigned int *novf = ccnt + nq, *oflag = ccnt + nq + 1;
    SME_HIP(hipMemsetAsync(ccnt, 0, (2 * (size_t)nq + 1) * sizeof(unsigned int), st));
    QWinArgs wa;
    wa.desc = qdesc;
    wa.qpos = qpos;
    wa.docno = dn;
    wa.tf = tf;
    wa.spk = ix->q_spk;
    wa.lut = lut;
    wa.max_tf = ix->max_tf;
    wa.skt = skt;
    wa.nrows = nrows_b;
    wa.qlut = qlut;
    wa.imp = ix->q_imp;
    wa.sbq = ix->q_sbq;
    wa.tfrow = ix->q_tfrow;
    wa.hstride = T << kQB;
    wa.dmin = ix->dmin;
    wa.T = T;
    wa.nwin = T >> 2;
    wa.reftie = reftie;
    wa.cap = cap;
    wa.alpha = ix->q_alpha;
    wa.th0 = th0;
    wa.thk = thk;
    uint32_t *gates = cx->q_gates.as<uint32_t>((size_t)nq);
    wa.gate = gates;
    wa.ccnt = ccnt;
    wa.cs = cs;
    wa.ck = ckk;
    wa.stats = qstats;
    wa.exper = 0;
#ifdef SME_EXPERIMENTS
    if (const char *qx = getenv("SME_QEXP")) wa.exper = atoi(qx);  // timing only: wrong results
#endif
    QFinalArgs fa{nullptr, nq, k, cap, ccnt, oflag, cs, ckk, d_out_docno, d_out_score, d_out_tie, th0, thk, ovf, novf};
    int n_round = nq;
    const int32_t *round_list = nullptr;
    // window lists: every 8th window (sample), the rest
    const int64_t nwin = wa.nwin;
    int32_t *wl = W[30].as<int32_t>(nwin + 1);
    // stages: the first two windows (under deep exact ties at the k-th score the
    // docno tie-break makes the docno prefix decisive) and every 2^L-th window,
    // then the windows 2^(L-1) mod 2^L, ..., then the odd ones -- 1/2^L, 1/2^L,
    // 1/2^(L-1), ..., 1/2 of the windows, each stage after a raise (and a
    // compaction) of every query's threshold and list.  Each stage doubles the
    // windows seen, so it appends about k documents over the raised threshold;
    // only the first one runs on the seed threshold, and L makes it small (about
    // 16 windows, 1/8 .. 1/256 of the index).
    // (auto: at least 16 windows, 8 from 1024 windows on -- a large index's first
    // stage on the seed threshold costs ~3.5x a last-stage window, and the extra raise
    // pass is cheap next to it: c5 (2,160 windows) -0.75 % per batch and 1,119 -> 72
    // overflowed lists, while c2's 245 windows lose 3 % to a ninth stage)
    const int64_t smin = cx->opt_win_stage_min > 0 ? cx->opt_win_stage_min : (nwin >= 1024 ? 8 : 16);
    int L = 3;
    while (L < 8 && (nwin >> (L + 1)) >= smin) L++;
    int64_t n_samp = 0, stage_start[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    {
      std::vector<int32_t> &h = cx->h_wlist;  // outlives the async copy
      h.assign((size_t)nwin, 0);
      auto stage_of = [L](int64_t xw) {
        if (xw < 2) return 0;
        const int t = __builtin_ctzll((unsigned long long)xw);
        return t >= L ? 0 : L - t;
      };
      for (int sg = 0; sg <= L; sg++) {
        stage_start[sg] = n_samp;
        for (int64_t xw = 0; xw < nwin; xw++)
          if (stage_of(xw) == sg) h[(size_t)n_samp++] = (int32_t)xw;
      }
      stage_start[L + 1] = n_samp;
      SME_HIP(hipMemcpyAsync(wl, h.data(), nwin * sizeof(int32_t), hipMemcpyHostToDevice, st));
    }
    auto launch_win = [&](const int32_t *wlist, int64_t nw) {
      wa.wlist = wlist;
      wa.nw = nw;
      const int64_t G = 8 * (int64_t)wa.nslices;
      const int64_t wg = ((nw + 7) / 8) * G;
      if (wg >= (int64_t(1) << 31)) throw Error(SME_ELIMIT, "query batch x windows too large for one launch");
      size_t dyn_lds = 0;
#ifdef SME_EXPERIMENTS
      // occupancy experiments: unused dynamic LDS per workgroup lowers the
      // workgroups per CU without changing the kernel's code
      if (const char *ql = getenv("SME_QLDS")) dyn_lds = (size_t)atoi(ql);
#endif
      if (wg > 0) {
        hipLaunchKernelGGL(k_gates, dim3((unsigned)std::min((nq + 255) / 256, 4096)), dim3(256), 0, st, th0, nq,
                           wa.alpha, gates);
        hipLaunchKernelGGL(k_query_win, dim3((unsigned)wg), dim3(kWNT), dyn_lds, st, wa);
      }
      SME_CHECK_LAUNCH();
    };
    for (int round = 0; round < kWinRounds && n_round > 0; round++) {
      if (round > 0) {
        hipLaunchKernelGGL(k_reset_cnt, dim3((unsigned)std::min((n_round + 255) / 256, 4096)), dim3(256), 0, st,
                           round_list, n_round, ccnt, oflag);
        hipLaunchKernelGGL(k_query_pos, dim3((unsigned)std::min((n_round + 255) / 256, 8192)), dim3(256), 0, st,
                           round_list, d_qoff, n_round, tbase, qpos);
      }
      wa.nq = n_round;
      // (auto: 128 queries per slice below 1024 windows -- c2's 245 windows: c3 kernel
      // 22.59 -> 22.34 ms, twice the workgroups per window --, 256 from 1024 on, where
      // the launch is large anyway and c5 does not gain)
      const int64_t qps = cx->opt_win_slice > 0 ? cx->opt_win_slice : (nwin >= 1024 ? 256 : 128);
      wa.nslices = (int)std::max<int64_t>(1, std::min<int64_t>(n_round / qps, 4096));
      if (round == 0 && cx->opt_win_sample && nwin >= 16) {
        for (int sg = 0; sg <= L; sg++) {
          if (sg > 0) {  // raise thresholds, keep each list's best k
            // lists of <= kRaiseSmall entries in a small-LDS pass (many workgroups per
            // CU), the longer ones deferred to the large-LDS instance
            SME_HIP(hipMemsetAsync(ndefer, 0, sizeof(unsigned int), st));
            const dim3 rg((unsigned)std::min(nq, 1 << 16));
            hipLaunchKernelGGL(k_query_raise<kRaiseSmall>, rg, dim3(64), 0, st, nq, k, cap, ccnt, oflag, cs, ckk, th0,
                               thk, nullptr, nullptr, defer, ndefer);
            if (cap <= 1024)
              hipLaunchKernelGGL(k_query_raise<1024>, rg, dim3(64), 0, st, nq, k, cap, ccnt, oflag, cs, ckk, th0, thk,
                                 defer, ndefer, nullptr, nullptr);
            else
              hipLaunchKernelGGL(k_query_raise<kCandMax>, rg, dim3(64), 0, st, nq, k, cap, ccnt, oflag, cs, ckk, th0,
                                 thk, defer, ndefer, nullptr, nullptr);
            SME_CHECK_LAUNCH();
          }
          launch_win(wl + stage_start[sg], stage_start[sg + 1] - stage_start[sg]);
        }
      } else {
        launch_win(nullptr, nwin);
      }
      if (round == 0) SME_HIP(hipEventRecord(e2, st));
      // overflow lists alternate between the two halves of `ovf`
      int32_t *out_list = ovf + (round & 1) * (nq + 1);
      SME_HIP(hipMemsetAsync(novf, 0, sizeof(unsigned int), st));
      fa.qlist = round_list;
      fa.n = n_round;
      fa.ovf = out_list;
      {
        SME_HIP(hipMemsetAsync(ndefer, 0, sizeof(unsigned int), st));
        QFinalArgs fb = fa;  // the deferred long lists
        fa.nlist = nullptr;
        fa.defer = defer;
        fa.ndefer = ndefer;
        fb.qlist = defer;
        fb.nlist = ndefer;
        fb.defer = nullptr;
        fb.ndefer = nullptr;
        const dim3 fg((unsigned)std::min(n_round, 1 << 16));
        hipLaunchKernelGGL(k_query_final<kRaiseSmall>, fg, dim3(64), 0, st, fa);
        if (cap <= 1024)
          hipLaunchKernelGGL(k_query_final<1024>, fg, dim3(64), 0, st, fb);
        else
          hipLaunchKernelGGL(k_query_final<kCandMax>, fg, dim3(64), 0, st, fb);
      }
      SME_CHECK_LAUNCH();
      unsigned int h_novf = 0;
      SME_HIP(hipMemcpyAsync(&h_novf, novf, sizeof h_novf, hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
      n_round = (int)h_novf;
      round_list = out_list;
      n_ovf += round == 0 ? n_round : 0;
      if (cap < k) break;  // no bound can be raised: every overflowed query to the fallback
    }
    if (n_round > 0) {  // still overflowing: the block-max sweep (on the tile skip table) if it fits
      size_t fr2 = 0, tot2 = 0;
      SME_HIP(hipMemGetInfo(&fr2, &tot2));
      const double tbudget = cx->opt_query_budget > 0 ? (double)cx->opt_query_budget
                                                      : (double)fr2 / 2.0 + (double)W[60].cap;
      if ((double)nrows_b * (double)(T + 1) * 4.0 <= tbudget || nq == 1) {
        if (build_sk) build_sk();
        QBmArgs ob = qa;
        ob.sk = sk;
        ob.qlut = qlut;
        ob.qorder = round_list;
        ob.nq = n_round;
        launch_bm(ob);
        SME_CHECK_LAUNCH();
      } else {
        // the list lives in this context's workspace, which the sub-batches reuse
        std::vector<int32_t> hl((size_t)n_round);
        SME_HIP(hipMemcpyAsync(hl.data(), round_list, n_round * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        SME_HIP(hipStreamSynchronize(st));
        // the nested calls store their own timings in the context: collected
        // here and added to this call's below (with the split flag)
        subset_ran = true;
        if (n_round < nq) {
          query_subset(ix, d_terms, d_qoff, nq, hl.data(), n_round, k, d_out_docno, d_out_score, d_out_tie, st, reftie);
          sub_times.add(cx);
        } else {  // every query of the batch: two compact halves (each recursion has fewer queries)
          const int h = n_round / 2;
          query_subset(ix, d_terms, d_qoff, nq, hl.data(), h, k, d_out_docno, d_out_score, d_out_tie, st, reftie);
          sub_times.add(cx);
          query_subset(ix, d_terms, d_qoff, nq, hl.data() + h, n_round - h, k, d_out_docno, d_out_score, d_out_tie,
                       st, reftie);
          sub_times.add(cx);
        }
      }
    }
    cx->last_query_fallback = n_round;
  } else if (tiled) {
    SME_HIP(hipEventRecord(e1, st));
    launch_bm(qa);
    SME_CHECK_LAUNCH();
    SME_HIP(hipEventRecord(e2, st));
  } else {
    // the longest query picks the kernel: the register lists take <= 128 terms,
    // the LDS list <= 1024
    if (h_mx == 0 && nq > 0) {
      hipLaunchKernelGGL(k_max_qlen, dim3(std::min((nq + 255) / 256, 1024)), dim3(256), 0, st, d_qoff, nq, err + 1);
      SME_HIP(hipMemcpyAsync(&h_mx, err + 1, sizeof(int), hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
    }
    if (h_mx > kMaxQTermsList) throw Error(SME_ELIMIT, "a query has more than 1024 terms");
    list_kernel = k > 32 || h_mx > kMaxQTerms;
    SME_HIP(hipEventRecord(e1, st));
    const unsigned grid = (unsigned)std::min(nq, 1 << 20);
    if (list_kernel)  // k > 32 or a query of more than 128 terms: the LDS candidate list
      hipLaunchKernelGGL((k_query<1, true>), dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, V,
                         d_terms, d_qoff, nq, k, d_out_docno, d_out_score, d_out_tie, reftie, err);
    else if (k <= 16)
      hipLaunchKernelGGL((k_query<16, false>), dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, V,
                         d_terms, d_qoff, nq, k, d_out_docno, d_out_score, d_out_tie, reftie, err);
    else
      hipLaunchKernelGGL((k_query<32, false>), dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, V,
                         d_terms, d_qoff, nq, k, d_out_docno, d_out_score, d_out_tie, reftie, err);
    SME_CHECK_LAUNCH();
    SME_HIP(hipEventRecord(e2, st));
  }
  SME_HIP(hipEventRecord(e3, st));
  int h_err = 0;
  SME_HIP(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  float ms = 0, pms = 0, sms = 0, fms = 0;
  SME_HIP(hipEventElapsedTime(&ms, e1, e2));
  SME_HIP(hipEventElapsedTime(&pms, ep, e0));
  SME_HIP(hipEventElapsedTime(&sms, e0, e1));
  SME_HIP(hipEventElapsedTime(&fms, e2, e3));
  cx->last_query_ms = ms;
  cx->last_query_prep_ms = pms;
  cx->last_query_seed_ms = sms;
  cx->last_query_final_ms = fms;
  cx->last_query_total_ms = sms + ms + fms;
  cx->last_query_overflow = n_ovf;
  cx->last_query_index_ms = tiled ? ix->q_prep_ms : 0.0f;
  cx->last_query_tiled = tiled;
  cx->last_query_name = win ? "k_query_win" : tiled ? "k_query_bm" : "k_query";
  cx->last_query_split = subset_ran;
  if (subset_ran) {  // the nested batches' kernel time (their events were not on this call's)
    cx->last_query_ms += sub_times.ms;
    cx->last_query_prep_ms += sub_times.prep;
    cx->last_query_seed_ms += sub_times.seed;
    cx->last_query_final_ms += sub_times.fin;
    cx->last_query_total_ms += sub_times.tot;
  }
  (void)hipEventDestroy(ep);
  for (hipEvent_t e : {e0, e1, e2, e3}) (void)hipEventDestroy(e);
  if (qstats) {
    uint64_t h[8];
    SME_HIP(hipMemcpy(h, qstats, sizeof h, hipMemcpyDeviceToHost));
    if (win)
      fprintf(stderr, "SME_QSTATS pairs=%llu sparse_postings=%llu subblocks_over_gate=%llu heavy_terms=%llu "
              "docs_over_gate=%llu kept=%llu\n", (unsigned long long)h[0], (unsigned long long)h[1],
              (unsigned long long)h[2], (unsigned long long)h[3], (unsigned long long)h[4], (unsigned long long)h[5]);
    else
      fprintf(stderr, "SME_QSTATS tiles=%llu blocks_gated=%llu candidates=%llu compactions=%llu\n",
              (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2], (unsigned long long)h[3]);
  }
  if (h_err) throw Error(SME_ELIMIT, list_kernel ? "a query has more than 1024 terms" : "a query has more than 128 terms");
}

static void query_subset(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, const int32_t *h_qlist,
                         int n, int k, int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie,
                         hipStream_t st, int tie_bits) {
  const std::vector<int32_t> ql(h_qlist, h_qlist + n);
  std::vector<int64_t> qo((size_t)nq + 1);
  SME_HIP(hipMemcpyAsync(qo.data(), d_qoff, (nq + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  const int64_t t0 = qo[0], nt = qo[nq] - t0;
  std::vector<int32_t> all((size_t)std::max<int64_t>(nt, 1));
  if (nt > 0) SME_HIP(hipMemcpy(all.data(), d_terms + t0, nt * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<int32_t> sterms;
  std::vector<int64_t> soff(1, 0);
  for (int i = 0; i < n; i++) {
    const int64_t q = ql[i];
    for (int64_t j = qo[q]; j < qo[q + 1]; j++) sterms.push_back(all[(size_t)(j - t0)]);
    soff.push_back((int64_t)sterms.size());
  }
  DevBuf b_terms, b_off, b_d, b_s, b_t, b_l;
  int32_t *dt = b_terms.as<int32_t>(std::max<size_t>(sterms.size(), 1));
  int64_t *doff = b_off.as<int64_t>(soff.size());
  int32_t *od = b_d.as<int32_t>((size_t)n * k);
  double *os = b_s.as<double>((size_t)n * k);
  uint32_t *ot = d_out_tie ? b_t.as<uint32_t>((size_t)n * k) : nullptr;
  int32_t *dl = b_l.as<int32_t>(n);
  if (!sterms.empty())
    SME_HIP(hipMemcpyAsync(dt, sterms.data(), sterms.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(doff, soff.data(), soff.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(dl, ql.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, st));
  query_topk(ix, dt, doff, n, k, od, os, ot, st, tie_bits);  // splits by itself until a subset's tables fit
  hipLaunchKernelGGL(k_scatter_rows, dim3((unsigned)std::min<int64_t>(((int64_t)n * k + 255) / 256, 4096)), dim3(256),
                     0, st, dl, n, k, od, os, ot, d_out_docno, d_out_score, d_out_tie);
  SME_CHECK_LAUNCH();
  SME_HIP(hipStreamSynchronize(st));  // the staging buffers are freed on return
}


// ---------------------------------------------------------------------------
// processContent on one string (query parsing), single lane
// ---------------------------------------------------------------------------
__global__ void k_tokenize_one(const uint8_t *b, int64_t n, uint16_t *units, uint16_t *work, int64_t work_cap,
                               uint16_t *out, int64_t out_cap, int64_t *offs, int cap_tok, int *ntok, int *err) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int64_t nu = 0;
  for (int64_t p = 0; p < n;) {
    uint16_t tmp[2];
    int k;
    int used = utf8_step(b, p, n, tmp, &k);
    for (int x = 0; x < k; x++) units[nu++] = tmp[x];
    p += used;
  }
  int cnt = 0;
  int64_t o = 0;
  offs[0] = 0;
  TagScan sc;
  sc.t = units;
  sc.n = (int)nu;
  Stemmer stm;
  sc.run([&](int u0, int u1) {
    normalize_raw(units + u0, u1 - u0, work, (int)work_cap, [&](const uint16_t *p, int l) {
      if (is_stopword(p, l)) return;
      for (int i = 0; i < l; i++) stm.b[i] = p[i];
      stm.len = l;
      stm.run();
      if (cnt >= cap_tok || o + stm.len > out_cap) {
        *err = 1;
        return;
      }
      for (int i = 0; i < stm.len; i++) out[o + i] = stm.b[i];
      o += stm.len;
      offs[++cnt] = o;
    });
  });
  *ntok = cnt;
}

void tokenize_string(sme_ctx *cx, const uint8_t *h_utf8, size_t n, std::vector<std::vector<uint16_t>> &out,
                     hipStream_t st) {
  auto &W = cx->ws;
  const int64_t cap_tok = (int64_t)n + 4;
  uint8_t *d_b = W[48].as<uint8_t>(n + 1);
  uint16_t *units = W[49].as<uint16_t>(n + 4);
  uint16_t *work = W[50].as<uint16_t>(4 * n + 64);
  uint16_t *tokbuf = W[51].as<uint16_t>(2 * n + 16);
  int64_t *offs = W[52].as<int64_t>(cap_tok + 1);
  int *cnt = W[53].as<int>(4);
  if (n) SME_HIP(hipMemcpyAsync(d_b, h_utf8, n, hipMemcpyHostToDevice, st));
  SME_HIP(hipMemsetAsync(cnt, 0, 4 * sizeof(int), st));
  hipLaunchKernelGGL(k_tokenize_one, dim3(1), dim3(64), 0, st, d_b, (int64_t)n, units, work, (int64_t)(4 * n + 64),
                     tokbuf, (int64_t)(2 * n + 16), offs, (int)cap_tok, cnt, cnt + 1);
  SME_CHECK_LAUNCH();
  int h[2];
  SME_HIP(hipMemcpyAsync(h, cnt, sizeof h, hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  if (h[1]) throw Error(SME_ELIMIT, "tokenize output capacity");
  std::vector<int64_t> ho(h[0] + 1);
  SME_HIP(hipMemcpy(ho.data(), offs, ho.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
  std::vector<uint16_t> hb(ho.back());
  if (!hb.empty()) SME_HIP(hipMemcpy(hb.data(), tokbuf, hb.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
  out.clear();
  for (int i = 0; i < h[0]; i++) out.emplace_back(hb.begin() + ho[i], hb.begin() + ho[i + 1]);
}

// ---------------------------------------------------------------------------
// term lookup: binary search over the rank-ordered vocabulary
// ---------------------------------------------------------------------------
__global__ void k_lookup(const int64_t *toff, const uint16_t *tchars, int64_t V, const int64_t *qo,
                         const uint16_t *qc, int n, int32_t *ids) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint16_t *a = qc + qo[i];
    const int64_t al = qo[i + 1] - qo[i];
    int64_t lo = 0, hi = V - 1, res = -1;
    while (lo <= hi) {
      int64_t mid = (lo + hi) >> 1;
      const uint16_t *b = tchars + toff[mid];
      int64_t bl = toff[mid + 1] - toff[mid], m = al < bl ? al : bl;
      int c = 0;
      for (int64_t x = 0; x < m && c == 0; x++) c = (int)b[x] - (int)a[x];
      if (c == 0) c = (int)(bl - al);
      if (c == 0) {
        res = mid;
        break;
      }
      if (c < 0)
        lo = mid + 1;
      else
        hi = mid - 1;
    }
    ids[i] = (int32_t)res;
  }
}

// K > 1: the forward index is keyed by k_gram[0] and its Hashtable keeps the
// LAST k-gram (TermDF order) with that first element (IntDocVectorsForwardIndex
// .java:107-120, T11): the last gram whose first component is the term id.
__global__ void k_gram_last(const int32_t *gram, int64_t V, int K, int n, int32_t *ids) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int32_t t = ids[i];
    if (t < 0) continue;
    int64_t lo = 0, hi = V;  // first gram with first component > t
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (gram[m * K] <= t)
        lo = m + 1;
      else
        hi = m;
    }
    ids[i] = (lo > 0 && gram[(lo - 1) * K] == t) ? (int32_t)(lo - 1) : -1;
  }
}

// 128-bit fingerprints of every index term's string (K = 1) or k-gram (the
// component terms' fingerprints chained): two independent 64-bit mixes of the
// UTF-16 units, for the multi-GPU df exchange (dist.py: equal terms on two
// shards get equal fingerprints without sorting strings on the host).
__device__ __forceinline__ void fp_string(const uint16_t *c, int64_t n, uint64_t &a, uint64_t &b) {
  a = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  b = 0xC2B2AE3D27D4EB4Full + (uint64_t)n * 0x165667B19E3779F9ull;
  for (int64_t i = 0; i < n; i++) {
    a = fmix64(a ^ ((uint64_t)c[i] + 0x100));
    b = (b ^ (uint64_t)c[i]) * 0x100000001B3ull + 0x9E3779B97F4A7C15ull;
  }
  b = fmix64(b);
}
__global__ void k_term_fp(const int64_t *toff, const uint16_t *tch, const int32_t *gram, int K, int64_t V,
                          uint64_t *out) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    uint64_t a = 0, b = 0;
    if (K == 1) {
      fp_string(tch + toff[t], toff[t + 1] - toff[t], a, b);
    } else {
      a = 0x243F6A8885A308D3ull;
      b = 0x13198A2E03707344ull;
      for (int g = 0; g < K; g++) {
        const int32_t c = gram[t * K + g];
        uint64_t x, y;
        fp_string(tch + toff[c], toff[c + 1] - toff[c], x, y);
        a = fmix64(a ^ x) + (uint64_t)g;
        b = fmix64(b + y) ^ (uint64_t)g;
      }
    }
    out[2 * t] = a;
    out[2 * t + 1] = b;
  }
}
void term_fingerprints(sme_index *ix, uint64_t *d_out, hipStream_t st) {
  if (ix->V <= 0) return;
  hipLaunchKernelGGL(k_term_fp, dim3((unsigned)std::min<int64_t>((ix->V + 255) / 256, 65536)), dim3(256), 0, st,
                     (const int64_t *)ix->d_term_off.p, (const uint16_t *)ix->d_term_chars.p,
                     ix->K > 1 ? (const int32_t *)ix->d_gram.p : nullptr, ix->K, ix->V, d_out);
  SME_CHECK_LAUNCH();
}

void lookup_terms(sme_index *ix, const std::vector<std::vector<uint16_t>> &terms, int32_t *ids, hipStream_t st) {
  const int n = (int)terms.size();
  if (n == 0) return;
  std::vector<int64_t> qo(n + 1, 0);
  for (int i = 0; i < n; i++) qo[i + 1] = qo[i] + (int64_t)terms[i].size();
  std::vector<uint16_t> qc(qo[n] + 1);
  for (int i = 0; i < n; i++) std::copy(terms[i].begin(), terms[i].end(), qc.begin() + qo[i]);
  auto &W = ix->ctx->ws;
  int64_t *d_qo = W[54].as<int64_t>(n + 1);
  uint16_t *d_qc = W[48].as<uint16_t>(qc.size());
  int32_t *d_ids = W[49].as<int32_t>(n);
  SME_HIP(hipMemcpyAsync(d_qo, qo.data(), qo.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_qc, qc.data(), qc.size() * sizeof(uint16_t), hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_lookup, dim3((n + 255) / 256), dim3(256), 0, st, (const int64_t *)ix->d_term_off.p,
                     (const uint16_t *)ix->d_term_chars.p, ix->Vt, d_qo, d_qc, n, d_ids);
  if (ix->K > 1)
    hipLaunchKernelGGL(k_gram_last, dim3((n + 255) / 256), dim3(256), 0, st, (const int32_t *)ix->d_gram.p, ix->V,
                       ix->K, n, d_ids);
  SME_CHECK_LAUNCH();
  SME_HIP(hipMemcpyAsync(ids, d_ids, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
}

}  // namespace sme
