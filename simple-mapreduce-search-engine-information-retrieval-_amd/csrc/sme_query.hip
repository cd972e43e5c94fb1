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
// per query with fp64 LDS accumulators over 4096-document tiles, k <= 32),
// which takes batches holding a longer query.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sme_internal.hpp"
#include "sme_text.hpp"

namespace sme {

constexpr int kQNT = 256;
constexpr int kTile = 4096;
constexpr int kQPer = 4;  // postings per lane per step
constexpr int kMaxQTerms = 128;
constexpr int kLutLds = 256;  // 1 + ln(tf) for tf < 256 from LDS, the rare rest from HBM

__device__ __forceinline__ bool better(double as, int32_t ad, double bs, int32_t bd) {
  return as > bs || (as == bs && ad < bd);
}

// insert (s, d) into the descending register list ts/td (fully unrolled: no
// dynamic register indexing)
template <int K>
__device__ __forceinline__ void topk_insert(double (&ts)[K], int32_t (&td)[K], double s, int32_t d) {
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
__device__ __forceinline__ void emit_topk(double (&ts)[KMAX], int32_t (&td)[KMAX], int k, int q, int32_t *out_d,
                                          double *out_s, double *red_s, int32_t *red_d, int32_t *red_t) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int r = 0; r < k; r++) {
    double bs = ts[0];
    int32_t bd = td[0];
    int32_t bt = tid;
    for (int o = 32; o > 0; o >>= 1) {
      double os = __shfl_xor(bs, o, 64);
      int32_t od = __shfl_xor(bd, o, 64), ot = __shfl_xor(bt, o, 64);
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
      td[KMAX - 1] = 0x7FFFFFFF;
    }
    if (tid == 0) {
      const bool valid = bs != -INFINITY;
      out_d[(int64_t)q * k + r] = valid ? bd : -1;
      out_s[(int64_t)q * k + r] = valid ? bs : 0.0;
    }
    __syncthreads();
  }
}

template <int KMAX>
__global__ __launch_bounds__(kQNT) void k_query(const int64_t *__restrict__ off, const int32_t *__restrict__ docno,
                                                const int32_t *__restrict__ tf, const double *__restrict__ lut,
                                                int max_tf, const double *__restrict__ idf, int64_t V,
                                                const int32_t *__restrict__ terms, const int64_t *__restrict__ qoff,
                                                int nq, int k, int32_t *out_d, double *out_s, int *err) {
  __shared__ double acc[kTile];
  __shared__ double s_lut[kLutLds];
  __shared__ int64_t cur[kMaxQTerms], endp[kMaxQTerms];
  __shared__ double tidf[kMaxQTerms];
  __shared__ int32_t s_next;
  __shared__ unsigned long long s_stop;
  __shared__ double red_s[kQNT / 64];
  __shared__ int32_t red_d[kQNT / 64], red_t[kQNT / 64];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (int j = tid; j < kTile; j += kQNT) acc[j] = -1.0;  // untouched (weights are >= 0)
  for (int j = tid; j < kLutLds; j += kQNT) s_lut[j] = j <= max_tf ? lut[j] : 0.0;
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int64_t q0 = qoff[q];
    int nt = (int)(qoff[q + 1] - q0);
    if (nt > kMaxQTerms) {
      if (tid == 0) atomicOr(err, 1);
      nt = kMaxQTerms;
    }
    if (tid == 0) s_next = 0x7FFFFFFF;
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
    int32_t td[KMAX];
#pragma unroll
    for (int j = 0; j < KMAX; j++) {
      ts[j] = -INFINITY;
      td[j] = 0x7FFFFFFF;
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
      for (int j = tid; j < kTile; j += kQNT) {
        const double sc = acc[j];
        if (sc < 0.0) continue;
        acc[j] = -1.0;
        topk_insert<KMAX>(ts, td, sc, lo + j);
      }
      __syncthreads();
    }
    emit_topk<KMAX>(ts, td, k, q, out_d, out_s, red_s, red_d, red_t);
  }
}



// ---------------------------------------------------------------------------
// Tiled, impact-gated scoring (default path).
//
// The docno axis is cut into tiles of kWTile documents from the index's
// smallest docno.  Per batch: a skip table gives, for every DISTINCT batch term
// and every tile, the term's first posting in the tile; terms covering >= 1/div
// of the docno span (the Zipf head) also get two dense byte rows, the tf of
// every document and its IMPACT q = floor(w * alpha) + 1 (w = lut[tf] * idf, the
// exact fp64 weight; 0 where absent), alpha = 253.5 / (largest weight of any
// batch term), so q <= 255 and q >= 1 exactly where the term occurs.
//
// One wave per query sweeps the tiles.  Per tile it sums the impacts of its
// terms into packed u16 lanes (A(d) = sum_j q_j(d) is an integer, order-free:
// dense terms by two byte permutes + adds per dword of four documents, posting
// terms by LDS atomic adds).  Since q_j > w_j * alpha, A(d) > alpha * R(d) where
// R is the real sum of d's weights, so a document whose fp64 score S(d) can
// reach the current k-th best score th has A(d) >= gate = floor(alpha * th *
// (1 - 2^-40)) (the factor absorbs every rounding).  Only
// those candidates are scored exactly: S(d) = the left-to-right fp64 sum of
// lut[tf] * idf over the query's terms in token order (tf from the dense tf row
// or a binary search of the tile's postings), bit-identical to the reference's
// `score += (1 + Math.log(tf)) * idf` (IntDocVectorsForwardIndex.java:197-213).
// Candidates that beat th go to a per-wave LDS buffer of C entries; when it
// fills, a bitonic sort (score desc, docno asc) keeps the best k and raises th.
// ---------------------------------------------------------------------------
#ifndef SME_QTB
#define SME_QTB 10
#endif
constexpr int kWBits = SME_QTB;     // tile = 2^kWBits documents
constexpr int kWTile = 1 << kWBits;
constexpr int kDPL = kWTile / 64;   // documents per lane in a tile (16 at 1024)
constexpr int kIMaxTerms = 64;      // lane j holds query term j
constexpr int kWLut = 256;          // 1 + ln(tf) for tf < 256 from LDS
constexpr int kTfRows = 4;          // LDS tf rows per tile (terms beyond: dense row bytes / binary search)
static_assert(kDPL % 16 == 0 && kDPL <= 32, "tile must be 1024 or 2048 documents");

__device__ __forceinline__ uint32_t impact(double l, double widf, double alpha) {
  return (uint32_t)floor(__dmul_rn(__dmul_rn(l, widf), alpha)) + 1u;
}
__device__ __forceinline__ double rld(double v, int l) { return __longlong_as_double(rl64(__double_as_longlong(v), l)); }
__device__ __forceinline__ uint32_t pkmax_u16(uint32_t a, uint32_t b) {
  const uint32_t lo = max(a & 0xFFFFu, b & 0xFFFFu), hi = max(a >> 16, b >> 16);
  return lo | (hi << 16);
}
__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

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
constexpr int kSkipChunk = 2048;  // postings per block in k_skip_fill
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
      const int64_t j = ((int64_t)docno[b + i] - dmin) >> kWBits;
      const int64_t jp = i == 0 ? -1 : (((int64_t)docno[b + i - 1] - dmin) >> kWBits);
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
// rows with df = 0 (possible only for empty terms) never get a posting: all zeros
__global__ void k_skip_zero_rows(const int64_t *rdf, int64_t nrows, int64_t T, int32_t *sk) {
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x)
    if (rdf[r] == 0)
      for (int64_t j = threadIdx.x; j <= T; j += blockDim.x) sk[r * (T + 1) + j] = 0;
}

// Per batch row: the largest weight of the term (its max tf is the first
// posting of the reduce-order CSR, tf desc) folded into wmax (non-negative
// doubles order like their bit patterns), and whether the term gets dense rows:
// postings covering >= 1/div of the docno span, every tf <= 255.  A row costs
// span bytes against >= 8 B x span / div of (docno, tf) postings.
__global__ void k_row_stats(const int32_t *term_of_row, const int64_t *rdf, int64_t nrows, const int64_t *off,
                            const int32_t *tf_o, const double *lut, const double *idf, int64_t span, int64_t div,
                            int32_t *flag, unsigned long long *wmax_bits) {
  unsigned long long wm = 0;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows + 1; r += (int64_t)gridDim.x * blockDim.x) {
    int32_t fl = 0;
    if (r < nrows && rdf[r] > 0) {
      const int32_t t = term_of_row[r];
      const int32_t mt = tf_o[off[t]];
      const unsigned long long wb = (unsigned long long)__double_as_longlong(__dmul_rn(lut[mt], idf[t]));
      wm = wb > wm ? wb : wm;
      fl = (div > 0 && rdf[r] * div >= span && mt <= 255) ? 1 : 0;
    }
    flag[r] = fl;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long u = __shfl_xor(wm, o, 64);
    wm = u > wm ? u : wm;
  }
  if ((threadIdx.x & 63) == 0 && wm) atomicMax(wmax_bits, wm);
}
__global__ void k_dense_rows(const int32_t *flag, const int32_t *scan, int64_t nrows, int64_t cap, int32_t *drow) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x)
    drow[r] = (flag[r] && scan[r] < cap) ? scan[r] : -1;
}
// Within a tile a dense row is stored lane-major: byte kDPL * l + b holds
// document 64 b + l, so lane l's kDPL-byte load carries the documents it owns.
__device__ __forceinline__ int64_t dense_pos(int64_t x) {
  const int64_t r = x & (kWTile - 1);
  return (x - r) + kDPL * (r & 63) + (r >> 6);
}
// tf and impact bytes at docno - dmin for every posting of a dense row, over the
// batch rows' postings as one flat list (chunks of kSkipChunk, like k_skip_fill)
// so a head term's million postings spread over the whole chip
__global__ __launch_bounds__(256) void k_dense_fill(const int64_t *rpre, int64_t nrows, const int32_t *drow,
                                                    const int32_t *term_of_row, const int64_t *off,
                                                    const int32_t *docno, const int32_t *tf, const double *lut,
                                                    const double *idf, const unsigned long long *wmax_bits,
                                                    int64_t dmin, int64_t stride, uint8_t *dtf, uint8_t *dq) {
  const double wmax = __longlong_as_double((long long)*wmax_bits);
  const double alpha = wmax > 0.0 ? 253.5 / wmax : 1.0;
  const int64_t total = rpre[nrows];
  for (int64_t x0 = (int64_t)blockIdx.x * kSkipChunk; x0 < total; x0 += (int64_t)gridDim.x * kSkipChunk) {
    const int64_t x1 = x0 + kSkipChunk < total ? x0 + kSkipChunk : total;
    int64_t lo = 0, hi = nrows;  // row of x0
    while (hi - lo > 1) {
      const int64_t m = (lo + hi) >> 1;
      if (rpre[m] <= x0) lo = m;
      else hi = m;
    }
    int64_t row = lo, rb = rpre[row], re = rpre[row + 1];
    for (int64_t x = x0 + threadIdx.x; x < x1; x += blockDim.x) {
      while (x >= re) {
        row++;
        rb = re;
        re = rpre[row + 1];
      }
      const int32_t d = drow[row];
      if (d < 0) continue;
      const int32_t t = term_of_row[row];
      const int64_t p = off[t] + (x - rb);
      const int32_t f = tf[p];  // <= 255 (k_row_stats)
      const int64_t pos = (int64_t)d * stride + dense_pos((int64_t)docno[p] - dmin);
      dtf[pos] = (uint8_t)f;
      dq[pos] = (uint8_t)impact(lut[f], idf[t], alpha);
    }
  }
}

// Query order for cache sharing: queries sorted by their heaviest term (largest
// df, then smaller id) and second heaviest, so concurrent waves on one XCD read
// the same rows / posting ranges.
__global__ void k_query_keys(const int32_t *terms, const int64_t *qoff, int nq, const int64_t *off, int64_t V,
                             uint64_t *keys, int32_t *idx) {
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
    keys[q] = ((uint64_t)t1 << 32) | t2;
    idx[q] = q;
  }
}

// Bitonic sort of n (power of two) entries of one wave's LDS buffer, best
// first (score desc, docno asc).  The workgroup is one wave, so the barriers
// only order the LDS traffic.
__device__ __forceinline__ void wave_sort(double *s, int32_t *d, int n) {
  const int lane = threadIdx.x;
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (n >> 1); i += 64) {
        const int lo = ((i & ~(stride - 1)) << 1) | (i & (stride - 1)), hi = lo + stride;
        const double as = s[lo], bs = s[hi];
        const int32_t ad = d[lo], bd = d[hi];
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

template <int C>
__global__ __launch_bounds__(64) void k_query_imp(
    const int64_t *__restrict__ off, const int32_t *__restrict__ docno, const int32_t *__restrict__ tf,
    const double *__restrict__ lut, int max_tf, const double *__restrict__ idf, int64_t V,
    const int32_t *__restrict__ row_of, const int32_t *__restrict__ sk, int64_t dmin, int64_t T,
    const int32_t *__restrict__ terms, const int64_t *__restrict__ qoff, const int32_t *__restrict__ qorder, int nq,
    int k, int32_t *out_d, double *out_s, const uint8_t *__restrict__ dtf, const uint8_t *__restrict__ dq,
    const int32_t *__restrict__ drow, int64_t dstride, const unsigned long long *__restrict__ wmax_bits, int sh,
    unsigned long long *stats, int exper) {
  __shared__ uint32_t lacc[kDPL / 2 * 64];  // posting terms' impact sums, u16 pairs (documents 128 m + l, + 64)
  __shared__ double bs[C];
  __shared__ int32_t bd[C];
  __shared__ double s_lut[kWLut];
  // tf bytes of the tile for the first kTfRows query terms with postings in it
  // (lane-major like the dense rows), read when candidates are scored exactly
  __shared__ uint8_t trow[kTfRows * kWTile];
  __shared__ uint32_t s_big;  // slots whose term has a tf > 255 in the tile
  const int lane = threadIdx.x;
  for (int j = lane; j < kWLut; j += 64) s_lut[j] = (j >= 1 && j <= max_tf) ? lut[j] : 0.0;
  const double wmax = __longlong_as_double((long long)*wmax_bits);
  // dense impacts are bytes at scale alpha; posting terms' impacts and the
  // gate use alpha * 2^sh (the dense sums are shifted by sh before the gate)
  const double alpha = wmax > 0.0 ? 253.5 / wmax : 1.0;
  const double alpha_s = __dmul_rn(alpha, (double)(1 << sh));
  __syncthreads();
  // queries in `qorder` (heaviest terms first) are dealt in 8 contiguous slices,
  // slice x to the blocks b with b % 8 == x, which share an XCD and its L2
  const int slice = (nq + 7) >> 3;
  for (int qi = blockIdx.x; qi < 8 * slice; qi += gridDim.x) {
    const int pos = (qi & 7) * slice + (qi >> 3);
    if (pos >= nq) continue;
    const int q = qorder ? qorder[pos] : pos;
    const int64_t q0 = qoff[q];
    const int nt = (int)(qoff[q + 1] - q0);  // <= kIMaxTerms (host checked)
    // lane j < nt holds term j: postings base, df, idf, skip row, dense rows
    int64_t mb = 0;
    int32_t mdf = 0;
    double midf = 0.0;
    const int32_t *mrow = sk;
    int32_t nx = 0x7FFFFFFF;
    int64_t mdr = -1;
    if (lane < nt) {
      const int32_t t = terms[q0 + lane];
      if (t >= 0 && t < V) {  // unknown (-1) and out-of-range ids are skipped
        mb = off[t];
        mdf = (int32_t)(off[t + 1] - mb);
        midf = idf[t];
        mrow = sk + (int64_t)row_of[t] * (T + 1);
        if (mdf > 0) {
          nx = (int32_t)(((int64_t)docno[mb] - dmin) >> kWBits);
          if (drow != nullptr) mdr = drow[row_of[t]];
        }
      }
    }
    const bool isd = mdr >= 0;
    const uint64_t dmask = (uint64_t)__ballot(isd);
    const int64_t mro = isd ? mdr * dstride : 0;  // this lane's dense row offset (impact / tf rows)
    int cnt = 0;  // buffer fill (wave-uniform)
    uint32_t st_tiles = 0, st_gated = 0, st_cand = 0, st_comp = 0, st_sparse = 0;  // SME_QSTATS
    bool th_ok = false;
    double th_s = 0.0;
    int32_t th_d = 0;
    uint32_t gate = 1;  // touched documents only until k of them are held
    // sort the buffer, keep the best k, raise th and the gate
    auto compact = [&]() {
      st_comp++;
      int n2 = 2;
      while (n2 < cnt) n2 <<= 1;
      for (int i = cnt + lane; i < n2; i += 64) {
        bs[i] = -INFINITY;
        bd[i] = 0x7FFFFFFF;
      }
      __syncthreads();
      wave_sort(bs, bd, n2);
      cnt = min(cnt, k);
      if (cnt >= k) {
        th_ok = true;
        th_s = bs[k - 1];
        th_d = bd[k - 1];
        const double g = floor(__dmul_rn(__dmul_rn(th_s, alpha_s), 1.0 - 0x1p-40));
        gate = g > 1.0 ? (uint32_t)g : 1u;
      }
    };
    int32_t tile = nx;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tile = min(tile, __shfl_xor(tile, o, 64));
    int32_t mc = 0, me = 0;
    if (tile != 0x7FFFFFFF && lane < nt && mdf > 0) {
      mc = mrow[tile];
      me = mrow[tile + 1];
    }
    while (tile != 0x7FFFFFFF) {  // wave-uniform
      // loads for the next step overlap this tile's work: the next tile of this
      // term, and (for the common case that it is tile + 1) its range end
      nx = 0x7FFFFFFF;
      int32_t me1 = 0;
      if (lane < nt && me < mdf) {
        nx = (int32_t)(((int64_t)docno[mb + me] - dmin) >> kWBits);
        me1 = tile + 2 <= T ? mrow[tile + 2] : mdf;
      } else if (lane < nt) {
        me1 = mdf;
      }
      const int64_t dbase = dmin + ((int64_t)tile << kWBits);
      const int64_t tbyte = (int64_t)tile << kWBits;
      const uint64_t amask = (uint64_t)__ballot(lane < nt && me > mc);  // terms with postings in the tile
      const uint64_t dm = amask & dmask, sm = amask & ~dmask;
      uint64_t rmask = amask;  // the first kTfRows terms of amask own an LDS tf row (slot = rank in amask)
#pragma unroll
      for (int x = 0; x < kTfRows; x++) rmask &= rmask - 1;
      rmask = amask & ~rmask;
      const int64_t plo = mb + mc, phi = mb + me;  // this lane's term: postings in the tile
      uint32_t a[kDPL / 2];
      st_tiles++;
      // dense terms: kDPL impact bytes per lane, four terms' loads in flight;
      // the first four are issued before the posting pass so both overlap
      uint64_t dmr = dm;
      auto dense_load = [&](uint4 (&v)[4][kDPL / 16]) {
#pragma unroll
        for (int g = 0; g < 4; g++) {
          if (dmr) {
            const int j = (int)__builtin_ctzll(dmr);
            dmr &= dmr - 1;
            const uint8_t *pj = dq + rl64(mro, j) + tbyte + kDPL * lane;
#pragma unroll
            for (int c = 0; c < kDPL / 16; c++) v[g][c] = *reinterpret_cast<const uint4 *>(pj + 16 * c);
          } else {
#pragma unroll
            for (int c = 0; c < kDPL / 16; c++) v[g][c] = make_uint4(0, 0, 0, 0);
          }
        }
      };
      auto dense_add = [&](const uint4 (&v)[4][kDPL / 16]) {
#pragma unroll
        for (int g = 0; g < 4; g++)
#pragma unroll
          for (int c = 0; c < kDPL / 16; c++) {
            const uint32_t w4[4] = {v[g][c].x, v[g][c].y, v[g][c].z, v[g][c].w};
#pragma unroll
            for (int u = 0; u < 4; u++) {
              a[8 * c + 2 * u] += __builtin_amdgcn_perm(0u, w4[u], 0x0C010C00u);
              a[8 * c + 2 * u + 1] += __builtin_amdgcn_perm(0u, w4[u], 0x0C030C02u);
            }
          }
      };
      uint4 v0[4][kDPL / 16];
      dense_load(v0);
      if (sm && !(exper & 2)) {
        st_sparse++;
        // posting terms: impacts added into LDS (order-free integer sums)
#pragma unroll
        for (int m = 0; m < kDPL / 2; m++) lacc[m * 64 + lane] = 0;
        {
          int sl = 0;
          for (uint64_t m = rmask; m; m &= m - 1, sl++)
            if ((sm >> __builtin_ctzll(m)) & 1)
#pragma unroll
              for (int c = 0; c < kDPL / 16; c++)
                *reinterpret_cast<uint4 *>(trow + (sl << kWBits) + kDPL * lane + 16 * c) = make_uint4(0, 0, 0, 0);
        }
        if (lane == 0) s_big = 0;
        __syncthreads();
        // the tile's postings of all posting terms as one list, 256 per step:
        // entry x belongs to the last term j of sm with pre_j <= x
        const int32_t cj = ((sm >> lane) & 1) ? me - mc : 0;
        const int32_t incl = wave_incl_sum(cj), prej = incl - cj;
        const int32_t total = __shfl(incl, 63, 64);
        for (int32_t x0 = 0; x0 < total; x0 += 256) {
          const int nu = min(4, (total - x0 + 63) >> 6);  // 64-entry chunks in this step (wave-uniform)
          int32_t dv[4], fv[4], sv[4];
          double wv[4];
#pragma unroll
          for (int u = 0; u < 4; u++) {
            dv[u] = 0;
            fv[u] = 0;
            wv[u] = 0.0;
            sv[u] = kTfRows;
            if (u < nu) {
              const int32_t x = x0 + 64 * u + lane;
              int64_t pb = 0;
              double wj = 0.0;
              int sj = kTfRows;
              for (uint64_t m = sm; m; m &= m - 1) {
                const int j = (int)__builtin_ctzll(m);
                const int32_t pj = __builtin_amdgcn_readlane(prej, j);
                if (x >= pj) {
                  pb = rl64(plo, j) - pj;
                  wj = rld(midf, j);
                  sj = ((rmask >> j) & 1) ? __popcll(amask & ((1ull << j) - 1)) : kTfRows;
                }
              }
              if (x < total) {
                dv[u] = docno[pb + x];
                fv[u] = tf[pb + x];
              }
              wv[u] = wj;
              sv[u] = sj;
            }
          }
#pragma unroll
          for (int u = 0; u < 4; u++) {
            if (fv[u] == 0) continue;
            const int r = (int)((int64_t)dv[u] - dbase);
            if (sv[u] < kTfRows) {
              trow[(sv[u] << kWBits) + kDPL * (r & 63) + (r >> 6)] = (uint8_t)(fv[u] > 255 ? 0 : fv[u]);
              if (fv[u] > 255) atomicOr(&s_big, 1u << sv[u]);
            }
            const double l = fv[u] < kWLut ? s_lut[fv[u]] : lut[fv[u]];
            atomicAdd(&lacc[((r >> 7) << 6) | (r & 63)], impact(l, wv[u], alpha_s) << (((r >> 6) & 1) << 4));
          }
        }
        __syncthreads();
      }
#pragma unroll
      for (int m = 0; m < kDPL / 2; m++) a[m] = 0;
      dense_add(v0);
      while (dmr) {
        uint4 v[4][kDPL / 16];
        dense_load(v);
        dense_add(v);
      }
      // A = (dense sums << sh) + posting-term sums: u16 fields never carry
      // (host: 255 * 2^sh * terms <= 65535)
#pragma unroll
      for (int m = 0; m < kDPL / 2; m++) a[m] = (a[m] << sh) + (sm && !(exper & 2) ? lacc[m * 64 + lane] : 0u);
      // gate: most tiles hold no document whose impact sum reaches it
      uint32_t mx = a[0];
#pragma unroll
      for (int m = 1; m < kDPL / 2; m++) mx = pkmax_u16(mx, a[m]);
      if (!(exper & 1) && __ballot(max(mx & 0xFFFFu, mx >> 16) >= gate) != 0) {
        uint32_t cm = 0;
#pragma unroll
        for (int b = 0; b < kDPL; b++)
          if (((a[b >> 1] >> ((b & 1) << 4)) & 0xFFFFu) >= gate) cm |= 1u << b;
        st_gated++;
        if (stats) st_cand += (uint32_t)__popc(cm);
        // dense terms that own a tf row: copy the tile's tf bytes
        {
          int sl = 0;
          for (uint64_t m = rmask; m; m &= m - 1, sl++) {
            const int j = (int)__builtin_ctzll(m);
            if (!((dmask >> j) & 1)) continue;
            const uint8_t *pj = dtf + rl64(mro, j) + tbyte + kDPL * lane;
#pragma unroll
            for (int c = 0; c < kDPL / 16; c++)
              *reinterpret_cast<uint4 *>(trow + (sl << kWBits) + kDPL * lane + 16 * c) =
                  *reinterpret_cast<const uint4 *>(pj + 16 * c);
          }
        }
        __syncthreads();
        const uint32_t bigs = sm ? s_big : 0u;
        for (;;) {
          const bool have = cm != 0;
          if (__ballot(have) == 0) break;  // wave-uniform
          double S = 0.0;
          int32_t d = 0x7FFFFFFF;
          bool keep = false;
          if (have) {
            const int b = (int)__builtin_ctz(cm);
            cm &= cm - 1;
            d = (int32_t)(dbase + ((b << 6) | lane));
            // exact score: query-token order, fp64, as rank() accumulates it
            int sl = 0;
            for (uint64_t m = amask; m; m &= m - 1, sl++) {
              const int j = (int)__builtin_ctzll(m);
              int f = 0;
              if (sl < kTfRows && !((bigs >> sl) & 1)) {
                f = trow[(sl << kWBits) + kDPL * lane + b];
              } else if ((dmask >> j) & 1) {
                f = dtf[rl64(mro, j) + tbyte + kDPL * lane + b];
              } else {
                int64_t lo = rl64(plo, j);
                const int64_t e = rl64(phi, j);
                int64_t hi = e;
                while (lo < hi) {
                  const int64_t mid = (lo + hi) >> 1;
                  if (docno[mid] < d) lo = mid + 1;
                  else hi = mid;
                }
                if (lo < e && docno[lo] == d) f = tf[lo];
              }
              if (f != 0) S = __dadd_rn(S, __dmul_rn(f < kWLut ? s_lut[f] : lut[f], rld(midf, j)));
            }
            keep = !th_ok || better(S, d, th_s, th_d);
          }
          const uint64_t km = (uint64_t)__ballot(keep);
          if (keep) {
            const int pos = cnt + (int)lane_prefix(km);
            bs[pos] = S;
            bd[pos] = d;
          }
          cnt += __popcll(km);
          if (cnt > C - 64) compact();
        }
      }
      int32_t nt_ = nx;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) nt_ = min(nt_, __shfl_xor(nt_, o, 64));
      if (nt_ == tile + 1) {
        mc = me;
        me = me1;
      } else if (nt_ != 0x7FFFFFFF && lane < nt && mdf > 0) {
        mc = mrow[nt_];
        me = mrow[nt_ + 1];
      }
      tile = nt_;
    }
    __syncthreads();
    compact();
    if (stats) {
      uint32_t c = st_cand;
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0) {
        atomicAdd(stats + 0, (unsigned long long)st_tiles);
        atomicAdd(stats + 1, (unsigned long long)st_gated);
        atomicAdd(stats + 2, (unsigned long long)c);
        atomicAdd(stats + 3, (unsigned long long)st_comp);
        atomicAdd(stats + 4, (unsigned long long)st_sparse);
      }
    }
    for (int r = lane; r < k; r += 64) {
      out_d[(int64_t)q * k + r] = r < cnt ? bd[r] : -1;
      out_s[(int64_t)q * k + r] = r < cnt ? bs[r] : 0.0;
    }
    __syncthreads();
  }
}

void query_topk(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, int k, int32_t *d_out_docno,
                double *d_out_score, hipStream_t st) {
  if (k < 1) throw Error(SME_EINVAL, "k must be >= 1");
  if (k > 448) throw Error(SME_ELIMIT, "top-k with k > 448");
  if (nq <= 0) return;
  auto &W = ix->ctx->ws;
  int *err = W[63].as<int>(4);
  unsigned long long *wmax = reinterpret_cast<unsigned long long *>(err + 2);
  SME_HIP(hipMemsetAsync(err, 0, 4 * sizeof(int), st));
  const int64_t *off = (const int64_t *)ix->d_off.p;
  const int32_t *dn = (const int32_t *)ix->d_docno_d.p;
  const int32_t *tf = (const int32_t *)ix->d_tf_d.p;
  const double *lut = (const double *)ix->d_lut.p;
  const double *idf = (const double *)ix->d_idf.p;
  const int64_t V = ix->V;
  hipEvent_t ep;
  SME_HIP(hipEventCreate(&ep));
  SME_HIP(hipEventRecord(ep, st));
  // Tiled path unless a query is longer than kIMaxTerms or the batch's skip
  // table would be unreasonably large; SME_QUERY_KERNEL=stream forces the
  // streaming kernel (tests run both).
  const char *force = getenv("SME_QUERY_KERNEL");
  bool tiled = V > 0 && ix->P > 0 && ix->dmax >= ix->dmin && !(force && strcmp(force, "stream") == 0);
  const int64_t T = tiled ? ((ix->dmax - ix->dmin) >> kWBits) + 1 : 0;
  const int32_t *row_of = nullptr, *sk = nullptr, *drow = nullptr;
  const uint8_t *dtf = nullptr, *dq = nullptr;
  int64_t dstride = 0;
  int h_mx = 0;
  if (tiled) {
    hipLaunchKernelGGL(k_max_qlen, dim3(std::min((nq + 255) / 256, 1024)), dim3(256), 0, st, d_qoff, nq, err + 1);
    SME_HIP(hipMemcpyAsync(&h_mx, err + 1, sizeof(int), hipMemcpyDeviceToHost, st));
    int64_t nterm = 0;
    SME_HIP(hipMemcpyAsync(&nterm, d_qoff + nq, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    tiled = h_mx <= kIMaxTerms;
    if (tiled) {
      // distinct batch terms -> rows of the skip table
      int32_t *mark = W[55].as<int32_t>(V + 1), *rowo = W[56].as<int32_t>(V + 1);
      SME_HIP(hipMemsetAsync(mark, 0, (V + 1) * sizeof(int32_t), st));
      if (nterm > 0)
        hipLaunchKernelGGL(k_mark_terms, dim3((unsigned)std::min<int64_t>((nterm + 255) / 256, 8192)), dim3(256), 0, st,
                           d_terms, nterm, V, mark);
      size_t tbb = 0;
      SME_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tbb, mark, rowo, (int)V + 1, st));
      SME_HIP(hipcub::DeviceScan::ExclusiveSum(ix->ctx->cub_tmp.get(tbb), tbb, mark, rowo, (int)V + 1, st));
      int32_t nrows32 = 0;
      SME_HIP(hipMemcpyAsync(&nrows32, rowo + V, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      SME_HIP(hipStreamSynchronize(st));
      const int64_t nrows = nrows32;
      if ((double)nrows * (double)(T + 1) * 4.0 > 8.0e9) {
        tiled = false;
      } else {
        row_of = rowo;
        int32_t *skw = W[60].as<int32_t>(std::max<int64_t>(nrows, 1) * (T + 1));
        sk = skw;
        if (nrows > 0) {
          int32_t *tor = W[57].as<int32_t>(nrows + 1);
          int64_t *rdf = W[58].as<int64_t>(nrows + 1), *rpre = W[59].as<int64_t>(nrows + 1);
          const unsigned gV = (unsigned)std::min<int64_t>((V + 255) / 256, 8192);
          hipLaunchKernelGGL(k_term_rows, dim3(gV), dim3(256), 0, st, mark, rowo, V, off, tor, rdf);
          SME_HIP(hipMemsetAsync(rdf + nrows, 0, sizeof(int64_t), st));
          SME_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tbb, rdf, rpre, (int)nrows + 1, st));
          SME_HIP(hipcub::DeviceScan::ExclusiveSum(ix->ctx->cub_tmp.get(tbb), tbb, rdf, rpre, (int)nrows + 1, st));
          SME_HIP(hipMemsetAsync(skw, 0x7F, (size_t)nrows * (T + 1) * sizeof(int32_t), st));
          hipLaunchKernelGGL(k_skip_zero_rows, dim3((unsigned)std::min<int64_t>(nrows, 4096)), dim3(256), 0, st, rdf,
                             nrows, T, skw);
          hipLaunchKernelGGL(k_skip_fill, dim3(16384), dim3(256), 0, st, rpre, nrows, tor, off, dn, ix->dmin, T, skw);
          hipLaunchKernelGGL(k_skip_suffix, dim3((unsigned)std::min<int64_t>((nrows + 3) / 4, 16384)), dim3(256), 0,
                             st, nrows, T, skw);
          // largest weight of the batch (impact scale) and the dense-row terms
          // (SME_QDENSE=div, 0 = posting path only; tests run several)
          const char *ed = getenv("SME_QDENSE");
          const int64_t ddiv = ed ? atoll(ed) : 32;
          const int64_t span = ix->dmax - ix->dmin + 1, stride = T << kWBits;
          int32_t *flag = W[53].as<int32_t>(nrows + 1), *dscan = W[54].as<int32_t>(nrows + 1);
          const unsigned gR = (unsigned)std::min<int64_t>((nrows + 256) / 256, 8192);
          hipLaunchKernelGGL(k_row_stats, dim3(gR), dim3(256), 0, st, tor, rdf, nrows, off,
                             (const int32_t *)ix->d_tf_o.p, lut, idf, span, ddiv, flag, wmax);
          SME_CHECK_LAUNCH();
          if (ddiv > 0) {
            const int64_t cap = std::max<int64_t>(1, (int64_t)2e9 / stride);
            SME_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tbb, flag, dscan, (int)nrows + 1, st));
            SME_HIP(hipcub::DeviceScan::ExclusiveSum(ix->ctx->cub_tmp.get(tbb), tbb, flag, dscan, (int)nrows + 1, st));
            int32_t ndense = 0;
            SME_HIP(hipMemcpyAsync(&ndense, dscan + nrows, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            SME_HIP(hipStreamSynchronize(st));
            const int64_t nd = std::min<int64_t>(ndense, cap);
            if (nd > 0) {
              int32_t *drw = W[62].as<int32_t>(nrows);
              uint8_t *dns = W[61].as<uint8_t>(2 * nd * stride);
              SME_HIP(hipMemsetAsync(dns, 0, (size_t)(2 * nd * stride), st));
              hipLaunchKernelGGL(k_dense_rows, dim3(gR), dim3(256), 0, st, flag, dscan, nrows, cap, drw);
              hipLaunchKernelGGL(k_dense_fill, dim3(16384), dim3(256), 0, st, rpre, nrows, drw, tor, off, dn, tf, lut,
                                 idf, wmax, ix->dmin, stride, dns, dns + nd * stride);
              SME_CHECK_LAUNCH();
              dtf = dns;
              dq = dns + nd * stride;
              drow = drw;
              dstride = stride;
            }
          }
        }
      }
    }
  }
  if (!tiled && k > 32) throw Error(SME_ENOTIMPL, "top-k with k > 32 for queries of more than 64 terms");
  int sh = 0;
  const int32_t *qord = nullptr;
  if (tiled) {
    // impact shift: 255 * 2^sh * (terms per query) <= 65535 keeps the u16 sums exact
    sh = 0;
    while (sh < 5 && 255 * (2 << sh) * std::max(h_mx, 1) <= 65535) sh++;
    // heaviest-term query order (SME_QORDER=0: batch order)
    const char *eo = getenv("SME_QORDER");
    if (!(eo && atoi(eo) == 0)) {
      uint64_t *qk = W[46].as<uint64_t>(2 * (size_t)nq);
      int32_t *qi = W[45].as<int32_t>(2 * (size_t)nq);
      hipLaunchKernelGGL(k_query_keys, dim3(std::min((nq + 255) / 256, 4096)), dim3(256), 0, st, d_terms, d_qoff, nq, off,
                         V, qk, qi);
      size_t tbb = 0;
      SME_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tbb, qk, qk + nq, qi, qi + nq, nq, 0, 64, st));
      SME_HIP(hipcub::DeviceRadixSort::SortPairs(ix->ctx->cub_tmp.get(tbb), tbb, qk, qk + nq, qi, qi + nq, nq, 0, 64,
                                                 st));
      qord = qi + nq;
    }
  }
  // events on the launch stream bracket the scoring kernel (bench.py roofline)
  hipEvent_t e0, e1;
  SME_HIP(hipEventCreate(&e0));
  SME_HIP(hipEventCreate(&e1));
  SME_HIP(hipEventRecord(e0, st));
  const char *ex = getenv("SME_QEXP");  // timing experiments only (wrong results): 1 no candidates, 2 no postings
  const int qexp = ex ? atoi(ex) : 0;
  unsigned long long *qstats = nullptr;
  const char *eq = getenv("SME_QSTATS");
  if (eq && atoi(eq)) {
    qstats = reinterpret_cast<unsigned long long *>(W[47].as<uint64_t>(8));
    SME_HIP(hipMemsetAsync(qstats, 0, 8 * sizeof(uint64_t), st));
  }
  if (tiled) {
    const unsigned wgrid = (unsigned)std::min<int64_t>(8 * (((int64_t)nq + 7) / 8), 1 << 30);
#define SME_QI(C)                                                                                                \
  hipLaunchKernelGGL(k_query_imp<C>, dim3(wgrid), dim3(64), 0, st, off, dn, tf, lut, ix->max_tf, idf, V, row_of, sk, \
                     ix->dmin, T, d_terms, d_qoff, qord, nq, k, d_out_docno, d_out_score, dtf, dq, drow, dstride,    \
                     (const unsigned long long *)wmax, sh, qstats, qexp)
    if (k <= 64) SME_QI(128);
    else if (k <= 192) SME_QI(256);
    else SME_QI(512);
#undef SME_QI
  } else if (k <= 16) {
    const unsigned grid = (unsigned)std::min(nq, 1 << 20);
    hipLaunchKernelGGL(k_query<16>, dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, V, d_terms,
                       d_qoff, nq, k, d_out_docno, d_out_score, err);
  } else {
    const unsigned grid = (unsigned)std::min(nq, 1 << 20);
    hipLaunchKernelGGL(k_query<32>, dim3(grid), dim3(kQNT), 0, st, off, dn, tf, lut, ix->max_tf, idf, V, d_terms,
                       d_qoff, nq, k, d_out_docno, d_out_score, err);
  }
  SME_CHECK_LAUNCH();
  SME_HIP(hipEventRecord(e1, st));
  int h_err = 0;
  SME_HIP(hipMemcpyAsync(&h_err, err, sizeof(int), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  float ms = 0, pms = 0;
  SME_HIP(hipEventElapsedTime(&ms, e0, e1));
  SME_HIP(hipEventElapsedTime(&pms, ep, e0));
  ix->ctx->last_query_ms = ms;
  ix->ctx->last_query_prep_ms = pms;
  (void)hipEventDestroy(ep);
  ix->ctx->last_query_tiled = tiled;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (qstats) {
    uint64_t h[8];
    SME_HIP(hipMemcpy(h, qstats, sizeof h, hipMemcpyDeviceToHost));
    fprintf(stderr, "SME_QSTATS tiles=%llu gated=%llu candidates=%llu compactions=%llu sparse_tiles=%llu\n",
            (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2], (unsigned long long)h[3],
            (unsigned long long)h[4]);
  }
  if (h_err) throw Error(SME_ELIMIT, "a query has more than 128 terms");
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
