// sme_timsort.hip -- SME_TIE_JAVA7: rank()'s printed list as a Java 7 JVM
// produces it (IntDocVectorsForwardIndex.java:192-222, DocScore.compareTo
// :363-365).
//
// rank() appends one DocScore per document in first-encounter order (query
// tokens in order, each term's postings in reduce order: tf desc, docno asc),
// adds (1 + ln tf) * idf per (token, posting), then Collections.sort(scores).
// On Java 7 that is ComparableTimSort, and DocScore.compareTo =
// (int)Math.ceil(o.score - score) is not a total order (it is 0 for score gaps
// in (-1, 0]), so the result depends on the whole list and on TimSort's exact
// sequence of comparisons -- no per-document key reproduces it.  This path
// therefore builds every query's full list on the device and runs TimSort
// itself, one thread per query:
//   k_j7_bound  per query: sum of its known terms' df (the list's upper bound)
//   k_j7_list   one wave per query: the first-encounter list -- a posting is new
//               when no earlier token's term holds its document (binary search in
//               that term's docno-order postings); a new document's score is the
//               left-to-right fp64 sum over its tokens, as rank() accumulates
//   k_j7_sort   one thread per query: OpenJDK 7 GA ComparableTimSort (runs,
//               binary insertion to minRun, the GA mergeCollapse invariant,
//               gallopLeft / gallopRight, mergeLo / mergeHi, MIN_GALLOP 7), every
//               test the Java source asks (< 0, <= 0, > 0, >= 0) on compareTo;
//               a merge that finds the contract violated is where Java throws
//               IllegalArgumentException("Comparison method violates its general
//               contract!"): that query's row is all docno -2.
// The same algorithm restated on the CPU is oracle/oracle_index.c (order 3),
// which the tests hold this path to.  It is a compatibility mode, not the
// serving path: its cost is the lists (16 B per candidate) and a serial sort.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <vector>

#include "sme_internal.hpp"

namespace sme {
namespace {

struct DS {  // DocScore: score, docId
  double s;
  int32_t d, pad;
};
static_assert(sizeof(DS) == 16, "DocScore record");

// a.compareTo(b): (int)Math.ceil(b.score - a.score); Java's double -> int cast
// maps NaN to 0 and saturates
__device__ __forceinline__ int ds_cmp(const DS &a, const DS &b) {
  const double x = ceil(__dsub_rn(b.s, a.s));
  if (x != x) return 0;
  if (x >= 2147483647.0) return INT_MAX;
  if (x <= -2147483648.0) return INT_MIN;
  return (int)x;
}

// System.arraycopy semantics (overlap-safe)
__device__ void ds_move(DS *dst, const DS *src, int n) {
  if (dst < src) {
    for (int i = 0; i < n; i++) dst[i] = src[i];
  } else if (dst > src) {
    for (int i = n - 1; i >= 0; i--) dst[i] = src[i];
  }
}

constexpr int kMinMerge = 32, kMinGallop = 7, kMaxRuns = 85;

struct TS {
  DS *a, *tmp;
  int min_gallop, stack;
  int base[kMaxRuns], len[kMaxRuns];
  int err;  // 1: IllegalArgumentException, 2: run stack past kMaxRuns
};

__device__ int count_run(DS *a, int lo, int hi) {
  int runHi = lo + 1;
  if (runHi == hi) return 1;
  if (ds_cmp(a[runHi++], a[lo]) < 0) {  // strictly descending: reversed
    while (runHi < hi && ds_cmp(a[runHi], a[runHi - 1]) < 0) runHi++;
    for (int l = lo, h = runHi - 1; l < h; l++, h--) {
      const DS t = a[l];
      a[l] = a[h];
      a[h] = t;
    }
  } else {
    while (runHi < hi && ds_cmp(a[runHi], a[runHi - 1]) >= 0) runHi++;
  }
  return runHi - lo;
}

__device__ void binary_sort(DS *a, int lo, int hi, int start) {
  if (start == lo) start++;
  for (; start < hi; start++) {
    const DS pivot = a[start];
    int left = lo, right = start;
    while (left < right) {
      const int mid = (int)(((unsigned)left + (unsigned)right) >> 1);
      if (ds_cmp(pivot, a[mid]) < 0) right = mid;
      else left = mid + 1;
    }
    ds_move(a + left + 1, a + left, start - left);
    a[left] = pivot;
  }
}

__device__ int min_run(int n) {
  int r = 0;
  while (n >= kMinMerge) {
    r |= n & 1;
    n >>= 1;
  }
  return n + r;
}

__device__ int gallop_left(const DS &key, const DS *a, int base, int len, int hint) {
  int lastOfs = 0, ofs = 1;
  if (ds_cmp(key, a[base + hint]) > 0) {
    const int maxOfs = len - hint;
    while (ofs < maxOfs && ds_cmp(key, a[base + hint + ofs]) > 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    lastOfs += hint;
    ofs += hint;
  } else {
    const int maxOfs = hint + 1;
    while (ofs < maxOfs && ds_cmp(key, a[base + hint - ofs]) <= 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    const int t = lastOfs;
    lastOfs = hint - ofs;
    ofs = hint - t;
  }
  lastOfs++;
  while (lastOfs < ofs) {
    const int m = lastOfs + (int)((unsigned)(ofs - lastOfs) >> 1);
    if (ds_cmp(key, a[base + m]) > 0) lastOfs = m + 1;
    else ofs = m;
  }
  return ofs;
}

__device__ int gallop_right(const DS &key, const DS *a, int base, int len, int hint) {
  int ofs = 1, lastOfs = 0;
  if (ds_cmp(key, a[base + hint]) < 0) {
    const int maxOfs = hint + 1;
    while (ofs < maxOfs && ds_cmp(key, a[base + hint - ofs]) < 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    const int t = lastOfs;
    lastOfs = hint - ofs;
    ofs = hint - t;
  } else {
    const int maxOfs = len - hint;
    while (ofs < maxOfs && ds_cmp(key, a[base + hint + ofs]) >= 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    lastOfs += hint;
    ofs += hint;
  }
  lastOfs++;
  while (lastOfs < ofs) {
    const int m = lastOfs + (int)((unsigned)(ofs - lastOfs) >> 1);
    if (ds_cmp(key, a[base + m]) < 0) ofs = m;
    else lastOfs = m + 1;
  }
  return ofs;
}

// mergeLo: run 1 (the shorter) copied to tmp, merged forward
__device__ void merge_lo(TS &t, int base1, int len1, int base2, int len2) {
  DS *a = t.a, *tmp = t.tmp;
  ds_move(tmp, a + base1, len1);
  int cursor1 = 0, cursor2 = base2, dest = base1;
  a[dest++] = a[cursor2++];
  if (--len2 == 0) {
    ds_move(a + dest, tmp + cursor1, len1);
    return;
  }
  if (len1 == 1) {
    ds_move(a + dest, a + cursor2, len2);
    a[dest + len2] = tmp[cursor1];
    return;
  }
  int minGallop = t.min_gallop;
  for (;;) {
    int count1 = 0, count2 = 0;
    bool brk = false;
    do {
      if (ds_cmp(a[cursor2], tmp[cursor1]) < 0) {
        a[dest++] = a[cursor2++];
        count2++;
        count1 = 0;
        if (--len2 == 0) {
          brk = true;
          break;
        }
      } else {
        a[dest++] = tmp[cursor1++];
        count1++;
        count2 = 0;
        if (--len1 == 1) {
          brk = true;
          break;
        }
      }
    } while ((count1 | count2) < minGallop);
    if (brk) break;
    do {
      count1 = gallop_right(a[cursor2], tmp, cursor1, len1, 0);
      if (count1 != 0) {
        ds_move(a + dest, tmp + cursor1, count1);
        dest += count1;
        cursor1 += count1;
        len1 -= count1;
        if (len1 <= 1) {
          brk = true;
          break;
        }
      }
      a[dest++] = a[cursor2++];
      if (--len2 == 0) {
        brk = true;
        break;
      }
      count2 = gallop_left(tmp[cursor1], a, cursor2, len2, 0);
      if (count2 != 0) {
        ds_move(a + dest, a + cursor2, count2);
        dest += count2;
        cursor2 += count2;
        len2 -= count2;
        if (len2 == 0) {
          brk = true;
          break;
        }
      }
      a[dest++] = tmp[cursor1++];
      if (--len1 == 1) {
        brk = true;
        break;
      }
      minGallop--;
    } while (count1 >= kMinGallop || count2 >= kMinGallop);
    if (brk) break;
    if (minGallop < 0) minGallop = 0;
    minGallop += 2;
  }
  t.min_gallop = minGallop < 1 ? 1 : minGallop;
  if (len1 == 1) {
    ds_move(a + dest, a + cursor2, len2);
    a[dest + len2] = tmp[cursor1];
  } else if (len1 == 0) {
    t.err = 1;  // "Comparison method violates its general contract!"
  } else {
    ds_move(a + dest, tmp + cursor1, len1);
  }
}

// mergeHi: run 2 (the shorter) copied to tmp, merged backward
__device__ void merge_hi(TS &t, int base1, int len1, int base2, int len2) {
  DS *a = t.a, *tmp = t.tmp;
  ds_move(tmp, a + base2, len2);
  int cursor1 = base1 + len1 - 1, cursor2 = len2 - 1, dest = base2 + len2 - 1;
  a[dest--] = a[cursor1--];
  if (--len1 == 0) {
    ds_move(a + dest - (len2 - 1), tmp, len2);
    return;
  }
  if (len2 == 1) {
    dest -= len1;
    cursor1 -= len1;
    ds_move(a + dest + 1, a + cursor1 + 1, len1);
    a[dest] = tmp[cursor2];
    return;
  }
  int minGallop = t.min_gallop;
  for (;;) {
    int count1 = 0, count2 = 0;
    bool brk = false;
    do {
      if (ds_cmp(tmp[cursor2], a[cursor1]) < 0) {
        a[dest--] = a[cursor1--];
        count1++;
        count2 = 0;
        if (--len1 == 0) {
          brk = true;
          break;
        }
      } else {
        a[dest--] = tmp[cursor2--];
        count2++;
        count1 = 0;
        if (--len2 == 1) {
          brk = true;
          break;
        }
      }
    } while ((count1 | count2) < minGallop);
    if (brk) break;
    do {
      count1 = len1 - gallop_right(tmp[cursor2], a, base1, len1, len1 - 1);
      if (count1 != 0) {
        dest -= count1;
        cursor1 -= count1;
        len1 -= count1;
        ds_move(a + dest + 1, a + cursor1 + 1, count1);
        if (len1 == 0) {
          brk = true;
          break;
        }
      }
      a[dest--] = tmp[cursor2--];
      if (--len2 == 1) {
        brk = true;
        break;
      }
      count2 = len2 - gallop_left(a[cursor1], tmp, 0, len2, len2 - 1);
      if (count2 != 0) {
        dest -= count2;
        cursor2 -= count2;
        len2 -= count2;
        ds_move(a + dest + 1, tmp + cursor2 + 1, count2);
        if (len2 <= 1) {
          brk = true;
          break;
        }
      }
      a[dest--] = a[cursor1--];
      if (--len1 == 0) {
        brk = true;
        break;
      }
      minGallop--;
    } while (count1 >= kMinGallop || count2 >= kMinGallop);
    if (brk) break;
    if (minGallop < 0) minGallop = 0;
    minGallop += 2;
  }
  t.min_gallop = minGallop < 1 ? 1 : minGallop;
  if (len2 == 1) {
    dest -= len1;
    cursor1 -= len1;
    ds_move(a + dest + 1, a + cursor1 + 1, len1);
    a[dest] = tmp[cursor2];
  } else if (len2 == 0) {
    t.err = 1;  // IllegalArgumentException
  } else {
    ds_move(a + dest - (len2 - 1), tmp, len2);
  }
}

__device__ void merge_at(TS &t, int i) {
  int base1 = t.base[i], len1 = t.len[i];
  const int base2 = t.base[i + 1];
  int len2 = t.len[i + 1];
  t.len[i] = len1 + len2;
  if (i == t.stack - 3) {
    t.base[i + 1] = t.base[i + 2];
    t.len[i + 1] = t.len[i + 2];
  }
  t.stack--;
  const int k = gallop_right(t.a[base2], t.a, base1, len1, 0);
  base1 += k;
  len1 -= k;
  if (len1 == 0) return;
  len2 = gallop_left(t.a[base1 + len1 - 1], t.a, base2, len2, len2 - 1);
  if (len2 == 0) return;
  if (len1 <= len2) merge_lo(t, base1, len1, base2, len2);
  else merge_hi(t, base1, len1, base2, len2);
}

// OpenJDK 7 GA mergeCollapse (the invariant before the JDK-8072909 fix)
__device__ void merge_collapse(TS &t) {
  while (t.stack > 1 && !t.err) {
    int n = t.stack - 2;
    if (n > 0 && t.len[n - 1] <= t.len[n] + t.len[n + 1]) {
      if (t.len[n - 1] < t.len[n + 1]) n--;
      merge_at(t, n);
    } else if (t.len[n] <= t.len[n + 1]) {
      merge_at(t, n);
    } else {
      break;
    }
  }
}

__device__ void merge_force_collapse(TS &t) {
  while (t.stack > 1 && !t.err) {
    int n = t.stack - 2;
    if (n > 0 && t.len[n - 1] < t.len[n + 1]) n--;
    merge_at(t, n);
  }
}

// ComparableTimSort.sort(a, 0, n); tmp holds >= n / 2 records.  0, or the error
__device__ int timsort7(DS *a, int n, DS *tmp) {
  if (n < 2) return 0;
  int lo = 0, rem = n;
  if (rem < kMinMerge) {
    const int initRunLen = count_run(a, lo, n);
    binary_sort(a, lo, n, lo + initRunLen);
    return 0;
  }
  TS t;
  t.a = a;
  t.tmp = tmp;
  t.min_gallop = kMinGallop;
  t.stack = 0;
  t.err = 0;
  const int minRun = min_run(rem);
  do {
    int runLen = count_run(a, lo, n);
    if (runLen < minRun) {
      const int force = rem <= minRun ? rem : minRun;
      binary_sort(a, lo, lo + force, lo + runLen);
      runLen = force;
    }
    if (t.stack == kMaxRuns) {
      t.err = 2;
      break;
    }
    t.base[t.stack] = lo;
    t.len[t.stack] = runLen;
    t.stack++;
    merge_collapse(t);
    lo += runLen;
    rem -= runLen;
  } while (rem != 0 && !t.err);
  merge_force_collapse(t);
  return t.err;
}

__device__ __forceinline__ bool valid_term(int32_t t, int64_t V) { return t >= 0 && t < V; }

// tf of document d in term t (its docno-order postings), 0 if absent
__device__ int32_t tf_in(const int64_t *off, const int32_t *dn, const int32_t *tf, int32_t t, int32_t d) {
  int64_t lo = off[t], hi = off[t + 1];
  const int64_t e = hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (dn[mid] < d) lo = mid + 1;
    else hi = mid;
  }
  return (lo < e && dn[lo] == d) ? tf[lo] : 0;
}

__global__ void k_j7_bound(const int32_t *terms, const int64_t *qoff, int nq, int64_t V, const int64_t *off,
                           int64_t *U) {
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nq; q += gridDim.x * blockDim.x) {
    int64_t u = 0;
    for (int64_t i = qoff[q]; i < qoff[q + 1]; i++) {
      const int32_t t = terms[i];
      if (valid_term(t, V)) u += off[t + 1] - off[t];
    }
    U[q] = u;
  }
}

struct J7List {
  const int32_t *terms;
  const int64_t *qoff;
  int q_lo, q_hi;
  int64_t V;
  const int64_t *off;
  const int32_t *dn_o, *tf_o, *dn_d, *tf_d;
  const double *lut, *idf;
  const int64_t *lbase;  // list start of every query (exclusive scan of k_j7_bound)
  int64_t l0;            // lbase of q_lo: the chunk's lists start at list[0]
  DS *list;
  int32_t *cnt;
};

__global__ __launch_bounds__(64) void k_j7_list(J7List a) {
  const int lane = threadIdx.x;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int q = a.q_lo + blockIdx.x; q < a.q_hi; q += gridDim.x) {
    const int64_t q0 = a.qoff[q];
    const int nt = (int)(a.qoff[q + 1] - q0);
    DS *L = a.list + (a.lbase[q] - a.l0);
    int64_t n = 0;
    for (int i = 0; i < nt; i++) {
      const int32_t t = a.terms[q0 + i];
      if (!valid_term(t, a.V)) continue;  // getValue: an unknown term is skipped
      const int64_t b = a.off[t], df = a.off[t + 1] - b;
      for (int64_t p0 = 0; p0 < df; p0 += 64) {
        const int64_t p = p0 + lane;
        bool fresh = false;
        int32_t d = 0;
        double S = 0.0;
        if (p < df) {
          d = a.dn_o[b + p];
          const int32_t f = a.tf_o[b + p];
          fresh = true;
          for (int j = 0; j < i && fresh; j++) {  // scores.indexOf found it under an earlier token
            const int32_t tj = a.terms[q0 + j];
            if (valid_term(tj, a.V) && tf_in(a.off, a.dn_d, a.tf_d, tj, d) != 0) fresh = false;
          }
          if (fresh) {
            // score.score += (1 + ln tf) * idf over the tokens holding d, in token order
            for (int j = i; j < nt; j++) {
              const int32_t tj = a.terms[q0 + j];
              if (!valid_term(tj, a.V)) continue;
              const int32_t fj = tj == t ? f : tf_in(a.off, a.dn_d, a.tf_d, tj, d);
              if (fj != 0) S = __dadd_rn(S, __dmul_rn(a.lut[fj], a.idf[tj]));
            }
          }
        }
        const uint64_t m = (uint64_t)__ballot(fresh);
        if (fresh) L[n + __popcll(m & lt)] = DS{S, d, 0};
        n += __popcll(m);
      }
    }
    if (lane == 0) a.cnt[q] = (int32_t)n;
  }
}

__global__ __launch_bounds__(64) void k_j7_sort(int q_lo, int q_hi, const int64_t *lbase, int64_t l0, DS *list,
                                                DS *tmp, const int32_t *cnt, int k, int32_t *out_d, double *out_s,
                                                uint32_t *out_t, int *err) {
  const int q = q_lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= q_hi) return;
  const int64_t o = lbase[q] - l0;
  DS *L = list + o;
  const int n = cnt[q];
  const int e = timsort7(L, n, tmp + o);
  if (e == 2) atomicOr(err, 2);
  for (int r = 0; r < k; r++) {
    const int64_t x = (int64_t)q * k + r;
    out_d[x] = e ? -2 : r < n ? L[r].d : -1;
    out_s[x] = (!e && r < n) ? L[r].s : 0.0;
    if (out_t) out_t[x] = 0xFFFFFFFFu;
  }
}

}  // namespace

void query_topk_java7(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, int k,
                      int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie, hipStream_t st) {
  sme_ctx *cx = ix->ctx;
  auto &W = cx->ws;
  const int64_t V = ix->V;
  const int64_t *off = (const int64_t *)ix->d_off.p;
  int64_t *U = W[48].as<int64_t>((size_t)nq + 1);
  int64_t *lbase = W[49].as<int64_t>((size_t)nq + 1);
  int32_t *cnt = W[50].as<int32_t>((size_t)nq + 1);
  int *err = W[51].as<int>(4);
  SME_HIP(hipMemsetAsync(err, 0, sizeof(int), st));
  SME_HIP(hipMemsetAsync(U + nq, 0, sizeof(int64_t), st));
  hipLaunchKernelGGL(k_j7_bound, dim3(std::min((nq + 255) / 256, 4096)), dim3(256), 0, st, d_terms, d_qoff, nq, V, off, U);
  excl_scan(U, lbase, (int64_t)nq + 1, cx->ws[23], st);
  std::vector<int64_t> hb((size_t)nq + 1);
  SME_HIP(hipMemcpyAsync(hb.data(), lbase, hb.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  // chunks of queries whose lists (and TimSort's tmp of the same size) fit an
  // eighth of the free HBM
  size_t fr = 0, tot = 0;
  SME_HIP(hipMemGetInfo(&fr, &tot));
  const int64_t cap = std::max<int64_t>(1, (int64_t)(fr / 8 / (2 * sizeof(DS))));
  J7List a{d_terms, d_qoff, 0, 0, V, off, (const int32_t *)ix->d_docno_o.p, (const int32_t *)ix->d_tf_o.p,
           (const int32_t *)ix->d_docno_d.p, (const int32_t *)ix->d_tf_d.p, (const double *)ix->d_lut.p,
           (const double *)ix->d_idf.p, lbase, 0, nullptr, cnt};
  int q_lo = 0;
  while (q_lo < nq) {
    int q_hi = q_lo + 1;
    if (hb[q_hi] - hb[q_lo] > cap)
      throw Error(SME_ELIMIT, "SME_TIE_JAVA7: one query's candidate list exceeds an eighth of the free HBM");
    while (q_hi < nq && hb[q_hi + 1] - hb[q_lo] <= cap) q_hi++;
    const int64_t len = std::max<int64_t>(hb[q_hi] - hb[q_lo], 1);
    DS *list = reinterpret_cast<DS *>(W[52].as<uint8_t>((size_t)len * sizeof(DS)));
    DS *tmp = reinterpret_cast<DS *>(W[53].as<uint8_t>((size_t)len * sizeof(DS)));
    a.q_lo = q_lo;
    a.q_hi = q_hi;
    a.l0 = hb[q_lo];
    a.list = list;
    const int nqc = q_hi - q_lo;
    hipLaunchKernelGGL(k_j7_list, dim3((unsigned)std::min(nqc, 65536)), dim3(64), 0, st, a);
    hipLaunchKernelGGL(k_j7_sort, dim3((unsigned)((nqc + 63) / 64)), dim3(64), 0, st, q_lo, q_hi, lbase, hb[q_lo],
                       list, tmp, cnt, k, d_out_docno, d_out_score, d_out_tie, err);
    SME_CHECK_LAUNCH();
    SME_HIP(hipStreamSynchronize(st));  // (the chunk's list buffers are reused by the next chunk)
    q_lo = q_hi;
  }
  int h_err = 0;
  SME_HIP(hipMemcpy(&h_err, err, sizeof(int), hipMemcpyDeviceToHost));
  if (h_err & 2) throw Error(SME_ELIMIT, "SME_TIE_JAVA7: TimSort run stack deeper than 85 runs");
  cx->last_query_name = "k_j7_sort";
  cx->last_query_tiled = false;
}

}  // namespace sme
