// sme_merge.hip -- the reference's reduce output from doc shards (last row).
//
// With W doc shards every term's postings are split W ways, while the job's
// output is one globally reduced postings list per term in R term-partitioned
// part files (partition (Arrays.hashCode(k_gram) & MAX_VALUE) % R, TermDF.java
// :79-81; one reducer per partition, TermKGramDocIndexer.java:189-211,246).
// Partition p is produced by rank p % W:
//
//   pack   (every shard)  its terms grouped by owner rank, one self-describing
//          blob per owner: the terms (UTF-16, in the shard's String.compareTo
//          order), their postings in reduce order, and -- for the owner of the
//          " " doc-counter key's partition -- the docnos of the shard's records
//          (the map task's doc-counter postings, TermKGramDocIndexer.java:84-90,126)
//   (all_to_all of the blobs over RCCL / gloo, dist.reference_partitions)
//   merge  (every owner)  the W received blobs -> one index holding the owned
//          partitions' terms: term order = a rank by binary search of every
//          term in the other pieces' sorted term lists (String.compareTo), equal
//          strings -> one term; postings = MyReducer.reduce over the
//          concatenated map outputs: sorted by docno, equal docnos merged by
//          summing tf (a docid duplicated across shards), stably sorted by tf
//          desc; the doc counter = every map task's list, each starting at (0,0).
//          The serializer (sme_serial.hip) then writes its partitions' records.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sme_internal.hpp"

namespace sme {

namespace {

constexpr uint64_t kPieceMagic = 0x3145434549505A53ull;  // "SZPIECE1"

struct PieceHdr {  // 64 bytes, at the start of every blob
  uint64_t magic;
  int64_t nterms, nunits, npost, nrec;
  int32_t dmin, dmax;  // docno range of the shard's records (dmin > dmax: none)
  int64_t pad[2];
};
static_assert(sizeof(PieceHdr) == 64, "piece header");

struct PieceLayout {  // byte offsets of the sections of a blob
  int64_t term_off, term_chars, post_off, docno, tf, rec, total;
};
inline int64_t al16(int64_t x) { return (x + 15) & ~int64_t(15); }
PieceLayout layout_of(const PieceHdr &h) {
  PieceLayout L;
  L.term_off = 64;
  L.term_chars = L.term_off + al16(8 * (h.nterms + 1));
  L.post_off = L.term_chars + al16(2 * h.nunits);
  L.docno = L.post_off + al16(8 * (h.nterms + 1));
  L.tf = L.docno + al16(4 * h.npost);
  L.rec = L.tf + al16(4 * h.npost);
  L.total = L.rec + al16(4 * h.nrec);
  return L;
}

// partition of a term: Arrays.hashCode(k_gram) = fold of 31 * h + s.hashCode()
// over the components from 1 (K = 1: 31 + s.hashCode()); a K >= 2 gram is its
// components joined by U+0000 (never inside a term: 0 is a split character)
__global__ void k_term_owner(const int64_t *toff, const uint16_t *tch, int64_t V, int R, int world, int32_t *owner) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h = 0, ah = 1u;
    for (int64_t i = toff[t]; i < toff[t + 1]; i++) {
      if (tch[i] == 0) {
        ah = 31u * ah + h;
        h = 0;
      } else {
        h = 31u * h + tch[i];
      }
    }
    ah = 31u * ah + h;
    owner[t] = (int32_t)((uint32_t)((int32_t)(ah & 0x7fffffffu) % R) % (uint32_t)world);
  }
}
// K >= 2: every gram as one string, its component terms joined by U+0000.  The
// strings' UTF-16 order is TermDF.compareTo's (TermDF.java:64-70): at the first
// differing component either a unit differs inside it, or one component is a
// prefix of the other and the shorter one meets U+0000, below every term unit
__global__ void k_gram_join_len(const int32_t *gram, int K, const int64_t *toff, int64_t V, int64_t *len) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t l = K - 1;
    for (int j = 0; j < K; j++) {
      const int64_t c = gram[t * K + j];
      l += toff[c + 1] - toff[c];
    }
    len[t] = l;
  }
}
__global__ void k_gram_join_write(const int32_t *gram, int K, const int64_t *toff, const uint16_t *tch, int64_t V,
                                  const int64_t *joff, uint16_t *jch) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    uint16_t *o = jch + joff[t];
    for (int j = 0; j < K; j++) {
      const int64_t c = gram[t * K + j];
      if (j > 0) *o++ = 0;
      for (int64_t i = toff[c]; i < toff[c + 1]; i++) *o++ = tch[i];
    }
  }
}
__global__ void k_owner_flags(const int32_t *owner, int64_t V, int o, uint8_t *f) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x)
    f[t] = owner[t] == o;
}
__global__ void k_sel_lens(const int32_t *sel, int64_t n, const int64_t *toff, const int64_t *off, int64_t *ulen,
                           int64_t *plen) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = sel[i];
    ulen[i] = toff[t + 1] - toff[t];
    plen[i] = off[t + 1] - off[t];
  }
}
// one wave per selected term: its units and postings into the blob
__global__ void k_pack_terms(const int32_t *sel, int64_t n, const int64_t *toff, const uint16_t *tch,
                             const int64_t *off, const int32_t *docno_o, const int32_t *tf_o, const int64_t *nuoff,
                             const int64_t *npoff, uint16_t *out_ch, int32_t *out_dn, int32_t *out_tf) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t i = blockIdx.x * wpb + (threadIdx.x >> 6); i < n; i += (int64_t)gridDim.x * wpb) {
    const int64_t t = sel[i];
    const int64_t u0 = toff[t], ul = toff[t + 1] - u0, p0 = off[t], pl = off[t + 1] - p0;
    for (int64_t k = lane; k < ul; k += 64) out_ch[nuoff[i] + k] = tch[u0 + k];
    for (int64_t k = lane; k < pl; k += 64) {
      out_dn[npoff[i] + k] = docno_o[p0 + k];
      out_tf[npoff[i] + k] = tf_o[p0 + k];
    }
  }
}

struct PieceDev {  // a received piece's term list (device pointers)
  const int64_t *toff;
  const uint16_t *tch;
  int64_t n;
};

// String.compareTo of units a[0, la) and b[0, lb)
__device__ __forceinline__ int cmp_units(const uint16_t *a, int64_t la, const uint16_t *b, int64_t lb) {
  const int64_t m = la < lb ? la : lb;
  for (int64_t i = 0; i < m; i++)
    if (a[i] != b[i]) return (int)a[i] - (int)b[i];
  return la < lb ? -1 : (la > lb ? 1 : 0);
}
// first index of piece p whose term is >= s (upper: > s)
__device__ int64_t piece_bound(const PieceDev &p, const uint16_t *s, int64_t ls, bool upper) {
  int64_t lo = 0, hi = p.n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    const int c = cmp_units(p.tch + p.toff[m], p.toff[m + 1] - p.toff[m], s, ls);
    if (c < 0 || (upper && c == 0))
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}
// rank of every term of every piece in the merged sequence (equal strings
// adjacent, in piece order); first: no earlier piece holds the string
__global__ void k_merge_rank(const PieceDev *pcs, int np, const int64_t *base, int64_t Vt, int64_t *pos,
                             uint8_t *first_at) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vt; j += (int64_t)gridDim.x * blockDim.x) {
    int a = 0;
    while (a + 1 < np && base[a + 1] <= j) a++;
    const int64_t i = j - base[a];
    const PieceDev &pa = pcs[a];
    const uint16_t *s = pa.tch + pa.toff[i];
    const int64_t ls = pa.toff[i + 1] - pa.toff[i];
    int64_t r = i;
    bool first = true;
    for (int b = 0; b < np; b++) {
      if (b == a || pcs[b].n == 0) continue;
      const int64_t lb = piece_bound(pcs[b], s, ls, false);
      if (b < a) {
        const int64_t ub = piece_bound(pcs[b], s, ls, true);
        r += ub;
        if (ub > lb) first = false;
      } else {
        r += lb;
      }
    }
    pos[j] = r;
    first_at[r] = first ? 1 : 0;
  }
}
__global__ void k_merge_scatter(const PieceDev *pcs, int np, const int64_t *base, const int64_t *post_base,
                                const int64_t *const *poff, int64_t Vt, const int64_t *pos, int64_t *at_pos,
                                int64_t *cnt_at_pos) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < Vt; j += (int64_t)gridDim.x * blockDim.x) {
    int a = 0;
    while (a + 1 < np && base[a + 1] <= j) a++;
    const int64_t i = j - base[a];
    at_pos[pos[j]] = j;
    cnt_at_pos[pos[j]] = poff[a][i + 1] - poff[a][i];
  }
}
// gid of every merged position: inclusive count of first flags - 1
__global__ void k_gid_at(const uint8_t *first_at, const int64_t *excl, int64_t Vt, int64_t *gid_at) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < Vt; p += (int64_t)gridDim.x * blockDim.x)
    gid_at[p] = excl[p] + first_at[p] - 1;
}
__global__ void k_first_flags_i64(const uint8_t *f, int64_t n, int64_t *v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = f[i];
}
// merged term strings: the first occurrence of every gid; term lengths
__global__ void k_gid_terms(const PieceDev *pcs, int np, const int64_t *base, const uint8_t *first_at,
                            const int64_t *at_pos, const int64_t *gid_at, int64_t Vt, int64_t *src_j, int64_t *glen) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < Vt; p += (int64_t)gridDim.x * blockDim.x) {
    if (!first_at[p]) continue;
    const int64_t j = at_pos[p];
    int a = 0;
    while (a + 1 < np && base[a + 1] <= j) a++;
    const int64_t i = j - base[a];
    src_j[gid_at[p]] = j;
    glen[gid_at[p]] = pcs[a].toff[i + 1] - pcs[a].toff[i];
  }
}
__global__ void k_gid_chars(const PieceDev *pcs, int np, const int64_t *base, const int64_t *src_j, int64_t V,
                            const int64_t *goff, uint16_t *gch) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t g = blockIdx.x * wpb + (threadIdx.x >> 6); g < V; g += (int64_t)gridDim.x * wpb) {
    const int64_t j = src_j[g];
    int a = 0;
    while (a + 1 < np && base[a + 1] <= j) a++;
    const int64_t i = j - base[a];
    const uint16_t *s = pcs[a].tch + pcs[a].toff[i];
    const int64_t l = goff[g + 1] - goff[g];
    for (int64_t k = lane; k < l; k += 64) gch[goff[g] + k] = s[k];
  }
}
// postings of every piece term into its merged slot: one wave per term
__global__ void k_merge_postings(int np, const int64_t *base, const int64_t *const *poff, const int32_t *const *pdn,
                                 const int32_t *const *ptf, int64_t Vt, const int64_t *pos, const int64_t *pstart_at,
                                 const int64_t *gid_at, int32_t *cdn, int32_t *ctf, uint32_t *cgid,
                                 unsigned int *max_tf) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  uint32_t m = 0;
  for (int64_t j = blockIdx.x * wpb + (threadIdx.x >> 6); j < Vt; j += (int64_t)gridDim.x * wpb) {
    int a = 0;
    while (a + 1 < np && base[a + 1] <= j) a++;
    const int64_t i = j - base[a];
    const int64_t p0 = poff[a][i], pl = poff[a][i + 1] - p0, d0 = pstart_at[pos[j]];
    const uint32_t g = (uint32_t)gid_at[pos[j]];
    for (int64_t k = lane; k < pl; k += 64) {
      const int32_t tf = ptf[a][p0 + k];
      cdn[d0 + k] = pdn[a][p0 + k];
      ctf[d0 + k] = tf;
      cgid[d0 + k] = g;
      m = max(m, (uint32_t)tf);
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  if (lane == 0 && m) atomicMax(max_tf, m);
}
__global__ void k_gid_offsets(const uint8_t *first_at, const int64_t *gid_at, const int64_t *pstart_at, int64_t Vt,
                              int64_t *off) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < Vt; p += (int64_t)gridDim.x * blockDim.x)
    if (first_at[p]) off[gid_at[p]] = pstart_at[p];
}
__global__ void k_keys_docno(const int32_t *dn, int64_t n, uint32_t *k, uint32_t *v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    k[i] = (uint32_t)dn[i] ^ 0x80000000u;  // signed order
    v[i] = (uint32_t)i;
  }
}
__global__ void k_keys_gid(const uint32_t *gid, const uint32_t *perm, int64_t n, uint32_t *k) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    k[i] = gid[perm[i]];
}
// after the (gid, docno) sort: run heads of equal (gid, docno)
__global__ void k_dup_heads(const uint32_t *perm, const uint32_t *gid, const int32_t *dn, int64_t n, uint8_t *head) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t x = perm[i];
    head[i] = i == 0 || gid[perm[i - 1]] != gid[x] || dn[perm[i - 1]] != dn[x];
  }
}
// MyReducer.reduce :202-210: equal docnos of a term become one posting, tf summed
__global__ void k_dup_merge(const uint32_t *perm, const uint32_t *gid, const int32_t *dn, const int32_t *tf,
                            const uint8_t *head, const int64_t *slot, int64_t n, uint32_t *ogid, int32_t *odn,
                            int32_t *otf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t x = perm[i];
    const int64_t s = slot[i] + head[i] - 1;
    if (head[i]) {
      ogid[s] = gid[x];
      odn[s] = dn[x];
    }
    atomicAdd(&otf[s], tf[x]);
  }
}
__global__ void k_count_gid(const uint32_t *gid, int64_t n, int64_t *off) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (i == 0 || gid[i] != gid[i - 1]) off[gid[i]] = i;
}
// (gid, tf desc) keys of the items in `perm` order (perm: nullptr = identity)
__global__ void k_keys_gid_tf(const uint32_t *gid, const int32_t *tf, const uint32_t *perm, int64_t n, int tfb,
                              uint32_t mtf, uint64_t *k, uint32_t *v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t x = perm ? perm[i] : (uint32_t)i;
    k[i] = ((uint64_t)gid[x] << tfb) | (uint64_t)(mtf - (uint32_t)tf[x]);
    v[i] = x;
  }
}
__global__ void k_gather_posts(const uint32_t *perm, const int32_t *dn, const int32_t *tf, int64_t n, int32_t *odn,
                               int32_t *otf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t x = perm[i];
    odn[i] = dn[x];
    otf[i] = tf[x];
  }
}
__global__ void k_max_i32(const int32_t *a, int64_t n, unsigned int *mx) {
  uint32_t m = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = max(m, (uint32_t)a[i]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}
__global__ void k_split_firsts(const int64_t *rbase, int np, int64_t N, uint8_t *first) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t f = 0;
    for (int a = 0; a < np; a++) f |= rbase[a] == i && rbase[a + 1] > i;
    first[i] = f;
  }
}

unsigned grid_n(int64_t n, int nt = 256, int cap = 16384) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + nt - 1) / nt, cap));
}
int bits_of(uint64_t v) {
  int b = 1;
  while (b < 64 && (1ull << b) <= v) b++;
  return b;
}
template <typename T>
T rd1(const T *d, hipStream_t st) {
  T h;
  SME_HIP(hipMemcpyAsync(&h, d, sizeof(T), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  return h;
}

}  // namespace

void pack_pieces(sme_index *ix, int world, uint8_t *d_out, uint64_t *sizes, hipStream_t st) {
  if (ix->job != 0 || ix->records_only) throw Error(SME_EINVAL, "reference-layout pieces need a TermKGramDocIndexer index");
  if (world < 1 || world > 65536) throw Error(SME_EINVAL, "world out of range");
  sme_ctx *cx = ix->ctx;
  auto &W = cx->ws;
  const int64_t V = ix->V;
  const int R = ix->R;
  const int part_sp = (31 + 32) % R;  // Arrays.hashCode({" "}), partition of the doc counter
  const int32_t sp_owner = part_sp % world;
  // the index terms' strings: the vocabulary (K = 1) or the grams' joined
  // component strings (K >= 2)
  const int64_t *toff = (const int64_t *)ix->d_term_off.p;
  const uint16_t *tch = (const uint16_t *)ix->d_term_chars.p;
  DevBuf jo, jc, jl;
  jo.pool = jc.pool = jl.pool = &cx->pool;
  if (ix->K > 1 && V > 0) {
    int64_t *len = jl.as<int64_t>(V + 1);
    int64_t *joff = jo.as<int64_t>(V + 1);
    hipLaunchKernelGGL(k_gram_join_len, dim3(grid_n(V)), dim3(256), 0, st, (const int32_t *)ix->d_gram.p, ix->K, toff,
                       V, len);
    SME_HIP(hipMemsetAsync(len + V, 0, sizeof(int64_t), st));
    excl_scan(len, joff, V + 1, W[9], st);
    const int64_t nu = rd1(joff + V, st);
    uint16_t *jch = jc.as<uint16_t>(nu + 1);
    hipLaunchKernelGGL(k_gram_join_write, dim3(grid_n(V)), dim3(256), 0, st, (const int32_t *)ix->d_gram.p, ix->K,
                       toff, tch, V, joff, jch);
    SME_CHECK_LAUNCH();
    toff = joff;
    tch = jch;
  }
  int32_t *owner = W[0].as<int32_t>(V + 1);
  if (V > 0)
    hipLaunchKernelGGL(k_term_owner, dim3(grid_n(V)), dim3(256), 0, st, toff, tch, V, R, world, owner);
  uint8_t *flag = W[1].as<uint8_t>(V + 1);
  int32_t *sel = W[2].as<int32_t>(V + 1);
  int32_t *d_n = W[3].as<int32_t>(4);
  int64_t *ulen = W[4].as<int64_t>(V + 2), *plen = W[5].as<int64_t>(V + 2);
  int64_t *uoff = W[6].as<int64_t>(V + 2), *poff = W[7].as<int64_t>(V + 2);
  int64_t at = 0;
  for (int o = 0; o < world; o++) {
    int64_t n = 0;
    if (V > 0) {
      hipLaunchKernelGGL(k_owner_flags, dim3(grid_n(V)), dim3(256), 0, st, owner, V, o, flag);
      select_flagged(flag, V, sel, d_n, W[8], W[9], st);
      n = rd1(d_n, st);
    }
    if (n > 0)
      hipLaunchKernelGGL(k_sel_lens, dim3(grid_n(n)), dim3(256), 0, st, sel, n, toff, (const int64_t *)ix->d_off.p,
                         ulen, plen);
    SME_HIP(hipMemsetAsync(ulen + n, 0, sizeof(int64_t), st));
    SME_HIP(hipMemsetAsync(plen + n, 0, sizeof(int64_t), st));
    excl_scan(ulen, uoff, n + 1, W[9], st);
    excl_scan(plen, poff, n + 1, W[9], st);
    PieceHdr h{};
    h.magic = kPieceMagic;
    h.nterms = n;
    h.nunits = rd1(uoff + n, st);
    h.npost = rd1(poff + n, st);
    h.nrec = o == sp_owner ? ix->N : 0;
    h.dmin = (int32_t)(ix->N > 0 ? ix->dmin : 1);
    h.dmax = (int32_t)(ix->N > 0 ? ix->dmax : 0);
    h.pad[0] = ix->K;  // components per term (joined by U+0000 when K >= 2)
    const PieceLayout L = layout_of(h);
    sizes[o] = (uint64_t)L.total;
    if (d_out) {
      uint8_t *b = d_out + at;
      SME_HIP(hipMemcpyAsync(b, &h, sizeof h, hipMemcpyHostToDevice, st));
      SME_HIP(hipMemcpyAsync(b + L.term_off, uoff, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
      SME_HIP(hipMemcpyAsync(b + L.post_off, poff, (n + 1) * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
      if (n > 0)
        hipLaunchKernelGGL(k_pack_terms, dim3(grid_n(n * 64)), dim3(256), 0, st, sel, n, toff, tch,
                           (const int64_t *)ix->d_off.p, (const int32_t *)ix->d_docno_o.p,
                           (const int32_t *)ix->d_tf_o.p, uoff, poff, (uint16_t *)(b + L.term_chars),
                           (int32_t *)(b + L.docno), (int32_t *)(b + L.tf));
      if (h.nrec > 0)
        SME_HIP(hipMemcpyAsync(b + L.rec, ix->d_rec_docno.p, h.nrec * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
      SME_CHECK_LAUNCH();
      SME_HIP(hipStreamSynchronize(st));  // the host header copy and the scratch are reused by the next owner
    }
    at += L.total;
  }
}

sme_index *merge_pieces(sme_ctx *cx, const uint8_t *d_blobs, const uint64_t *sizes, int np, hipStream_t st) {
  if (np < 1) throw Error(SME_EINVAL, "no pieces");
  auto &W = cx->ws;
  std::vector<PieceHdr> hd(np);
  std::vector<PieceLayout> lay(np);
  std::vector<const uint8_t *> bp(np);
  int64_t at = 0;
  for (int a = 0; a < np; a++) {
    bp[a] = d_blobs + at;
    SME_HIP(hipMemcpy(&hd[a], bp[a], sizeof(PieceHdr), hipMemcpyDeviceToHost));
    if (hd[a].magic != kPieceMagic) throw Error(SME_EINVAL, "not a piece blob (sme_index_pack_pieces)");
    lay[a] = layout_of(hd[a]);
    if ((uint64_t)lay[a].total != sizes[a]) throw Error(SME_EINVAL, "piece blob size mismatch");
    if (std::max<int64_t>(hd[a].pad[0], 1) != std::max<int64_t>(hd[0].pad[0], 1))
      throw Error(SME_EINVAL, "pieces of different k-gram lengths");
    at += lay[a].total;
  }
  std::vector<PieceDev> hp(np);
  std::vector<int64_t> base(np + 1, 0), pbase(np + 1, 0), rbase(np + 1, 0);
  std::vector<const int64_t *> hpoff(np);
  std::vector<const int32_t *> hpdn(np), hptf(np);
  bool ordered = true;  // record docno ranges disjoint and increasing with the piece index
  int64_t last_max = INT64_MIN;
  for (int a = 0; a < np; a++) {
    hp[a] = PieceDev{(const int64_t *)(bp[a] + lay[a].term_off), (const uint16_t *)(bp[a] + lay[a].term_chars),
                     hd[a].nterms};
    hpoff[a] = (const int64_t *)(bp[a] + lay[a].post_off);
    hpdn[a] = (const int32_t *)(bp[a] + lay[a].docno);
    hptf[a] = (const int32_t *)(bp[a] + lay[a].tf);
    base[a + 1] = base[a] + hd[a].nterms;
    pbase[a + 1] = pbase[a] + hd[a].npost;
    rbase[a + 1] = rbase[a] + hd[a].nrec;
    if (hd[a].dmin <= hd[a].dmax) {
      if ((int64_t)hd[a].dmin <= last_max) ordered = false;
      last_max = hd[a].dmax;
    }
  }
  const int64_t Vt = base[np], Pt = pbase[np], N = rbase[np];
  // small device tables of the pieces
  PieceDev *d_pcs = W[10].as<PieceDev>(np);
  int64_t *d_base = W[11].as<int64_t>(np + 1);
  const int64_t **d_poff = (const int64_t **)W[12].as<uint64_t>(np);
  const int32_t **d_pdn = (const int32_t **)W[13].as<uint64_t>(np);
  const int32_t **d_ptf = (const int32_t **)W[14].as<uint64_t>(np);
  int64_t *d_rbase = W[15].as<int64_t>(np + 1);
  SME_HIP(hipMemcpyAsync(d_pcs, hp.data(), np * sizeof(PieceDev), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_base, base.data(), (np + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_poff, hpoff.data(), np * sizeof(void *), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_pdn, hpdn.data(), np * sizeof(void *), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_ptf, hptf.data(), np * sizeof(void *), hipMemcpyHostToDevice, st));
  SME_HIP(hipMemcpyAsync(d_rbase, rbase.data(), (np + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));

  sme_index *ix = new sme_index(cx);
  std::unique_ptr<sme_index> guard(ix);
  // K >= 2: each merged term is a gram's joined component strings (no gram
  // table: the serializer splits the strings at U+0000)
  ix->K = (int)std::max<int64_t>(hd[0].pad[0], 1);
  ix->R = cx->cfg.num_partitions;
  ix->idf_mode = cx->cfg.idf_mode;
  ix->records_only = true;
  ix->N = N;
  // 1. merged vocabulary
  int64_t V = 0;
  int64_t *pos = W[16].as<int64_t>(Vt + 1);
  uint8_t *first_at = W[17].as<uint8_t>(Vt + 1);
  int64_t *at_pos = W[18].as<int64_t>(Vt + 1), *cnt_at = W[19].as<int64_t>(Vt + 1);
  int64_t *excl = W[20].as<int64_t>(Vt + 1), *gid_at = W[21].as<int64_t>(Vt + 1);
  int64_t *pstart = W[22].as<int64_t>(Vt + 1);
  if (Vt > 0) {
    hipLaunchKernelGGL(k_merge_rank, dim3(grid_n(Vt)), dim3(256), 0, st, d_pcs, np, d_base, Vt, pos, first_at);
    hipLaunchKernelGGL(k_merge_scatter, dim3(grid_n(Vt)), dim3(256), 0, st, d_pcs, np, d_base, (const int64_t *)nullptr,
                       d_poff, Vt, pos, at_pos, cnt_at);
    hipLaunchKernelGGL(k_first_flags_i64, dim3(grid_n(Vt)), dim3(256), 0, st, first_at, Vt, excl);
    excl_scan(excl, excl, Vt, W[23], st);
    hipLaunchKernelGGL(k_gid_at, dim3(grid_n(Vt)), dim3(256), 0, st, first_at, excl, Vt, gid_at);
    SME_CHECK_LAUNCH();
    V = rd1(gid_at + Vt - 1, st) + 1;
  }
  ix->V = ix->Vt = V;
  int64_t *term_off = ix->d_term_off.as<int64_t>(V + 1);
  if (V > 0) {
    int64_t *src_j = W[24].as<int64_t>(V + 1), *glen = W[25].as<int64_t>(V + 1);
    hipLaunchKernelGGL(k_gid_terms, dim3(grid_n(Vt)), dim3(256), 0, st, d_pcs, np, d_base, first_at, at_pos, gid_at, Vt,
                       src_j, glen);
    SME_HIP(hipMemsetAsync(glen + V, 0, sizeof(int64_t), st));
    excl_scan(glen, term_off, V + 1, W[23], st);
    const int64_t tchars = rd1(term_off + V, st);
    uint16_t *gch = ix->d_term_chars.as<uint16_t>(tchars + 1);
    hipLaunchKernelGGL(k_gid_chars, dim3(grid_n(V * 64)), dim3(256), 0, st, d_pcs, np, d_base, src_j, V, term_off, gch);
    SME_CHECK_LAUNCH();
  } else {
    SME_HIP(hipMemsetAsync(term_off, 0, sizeof(int64_t), st));
    ix->d_term_chars.get(16);
  }
  // 2. postings grouped by merged term (pieces in order inside a term)
  int64_t P = Pt;
  int64_t *off = ix->d_off.as<int64_t>(V + 1);
  int32_t *docno_o = nullptr, *tf_o = nullptr;
  int32_t mtf = 0;
  if (Pt > 0) {
    SME_HIP(hipMemsetAsync(cnt_at + Vt, 0, sizeof(int64_t), st));
    excl_scan(cnt_at, pstart, Vt + 1, W[23], st);
    int32_t *cdn = W[26].as<int32_t>(Pt), *ctf = W[27].as<int32_t>(Pt);
    uint32_t *cgid = W[28].as<uint32_t>(Pt);
    unsigned int *d_mtf = W[3].as<unsigned int>(4);
    SME_HIP(hipMemsetAsync(d_mtf, 0, sizeof(unsigned int), st));
    hipLaunchKernelGGL(k_merge_postings, dim3(grid_n(Vt * 64)), dim3(256), 0, st, np, d_base, d_poff, d_pdn, d_ptf, Vt,
                       pos, pstart, gid_at, cdn, ctf, cgid, d_mtf);
    SME_CHECK_LAUNCH();
    const uint32_t *perm = nullptr;  // item order so far (nullptr: the grouped order)
    uint32_t *k0 = W[29].as<uint32_t>(Pt), *k1 = W[30].as<uint32_t>(Pt);
    uint32_t *v0 = W[31].as<uint32_t>(Pt), *v1 = W[32].as<uint32_t>(Pt);
    uint32_t *rscr = W[33].as<uint32_t>(kv_sort_scratch(Pt) / sizeof(uint32_t) + 1);
    if (!ordered) {
      // MyReducer.reduce: sort by docno (stable), then by term -> (gid, docno); equal
      // (gid, docno) -- a docid duplicated across shards -- merge with tf summed
      hipLaunchKernelGGL(k_keys_docno, dim3(grid_n(Pt)), dim3(256), 0, st, cdn, Pt, k0, v0);
      uint32_t *pv = kv_sort<uint32_t>(k0, v0, k1, v1, Pt, 32, rscr, st);
      uint32_t *pk = pv == v0 ? k1 : k0;  // a free key buffer
      uint32_t *pv2 = pv == v0 ? v1 : v0;
      hipLaunchKernelGGL(k_keys_gid, dim3(grid_n(Pt)), dim3(256), 0, st, cgid, pv, Pt, pk);
      uint32_t *pk2 = pk == k0 ? k1 : k0;
      const uint32_t *srt = kv_sort<uint32_t>(pk, pv, pk2, pv2, Pt, bits_of((uint64_t)std::max<int64_t>(V, 1)), rscr, st);
      uint8_t *head = W[34].as<uint8_t>(Pt);
      int64_t *slot = W[35].as<int64_t>(Pt + 1);
      hipLaunchKernelGGL(k_dup_heads, dim3(grid_n(Pt)), dim3(256), 0, st, srt, cgid, cdn, Pt, head);
      hipLaunchKernelGGL(k_first_flags_i64, dim3(grid_n(Pt)), dim3(256), 0, st, head, Pt, slot);
      SME_HIP(hipMemsetAsync(slot + Pt, 0, sizeof(int64_t), st));
      excl_scan(slot, slot, Pt + 1, W[23], st);
      P = rd1(slot + Pt, st);
      uint32_t *mgid = W[36].as<uint32_t>(P);
      int32_t *mdn = W[37].as<int32_t>(P), *mtf2 = W[38].as<int32_t>(P);
      SME_HIP(hipMemsetAsync(mtf2, 0, P * sizeof(int32_t), st));
      hipLaunchKernelGGL(k_dup_merge, dim3(grid_n(Pt)), dim3(256), 0, st, srt, cgid, cdn, ctf, head, slot, Pt, mgid,
                         mdn, mtf2);
      SME_CHECK_LAUNCH();
      cgid = mgid;
      cdn = mdn;
      ctf = mtf2;
      SME_HIP(hipMemsetAsync(d_mtf, 0, sizeof(unsigned int), st));
      // max tf after merging, and the term offsets of the merged postings
      SME_HIP(hipMemsetAsync(off, 0, (V + 1) * sizeof(int64_t), st));
      hipLaunchKernelGGL(k_count_gid, dim3(grid_n(P)), dim3(256), 0, st, cgid, P, off);
      SME_CHECK_LAUNCH();
      hipLaunchKernelGGL(k_max_i32, dim3(grid_n(P)), dim3(256), 0, st, ctf, P, d_mtf);
      SME_CHECK_LAUNCH();
      mtf = (int32_t)rd1(d_mtf, st);
    } else {
      mtf = (int32_t)rd1(d_mtf, st);
      hipLaunchKernelGGL(k_gid_offsets, dim3(grid_n(Vt)), dim3(256), 0, st, first_at, gid_at, pstart, Vt, off);
    }
    SME_HIP(hipMemcpyAsync(off + V, &P, sizeof(int64_t), hipMemcpyHostToDevice, st));
    // stable by (term, tf desc): the reducer's final Collections.sort (:211)
    const int tfb = bits_of((uint64_t)std::max(mtf, 1));
    uint64_t *q0 = W[39].as<uint64_t>(P), *q1 = W[40].as<uint64_t>(P);
    hipLaunchKernelGGL(k_keys_gid_tf, dim3(grid_n(P)), dim3(256), 0, st, cgid, ctf, perm, P, tfb, (uint32_t)mtf, q0,
                       v0);
    const uint32_t *fin = kv_sort<uint64_t>(q0, v0, q1, v1, P, bits_of((uint64_t)std::max<int64_t>(V, 1)) + tfb, rscr,
                                            st);
    docno_o = ix->d_docno_o.as<int32_t>(P + 1);
    tf_o = ix->d_tf_o.as<int32_t>(P + 1);
    hipLaunchKernelGGL(k_gather_posts, dim3(grid_n(P)), dim3(256), 0, st, fin, cdn, ctf, P, docno_o, tf_o);
    SME_CHECK_LAUNCH();
  } else {
    SME_HIP(hipMemsetAsync(off, 0, (V + 1) * sizeof(int64_t), st));
    ix->d_docno_o.get(16);
    ix->d_tf_o.get(16);
  }
  ix->P = P;
  ix->max_tf = mtf;
  // 3. doc-counter postings: every piece's records, each map task's list from (0,0)
  int32_t *rdn = ix->d_rec_docno.as<int32_t>(N + 1);
  for (int a = 0; a < np; a++)
    if (hd[a].nrec > 0)
      SME_HIP(hipMemcpyAsync(rdn + rbase[a], bp[a] + lay[a].rec, hd[a].nrec * sizeof(int32_t),
                             hipMemcpyDeviceToDevice, st));
  if (N > 0) {
    uint8_t *fst = ix->d_rec_first.as<uint8_t>(N);
    hipLaunchKernelGGL(k_split_firsts, dim3(grid_n(N)), dim3(256), 0, st, d_rbase, np, N, fst);
    SME_CHECK_LAUNCH();
  }
  SME_HIP(hipStreamSynchronize(st));
  guard.release();
  return ix;
}

}  // namespace sme
