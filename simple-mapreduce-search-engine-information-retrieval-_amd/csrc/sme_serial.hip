// sme_serial.hip -- the reduce output as the reference writes it: per reducer
// partition, records in key order, framed as in a SequenceFile body
// (int32 recLen, int32 keyLen, key bytes, value bytes; big-endian).
//
//   partition  HashPartitioner: (TermDF.hashCode & MAX_VALUE) % R, TermDF.hashCode =
//              Arrays.hashCode(k_gram)                       C/sa/edu/kaust/io/TermDF.java:79-81
//   key        TermDF.write: int32 k, k x writeUTF, int32 df TermDF.java:50-56 (df = 1 for real
//              terms, N for " ": TermKGramDocIndexer.java:116,175-183)
//   value      ArrayListWritable.write: int32 n, writeUTF(class name), n x PostingWritable
//              C/edu/umd/cloud9/io/array/ArrayListWritable.java:90-105, PostingWritable.java:46-49
//   " " record postings: (0,0) then the previous record's (docno,1) for every later record
//              (the mapper's shared posting object, TermKGramDocIndexer.java:84-90,126,132-133)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sme_internal.hpp"

namespace sme {

constexpr int kClassLen = 31;

__device__ __forceinline__ int mutf8_unit_len(uint16_t c) { return (c >= 1 && c <= 0x7F) ? 1 : (c > 0x7FF ? 3 : 2); }

__device__ __forceinline__ void put_be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

// index term t has K components: the term ids gram[t*K ..] (K > 1 with a gram
// table), or -- gram == nullptr -- the segments of term t's own string split at
// U+0000 (K = 1: the whole string; a K >= 2 index merged from shard pieces
// stores each gram as its components joined by U+0000, sme_merge.hip).  f(units,
// length) is called per component in order.
template <typename F>
__device__ __forceinline__ void for_each_comp(const int64_t *toff, const uint16_t *tch, const int32_t *gram, int K,
                                              int64_t t, F f) {
  if (gram) {
    for (int j = 0; j < K; j++) {
      const int64_t c = gram[t * K + j];
      f(tch + toff[c], toff[c + 1] - toff[c]);
    }
    return;
  }
  const uint16_t *u = tch + toff[t];
  const int64_t l = toff[t + 1] - toff[t];
  int64_t s = 0;
  for (int64_t i = 0; i <= l; i++)
    if (i == l || u[i] == 0) {
      f(u + s, i - s);
      s = i + 1;
    }
}

// Partition byte totals are summed in LDS first (one global atomic per block
// and partition): with few partitions, per-term global atomics on R addresses
// serialise (24 ms for the 2 M terms of c2 at R = 1).
constexpr int kSerLdsParts = 1024;
__global__ __launch_bounds__(256) void k_ser_sizes(const int64_t *toff, const uint16_t *tch, const int32_t *gram, int K,
                                                   const int64_t *off, int64_t V, int R, int64_t *rec_bytes,
                                                   uint32_t *part, uint32_t *idx, unsigned long long *psum) {
  __shared__ unsigned long long s_ps[kSerLdsParts];
  const bool lds = R <= kSerLdsParts;
  if (lds)
    for (int i = threadIdx.x; i < R; i += blockDim.x) s_ps[i] = 0ull;
  __syncthreads();
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t ul = 0;
    uint32_t ah = 1u;  // Arrays.hashCode: 31 * h + String.hashCode per element, seed 1
    for_each_comp(toff, tch, gram, K, t, [&](const uint16_t *u, int64_t l) {
      uint32_t h = 0;
      for (int64_t i = 0; i < l; i++) {
        ul += mutf8_unit_len(u[i]);
        h = 31u * h + u[i];
      }
      ah = 31u * ah + h;
    });
    const int64_t df = off[t + 1] - off[t];
    const int64_t key = 4 + 2 * (int64_t)K + ul + 4;
    const int64_t val = 4 + (df > 0 ? 2 + kClassLen + 8 * df : 0);
    rec_bytes[t] = 8 + key + val;
    const uint32_t p = (uint32_t)((int32_t)(ah & 0x7fffffffu) % R);
    part[t] = p;
    idx[t] = (uint32_t)t;
    atomicAdd(lds ? &s_ps[p] : &psum[p], (unsigned long long)(8 + key + val));
  }
  if (lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += blockDim.x)
      if (s_ps[i]) atomicAdd(&psum[i], s_ps[i]);
  }
}

__global__ void k_ser_offsets(const uint32_t *grp_term, const int64_t *scan, int64_t V, const uint32_t *part,
                              uint32_t part_sp, int64_t sp_bytes, int64_t *rec_off) {
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < V; g += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t t = grp_term[g];
    rec_off[t] = scan[g] + (part[t] >= part_sp ? sp_bytes : 0);
  }
}

constexpr int64_t kSerBigDf = 8192;             // larger terms: posting stream in tiles (k_ser_big)
constexpr int64_t kSerTileBytes = 64 * 1024;    // stream bytes per tile

// Stream bytes [b0, b1) of a posting list's big-endian (docno, tf) words, at
// post + b0, written as aligned dwords: output dword at stream byte b = 4 f + s
// is v_alignbyte of the stream words f + 1 and f (each byte-swapped, so a
// little-endian store lays its bytes out big-endian); the unaligned head and
// tail bytes singly (byte stores of every posting cost 22 ms on c2).  Tiles of
// one stream meet on byte boundaries, so no byte is written twice.
__device__ __forceinline__ void ser_posts(uint8_t *post, const int32_t *dn, const int32_t *tf, int64_t b0, int64_t b1,
                                          int lane) {
  auto word = [&](int64_t f) -> uint32_t {
    const uint32_t v = (f & 1) ? (uint32_t)tf[f >> 1] : (uint32_t)dn[f >> 1];
    return __builtin_bswap32(v);
  };
  const int a = (int)((uintptr_t)(post + b0) & 3);
  const int64_t h = min((int64_t)((4 - a) & 3), b1 - b0);  // head bytes before the first aligned address
  if (lane < h) {
    const int64_t b = b0 + lane;
    post[b] = (uint8_t)(word(b >> 2) >> (8 * (b & 3)));
  }
  const int64_t s = b0 + h, nd = (b1 - s) >> 2;  // whole aligned dwords
  uint32_t *dst = reinterpret_cast<uint32_t *>(post + s);
  for (int64_t k = lane; k < nd; k += 64) {
    const int64_t b = s + 4 * k, f = b >> 2;
    const int sft = (int)(b & 3);
    dst[k] = sft == 0 ? word(f) : __builtin_amdgcn_alignbyte(word(f + 1), word(f), sft);
  }
  const int64_t t0 = s + 4 * nd;  // tail bytes
  if (lane < b1 - t0) {
    const int64_t b = t0 + lane;
    post[b] = (uint8_t)(word(b >> 2) >> (8 * (b & 3)));
  }
}

// big terms (df > kSerBigDf): tile counts and the byte offset of the posting
// stream inside the record
__global__ void k_ser_bigflags(const int64_t *off, int64_t V, uint8_t *f) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < V; t += (int64_t)gridDim.x * blockDim.x)
    f[t] = off[t + 1] - off[t] > kSerBigDf;
}
__global__ void k_ser_bigtiles(const int32_t *big, int64_t nbig, const int64_t *off, const int64_t *toff,
                               const uint16_t *tch, const int32_t *gram, int K, int64_t *ntile, int64_t *post_rel) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nbig; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = big[j], df = off[t + 1] - off[t];
    ntile[j] = (8 * df + kSerTileBytes - 1) / kSerTileBytes;
    int64_t ul = 0;
    for_each_comp(toff, tch, gram, K, t, [&](const uint16_t *u, int64_t l) {
      for (int64_t i = 0; i < l; i++) ul += mutf8_unit_len(u[i]);
    });
    post_rel[j] = 8 + (4 + 2 * (int64_t)K + ul + 4) + 4 + 2 + kClassLen;
  }
}

// one wave per index term
__global__ void k_ser_write(const int64_t *toff, const uint16_t *tch, const int32_t *gram, int K, const int64_t *off,
                            const int32_t *docno_o, const int32_t *tf_o, int64_t V, const int64_t *rec_off,
                            uint8_t *out) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t t = blockIdx.x * wpb + (threadIdx.x >> 6); t < V; t += (int64_t)gridDim.x * wpb) {
    const int64_t p0 = off[t], df = off[t + 1] - off[t];
    uint8_t *o = out + rec_off[t];
    // K = 1 and an all-ASCII term (every c2 / c5 term): each modified-UTF-8 byte
    // is one unit, and the lanes write the record header one byte each (a lane-0
    // byte loop per term cost most of the pass on c5's 8.9 M short terms)
    bool ascii = K == 1;
    if (ascii) {
      for (int64_t i = toff[t] + lane; i < toff[t + 1]; i += 64) ascii &= tch[i] >= 1 && tch[i] <= 0x7F;
      ascii = __all(ascii);
    }
    int64_t ul = 0;
    if (ascii) {
      ul = toff[t + 1] - toff[t];
    } else {
      for_each_comp(toff, tch, gram, K, t, [&](const uint16_t *u, int64_t l) {
        for (int64_t i = 0; i < l; i++) ul += mutf8_unit_len(u[i]);
      });
    }
    const int64_t key = 4 + 2 * (int64_t)K + ul + 4, val = 4 + (df > 0 ? 2 + kClassLen + 8 * df : 0);
    uint8_t *post = o + 8 + key + 4 + 2 + kClassLen;
    if (ascii) {
      const int64_t hdr = 14 + ul + 8 + (df > 0 ? 2 + kClassLen : 0);
      const uint16_t *u = tch + toff[t];
      for (int64_t j = lane; j < hdr; j += 64) {
        uint32_t b;
        auto be = [](uint32_t v, int64_t i) { return (v >> (8 * (3 - i))) & 0xFFu; };
        if (j < 4) b = be((uint32_t)(key + val), j);
        else if (j < 8) b = be((uint32_t)key, j - 4);
        else if (j < 12) b = be(1u, j - 8);
        else if (j < 14) b = j == 12 ? (uint32_t)(ul >> 8) & 0xFFu : (uint32_t)ul & 0xFFu;
        else if (j < 14 + ul) b = u[j - 14];
        else {
          const int64_t q = j - 14 - ul;
          if (q < 4) b = be(1u, q);  // stored df of a real term (T1)
          else if (q < 8) b = be((uint32_t)df, q - 4);
          else if (q == 8) b = 0;
          else if (q == 9) b = (uint32_t)kClassLen;
          else b = (uint8_t)"sa.edu.kaust.io.PostingWritable"[q - 10];
        }
        o[j] = (uint8_t)b;
      }
    } else if (lane == 0) {
      put_be32(o, (uint32_t)(key + val));
      put_be32(o + 4, (uint32_t)key);
      put_be32(o + 8, (uint32_t)K);
      uint8_t *q = o + 12;
      for_each_comp(toff, tch, gram, K, t, [&](const uint16_t *u, int64_t l) {  // writeUTF per element
        int64_t el = 0;
        for (int64_t i = 0; i < l; i++) el += mutf8_unit_len(u[i]);
        q[0] = (uint8_t)(el >> 8);
        q[1] = (uint8_t)el;
        q += 2;
        for (int64_t i = 0; i < l; i++) {
          uint16_t ch = u[i];
          if (ch >= 1 && ch <= 0x7F) {
            *q++ = (uint8_t)ch;
          } else if (ch > 0x7FF) {
            *q++ = (uint8_t)(0xE0 | ((ch >> 12) & 0x0F));
            *q++ = (uint8_t)(0x80 | ((ch >> 6) & 0x3F));
            *q++ = (uint8_t)(0x80 | (ch & 0x3F));
          } else {
            *q++ = (uint8_t)(0xC0 | ((ch >> 6) & 0x1F));
            *q++ = (uint8_t)(0x80 | (ch & 0x3F));
          }
        }
      });
      put_be32(q, 1u);  // stored df of a real term (T1)
      put_be32(q + 4, (uint32_t)df);
      if (df > 0) {
        q[8] = 0;
        q[9] = (uint8_t)kClassLen;
        for (int i = 0; i < kClassLen; i++) q[10 + i] = (uint8_t)"sa.edu.kaust.io.PostingWritable"[i];
      }
    }
    // postings: this wave writes those of small terms; a large term's stream is
    // cut into tiles written by many waves (k_ser_big), so one wave does not
    // write a 1 M-posting list alone (that tail cost c2 most of the pass)
    if (df > 0 && df <= kSerBigDf) ser_posts(post, docno_o + p0, tf_o + p0, 0, 8 * df, lane);
  }
}

// tiles of the large terms' posting streams: tile i of big term j covers stream
// bytes [i, i + 1) x kSerTileBytes (clamped); tile_off = exclusive scan of the
// terms' tile counts
__global__ void k_ser_big(const int32_t *big, int64_t nbig, const int64_t *tile_off, const int64_t *off,
                          const int32_t *docno_o, const int32_t *tf_o, const int64_t *rec_off,
                          const int64_t *post_rel, uint8_t *out) {
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64, ntiles = tile_off[nbig];
  for (int64_t x = blockIdx.x * wpb + (threadIdx.x >> 6); x < ntiles; x += (int64_t)gridDim.x * wpb) {
    int64_t lo = 0, hi = nbig;  // last j with tile_off[j] <= x
    while (hi - lo > 1) {
      const int64_t m = (lo + hi) >> 1;
      if (tile_off[m] <= x) lo = m;
      else hi = m;
    }
    const int64_t t = big[lo], p0 = off[t], nb = 8 * (off[t + 1] - p0);
    const int64_t b0 = (x - tile_off[lo]) * kSerTileBytes, b1 = min(nb, b0 + kSerTileBytes);
    ser_posts(out + rec_off[t] + post_rel[lo], docno_o + p0, tf_o + p0, b0, b1, lane);
  }
}

__global__ void k_ser_space(const int32_t *rec_docno, const uint8_t *first, int64_t N, uint8_t *o) {
  // key: k=1, writeUTF(" "), df = N ; value: n = N, class, postings
  const int64_t key = 11, val = 4 + 2 + kClassLen + 8 * N;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    put_be32(o, (uint32_t)(key + val));
    put_be32(o + 4, (uint32_t)key);
    put_be32(o + 8, 1u);
    o[12] = 0;
    o[13] = 1;
    o[14] = ' ';
    put_be32(o + 15, (uint32_t)N);
    put_be32(o + 19, (uint32_t)N);
    o[23] = 0;
    o[24] = (uint8_t)kClassLen;
    for (int i = 0; i < kClassLen; i++) o[25 + i] = (uint8_t)"sa.edu.kaust.io.PostingWritable"[i];
  }
  uint8_t *post = o + 25 + kClassLen;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
    // every map task's list starts with the fresh (0, 0) posting (merged shard
    // pieces: several tasks, `first` marks their first records)
    const bool f = i == 0 || (first && first[i]);
    put_be32(post + 8 * i, f ? 0u : (uint32_t)rec_docno[i - 1]);
    put_be32(post + 8 * i + 4, f ? 0u : 1u);
  }
}

__global__ void k_gather_bytes(const uint32_t *g, const int64_t *rb, int64_t n, int64_t *gb) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gb[i] = rb[g[i]];
}

void serialize_index(sme_index *ix, hipStream_t st) {
  if (ix->ser_ready) return;
  auto &W = ix->ctx->ws;
  const int64_t V = ix->V, N = ix->N;
  const int R = ix->R;
  const int32_t *gram = ix->K > 1 ? (const int32_t *)ix->d_gram.p : nullptr;
  int64_t *rec_bytes = W[48].as<int64_t>(V + 1);
  uint32_t *part = W[49].as<uint32_t>(V + 1), *idx = W[50].as<uint32_t>(V + 1);
  uint32_t *part2 = W[51].as<uint32_t>(V + 1), *idx2 = W[52].as<uint32_t>(V + 1);
  int64_t *grp_bytes = W[53].as<int64_t>(V + 1), *scan = W[54].as<int64_t>(V + 1);
  unsigned long long *psum = W[55].as<unsigned long long>(R + 1);
  // device time of the pass (sizes + partition sort + writes; the host reads the
  // partition sizes in between, so the two legs are timed separately)
  hipEvent_t ev[4];
  for (auto &e : ev) SME_HIP(hipEventCreate(&e));
  SME_HIP(hipEventRecord(ev[0], st));
  SME_HIP(hipMemsetAsync(psum, 0, (R + 1) * sizeof(unsigned long long), st));
  const int G = (int)std::min<int64_t>(std::max<int64_t>((V + 255) / 256, 1), 8192);
  if (V > 0)
    hipLaunchKernelGGL(k_ser_sizes, dim3(G), dim3(256), 0, st, (const int64_t *)ix->d_term_off.p,
                       (const uint16_t *)ix->d_term_chars.p, gram, ix->K, (const int64_t *)ix->d_off.p, V, R, rec_bytes,
                       part, idx, psum);
  SME_CHECK_LAUNCH();
  SME_HIP(hipEventRecord(ev[1], st));
  std::vector<unsigned long long> hps(R + 1);
  SME_HIP(hipMemcpyAsync(hps.data(), psum, (R + 1) * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  SME_HIP(hipStreamSynchronize(st));
  const uint32_t part_sp = (uint32_t)((31 + 32) % R);  // Arrays.hashCode({" "}) = 31 + 32
  const int64_t sp_bytes = N > 0 ? 8 + 11 + 4 + 2 + kClassLen + 8 * N : 0;
  ix->part_start.assign(R + 1, 0);
  for (int p = 0; p < R; p++) {
    ix->part_start[p + 1] = ix->part_start[p] + (int64_t)hps[p] + (p == (int)part_sp ? sp_bytes : 0);
  }
  const int64_t total = ix->part_start[R];
  uint8_t *out = ix->d_ser.as<uint8_t>(total + 16);
  SME_HIP(hipEventRecord(ev[2], st));
  if (V > 0) {
    int bits = 1;
    while ((1 << bits) < R) bits++;
    // terms grouped by partition, term order kept (stable LSD radix, sme_sort.hip);
    // the sort runs on a copy of the partition ids (part stays per term)
    uint32_t *pk = W[21].as<uint32_t>(V + 1);
    SME_HIP(hipMemcpyAsync(pk, part, V * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    uint32_t *rscr = W[20].as<uint32_t>(kv_sort_scratch(V) / sizeof(uint32_t) + 1);
    uint32_t *grp = kv_sort<uint32_t>(pk, idx, part2, idx2, V, bits, rscr, st, false);
    idx2 = grp;
    hipLaunchKernelGGL(k_gather_bytes, dim3(G), dim3(256), 0, st, idx2, rec_bytes, V, grp_bytes);
    excl_scan<int64_t>(grp_bytes, scan, V, W[22], st);
    int64_t *rec_off = grp_bytes;  // reuse after scan
    hipLaunchKernelGGL(k_ser_offsets, dim3(G), dim3(256), 0, st, idx2, scan, V, part, part_sp, sp_bytes, rec_off);
    hipLaunchKernelGGL(k_ser_write, dim3((unsigned)std::min<int64_t>((V + 3) / 4, 65536)), dim3(256), 0, st,
                       (const int64_t *)ix->d_term_off.p, (const uint16_t *)ix->d_term_chars.p, gram, ix->K,
                       (const int64_t *)ix->d_off.p, (const int32_t *)ix->d_docno_o.p, (const int32_t *)ix->d_tf_o.p,
                       V, rec_off, out);
    SME_CHECK_LAUNCH();
    // the large terms' posting streams, in tiles
    uint8_t *bflag = W[24].as<uint8_t>(V + 1);
    int32_t *big = W[25].as<int32_t>(V + 1), *d_nbig = W[30].as<int32_t>(4);
    hipLaunchKernelGGL(k_ser_bigflags, dim3(G), dim3(256), 0, st, (const int64_t *)ix->d_off.p, V, bflag);
    select_flagged(bflag, V, big, d_nbig, W[29], W[23], st);
    int32_t nbig = 0;
    SME_HIP(hipMemcpyAsync(&nbig, d_nbig, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    if (nbig > 0) {
      int64_t *ntile = W[26].as<int64_t>(nbig + 1), *tile_off = W[27].as<int64_t>(nbig + 1);
      int64_t *post_rel = W[28].as<int64_t>(nbig + 1);
      hipLaunchKernelGGL(k_ser_bigtiles, dim3((unsigned)std::min<int64_t>((nbig + 255) / 256, 4096)), dim3(256), 0, st,
                         big, (int64_t)nbig, (const int64_t *)ix->d_off.p, (const int64_t *)ix->d_term_off.p,
                         (const uint16_t *)ix->d_term_chars.p, gram, ix->K, ntile, post_rel);
      SME_HIP(hipMemsetAsync(ntile + nbig, 0, sizeof(int64_t), st));
      excl_scan<int64_t>(ntile, tile_off, nbig + 1, W[23], st);
      hipLaunchKernelGGL(k_ser_big, dim3(8192), dim3(256), 0, st, big, (int64_t)nbig, tile_off,
                         (const int64_t *)ix->d_off.p, (const int32_t *)ix->d_docno_o.p, (const int32_t *)ix->d_tf_o.p,
                         rec_off, post_rel, out);
      SME_CHECK_LAUNCH();
    }
  }
  if (N > 0) {
    hipLaunchKernelGGL(k_ser_space, dim3((unsigned)std::min<int64_t>((N + 255) / 256, 8192)), dim3(256), 0, st,
                       (const int32_t *)ix->d_rec_docno.p, (const uint8_t *)ix->d_rec_first.p, N,
                       out + ix->part_start[part_sp]);
    SME_CHECK_LAUNCH();
  }
  SME_HIP(hipEventRecord(ev[3], st));
  SME_HIP(hipStreamSynchronize(st));
  float m0 = 0, m1 = 0;
  SME_HIP(hipEventElapsedTime(&m0, ev[0], ev[1]));
  SME_HIP(hipEventElapsedTime(&m1, ev[2], ev[3]));
  for (auto &e : ev) (void)hipEventDestroy(e);
  ix->ser_ms = m0 + m1;
  ix->ser_ready = true;
  ix->h_parts.clear();
  ix->h_parts.resize((size_t)R);
  ix->h_parts_ready.assign(R, 0);
}

}  // namespace sme
