// sme_api.hip -- the C-ABI (include/sme.h).  Every entry point converts
// sme::Error / std::exception into a negative status and a thread-local message.
#include <hip/hip_runtime.h>
#include <string.h>

#include <sstream>
#include <string>
#include <vector>

#include <algorithm>
#include <system_error>
#include <thread>

#include "sme_internal.hpp"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

template <typename F>
int guard(F &&f) {
  try {
    f();
    g_err.clear();
    return SME_OK;
  } catch (const sme::Error &e) {
    return fail(e.code, e.what());
  } catch (const std::bad_alloc &) {
    return fail(SME_ENOMEM, "host allocation failed");
  } catch (const std::exception &e) {
    return fail(SME_EINVAL, e.what());
  }
}

hipStream_t stream_of(sme_ctx *cx, void *s) { return s ? (hipStream_t)s : cx->own_stream; }

// merged shard pieces (sme_merge_pieces) hold the reduce output only
void need_query_side(const sme_index *ix) {
  if (ix->records_only)
    throw sme::Error(SME_EINVAL, "records-only index (merged shard pieces): query the shard indexes");
}

void set_device(sme_ctx *cx) { SME_HIP(hipSetDevice(cx->device)); }

// DataInput.readUTF body -> UTF-16
bool read_mutf8(const uint8_t *p, size_t len, std::vector<uint16_t> &out) {
  size_t i = 0;
  while (i < len) {
    unsigned c = p[i];
    if (c < 0x80) {
      out.push_back((uint16_t)c);
      i++;
    } else if ((c & 0xE0) == 0xC0) {
      if (i + 1 >= len) return false;
      out.push_back((uint16_t)(((c & 0x1F) << 6) | (p[i + 1] & 0x3F)));
      i += 2;
    } else if ((c & 0xF0) == 0xE0) {
      if (i + 2 >= len) return false;
      out.push_back((uint16_t)(((c & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F)));
      i += 3;
    } else {
      return false;
    }
  }
  return true;
}

// standard UTF-8 -> UTF-16 (API inputs of already-processed terms)
std::vector<uint16_t> utf8_to_u16(const uint8_t *p, size_t n) {
  std::vector<uint16_t> o;
  size_t i = 0;
  while (i < n) {
    unsigned c = p[i];
    unsigned cp;
    int extra;
    if (c < 0x80) {
      cp = c;
      extra = 0;
    } else if ((c & 0xE0) == 0xC0) {
      cp = c & 0x1F;
      extra = 1;
    } else if ((c & 0xF0) == 0xE0) {
      cp = c & 0x0F;
      extra = 2;
    } else {
      cp = c & 0x07;
      extra = 3;
    }
    i++;
    for (int k = 0; k < extra && i < n; k++, i++) cp = (cp << 6) | (p[i] & 0x3F);
    if (cp >= 0x10000) {
      cp -= 0x10000;
      o.push_back((uint16_t)(0xD800 + (cp >> 10)));
      o.push_back((uint16_t)(0xDC00 + (cp & 0x3FF)));
    } else {
      o.push_back((uint16_t)cp);
    }
  }
  return o;
}

// DataOutput.writeUTF body of UTF-16 units
void u16_to_mutf8(const uint16_t *u, size_t n, std::vector<uint8_t> &o) {
  for (size_t i = 0; i < n; i++) {
    uint16_t c = u[i];
    if (c >= 1 && c <= 0x7F) {
      o.push_back((uint8_t)c);
    } else if (c > 0x7FF) {
      o.push_back((uint8_t)(0xE0 | ((c >> 12) & 0x0F)));
      o.push_back((uint8_t)(0x80 | ((c >> 6) & 0x3F)));
      o.push_back((uint8_t)(0x80 | (c & 0x3F)));
    } else {
      o.push_back((uint8_t)(0xC0 | ((c >> 6) & 0x1F)));
      o.push_back((uint8_t)(0x80 | (c & 0x3F)));
    }
  }
}

void ensure_host_terms(sme_index *ix) {
  if (ix->h_terms_ready) return;
  const int64_t Vt = ix->Vt;
  ix->h_term_off.resize(Vt + 1);
  SME_HIP(hipMemcpy(ix->h_term_off.data(), ix->d_term_off.p, (Vt + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  ix->h_term_chars.resize(ix->h_term_off[Vt] + 1);
  if (ix->h_term_off[Vt] > 0)
    SME_HIP(hipMemcpy(ix->h_term_chars.data(), ix->d_term_chars.p, ix->h_term_off[Vt] * sizeof(uint16_t),
                      hipMemcpyDeviceToHost));
  if (ix->K > 1 && ix->V > 0 && ix->d_gram.p) {  // (a merged K >= 2 index holds joined gram strings instead)
    ix->h_gram.resize((size_t)(ix->V * ix->K));
    SME_HIP(hipMemcpy(ix->h_gram.data(), ix->d_gram.p, ix->h_gram.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  ix->h_terms_ready = true;
}

// Device -> host copy of n bytes at d into dst.  Pinned dst (hipHostMalloc /
// hipHostRegister memory): one DMA.  Pageable dst: 64 MiB chunks DMA'd into
// the context's two pinned staging buffers while the host copies the previous
// chunk out of the other buffer, spread over up to 8 threads (one host thread
// moves ~10 GB/s; PCIe Gen5 x16 ~50 GB/s).  A plain pageable hipMemcpy of the
// c2 record stream ran at ~2 GB/s.
void copy_d2h(sme_ctx *cx, void *dst, const void *d, size_t n, hipStream_t st) {
  if (!n) return;
  hipPointerAttribute_t at{};
  bool pinned = false;
  if (hipPointerGetAttributes(&at, dst) == hipSuccess)
    pinned = at.type == hipMemoryTypeHost;
  else
    (void)hipGetLastError();  // pageable memory: not an error for the caller
  if (pinned) {
    SME_HIP(hipMemcpyAsync(dst, d, n, hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
    return;
  }
  constexpr size_t kStage = size_t(64) << 20;
  if (!cx->h_stage[0]) {
    for (auto &b : cx->h_stage) SME_HIP(hipHostMalloc(&b, kStage, hipHostMallocDefault));
    cx->h_stage_cap = kStage;
  }
  hipEvent_t ev[2];
  for (auto &e : ev) SME_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const size_t nch = (n + kStage - 1) / kStage;
  auto issue = [&](size_t c) {
    const size_t o = c * kStage, len = std::min(kStage, n - o);
    SME_HIP(hipMemcpyAsync(cx->h_stage[c & 1], (const uint8_t *)d + o, len, hipMemcpyDeviceToHost, st));
    SME_HIP(hipEventRecord(ev[c & 1], st));
  };
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const unsigned nth = std::min(8u, hw);
  try {
    issue(0);
    for (size_t c = 0; c < nch; c++) {
      SME_HIP(hipEventSynchronize(ev[c & 1]));
      if (c + 1 < nch) issue(c + 1);  // the other buffer's chunk was copied out last iteration
      const size_t o = c * kStage, len = std::min(kStage, n - o);
      const uint8_t *src = (const uint8_t *)cx->h_stage[c & 1];
      uint8_t *out = (uint8_t *)dst + o;
      const unsigned t = len >= (size_t(8) << 20) ? nth : 1u;
      const size_t per = (len + t - 1) / t;
      std::vector<std::thread> th;
      struct Joiner {  // joins every started thread on any exit (a joinable std::thread's destructor aborts)
        std::vector<std::thread> &v;
        ~Joiner() {
          for (auto &x : v)
            if (x.joinable()) x.join();
        }
      } joiner{th};
      for (unsigned i = 1; i < t; i++) {
        const size_t lo = std::min(len, i * per), hi = std::min(len, lo + per);
        if (hi <= lo) continue;
        try {
          th.emplace_back([=] { memcpy(out + lo, src + lo, hi - lo); });
        } catch (const std::system_error &) {  // no thread (EAGAIN): copy this slice here
          memcpy(out + lo, src + lo, hi - lo);
        }
      }
      memcpy(out, src, std::min(len, per));
    }
  } catch (...) {
    (void)hipStreamSynchronize(st);
    for (auto &e : ev) (void)hipEventDestroy(e);
    throw;
  }
  for (auto &e : ev) (void)hipEventDestroy(e);
}
}  // namespace

extern "C" {

const char *sme_last_error(void) { return g_err.c_str(); }

int sme_device_alloc(int device, size_t n, void **d) {
  return guard([&] {
    if (!d) throw sme::Error(SME_EINVAL, "null argument");
    SME_HIP(hipSetDevice(device));
    *d = nullptr;
    SME_HIP(hipMalloc(d, n ? n : 16));
  });
}

void sme_device_free(void *d) {
  if (d) (void)hipFree(d);
}

int sme_memcpy(void *dst, const void *src, size_t n, void *stream) {
  return guard([&] {
    if (n == 0) return;
    if (!dst || !src) throw sme::Error(SME_EINVAL, "null argument");
    if (stream)
      SME_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, (hipStream_t)stream));
    else
      SME_HIP(hipMemcpy(dst, src, n, hipMemcpyDefault));
  });
}
const char *sme_version(void) { return "sme 0.1 (gfx950)"; }

int sme_create(const sme_config *cfg, sme_ctx **out) {
  return guard([&] {
    if (!cfg || !out) throw sme::Error(SME_EINVAL, "null argument");
    if (cfg->k < 1) throw sme::Error(SME_EINVAL, "k must be >= 1");
    if (cfg->num_partitions < 1) throw sme::Error(SME_EINVAL, "num_partitions must be >= 1");
    if (cfg->idf_mode != SME_IDF_REFERENCE && cfg->idf_mode != SME_IDF_TRUE_DF)
      throw sme::Error(SME_EINVAL, "bad idf_mode");
    if (cfg->tiebreak != SME_TIE_DOCNO && cfg->tiebreak != SME_TIE_REFERENCE && cfg->tiebreak != SME_TIE_JAVA7)
      throw sme::Error(SME_EINVAL, "bad tiebreak");
    int ndev = 0;
    SME_HIP(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev) throw sme::Error(SME_EINVAL, "bad device ordinal");
    sme_ctx *cx = new sme_ctx();
    cx->cfg = *cfg;
    cx->device = cfg->device;
    try {
      set_device(cx);
      SME_HIP(hipStreamCreateWithFlags(&cx->own_stream, hipStreamNonBlocking));
      SME_HIP(hipStreamCreateWithFlags(&cx->aux_stream, hipStreamNonBlocking));
      SME_HIP(hipEventCreateWithFlags(&cx->ev_fork, hipEventDisableTiming));
      SME_HIP(hipEventCreateWithFlags(&cx->ev_join, hipEventDisableTiming));
    } catch (...) {
      delete cx;
      throw;
    }
    *out = cx;
  });
}

int sme_set_option(sme_ctx *cx, const char *name, int64_t v) {
  return guard([&] {
    if (!cx || !name) throw sme::Error(SME_EINVAL, "null argument");
    const std::string n(name);
    auto range = [&](int64_t lo, int64_t hi) {
      if (v < lo || v > hi) throw sme::Error(SME_EINVAL, "option " + n + " out of range");
    };
    if (n == "query_kernel") {
      range(0, 2);
      cx->opt_query_kernel = v;
    } else if (n == "heavy_div") {
      range(0, int64_t(1) << 40);
      cx->opt_heavy_div = v;
    } else if (n == "seed_tiles") {
      range(0, 8);
      cx->opt_seed_tiles = v;
    } else if (n == "query_order") {
      range(0, 1);
      cx->opt_query_order = v;
    } else if (n == "agg_two_pass") {
      range(0, 1);
      cx->opt_agg_two_pass = v;
    } else if (n == "agg_grid") {
      range(0, int64_t(1) << 30);
      cx->opt_agg_grid = v;
    } else if (n == "tok_grid") {
      range(1, int64_t(1) << 30);
      cx->opt_tok_grid = v;
    } else if (n == "cand_cap") {
      range(1, 2048);
      cx->opt_cand_cap = v;
    } else if (n == "win_sample") {
      range(0, 1);
      cx->opt_win_sample = v;
    } else if (n == "win_stage_min") {
      range(0, int64_t(1) << 20);
      cx->opt_win_stage_min = v;
    } else if (n == "kgram_rank") {
      range(0, 1);
      cx->opt_kgram_rank = v;
    } else if (n == "win_slice") {
      range(0, int64_t(1) << 30);
      cx->opt_win_slice = v;
    } else if (n == "seed_m") {
      range(0, 4096);
      cx->opt_seed_m = v;
    } else if (n == "query_table_budget") {
      range(0, int64_t(1) << 50);
      cx->opt_query_budget = v;
    } else if (n == "corpus_keep_bytes") {
      range(0, int64_t(1) << 50);
      cx->opt_corpus_keep = v;
    } else if (n == "raw_load_pct") {
      range(10, 90);
      cx->opt_raw_load_pct = v;
    } else if (n == "docid_terms") {
      range(0, 1);
      cx->opt_docid_terms = v;
    } else if (n == "sort_digit_bits") {
      if (v != 0) range(6, 11);
      cx->opt_sort_bits = v;
    } else if (n == "docid_split") {
      range(0, 2);
      cx->opt_docid_split = v;
    } else {
      throw sme::Error(SME_EINVAL, "unknown option " + n);
    }
  });
}

static void ctx_release(sme_ctx *cx) {
  (void)hipSetDevice(cx->device);
  (void)hipDeviceSynchronize();
  if (cx->own_stream) (void)hipStreamDestroy(cx->own_stream);
  if (cx->aux_stream) (void)hipStreamDestroy(cx->aux_stream);
  if (cx->ev_fork) (void)hipEventDestroy(cx->ev_fork);
  if (cx->ev_join) (void)hipEventDestroy(cx->ev_join);
  for (hipEvent_t e : cx->prof_events) (void)hipEventDestroy(e);
  for (auto &b : cx->h_stage)
    if (b) (void)hipHostFree(b);
  delete cx;
}

void sme_destroy(sme_ctx *cx) {
  if (!cx) return;
  cx->destroyed = true;
  if (cx->live_indexes == 0) ctx_release(cx);
}

int sme_load_docno_mapping(sme_ctx *cx, const uint8_t *m, size_t n) {
  return guard([&] {
    if (!cx || (!m && n)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    if (n < 4) throw sme::Error(SME_EINVAL, "mapping file shorter than its int32 count");
    int32_t cnt = (int32_t)(((uint32_t)m[0] << 24) | ((uint32_t)m[1] << 16) | ((uint32_t)m[2] << 8) | m[3]);
    if (cnt < 0) throw sme::Error(SME_EINVAL, "negative mapping count");
    std::vector<uint16_t> chars;
    std::vector<int64_t> off;
    off.push_back(0);
    off.push_back(0);  // "" sentinel at index 0 (readDocnoData)
    size_t p = 4;
    for (int32_t i = 0; i < cnt; i++) {
      if (p + 2 > n) throw sme::Error(SME_EINVAL, "truncated mapping file");
      size_t l = ((size_t)m[p] << 8) | m[p + 1];
      p += 2;
      if (p + l > n) throw sme::Error(SME_EINVAL, "truncated mapping file");
      if (!read_mutf8(m + p, l, chars)) throw sme::Error(SME_EINVAL, "bad modified UTF-8 in mapping file");
      p += l;
      off.push_back((int64_t)chars.size());
    }
    chars.push_back(0);
    hipStream_t st = cx->own_stream;
    uint16_t *dc = cx->map_chars.as<uint16_t>(chars.size());
    int64_t *doff = cx->map_off.as<int64_t>(off.size());
    SME_HIP(hipMemcpyAsync(dc, chars.data(), chars.size() * sizeof(uint16_t), hipMemcpyHostToDevice, st));
    SME_HIP(hipMemcpyAsync(doff, off.data(), off.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
    SME_HIP(hipStreamSynchronize(st));
    cx->map_n = (int64_t)off.size() - 1;
    cx->has_map = true;
    // The docid hash equals Arrays.binarySearch only when the entries {"", docids...}
    // are strictly ascending in String.compareTo (UTF-16 unit) order -- a sorted
    // file of distinct docids, as writeDocnoData produces.  Any other file (unsorted,
    // or with duplicates) keeps the device binary search, which then reproduces
    // binarySearch's result on that array exactly.
    bool distinct = true;
    for (size_t i = 1; i + 1 < off.size() && distinct; i++)
      distinct = std::lexicographical_compare(chars.begin() + off[i - 1], chars.begin() + off[i],
                                              chars.begin() + off[i], chars.begin() + off[i + 1]);
    sme::build_docid_hash(cx, distinct, st);
  });
}

int sme_number_documents(sme_ctx *cx, const uint8_t *corpus, size_t nbytes, const uint8_t **mapping, size_t *n) {
  return guard([&] {
    if (!cx || !mapping || !n || (!corpus && nbytes)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    hipStream_t st = cx->own_stream;
    sme::DevBuf buf;
    uint8_t *d = buf.as<uint8_t>(nbytes + 16);
    if (nbytes) SME_HIP(hipMemcpyAsync(d, corpus, nbytes, hipMemcpyHostToDevice, st));
    sme::number_documents(cx, d, nbytes, st, cx->mapping_out);
    *mapping = cx->mapping_out.data();
    *n = cx->mapping_out.size();
  });
}

int sme_split_points(sme_ctx *cx, const uint8_t *corpus, size_t nbytes, int world, uint64_t *cuts) {
  return guard([&] {
    if (!cx || !cuts || world < 1 || (!corpus && nbytes)) throw sme::Error(SME_EINVAL, "bad argument");
    set_device(cx);
    hipStream_t st = cx->own_stream;
    sme::DevBuf buf;
    uint8_t *d = buf.as<uint8_t>(nbytes + 16);
    if (nbytes) SME_HIP(hipMemcpyAsync(d, corpus, nbytes, hipMemcpyHostToDevice, st));
    sme::split_points(cx, d, nbytes, world, cuts, st);
  });
}

int sme_split_points_device(sme_ctx *cx, const void *d_corpus, size_t nbytes, int world, void *stream,
                            uint64_t *cuts) {
  return guard([&] {
    if (!cx || !cuts || world < 1 || (!d_corpus && nbytes)) throw sme::Error(SME_EINVAL, "bad argument");
    set_device(cx);
    sme::split_points(cx, (const uint8_t *)d_corpus, nbytes, world, cuts, stream_of(cx, stream));
  });
}

int sme_build_index_device(sme_ctx *cx, const void *d_corpus, size_t nbytes, void *stream, sme_index **out) {
  return guard([&] {
    if (!cx || !out || (!d_corpus && nbytes)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    hipStream_t st = stream_of(cx, stream);
    sme_index *ix = sme::build_index(cx, (const uint8_t *)d_corpus, nbytes, st);
    cx->last_profile = ix->profile;
    *out = ix;
  });
}

int sme_build_chargram_device(sme_ctx *cx, const void *d_corpus, size_t nbytes, void *stream, sme_index **out) {
  return guard([&] {
    if (!cx || !out || (!d_corpus && nbytes)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    hipStream_t st = stream_of(cx, stream);
    sme_index *ix = sme::build_index(cx, (const uint8_t *)d_corpus, nbytes, st, 1);
    cx->last_profile = ix->profile;
    *out = ix;
  });
}

int sme_build_chargram(sme_ctx *cx, const uint8_t *corpus, size_t nbytes, sme_index **out) {
  return guard([&] {
    if (!cx || !out || (!corpus && nbytes)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    hipStream_t st = cx->own_stream;
    sme::DevBuf buf;
    uint8_t *d = buf.as<uint8_t>(nbytes + 16);
    if (nbytes) SME_HIP(hipMemcpyAsync(d, corpus, nbytes, hipMemcpyHostToDevice, st));
    sme_index *ix = sme::build_index(cx, d, nbytes, st, 1);
    SME_HIP(hipStreamSynchronize(st));
    cx->last_profile = ix->profile;
    *out = ix;
  });
}

int sme_chargram_stats(const sme_index *ix, uint64_t *ngrams, uint64_t *npairs) {
  return guard([&] {
    if (!ix || !ngrams || !npairs) throw sme::Error(SME_EINVAL, "null argument");
    if (ix->job != 1) throw sme::Error(SME_EINVAL, "not a CharKGramTermIndexer output");
    *ngrams = (uint64_t)ix->cg_ngrams;
    *npairs = (uint64_t)ix->cg_pairs;
  });
}

int sme_chargram_partition_text(sme_index *ix, int part, const uint8_t **buf, size_t *n) {
  if (ix && ix->job != 1) return fail(SME_EINVAL, "not a CharKGramTermIndexer output");
  return sme_index_partition_records(ix, part, buf, n);
}

int sme_build_index(sme_ctx *cx, const uint8_t *corpus, size_t nbytes, sme_index **out) {
  return guard([&] {
    if (!cx || !out || (!corpus && nbytes)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    hipStream_t st = cx->own_stream;
    // the corpus's device copy is kept in the context (no hipMalloc per build);
    // a pinned host corpus is copied at DMA rate
    uint8_t *d = cx->h_corpus_dev.as<uint8_t>(nbytes + 16);
    if (nbytes) SME_HIP(hipMemcpyAsync(d, corpus, nbytes, hipMemcpyHostToDevice, st));
    sme_index *ix = sme::build_index(cx, d, nbytes, st);
    SME_HIP(hipStreamSynchronize(st));
    // a large copy is not held for the context's lifetime: it would also shrink
    // the HBM that sme_index_prepare_queries sizes its heavy rows from
    if ((int64_t)nbytes > cx->opt_corpus_keep) cx->h_corpus_dev.release();
    cx->last_profile = ix->profile;
    *out = ix;
  });
}

void sme_index_free(sme_index *ix) {
  if (!ix) return;
  sme_ctx *cx = ix->ctx;
  (void)hipSetDevice(cx->device);
  (void)hipDeviceSynchronize();
  delete ix;  // buffers go back to the context's pool
  if (cx->live_indexes == 0 && cx->destroyed) ctx_release(cx);
}

int sme_index_stats(const sme_index *ix, uint64_t *N, uint64_t *V, uint64_t *P) {
  return guard([&] {
    if (!ix) throw sme::Error(SME_EINVAL, "null index");
    if (N) *N = (uint64_t)ix->N;
    if (V) *V = (uint64_t)ix->V;
    if (P) *P = (uint64_t)ix->P;
  });
}

int sme_index_partition_records(sme_index *ix, int part, const uint8_t **buf, size_t *n) {
  return guard([&] {
    if (!ix || !buf || !n) throw sme::Error(SME_EINVAL, "null argument");
    if (part < 0 || part >= ix->R) throw sme::Error(SME_EINVAL, "partition out of range");
    set_device(ix->ctx);
    hipStream_t st = ix->ctx->own_stream;
    sme::serialize_index(ix, st);
    const int64_t a = ix->part_start[part], b = ix->part_start[part + 1];
    if (!ix->h_parts_ready[part]) {
      // default-initialised (not zero-filled) host storage, filled straight from HBM
      ix->h_parts[part].reset(new uint8_t[(size_t)(b - a) + 1]);
      copy_d2h(ix->ctx, ix->h_parts[part].get(), (const uint8_t *)ix->d_ser.p + a, (size_t)(b - a), st);
      ix->h_parts_ready[part] = 1;
    }
    *buf = ix->h_parts[part].get();
    *n = (size_t)(b - a);
  });
}

int sme_index_serialize(sme_index *ix, uint64_t *part_offsets, float *device_ms) {
  return guard([&] {
    if (!ix) throw sme::Error(SME_EINVAL, "null index");
    set_device(ix->ctx);
    sme::serialize_index(ix, ix->ctx->own_stream);
    if (part_offsets)
      for (int p = 0; p <= ix->R; p++) part_offsets[p] = (uint64_t)ix->part_start[p];
    if (device_ms) *device_ms = ix->ser_ms;
  });
}

int sme_index_copy_records(sme_index *ix, int part, void *dst, size_t cap, size_t *n) {
  return guard([&] {
    if (!ix || !n || (!dst && cap)) throw sme::Error(SME_EINVAL, "null argument");
    if (part < -1 || part >= ix->R) throw sme::Error(SME_EINVAL, "partition out of range");
    set_device(ix->ctx);
    hipStream_t st = ix->ctx->own_stream;
    sme::serialize_index(ix, st);
    const int64_t a = part < 0 ? 0 : ix->part_start[part], b = part < 0 ? ix->part_start[ix->R] : ix->part_start[part + 1];
    if ((size_t)(b - a) > cap) throw sme::Error(SME_EINVAL, "destination smaller than the records");
    copy_d2h(ix->ctx, dst, (const uint8_t *)ix->d_ser.p + a, (size_t)(b - a), st);
    *n = (size_t)(b - a);
  });
}

int sme_index_csr(sme_index *ix, const int64_t **offsets, const int32_t **docno, const int32_t **tf,
                  const int32_t **true_df) {
  return guard([&] {
    if (!ix) throw sme::Error(SME_EINVAL, "null index");
    set_device(ix->ctx);
    if (!ix->h_csr_ready) {
      ix->h_off.resize(ix->V + 1);
      ix->h_docno.resize(ix->P);
      ix->h_tf.resize(ix->P);
      ix->h_df.resize(ix->V);
      SME_HIP(hipMemcpy(ix->h_off.data(), ix->d_off.p, (ix->V + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
      if (ix->P) {
        SME_HIP(hipMemcpy(ix->h_docno.data(), ix->d_docno_o.p, ix->P * sizeof(int32_t), hipMemcpyDeviceToHost));
        SME_HIP(hipMemcpy(ix->h_tf.data(), ix->d_tf_o.p, ix->P * sizeof(int32_t), hipMemcpyDeviceToHost));
      }
      for (int64_t t = 0; t < ix->V; t++) ix->h_df[t] = (int32_t)(ix->h_off[t + 1] - ix->h_off[t]);
      ix->h_csr_ready = true;
    }
    if (offsets) *offsets = ix->h_off.data();
    if (docno) *docno = ix->h_docno.data();
    if (tf) *tf = ix->h_tf.data();
    if (true_df) *true_df = ix->h_df.data();
  });
}

int sme_index_device_arrays(sme_index *ix, const int64_t **d_offsets, const int32_t **d_docno,
                            const double **d_weight) {
  return guard([&] {
    if (!ix) throw sme::Error(SME_EINVAL, "null index");
    need_query_side(ix);
    if (d_offsets) *d_offsets = (const int64_t *)ix->d_off.p;
    if (d_docno) *d_docno = (const int32_t *)ix->d_docno_d.p;
    if (d_weight) *d_weight = (const double *)ix->d_w.p;
  });
}

int sme_index_term(sme_index *ix, int64_t t, const uint8_t **utf8, size_t *n) {
  return guard([&] {
    if (!ix || !utf8 || !n) throw sme::Error(SME_EINVAL, "null argument");
    if (t < 0 || t >= ix->V) throw sme::Error(SME_EINVAL, "term id out of range");
    set_device(ix->ctx);
    ensure_host_terms(ix);
    ix->h_term_tmp.clear();
    const bool joined = ix->K > 1 && ix->h_gram.empty();  // merged pieces: components joined by U+0000
    const int64_t c = (ix->K > 1 && !joined) ? (int64_t)ix->h_gram[(size_t)(t * ix->K)] : t;  // k_gram[0] of a k-gram
    const uint16_t *u = ix->h_term_chars.data() + ix->h_term_off[c];
    size_t len = (size_t)(ix->h_term_off[c + 1] - ix->h_term_off[c]);
    if (joined)
      for (size_t i = 0; i < len; i++)
        if (u[i] == 0) {
          len = i;
          break;
        }
    u16_to_mutf8(u, len, ix->h_term_tmp);
    *utf8 = ix->h_term_tmp.data();
    *n = ix->h_term_tmp.size();
  });
}

int sme_tokenize(sme_ctx *cx, const uint8_t *utf8, size_t n, uint8_t *buf, size_t cap, int64_t *offs, int cap_tok,
                 int *ntok) {
  return guard([&] {
    if (!cx || !buf || !offs || !ntok || (!utf8 && n)) throw sme::Error(SME_EINVAL, "null argument");
    set_device(cx);
    std::vector<std::vector<uint16_t>> toks;
    sme::tokenize_string(cx, utf8, n, toks, cx->own_stream);
    if ((int)toks.size() > cap_tok) throw sme::Error(SME_ELIMIT, "more tokens than cap_tok");
    std::vector<uint8_t> o;
    offs[0] = 0;
    for (size_t i = 0; i < toks.size(); i++) {
      u16_to_mutf8(toks[i].data(), toks[i].size(), o);
      offs[i + 1] = (int64_t)o.size();
    }
    if (o.size() > cap) throw sme::Error(SME_ELIMIT, "token buffer too small");
    if (!o.empty()) memcpy(buf, o.data(), o.size());
    *ntok = (int)toks.size();
  });
}

int sme_lookup_terms(sme_index *ix, const uint8_t *terms, const int64_t *offs, int n, int32_t *term_ids) {
  return guard([&] {
    if (!ix || !offs || !term_ids || n < 0) throw sme::Error(SME_EINVAL, "null argument");
    set_device(ix->ctx);
    std::vector<std::vector<uint16_t>> q(n);
    for (int i = 0; i < n; i++) q[i] = utf8_to_u16(terms + offs[i], (size_t)(offs[i + 1] - offs[i]));
    sme::lookup_terms(ix, q, term_ids, ix->ctx->own_stream);
  });
}

int sme_index_prepare_queries(sme_index *ix, void *stream, float *ms) {
  return guard([&] {
    if (!ix) throw sme::Error(SME_EINVAL, "null index");
    need_query_side(ix);
    if (ix->job != 0) throw sme::Error(SME_EINVAL, "not a TermKGramDocIndexer index");
    set_device(ix->ctx);
    sme::prepare_queries(ix, stream_of(ix->ctx, stream));
    if (ms) *ms = ix->q_prep_ms;
  });
}

int sme_query_topk_device(sme_index *ix, const int32_t *d_term_ids, const int64_t *d_q_offsets, int nq, int k,
                          int32_t *d_out_docno, double *d_out_score, void *stream) {
  return guard([&] {
    if (!ix || (nq > 0 && (!d_term_ids || !d_q_offsets || !d_out_docno || !d_out_score)))
      throw sme::Error(SME_EINVAL, "null argument");
    need_query_side(ix);
    set_device(ix->ctx);
    sme::query_topk(ix, d_term_ids, d_q_offsets, nq, k, d_out_docno, d_out_score, nullptr,
                    stream_of(ix->ctx, stream));
  });
}

int sme_query_topk_device_tie(sme_index *ix, const int32_t *d_term_ids, const int64_t *d_q_offsets, int nq, int k,
                              int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie, void *stream) {
  return guard([&] {
    if (!ix || (nq > 0 && (!d_term_ids || !d_q_offsets || !d_out_docno || !d_out_score || !d_out_tie)))
      throw sme::Error(SME_EINVAL, "null argument");
    need_query_side(ix);
    set_device(ix->ctx);
    sme::query_topk(ix, d_term_ids, d_q_offsets, nq, k, d_out_docno, d_out_score, d_out_tie,
                    stream_of(ix->ctx, stream));
  });
}

static int query_topk_host(sme_index *ix, const int32_t *term_ids, const int64_t *q_offsets, int nq, int k,
                           int32_t *out_docno, double *out_score, uint32_t *out_tie) {
  return guard([&] {
    if (!ix || (nq > 0 && (!term_ids || !q_offsets || !out_docno || !out_score)))
      throw sme::Error(SME_EINVAL, "null argument");
    need_query_side(ix);
    if (nq <= 0) return;
    set_device(ix->ctx);
    hipStream_t st = ix->ctx->own_stream;
    const int64_t nt = q_offsets[nq];
    for (int q = 0; q < nq; q++)
      if (q_offsets[q + 1] < q_offsets[q] || q_offsets[q] < 0) throw sme::Error(SME_EINVAL, "q_offsets not ascending");
    for (int64_t i = 0; i < nt; i++)
      if (term_ids[i] < -1 || term_ids[i] >= ix->V)
        throw sme::Error(SME_EINVAL, "term id " + std::to_string(term_ids[i]) + " outside [-1, V)");
    sme::DevBuf a, b, c, d, e;
    int32_t *dt = a.as<int32_t>(nt + 1);
    int64_t *dq = b.as<int64_t>(nq + 1);
    int32_t *dd = c.as<int32_t>((size_t)nq * k);
    double *ds = d.as<double>((size_t)nq * k);
    uint32_t *dtie = out_tie ? e.as<uint32_t>((size_t)nq * k) : nullptr;
    if (nt) SME_HIP(hipMemcpyAsync(dt, term_ids, nt * sizeof(int32_t), hipMemcpyHostToDevice, st));
    SME_HIP(hipMemcpyAsync(dq, q_offsets, (nq + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
    sme::query_topk(ix, dt, dq, nq, k, dd, ds, dtie, st);
    SME_HIP(hipMemcpyAsync(out_docno, dd, (size_t)nq * k * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipMemcpyAsync(out_score, ds, (size_t)nq * k * sizeof(double), hipMemcpyDeviceToHost, st));
    if (out_tie)
      SME_HIP(hipMemcpyAsync(out_tie, dtie, (size_t)nq * k * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    SME_HIP(hipStreamSynchronize(st));
  });
}

int sme_query_topk(sme_index *ix, const int32_t *term_ids, const int64_t *q_offsets, int nq, int k,
                   int32_t *out_docno, double *out_score) {
  return query_topk_host(ix, term_ids, q_offsets, nq, k, out_docno, out_score, nullptr);
}

int sme_query_topk_tie(sme_index *ix, const int32_t *term_ids, const int64_t *q_offsets, int nq, int k,
                       int32_t *out_docno, double *out_score, uint32_t *out_tie) {
  if (nq > 0 && !out_tie) return fail(SME_EINVAL, "null argument");
  return query_topk_host(ix, term_ids, q_offsets, nq, k, out_docno, out_score, out_tie);
}

int sme_index_term_fingerprints(sme_index *ix, uint64_t *d_out, void *stream) {
  return guard([&] {
    if (!ix || (!d_out && ix->V > 0)) throw sme::Error(SME_EINVAL, "null argument");
    if (ix->job != 0) throw sme::Error(SME_EINVAL, "not a TermKGramDocIndexer index");
    set_device(ix->ctx);
    hipStream_t st = stream_of(ix->ctx, stream);
    sme::term_fingerprints(ix, d_out, st);
    SME_HIP(hipStreamSynchronize(st));
  });
}

int sme_df_owner_pack(sme_ctx *ctx, const uint64_t *d_fp, const int64_t *d_df, int64_t n, int world,
                      uint64_t *d_send_fp, int64_t *d_send_df, int64_t *d_pos, int64_t *counts, void *stream) {
  return guard([&] {
    if (!ctx || !counts || n < 0 || (n > 0 && (!d_fp || !d_df || !d_send_fp || !d_send_df || !d_pos)))
      throw sme::Error(SME_EINVAL, "bad argument");
    set_device(ctx);
    sme::dfx_pack(ctx, d_fp, d_df, n, world, d_send_fp, d_send_df, d_pos, counts, stream_of(ctx, stream));
  });
}

int sme_df_owner_sum(sme_ctx *ctx, const uint64_t *d_fp, const int64_t *d_df, int64_t n, int64_t *d_out,
                     int64_t *distinct, void *stream) {
  return guard([&] {
    if (!ctx || !distinct || n < 0 || (n > 0 && (!d_fp || !d_df || !d_out)))
      throw sme::Error(SME_EINVAL, "bad argument");
    set_device(ctx);
    sme::dfx_sum(ctx, d_fp, d_df, n, d_out, distinct, stream_of(ctx, stream));
  });
}

int sme_df_owner_unpack(sme_ctx *ctx, const int64_t *d_ret, const int64_t *d_pos, int64_t n, int64_t *d_out,
                        void *stream) {
  return guard([&] {
    if (!ctx || n < 0 || (n > 0 && (!d_ret || !d_pos || !d_out))) throw sme::Error(SME_EINVAL, "bad argument");
    set_device(ctx);
    hipStream_t st = stream_of(ctx, stream);
    sme::dfx_unpack(d_ret, d_pos, n, d_out, st);
    SME_HIP(hipStreamSynchronize(st));
  });
}

int sme_topk_merge_rows(sme_ctx *ctx, const double *d_score, const int32_t *d_docno, const uint32_t *d_tie,
                        int64_t rows, int m, int k, int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie,
                        void *stream) {
  return guard([&] {
    if (!ctx || rows < 0 || m < 0 || k < 1 || (rows > 0 && (!d_out_docno || !d_out_score || (m > 0 && (!d_score || !d_docno)))))
      throw sme::Error(SME_EINVAL, "bad argument");
    set_device(ctx);
    hipStream_t st = stream_of(ctx, stream);
    sme::merge_rows(d_score, d_docno, d_tie, rows, m, k, d_out_docno, d_out_score, d_out_tie, st);
    SME_HIP(hipStreamSynchronize(st));
  });
}

int sme_count_shared_keys(sme_ctx *ctx, const uint64_t *d_rows, int64_t n, int64_t *count, void *stream) {
  return guard([&] {
    if (!ctx || !count || n < 0 || (n > 0 && !d_rows)) throw sme::Error(SME_EINVAL, "bad argument");
    set_device(ctx);
    *count = sme::count_shared_keys(ctx, d_rows, n, stream_of(ctx, stream));
  });
}

int sme_index_reweight(sme_index *ix, int64_t n_global, const int64_t *d_df_global, void *stream) {
  return guard([&] {
    if (!ix || n_global < 0) throw sme::Error(SME_EINVAL, "bad argument");
    need_query_side(ix);
    set_device(ix->ctx);
    sme::reweight_index(ix, n_global, d_df_global, stream_of(ix->ctx, stream));
  });
}

int sme_index_record_docnos(sme_index *ix, const int32_t **d_docno, int64_t *n) {
  return guard([&] {
    if (!ix || !d_docno || !n) throw sme::Error(SME_EINVAL, "null argument");
    if (ix->job != 0) throw sme::Error(SME_EINVAL, "not a TermKGramDocIndexer index");
    *d_docno = (const int32_t *)ix->d_rec_docno.p;
    *n = ix->N;
  });
}

int sme_index_pack_pieces(sme_index *ix, int world, void *d_out, uint64_t *sizes, void *stream) {
  return guard([&] {
    if (!ix || !sizes) throw sme::Error(SME_EINVAL, "null argument");
    need_query_side(ix);
    set_device(ix->ctx);
    hipStream_t st = stream_of(ix->ctx, stream);
    sme::pack_pieces(ix, world, (uint8_t *)d_out, sizes, st);
    SME_HIP(hipStreamSynchronize(st));
  });
}

int sme_merge_pieces(sme_ctx *cx, const void *d_blobs, const uint64_t *sizes, int n, void *stream, sme_index **out) {
  return guard([&] {
    if (!cx || !d_blobs || !sizes || !out || n < 1) throw sme::Error(SME_EINVAL, "bad argument");
    set_device(cx);
    *out = sme::merge_pieces(cx, (const uint8_t *)d_blobs, sizes, n, stream_of(cx, stream));
  });
}

int sme_last_build_profile(const sme_ctx *cx, const char **json) {
  return guard([&] {
    if (!cx || !json) throw sme::Error(SME_EINVAL, "null argument");
    std::ostringstream os;
    os << "{";
    for (size_t i = 0; i < cx->last_profile.size(); i++)
      os << (i ? "," : "") << "\"" << cx->last_profile[i].first << "\":" << cx->last_profile[i].second;
    if (cx->last_query_ms >= 0) os << (cx->last_profile.empty() ? "" : ",") << "\"query_kernel\":" << cx->last_query_ms;
    if (cx->last_query_ms >= 0) os << ",\"query_prep\":" << cx->last_query_prep_ms;
    if (cx->last_query_ms >= 0) os << ",\"query_index\":" << cx->last_query_index_ms;
    if (cx->last_query_ms >= 0) os << ",\"query_kernel_name\":\"" << cx->last_query_name << "\"";
    if (cx->last_query_ms >= 0 && cx->last_query_name == std::string("k_query_win"))
      os << ",\"query_seed\":" << cx->last_query_seed_ms << ",\"query_final\":" << cx->last_query_final_ms
         << ",\"query_overflow\":" << cx->last_query_overflow << ",\"query_fallback\":" << cx->last_query_fallback << ",\"query_split\":" << (cx->last_query_split ? 1 : 0) << ",\"query_total\":" << cx->last_query_total_ms;
    os << "}";
    const_cast<sme_ctx *>(cx)->profile_json = os.str();
    *json = cx->profile_json.c_str();
  });
}

}  // extern "C"
