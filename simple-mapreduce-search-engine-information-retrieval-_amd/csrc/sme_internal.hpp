// sme_internal.hpp -- context and index objects behind the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "sme_common.hpp"

struct sme_ctx {
  sme::BufPool pool;  // declared first: destroyed after every DevBuf below
  sme_config cfg{};
  int device = 0;
  hipStream_t own_stream = nullptr;
  // a second stream for independent kernels of one build stage (the tf-desc
  // sort's segment classes), joined back by events
  hipStream_t aux_stream = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::vector<hipEvent_t> prof_events;  // Prof's reusable stage events
  // docno mapping: {"", docids...} as UTF-16 (TrecDocnoMapping.readDocnoData)
  sme::DevBuf map_chars, map_off;
  int64_t map_n = 0;  // entries including the "" sentinel
  bool has_map = false;
  sme::DevBuf map_slots;  // docid hash table (entry index + 1), see k_docno
  uint64_t map_mask = 0;
  bool map_hash_ok = false;  // built, and the mapping's docids are distinct
  // build workspace, reused across builds (see DevBuf)
  sme::DevBuf ws[128];  // 48..63 query / serializer / tokenizer / reweight, 64..127 build
  sme::DevBuf cub_tmp;
  sme::DevBuf q_gates;  // k_query_win: per-query gate of the current thresholds (k_gates)
  uint64_t vocab_long_cap = 0, vocab_ovf_cap = 0, raw_cap_hint = 0, lt_cap_hint = 0;  // learned across builds
  std::string profile_json;
  std::vector<std::pair<std::string, float>> last_profile;
  std::vector<uint8_t> mapping_out;  // last sme_number_documents result
  std::vector<int32_t> h_wlist;      // k_query_win window order of the last batch (source of an async copy)
  float last_query_ms = -1.0f;  // device time of the last query kernel launch
  float last_query_prep_ms = -1.0f;  // per-batch tables before it (skip / impact tables, query order)
  float last_query_index_ms = -1.0f;  // one-time heavy-row build of the index it ran on (prepare_queries)
  bool last_query_tiled = false;  // tiled path (k_query_win / k_query_bm) or the streaming k_query
  const char *last_query_name = "k_query";  // the scoring kernel that ran
  float last_query_seed_ms = 0.0f, last_query_final_ms = 0.0f, last_query_total_ms = 0.0f;
  int64_t last_query_overflow = 0;  // k_query_win queries whose first candidate list overflowed
  int64_t last_query_fallback = 0;  // of those, queries finally scored by k_query_bm
  bool last_query_split = false;     // the batch was split by query range (table budget)
  // Path options (sme_set_option).  Every setting gives identical results; they
  // exist so tests can hold each path to the others and benches can sweep them.
  int64_t opt_query_kernel = 0;   // "query_kernel": 0 window-major (auto), 1 streaming k_query, 2 block-max sweep
  int64_t opt_heavy_div = 128;    // "heavy_div": heavy rows for terms with df >= span / div (0: none)
  int64_t opt_seed_tiles = 4;     // "seed_tiles": best-bound tiles scored before the sweep (0..8)
  int64_t opt_query_order = 1;    // "query_order": 1 heaviest-term query order, 0 batch order
  int64_t opt_agg_two_pass = 0;   // "agg_two_pass": 1 = count + emit aggregation passes
  int64_t opt_agg_grid = 0;      // "agg_grid": aggregation workgroups (0 = auto)
  int64_t opt_tok_grid = 5120;    // "tok_grid": tokenizer workgroups (>= 1): four rounds of 5 per CU x 256 CUs
  int64_t opt_raw_load_pct = 40;  // "raw_load_pct": raw-vocabulary table load of the next build (10..90)
  int64_t opt_docid_terms = 1;    // "docid_terms": docid terms beside the word vocabulary (K4b; 0 = general path)
  int64_t opt_sort_bits = 0;      // "sort_digit_bits": most bits per digit of the term sort's LSD passes (6..11; 0 auto)
  int64_t opt_docid_split = 1;    // "docid_split": docid pairs beside the term sort (K6b): 1 past 22 merged id bits, 2 whenever the words need fewer, 0 never
  int64_t opt_cand_cap = 1024;    // "cand_cap": candidate list per query of k_query_win (1..2048; >= 1024: at least 16 k)
  int64_t opt_seed_m = 64;        // "seed_m": seed postings per term (k_query_seed; 0 = no seed)
  int64_t opt_kgram_rank = 0;     // "kgram_rank": 1 = K >= 2 gram keys by iterated ranking even when packed ids fit
  int64_t opt_win_slice = 0;      // "win_slice": queries per k_query_win workgroup slice (0 = auto: 128, 256 from 1024 windows)
  int64_t opt_win_sample = 1;     // "win_sample": 1 = every 8th window first, thresholds raised, then the rest
  int64_t opt_win_stage_min = 0;   // "win_stage_min": windows of the first stage (at least; the stage count follows; 0 = auto)
  int64_t opt_query_budget = 0;  // "query_table_budget": per-batch skip-table bytes (0: a quarter of free HBM)
  int64_t opt_corpus_keep = int64_t(16) << 30;  // "corpus_keep_bytes": host-corpus builds keep their device copy
                                                // (no hipMalloc next build) only up to this size
  // pinned host staging of device -> host record copies into pageable caller
  // memory (sme_index_copy_records): two buffers, DMA into one while the host
  // copies out of the other
  void *h_stage[2] = {nullptr, nullptr};
  size_t h_stage_cap = 0;
  // device copy of a host corpus (sme_build_index), kept across builds
  sme::DevBuf h_corpus_dev;
  // indexes borrow the context (its pool, workspace, stream): sme_destroy defers
  // the delete until the last index is freed, whatever order a host frees them in
  int live_indexes = 0;
  bool destroyed = false;
};

struct sme_index {
  sme_ctx *ctx = nullptr;
  int K = 1, R = 1, idf_mode = 0;
  int job = 0;               // 0 TermKGramDocIndexer index, 1 CharKGramTermIndexer output
  int64_t cg_ngrams = 0, cg_pairs = 0;  // job 1: distinct char k-grams, (gram, term) set entries
  int64_t N = 0, V = 0, P = 0;
  int64_t Vt = 0;  // term vocabulary size (V counts k-grams when K > 1)
  int32_t max_tf = 0;
  int64_t dmin = 0, dmax = -1;  // docno range of the records (query doc tiles)
  // sorted vocabulary (rank order): UTF-16 units
  sme::DevBuf d_term_off;    // int64 [V+1]
  sme::DevBuf d_term_chars;  // uint16
  // query-side CSR: postings per term in docno-ascending order, fp64 TF-IDF weights
  sme::DevBuf d_off;      // int64 [V+1]
  sme::DevBuf d_docno_d;  // int32 [P]
  sme::DevBuf d_tf_d;     // int32 [P]
  sme::DevBuf d_w;        // double [P]
  sme::DevBuf d_idf;      // double [V]   idf of every term (query side: w = lut[tf] * idf)
  sme::DevBuf d_gram;     // int32 [V * K]  term ids of every k-gram (K > 1)
  sme::DevBuf d_lut;      // double [max_tf + 1]  1 + ln(tf)
  // reduce-output CSR: (tf desc, docno asc) per term (MyReducer.reduce order)
  sme::DevBuf d_docno_o;  // int32 [P]
  sme::DevBuf d_tf_o;     // int32 [P]
  // docno of every record in input order (for the " " doc-counter postings)
  sme::DevBuf d_rec_docno;  // int32 [N]
  sme::DevBuf d_rec_first;  // u8 [N]: record starts a map task (split) -- merged shard pieces only
  bool records_only = false;  // merged shard pieces (sme_merge_pieces): reduce-order CSR + records, no query side
  // serialized partitions (lazily built)
  sme::DevBuf d_ser;
  std::vector<int64_t> part_start;  // R+1
  bool ser_ready = false;
  float ser_ms = 0.0f;  // device time of the k_ser_* pass (serialize_index)
  // host copies of the partitions (sme_index_partition_records), not zero-filled
  std::vector<std::unique_ptr<uint8_t[]>> h_parts;
  std::vector<char> h_parts_ready;
  // host copies (lazily)
  std::vector<int64_t> h_off;
  std::vector<int32_t> h_docno, h_tf, h_df;
  bool h_csr_ready = false;
  std::vector<int64_t> h_term_off;
  std::vector<uint16_t> h_term_chars;
  std::vector<int32_t> h_gram;
  std::vector<uint8_t> h_term_tmp;
  bool h_terms_ready = false;
  // query-side heavy rows (prepare_queries, sme_query.hip): tf byte rows, 16-doc
  // and 1024-doc block maxima of the terms covering >= 1/div of the docno span
  sme::DevBuf d_hrow_of;  // int32 [V] heavy row or -1
  // u8 [H][T * 1024] tf | imp | [H][T * 64] bm16 | [H][T] bm1k | [H][T * 256] sbq
  sme::DevBuf d_heavy;
  const uint8_t *q_tfrow = nullptr, *q_bm16 = nullptr, *q_bm1k = nullptr, *q_imp = nullptr;
  const uint8_t *q_sbq = nullptr;  // impact maxima of 4-document sub-blocks (k_query_win's second level)
  // k_query_win's sparse postings, one word per docno-order posting of a term
  // without a heavy row: (docno - dmin) mod 4096 | q(tf) << 12 | min(tf, 4095) << 20
  sme::DevBuf d_spk;
  const uint32_t *q_spk = nullptr;
  double q_alpha = 1.0;                 // impact scale 253.5 / (largest weight of any term)
  unsigned long long q_wmax_bits = 0;   // that weight's bits
  int64_t q_T = 0, q_H = 0, q_div = -1;
  bool q_ready = false;
  float q_prep_ms = 0.0f;
  // stage timings of the build that produced this index (ms)
  std::vector<std::pair<std::string, float>> profile;
  ~sme_index() { ctx->live_indexes--; }  // members (pooled buffers) are released after this body
  explicit sme_index(sme_ctx *c) : ctx(c) {
    c->live_indexes++;
    for (sme::DevBuf *b : {&d_term_off, &d_term_chars, &d_off, &d_docno_d, &d_tf_d, &d_w, &d_idf, &d_lut, &d_gram, &d_docno_o,
                           &d_tf_o, &d_rec_docno, &d_rec_first, &d_ser, &d_hrow_of, &d_heavy, &d_spk})
      b->pool = &c->pool;
  }
};

namespace sme {
// per-stage device-event timer of a build
struct Prof {
  // stage events come from a pool kept by the context (hipEventCreate per mark
  // cost host time between a build's launches); events of an abandoned Prof
  // (an exception) go back to the pool in the destructor
  hipStream_t st;
  std::vector<hipEvent_t> *pool;
  std::vector<std::pair<std::string, hipEvent_t>> ev;
  Prof(hipStream_t s, std::vector<hipEvent_t> *p) : st(s), pool(p) { mark("start"); }
  ~Prof() {
    for (auto &e : ev) pool->push_back(e.second);
  }
  void mark(const char *name) {
    hipEvent_t e;
    if (!pool->empty()) {
      e = pool->back();
      pool->pop_back();
    } else {
      SME_HIP(hipEventCreate(&e));
    }
    ev.emplace_back(name, e);
    SME_HIP(hipEventRecord(e, st));
  }
  std::vector<std::pair<std::string, float>> finish() {
    SME_HIP(hipEventSynchronize(ev.back().second));
    std::vector<std::pair<std::string, float>> out;
    for (size_t i = 1; i < ev.size(); i++) {
      float ms = 0;
      SME_HIP(hipEventElapsedTime(&ms, ev[i - 1].second, ev[i].second));
      out.emplace_back(ev[i].first, ms);
    }
    float tot = 0;
    SME_HIP(hipEventElapsedTime(&tot, ev.front().second, ev.back().second));
    out.emplace_back("total", tot);
    for (auto &p : ev) pool->push_back(p.second);
    ev.clear();
    return out;
  }
};

struct RecordSpans {
  uint64_t *rs, *re;  // record [rs, re) byte spans, in reader order
  int64_t nR;
  uint64_t *C;        // sorted positions of '<' whose markup is not "simple"
  int64_t nC;
};
void build_docid_hash(sme_ctx *cx, bool distinct, hipStream_t st);
RecordSpans find_records(sme_ctx *cx, const uint8_t *d_text, uint64_t n, hipStream_t st, Prof *prof);
void split_points(sme_ctx *cx, const uint8_t *d_text, uint64_t n, int world, uint64_t *h_cuts, hipStream_t st);
void number_documents(sme_ctx *cx, const uint8_t *d_text, uint64_t n, hipStream_t st, std::vector<uint8_t> &out);
sme_index *build_index(sme_ctx *cx, const uint8_t *d_text, uint64_t n, hipStream_t st, int job = 0);
// CharKGramTermIndexer stage over the file-order term stream (sme_chargram.hip)
void chargram_stage(sme_ctx *cx, sme_index *ix, const int32_t *tstream, int64_t M, int64_t V, const int64_t *term_off,
                    const uint16_t *term_chars, hipStream_t st, Prof *prof);
// stable LSD radix sort of (term id, packed posting) pairs (sme_sort.hip)
// (reg != nullptr: the first pass reads pair x from reg[i] + x - xoff[i], record i
// holding it -- the single-pass aggregation's layout)
// (xw != nullptr: K6b -- the keys are word ranks; the last pass writes word i's
// postings shifted by xw[i].x and keyed xw[i].y into Pout slots keyed 0xFFFFFFFF)
uint32_t *term_sort(uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, int64_t nrec, const int64_t *reg,
                    const int64_t *xoff, int64_t P, int bits, int64_t dmin, uint32_t F, int32_t *docno, int32_t *tf,
                    uint32_t *counts, hipStream_t st, const double *lut = nullptr, double idf = 0.0,
                    double *w = nullptr, int maxbits = 11, const uint2 *xw = nullptr, int64_t Pout = 0);
size_t term_sort_scratch(int64_t P);
// stable LSD radix sort of (key, u32 value) pairs by the key's low `bits` bits
// (sme_sort.hip; K = uint32_t or uint64_t); ping-pongs between (k0, v0) and
// (k1, v1) and returns the sorted values' buffer (keys beside it if keys_out)
template <typename K>
uint32_t *kv_sort(K *k0, uint32_t *v0, K *k1, uint32_t *v1, int64_t n, int bits, uint32_t *scratch, hipStream_t st,
                  bool keys_out = false);
size_t kv_sort_scratch(int64_t n);
// device-wide exclusive scan out[i] = sum in[0..i) (in == out allowed; scratch:
// one T per 4096 items), and flag compaction (ascending indices of the nonzero
// flags, their count to *d_count) -- hand-written, sme_sort.hip
template <typename T>
void excl_scan(const T *in, T *out, int64_t n, DevBuf &scratch, hipStream_t st);
void select_flagged(const uint8_t *flag, int64_t n, int32_t *out, int32_t *d_count, DevBuf &s1, DevBuf &s2,
                    hipStream_t st);
// SortPairs-shaped wrappers of kv_sort (separate in / out arrays; the inputs are
// clobbered): u32 values, or 64-bit values through a sorted index + gather
template <typename K>
void sort_pairs(K *keys_in, K *keys_out, uint32_t *vals_in, uint32_t *vals_out, int64_t n, int bits, DevBuf &radix,
                hipStream_t st);
template <typename K>
void sort_pairs_v64(K *keys_in, K *keys_out, const uint64_t *vals_in, uint64_t *vals_out, int64_t n, int bits,
                    DevBuf &ia, DevBuf &ib, DevBuf &radix, hipStream_t st);
// *d_max = the largest of n >= 1 values (non-negative integers)
template <typename T>
void reduce_max(const T *in, int64_t n, T *d_max, hipStream_t st);
// runs of equal keys (sorted input) -> (key, sum of vals) per run, *d_runs = count
void reduce_by_key_sum(const uint64_t *keys, const int32_t *vals, int64_t n, uint64_t *ukeys, int32_t *sums,
                       int64_t *d_runs, DevBuf &flags, DevBuf &pos, DevBuf &scan, hipStream_t st);
void serialize_index(sme_index *ix, hipStream_t st);
// reference-layout output from doc shards (sme_merge.hip): per-owner blobs of a
// shard's terms and postings, and the owner's merge of the received blobs
void pack_pieces(sme_index *ix, int world, uint8_t *d_out, uint64_t *sizes, hipStream_t st);
sme_index *merge_pieces(sme_ctx *cx, const uint8_t *d_blobs, const uint64_t *sizes, int np, hipStream_t st);
void reweight_index(sme_index *ix, int64_t N, const int64_t *d_gdf, hipStream_t st);
void prepare_queries(sme_index *ix, hipStream_t st);
// tie_bits: the reference tie word's tf width (24, or 22 when a query of the
// batch has > 256 terms); 0 = decided by this batch.  Only the nested calls of
// one batch (query-range splits, overflow subsets) pass it, so every query of a
// batch -- on every doc shard answering it -- gets the same tie words.
void query_topk(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, int k,
                int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie, hipStream_t st, int tie_bits = 0);
// SME_TIE_JAVA7 (sme_timsort.hip): every query's whole first-encounter list and
// the JDK 7 ComparableTimSort over it, one thread per query
void query_topk_java7(sme_index *ix, const int32_t *d_terms, const int64_t *d_qoff, int nq, int k,
                      int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie, hipStream_t st);
void tokenize_string(sme_ctx *cx, const uint8_t *h_utf8, size_t n, std::vector<std::vector<uint16_t>> &out,
                     hipStream_t st);
void term_fingerprints(sme_index *ix, uint64_t *d_out, hipStream_t st);
// multi-GPU df exchange steps (sme_dfx.hip): owner grouping, owner sums, return gather
void dfx_pack(sme_ctx *cx, const uint64_t *fp, const int64_t *df, int64_t n, int world, uint64_t *sfp, int64_t *sdf,
              int64_t *pos, int64_t *h_counts, hipStream_t st);
void dfx_sum(sme_ctx *cx, const uint64_t *fp, const int64_t *df, int64_t n, int64_t *out, int64_t *h_distinct,
             hipStream_t st);
void dfx_unpack(const int64_t *ret, const int64_t *pos, int64_t n, int64_t *out, hipStream_t st);
// owner-side steps of the N > 1 query path (sme_owner.hip): merge of the shards'
// top-k rows, and the count of keys that arrive from two or more ranks
void merge_rows(const double *s, const int32_t *d, const uint32_t *t, int64_t rows, int m, int k, int32_t *od,
                double *os, uint32_t *ot, hipStream_t st);
int64_t count_shared_keys(sme_ctx *cx, const uint64_t *rows, int64_t n, hipStream_t st);
void lookup_terms(sme_index *ix, const std::vector<std::vector<uint16_t>> &terms, int32_t *ids,
                  hipStream_t st);
}  // namespace sme
