/*
 * sme.h -- C-ABI of the MI355X-native index-build / TF-IDF / query hot path.
 *
 * "sme" = Simple MapReduce Engine.  This library replaces, as one batch call,
 * the reference's whole TermKGramDocIndexer job (map -> shuffle/sort ->
 * combine/reduce) and IntDocVectorsForwardIndex.rank():
 *
 *   sme_build_index*      <- TermKGramDocIndexer.run / MyMapper.map / MyReducer.reduce
 *                            C/sa/edu/kaust/indexing/TermKGramDocIndexer.java:119-160,168-213,227-283
 *   sme_load_docno_mapping<- MyMapper.configure -> TrecDocnoMapping.loadMapping/readDocnoData
 *                            TermKGramDocIndexer.java:93-117; C/edu/umd/cloud9/collection/trec/TrecDocnoMapping.java:75-77,137-155
 *   sme_index_partition_records <- SequenceFileOutputFormat part-NNNNN record stream
 *                            (TermDF.write TermDF.java:50-56, ArrayListWritable.write ArrayListWritable.java:90-105)
 *   sme_tokenize          <- GalagoTokenizer.processContent  C/ivory/tokenize/GalagoTokenizer.java:139-183
 *   sme_lookup_terms      <- IntDocVectorsForwardIndex.getValue(String[]) term lookup
 *                            C/sa/edu/kaust/fwindex/IntDocVectorsForwardIndex.java:131-184
 *   sme_query_topk        <- IntDocVectorsForwardIndex.rank()  IntDocVectorsForwardIndex.java:192-223
 * (C/ = ABDURRAHMAN-PA2-3-code/src/ of the reference; U+2010 hyphens in the real path.)
 *
 * Conventions: every int-returning function returns 0 (SME_OK) on success and
 * a negative SME_E* code on failure; sme_last_error() returns a thread-local
 * message for the last failure.  Inputs are borrowed for the duration of the
 * call; outputs returned through pointers are owned by the library until the
 * owning object is freed.  One sme_ctx per device; calls on one context must
 * be serialized by the caller (the reference's query class is not thread-safe
 * either: IntDocVectorsForwardIndex.java:63-65).
 */
#ifndef SME_H
#define SME_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SME_OK 0
#define SME_EINVAL -1    /* bad argument */
#define SME_EHIP -2      /* HIP runtime error */
#define SME_ENOMEM -3    /* device allocation failed */
#define SME_EPARSE -4    /* input the reference rejects (e.g. <DOCNO> without </DOCNO>: getDocid throws) */
#define SME_ENOMAP -5    /* no docno mapping loaded */
#define SME_ELIMIT -6    /* an implementation limit was hit (message says which) */
#define SME_ENOTIMPL -7  /* feature not built yet (message says which) */

/* idf_mode */
#define SME_IDF_REFERENCE 0 /* log10(N / stored_df); stored df of every real term is 1 */
#define SME_IDF_TRUE_DF 1   /* log10(N / df) with df = postings length, int division as the reference */

/* tiebreak */
#define SME_TIE_DOCNO 0     /* score desc, then docno asc (north-star contract) */
#define SME_TIE_REFERENCE 1 /* score desc, then the reference's printed order: rank() appends
                               candidates in first-encounter order (query token order, each term's
                               postings tf desc / docno asc) and Collections.sort over DocScore
                               (IntDocVectorsForwardIndex.java:195-215,363-365) is a stable sort by
                               score desc (its merge sort only asks compareTo <= 0 / > 0, which is
                               score order for finite scores), so equal scores keep that order */
#define SME_TIE_JAVA7 2     /* rank()'s list as a Java 7 JVM leaves it: Collections.sort is then
                               ComparableTimSort, and DocScore.compareTo = (int)Math.ceil(o.score -
                               score) -- 0 for score gaps in (-1, 0] -- is not a total order, so the
                               whole first-encounter list is sorted by the JDK 7 GA algorithm on the
                               device (one thread per query; a compatibility mode, not the serving
                               path).  A query whose sort Java aborts with IllegalArgumentException
                               ("Comparison method violates its general contract!") gets docno -2
                               in all k slots; tie words are 0xFFFFFFFF (no shard merge) */

typedef struct sme_ctx sme_ctx;
typedef struct sme_index sme_index;

typedef struct {
  int k;              /* K of the K-gram index (TermKGramDocIndexer args[0]); 1 = term index */
  int num_partitions; /* R reducers (conf.setNumReduceTasks(10) on the cluster, 1 in local mode) */
  int idf_mode;       /* SME_IDF_* used by the TF-IDF weight pass and sme_query_topk */
  int tiebreak;       /* SME_TIE_* */
  int device;         /* HIP device ordinal */
  int reserved[11];   /* must be zero */
} sme_config;

const char *sme_last_error(void);
const char *sme_version(void);

/* Device-memory plumbing for hosts without a HIP binding of their own (a JNI /
 * ctypes host passing d_df_global to sme_index_reweight, or reading a device
 * corpus back): allocation on `device`, and a copy in any direction
 * (hipMemcpyDefault; stream NULL = synchronous).  They run on the library's own
 * HIP runtime, so pointers from it and to it always agree. */
int sme_device_alloc(int device, size_t n, void **d);
void sme_device_free(void *d);
int sme_memcpy(void *dst, const void *src, size_t n, void *stream);

int sme_create(const sme_config *cfg, sme_ctx **out);
void sme_destroy(sme_ctx *ctx);

/* Path options of a context (no reference counterpart: the reference has one
 * code path).  Every value gives bit-identical results; the options exist so
 * tests can hold each device path to the others and benches can sweep them.
 *   "query_kernel"  0 window-major scoring with seeded thresholds (default), 1 streaming
 *                   k_query, 2 per-query block-max sweep k_query_bm
 *   "heavy_div"     heavy tf / impact rows for terms with df >= docno span / div (default 128; 0 none)
 *   "seed_m"        seed postings per term for the window path's threshold, 0..4096 (default 64)
 *   "cand_cap"      candidate list per query of the window path, 1..2048 (default 1024; >= 1024:
 *                   at least 16 k)
 *   "win_sample"    1 (default): sample windows first, thresholds raised, then the rest
 *   "win_stage_min" windows of the first sampled stage, at least (default 0 = auto: 16, or 8
 *                   for indexes of >= 1024 windows of 4096 documents; the stage count
 *                   follows, at most 9)
 *   "win_slice"     queries per window-path workgroup slice (default 0 = auto: 128, or 256 for
 *                   indexes of >= 1024 windows)
 *   "seed_tiles"    k_query_bm: best-bound tiles scored before the sweep, 0..8 (default 4)
 *   "query_order"   1 heaviest-term query order (default), 0 batch order
 *   "agg_two_pass"  1 count + emit aggregation passes (default 0: single pass)
 *   "kgram_rank"    1: K >= 2 gram keys by iterated ranking (the path of K * ceil(log2 V) > 63)
 *                   even when the packed term ids fit 64 bits (default 0: automatic)
 *   "agg_grid"      aggregation workgroups, 0 = auto (default 0)
 *   "tok_grid"      tokenizer workgroups, >= 1 (default 5120)
 *   "raw_load_pct"  raw-vocabulary table load of the next build, 10..90 (default 40)
 *   "docid_terms"   1 (default): a record's DOCNO token that is its own term (ASCII letters and
 *                   digits ending in a digit, unchanged by the stemmer) skips the per-distinct
 *                   vocabulary work and is ranked by a merge with the sorted word terms when the
 *                   docids ascend in file order; 0: every raw token through the general path
 *   "sort_digit_bits"  most bits per digit of the term sort's LSD passes, 6..11, or 0 (default:
 *                   11 -- two passes for up to 2^22 terms -- and 8 past 2^30 pairs)
 *   "docid_split"   1 (default): with docid terms (K4b) that push the term ids past 22 bits
 *                   while the word terms need fewer, each record's docid pair is kept beside
 *                   the sort of word-rank keys and merged into the CSR after it; 2: whenever
 *                   the word ranks need fewer bits than the merged ids; 0: one sort of all
 *                   pairs by merged id
 *   "query_table_budget"  bytes a batch's skip table may take (default 0 =
 *                   a quarter of the free HBM); a batch over it is split by
 *                   query range, and queries still overflowing their
 *                   candidate lists whose tile table does not fit run as their
 *                   own compact batch -- every batch of queries of <= 64 terms
 *                   is answered by the window-major scorer, for any k <= 448
 *   "corpus_keep_bytes"  sme_build_index keeps its device copy of the host
 *                   corpus for the next build (no hipMalloc) only up to this
 *                   many bytes (default 16 GiB); larger copies are freed after
 *                   the build, since HBM held there also shrinks the heavy-row
 *                   budget of sme_index_prepare_queries (1/4 of free HBM)
 * Unknown names and out-of-range values are SME_EINVAL. */
int sme_set_option(sme_ctx *ctx, const char *name, int64_t value);

/* Docno mapping file bytes: int32 N, then N x writeUTF(docid), docids sorted
 * (TrecDocnoMapping.writeDocnoData format).  Uploaded once; docno lookup is
 * Arrays.binarySearch over {"", docids...} on the device. */
int sme_load_docno_mapping(sme_ctx *ctx, const uint8_t *mapping_file, size_t n);

/* Docno assignment (NumberTrecDocuments.run + TrecDocnoMapping.writeDocnoData,
 * C/edu/umd/cloud9/collection/trec/NumberTrecDocuments.java:82-168,
 * TrecDocnoMapping.java:92-125): the distinct docids of the corpus's records in
 * UTF-8 byte order, numbered 1.., as the mapping FILE BYTES (int32 N, N x
 * writeUTF(docid)) that sme_load_docno_mapping takes.  *mapping is owned by ctx
 * until its next call. */
int sme_number_documents(sme_ctx *ctx, const uint8_t *corpus, size_t nbytes, const uint8_t **mapping, size_t *n);

/* Doc-shard cut points for `world` shards: cuts[0] = 0, cuts[world] =
 * nbytes, and cuts[g] = the first record start at or after nbytes * g / world,
 * i.e. shard g holds the records a Hadoop split [n g/W, n (g+1)/W) owns
 * (XMLInputFormat.java:110-143,173-198: a record belongs to the split its <DOC>
 * match begins in), found by one record-reader pass over the whole input so a
 * shard built from [cuts[g], cuts[g+1]) has exactly the single reader's records.
 * cuts: world + 1 host entries. */
int sme_split_points(sme_ctx *ctx, const uint8_t *corpus, size_t nbytes, int world, uint64_t *cuts);
int sme_split_points_device(sme_ctx *ctx, const void *d_corpus, size_t nbytes, int world, void *stream,
                            uint64_t *cuts);

/* Build from a host corpus (TREC <DOC>..</DOC> records, one split). Copies to HBM. */
int sme_build_index(sme_ctx *ctx, const uint8_t *corpus, size_t nbytes, sme_index **out);

/* Build from a corpus already resident in device memory (d_corpus on ctx's
 * device, nbytes long); stream may be NULL (default stream).  No host copies
 * of the corpus are made; this is the timed path of bench.py. */
int sme_build_index_device(sme_ctx *ctx, const void *d_corpus, size_t nbytes, void *stream,
                           sme_index **out);

/* CharKGramTermIndexer (C/sa/edu/kaust/indexing/CharKGramTermIndexer.java:74-211, the
 * other PA2-3 job): k = cfg.k (1..5) character k-grams of every '$'+token+'$', each
 * mapped to the set of tokens containing it (JDK 6 HashSet iteration order), written
 * as TextOutputFormat lines "gram\t[t1, t2, ...]\n" into cfg.num_partitions
 * HashPartitioner partitions in Text key order.  One split (one map task); no docno
 * mapping is needed (the job's mapper never reads docids).  The result is an
 * sme_index whose only accessors are the two below and sme_index_free. */
int sme_build_chargram(sme_ctx *ctx, const uint8_t *corpus, size_t nbytes, sme_index **out);
int sme_build_chargram_device(sme_ctx *ctx, const void *d_corpus, size_t nbytes, void *stream,
                              sme_index **out);
/* part-NNNNN text bytes of reduce partition `part` (host buffer owned by the index) */
int sme_chargram_partition_text(sme_index *ix, int part, const uint8_t **buf, size_t *n);
/* distinct k-grams (output lines) and (k-gram, token) set entries */
int sme_chargram_stats(const sme_index *ix, uint64_t *ngrams, uint64_t *npairs);

void sme_index_free(sme_index *ix);

/* N = records mapped (= df of the " " doc-counter key), V = distinct terms
 * (K-grams when K > 1) excluding the doc counter, P = postings (distinct
 * (term, docno)).  K > 1 needs K * ceil(log2(distinct terms)) <= 63. */
int sme_index_stats(const sme_index *ix, uint64_t *N, uint64_t *V, uint64_t *P);

/* Serialized records of reduce partition `part` in key order, framed as in a
 * SequenceFile body: int32 recLen(key+value), int32 keyLen, TermDF bytes,
 * ArrayListWritable<PostingWritable> bytes (all big-endian).  The buffer lives
 * on the host and is owned by ix. */
int sme_index_partition_records(sme_index *ix, int part, const uint8_t **buf, size_t *n);

/* The device half of the same output (the serializer kernels k_ser_*, run once
 * per index): part_offsets (R+1 host entries, may be NULL) gets the byte offset
 * of every partition in the concatenated record stream (partition order), and
 * *device_ms (may be NULL) the serializer's device time.  Replaces the reduce
 * tasks' record writes, TermKGramDocIndexer.java:275 (SequenceFileOutputFormat)
 * + TermDF.java:50-56 + ArrayListWritable.java:90-105. */
int sme_index_serialize(sme_index *ix, uint64_t *part_offsets, float *device_ms);

/* Copy the record bytes of partition `part` (part = -1: every partition, back
 * to back in partition order) from HBM into caller memory dst of cap bytes;
 * *n gets the bytes written.  Pinned dst (hipHostMalloc / hipHostRegister,
 * e.g. a pinned direct ByteBuffer) is one DMA; pageable dst goes through the
 * context's pinned staging buffers.  No intermediate host copy is kept. */
int sme_index_copy_records(sme_index *ix, int part, void *dst, size_t cap, size_t *n);

/* Host copies of the CSR in reduce-output order (tf desc, docno asc) over
 * terms in TermDF key order.  offsets has V+1 entries; true_df has V. */
int sme_index_csr(sme_index *ix, const int64_t **offsets, const int32_t **docno,
                  const int32_t **tf, const int32_t **true_df);

/* Device pointers of the query-side arrays (docno-ascending postings per term
 * and their fp64 TF-IDF weights), for callers that keep data in HBM. */
int sme_index_device_arrays(sme_index *ix, const int64_t **d_offsets, const int32_t **d_docno,
                            const double **d_weight);

/* Term string of index term t (modified-UTF-8 bytes as written by writeUTF);
 * for K > 1 (t is a k-gram) its first element k_gram[0], the forward-index key. */
int sme_index_term(sme_index *ix, int64_t t, const uint8_t **utf8, size_t *n);

/* GalagoTokenizer.processContent on one UTF-8 string, run through the same
 * device kernels as the build.  Tokens (modified UTF-8) are written back to back
 * into buf; offs[i]..offs[i+1] delimits token i (offs has cap_tok+1 entries). */
int sme_tokenize(sme_ctx *ctx, const uint8_t *utf8, size_t n, uint8_t *buf, size_t cap,
                 int64_t *offs, int cap_tok, int *ntok);

/* Map processed terms (UTF-8, offs delimits n terms) to index term ids; -1 if
 * absent (getValue skips unknown terms silently).  For K > 1 a term maps to the
 * LAST k-gram (TermDF order) starting with it, as the forward index's Hashtable
 * keeps it (IntDocVectorsForwardIndex.java:107-120). */
int sme_lookup_terms(sme_index *ix, const uint8_t *terms, const int64_t *offs, int n,
                     int32_t *term_ids);

/* Batched rank(): query q has term ids term_ids[q_offsets[q] .. q_offsets[q+1])
 * in query-token order (duplicates count twice, -1 entries are skipped; an id
 * outside [-1, V) is SME_EINVAL here and skipped like -1 by the device entry).
 * k <= 1792 (SME_ELIMIT above; k > 448 and queries of more than 64 terms take the
 * streaming kernel: up to 1024 terms, 256 in SME_TIE_REFERENCE order).
 * Writes k docnos / scores per query (score desc, docno asc), padded with
 * docno -1 / score 0 when fewer than k documents match. */
int sme_query_topk(sme_index *ix, const int32_t *term_ids, const int64_t *q_offsets, int nq,
                   int k, int32_t *out_docno, double *out_score);
/* The same plus every result's tie word (see sme_query_topk_device_tie). */
int sme_query_topk_tie(sme_index *ix, const int32_t *term_ids, const int64_t *q_offsets, int nq,
                       int k, int32_t *out_docno, double *out_score, uint32_t *out_tie);

/* Query-side structures of an index (the role the reference's forward index,
 * BuildIntDocVectorsForwardIndex.java:84-158, plays for rank()): heavy-term tf
 * and impact rows with their block maxima (at most a quarter of the free HBM --
 * counting the device blocks the context holds for reuse --, 64 GB), and one
 * 4-byte window-pass word per posting of the other terms (if 4 B per posting
 * fits a quarter of the free HBM; else the window-major scorer is
 * not used and batches take the block-max path).  Built once per index; the
 * impact rows and their scale depend on idf, so sme_index_reweight DROPS them:
 * call this after the last reweight (sme_query_topk* rebuilds them on first
 * use otherwise, inside that call).  *ms (may be NULL) gets the device time. */
int sme_index_prepare_queries(sme_index *ix, void *stream, float *ms);

/* Same with all arrays already in device memory (timed path). */
int sme_query_topk_device(sme_index *ix, const int32_t *d_term_ids, const int64_t *d_q_offsets,
                          int nq, int k, int32_t *d_out_docno, double *d_out_score, void *stream);

/* The same plus the tie word of every result (d_out_tie[nq * k], 0xFFFFFFFF
 * padding): 0 under SME_TIE_DOCNO; under SME_TIE_REFERENCE (first query token
 * holding the document) << 24 | (2^24 - 1 - its tf).  Results of doc shards
 * merge by (score desc, tie asc, docno asc) into the single index's order
 * (dist.py merge_topk_owner). */
int sme_query_topk_device_tie(sme_index *ix, const int32_t *d_term_ids, const int64_t *d_q_offsets,
                              int nq, int k, int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie,
                              void *stream);

/* 128-bit fingerprint of every index term (two u64 per term into device memory
 * d_out[2 V]): equal term strings (k-grams) on different shards get equal
 * fingerprints, so a multi-GPU df exchange can key the all-reduce on them
 * without gathering and sorting term strings (dist.py global_df). */
int sme_index_term_fingerprints(sme_index *ix, uint64_t *d_out, void *stream);

/* Global df of a doc-sharded build by owner rank (the reducer's df =
 * postings length summed over the map outputs, TermKGramDocIndexer.java:175-183).
 * Rows are (fp[2i], fp[2i+1], df[i]) in device memory; a row's owner is
 * fp[2i] % world.
 *   pack:   rows grouped by owner into send_fp[2n] / send_df[n] (owner 0's rows
 *           first, ...), pos[i] = send slot of row i, counts[world] (host) = rows
 *           per owner -- the layout of one all_to_all
 *   sum:    for every received row, out[i] = the sum of df over all received rows
 *           with the same 128-bit fingerprint; *distinct = fingerprints seen
 *   unpack: out[i] = ret[pos[i]] (the owners' sums, returned in send order, back
 *           in local row order)
 * Replaces the Hadoop shuffle's grouping of the doc-counter / df by key. */
int sme_df_owner_pack(sme_ctx *ctx, const uint64_t *d_fp, const int64_t *d_df, int64_t n, int world,
                      uint64_t *d_send_fp, int64_t *d_send_df, int64_t *d_pos, int64_t *counts, void *stream);
int sme_df_owner_sum(sme_ctx *ctx, const uint64_t *d_fp, const int64_t *d_df, int64_t n, int64_t *d_out,
                     int64_t *distinct, void *stream);
int sme_df_owner_unpack(sme_ctx *ctx, const int64_t *d_ret, const int64_t *d_pos, int64_t n, int64_t *d_out,
                        void *stream);

/* Query-owner merge (dist.merge_topk_owner): rows x m candidates
 * (d_score / d_docno / optional d_tie, row-major, any order, docno -1 pads, e.g.
 * the W shards' top-k lists of the queries this rank owns) -> per row the best k
 * in (score desc, tie asc, docno asc) order, docno -1 / score 0 / tie ~0 pads.
 * The tie word is sme_query_topk_tie's (0 in the north-star docno order), so the
 * merged rows equal one index's top-k (IntDocVectorsForwardIndex.java:215-222:
 * Collections.sort over the candidates, first k).  k <= 2048.  Device memory;
 * synchronized on return. */
int sme_topk_merge_rows(sme_ctx *ctx, const double *d_score, const int32_t *d_docno, const uint32_t *d_tie,
                        int64_t rows, int m, int k, int32_t *d_out_docno, double *d_out_score, uint32_t *d_out_tie,
                        void *stream);

/* Owner side of the cross-shard duplicate-docid check (dist.docno_duplicates):
 * d_rows = n (key, source rank) pairs (u64, keys zero-extended 32-bit docnos)
 * received by the keys' owner rank (grouped with sme_df_owner_pack); *count =
 * distinct keys that arrive from two or more source ranks.  A docid held by two
 * shards is one posting with summed tf in the reference's single reducer
 * (TermKGramDocIndexer.java:202-210), so per-shard scoring must refuse it. */
int sme_count_shared_keys(sme_ctx *ctx, const uint64_t *d_rows, int64_t n, int64_t *count, void *stream);

/* Recompute the fp64 TF-IDF weights of a doc-sharded index with global
 * statistics: n_global = records over all shards (all-reduced doc counter),
 * d_df_global = per local term the all-reduced df (device int64[V]) or NULL to
 * keep the shard's own df (SME_IDF_TRUE_DF only; reference mode uses stored df 1). */
int sme_index_reweight(sme_index *ix, int64_t n_global, const int64_t *d_df_global, void *stream);

/* Synthetic Zipfian TREC corpus generated directly in HBM (bench / tests; same
 * bytes as synth.py).  vocab/vocab_off/cdf are host arrays (V words, V+1
 * offsets, V cumulative probabilities).  *d_corpus is freed with sme_synth_free. */
int sme_synth_corpus(int device, const uint8_t *vocab, const int64_t *vocab_off, int64_t V, const double *cdf,
                     int64_t n_docs, int64_t d0, uint64_t seed, int len_lo, int len_hi, void **d_corpus,
                     size_t *nbytes);
void sme_synth_free(void *d_corpus);

/* Calibration (bench.py): achievable HBM bandwidth of a streaming device copy of
 * `bytes` (x reps, after a warm-up); *gbps = read + write bytes / kernel time. */
int sme_hbm_copy_bench(int device, size_t bytes, int reps, double *gbps);

/* Reference-layout output from doc shards (the job's R part files,
 * TermKGramDocIndexer.java:189-211,246-275): partition p is reduced by rank
 * p % world.  pack: this shard's terms grouped by owner rank as `world` blobs
 * laid out back to back at d_out (device memory; NULL = only fill sizes[world],
 * each blob's bytes): the terms (String.compareTo order), their postings in
 * reduce order, and the shard's record docnos for the owner of the " " doc
 * counter's partition.  merge: the n blobs a rank received (one per shard, in
 * shard order, back to back at d_blobs) -> a records-only index whose
 * partitions p with p % world == rank hold exactly what the reference's single
 * reducer writes for the shards' map tasks (postings merged per term by
 * MyReducer.reduce, :189-211: docno sort, equal docnos summed, stable tf-desc
 * sort; one doc-counter list per map task).  Read it with sme_index_serialize /
 * sme_index_copy_records; it has no query side (query entry points: SME_EINVAL). */
int sme_index_pack_pieces(sme_index *ix, int world, void *d_out, uint64_t *sizes, void *stream);
/* Device pointer to the docnos of the index's records in input order (*n = N;
 * the map task's doc-counter postings, TermKGramDocIndexer.java:84-90,126). */
int sme_index_record_docnos(sme_index *ix, const int32_t **d_docno, int64_t *n);
int sme_merge_pieces(sme_ctx *ctx, const void *d_blobs, const uint64_t *sizes, int n, void *stream,
                     sme_index **out);

/* Timing of the last build, per stage, in milliseconds (device events on the
 * build stream), as a JSON object; "tok_kernel" brackets exactly the tokenizer
 * launch and "query_kernel" (if a query batch ran) the last scoring launch. */
int sme_last_build_profile(const sme_ctx *ctx, const char **json);

#ifdef __cplusplus
}
#endif
#endif
