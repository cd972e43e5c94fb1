/*
 * oracle_index.c -- restatement of the index job (map + shuffle + reduce), its
 * output bytes, and the query ranking.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Record split   XMLRecordReader.next / readUntilMatch
 *                C/edu/umd/cloud9/collection/XMLInputFormat.java:110-143,173-198
 * docid          TrecDocument.getDocid  C/edu/umd/cloud9/collection/trec/TrecDocument.java:76-89
 * docno          TrecDocnoMapping.getDocno (Arrays.binarySearch) / readDocnoData
 *                C/edu/umd/cloud9/collection/trec/TrecDocnoMapping.java:67-69,137-155
 * map            TermKGramDocIndexer.MyMapper.map
 *                C/sa/edu/kaust/indexing/TermKGramDocIndexer.java:84-90,119-160
 * shuffle        [Hadoop] HashPartitioner on TermDF.hashCode (C/sa/edu/kaust/io/TermDF.java:79-81),
 *                key order TermDF.compareTo (TermDF.java:64-70)
 * reduce         TermKGramDocIndexer.MyReducer.reduce  TermKGramDocIndexer.java:168-213,
 *                PostingWritable.compareTo  C/sa/edu/kaust/io/PostingWritable.java:57-59
 * bytes          TermDF.write 50-56, ArrayListWritable.write
 *                C/edu/umd/cloud9/io/array/ArrayListWritable.java:90-105, PostingWritable.write 46-49
 * query          IntDocVectorsForwardIndex.rank / DocScore
 *                C/sa/edu/kaust/fwindex/IntDocVectorsForwardIndex.java:192-223,329-371
 *
 * This is the "ref-faithful" restatement: every map-output record is
 * materialised, sorted by string keys with a comparison merge sort, and reduced
 * with the reference's two list sorts.  It is deliberately not fast.
 */
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ------------------------------------------------------------------ */
/* error reporting                                                      */
static char g_err[256];
const char *or_last_error(void) { return g_err; }

/* ------------------------------------------------------------------ */
/* record reader                                                        */

/* readUntilMatch: advances *pos over bytes [.., n); returns 1 on full match.
 * withinBlock: bytes are appended to the record (we track the span instead). */
static int read_until_match(const uint8_t *b, size_t n, size_t *pos, size_t end, const char *m,
                            int withinBlock) {
  int ml = (int)strlen(m);
  int i = 0;
  for (;;) {
    if (*pos >= n) {
      (*pos)++;
      return 0; /* b == -1: EOF (pos still incremented, as the reference does) */
    }
    int c = b[*pos];
    (*pos)++;
    if (c == (unsigned char)m[i]) {
      i++;
      if (i >= ml) return 1;
    } else {
      i = 0;
    }
    if (!withinBlock && i == 0 && *pos >= end) return 0;
  }
}

typedef struct {
  size_t off, len;
} rec;

/* Records of one split [start, end) in the XMLRecordReader order. */
static int split_records(const uint8_t *b, size_t n, size_t start, size_t end, rec **out,
                         int *nout) {
  size_t pos = start;
  int cap = 16, cnt = 0;
  rec *r = (rec *)malloc(sizeof(rec) * cap);
  while (pos < end) {
    if (!read_until_match(b, n, &pos, end, "<DOC>", 0)) break;
    size_t rs = pos - 5;
    if (!read_until_match(b, n, &pos, end, "</DOC>", 1)) break;
    if (cnt == cap) {
      cap *= 2;
      r = (rec *)realloc(r, sizeof(rec) * cap);
    }
    r[cnt].off = rs;
    r[cnt].len = pos - rs;
    cnt++;
  }
  *out = r;
  *nout = cnt;
  return 0;
}

/* ------------------------------------------------------------------ */
/* docno mapping                                                        */
typedef struct {
  jstr *ids; /* ids[0] = "" sentinel */
  int n;     /* entries including sentinel */
} mapping;

static int read_u16be(const uint8_t *p) { return (p[0] << 8) | p[1]; }
static int32_t read_i32be(const uint8_t *p) {
  return (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
}

/* DataInput.readUTF: modified UTF-8 -> UTF-16 */
static int read_mutf8(const uint8_t *p, int len, jstr *out) {
  out->n = 0;
  int i = 0;
  while (i < len) {
    unsigned c = p[i];
    if (c < 0x80) {
      js_push(out, (uint16_t)c);
      i++;
    } else if ((c & 0xE0) == 0xC0) {
      if (i + 1 >= len) return -1;
      js_push(out, (uint16_t)(((c & 0x1F) << 6) | (p[i + 1] & 0x3F)));
      i += 2;
    } else if ((c & 0xF0) == 0xE0) {
      if (i + 2 >= len) return -1;
      js_push(out, (uint16_t)(((c & 0x0F) << 12) | ((p[i + 1] & 0x3F) << 6) | (p[i + 2] & 0x3F)));
      i += 3;
    } else {
      return -1;
    }
  }
  return 0;
}

static int load_mapping(const uint8_t *m, size_t n, mapping *mp) {
  if (n < 4) {
    snprintf(g_err, sizeof g_err, "mapping file too short");
    return -1;
  }
  int cnt = read_i32be(m);
  if (cnt < 0) {
    snprintf(g_err, sizeof g_err, "negative mapping count");
    return -1;
  }
  mp->n = cnt + 1;
  mp->ids = (jstr *)calloc((size_t)mp->n, sizeof(jstr));
  size_t p = 4;
  for (int i = 1; i < mp->n; i++) {
    if (p + 2 > n) {
      snprintf(g_err, sizeof g_err, "truncated mapping file");
      return -1;
    }
    int l = read_u16be(m + p);
    p += 2;
    if (p + (size_t)l > n) {
      snprintf(g_err, sizeof g_err, "truncated mapping file");
      return -1;
    }
    js_init(&mp->ids[i]);
    if (read_mutf8(m + p, l, &mp->ids[i]) < 0) {
      snprintf(g_err, sizeof g_err, "bad modified UTF-8 in mapping");
      return -1;
    }
    p += (size_t)l;
  }
  js_init(&mp->ids[0]);
  return 0;
}

/* Arrays.binarySearch(Object[], key) */
static int get_docno(const mapping *mp, const uint16_t *k, int kn) {
  int low = 0, high = mp->n - 1;
  while (low <= high) {
    int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
    int c = js_cmp(mp->ids[mid].p, mp->ids[mid].n, k, kn);
    if (c < 0)
      low = mid + 1;
    else if (c > 0)
      high = mid - 1;
    else
      return mid;
  }
  return -(low + 1);
}

/* TrecDocument.getDocid: trim(substring(indexOf("<DOCNO>")+7, indexOf("</DOCNO>", start))) */
static int get_docid(const jstr *doc, jstr *id) {
  static const char *o = "<DOCNO>", *c = "</DOCNO>";
  int start = -1;
  for (int i = 0; i + 7 <= doc->n && start < 0; i++) {
    int k = 0;
    while (k < 7 && doc->p[i + k] == (unsigned char)o[k]) k++;
    if (k == 7) start = i;
  }
  if (start < 0) {
    id->n = 0;
    return 0;
  }
  int end = -1;
  for (int i = start; i + 8 <= doc->n && end < 0; i++) {
    int k = 0;
    while (k < 8 && doc->p[i + k] == (unsigned char)c[k]) k++;
    if (k == 8) end = i;
  }
  if (end < 0 || end < start + 7) {
    snprintf(g_err, sizeof g_err, "StringIndexOutOfBoundsException in getDocid (no </DOCNO>)");
    return -1;
  }
  int b = start + 7, e = end;
  while (b < e && doc->p[b] <= 0x20) b++;
  while (e > b && doc->p[e - 1] <= 0x20) e--;
  js_set(id, doc->p + b, e - b);
  return 0;
}

/* ------------------------------------------------------------------ */
/* map output records                                                   */
typedef struct {
  const jstr *gram; /* K strings (points into a doc's token array), or NULL for " " */
  int docno, tf;
  int part;
} mrec;

typedef struct {
  jstr_list toks; /* stems of one record */
} docbuf;

static jstr SPACE_KEY; /* " " */
static int g_K;

static const jstr *gram_at(const mrec *r, int i) { return r->gram ? &r->gram[i] : &SPACE_KEY; }
static int gram_len(const mrec *r) { return r->gram ? g_K : 1; }

/* TermDF.compareTo */
static int key_cmp(const mrec *a, const mrec *b) {
  int al = gram_len(a), bl = gram_len(b);
  for (int i = 0; i < al && i < bl; i++) {
    const jstr *x = gram_at(a, i), *y = gram_at(b, i);
    int r = js_cmp(x->p, x->n, y->p, y->n);
    if (r) return r;
  }
  return al - bl;
}

/* Arrays.hashCode(Object[]) of the k-gram, HashPartitioner */
static int partition_of(const mrec *r, int R) {
  uint32_t h = 1;
  for (int i = 0; i < gram_len(r); i++) {
    const jstr *s = gram_at(r, i);
    h = 31u * h + (uint32_t)js_hash(s->p, s->n);
  }
  return (int)(((int32_t)h & 0x7fffffff) % R);
}

static int mrec_cmp(const mrec *a, const mrec *b) {
  if (a->part != b->part) return a->part - b->part;
  return key_cmp(a, b);
}

/* stable merge sort (the shuffle's order within a key does not matter for the
 * real terms; for " " we keep emission order, which the tests compare as a multiset) */
static void msort(mrec *a, mrec *tmp, size_t n) {
  if (n < 2) return;
  size_t h = n / 2;
  msort(a, tmp, h);
  msort(a + h, tmp, n - h);
  if (mrec_cmp(&a[h - 1], &a[h]) <= 0) return;
  size_t i = 0, j = h, k = 0;
  while (i < h && j < n) tmp[k++] = (mrec_cmp(&a[j], &a[i]) < 0) ? a[j++] : a[i++];
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, n * sizeof(mrec));
}

typedef struct {
  int docno, tf;
} posting;

/* ------------------------------------------------------------------ */
/* index                                                                */
typedef struct {
  jstr *gram; /* K strings (or 1 for " ") */
  int k;
  int df_field;      /* stored TermDF.df */
  posting *post;     /* reduce output order */
  int npost;
  int part;
} term_rec;

typedef struct or_index {
  int K, R;
  int N;             /* df of " " = number of records mapped */
  term_rec *terms;   /* global key order (" " first) */
  int nterms;
  uint8_t **part_bytes;
  size_t *part_len;
  int *lk;           /* lazily built: open-addressed table of the forward-index lookup (find_term) */
  int lk_cap;
} or_index;

static void stable_sort_postings(posting *a, posting *tmp, int n, int by_tf) {
  /* Collections.sort is a stable merge sort; take left while compare(left,right) <= 0.
   * reducer comparator: o1.docNo - o2.docNo;  PostingWritable.compareTo: o.tf - tf */
  if (n < 2) return;
  int h = n / 2;
  stable_sort_postings(a, tmp, h, by_tf);
  stable_sort_postings(a + h, tmp, n - h, by_tf);
  int i = 0, j = h, k = 0;
  while (i < h && j < n) {
    int32_t c = by_tf ? (int32_t)((uint32_t)a[j].tf - (uint32_t)a[i].tf)
                      : (int32_t)((uint32_t)a[i].docno - (uint32_t)a[j].docno);
    tmp[k++] = (c <= 0) ? a[i++] : a[j++];
  }
  while (i < h) tmp[k++] = a[i++];
  while (j < n) tmp[k++] = a[j++];
  memcpy(a, tmp, (size_t)n * sizeof(posting));
}

static void put_i32(uint8_t **p, int32_t v) {
  uint32_t u = (uint32_t)v;
  (*p)[0] = (uint8_t)(u >> 24);
  (*p)[1] = (uint8_t)(u >> 16);
  (*p)[2] = (uint8_t)(u >> 8);
  (*p)[3] = (uint8_t)u;
  *p += 4;
}

static const char *CLASSNAME = "sa.edu.kaust.io.PostingWritable";

static size_t key_bytes(const term_rec *t) {
  size_t s = 8;
  for (int i = 0; i < t->k; i++) s += 2 + (size_t)mutf8_len(t->gram[i].p, t->gram[i].n);
  return s;
}
static size_t val_bytes(const term_rec *t) {
  return 4 + (t->npost > 0 ? 2 + strlen(CLASSNAME) + 8 * (size_t)t->npost : 0);
}

/* SequenceFile record framing: int32 recLen(key+value), int32 keyLen, key, value */
static void serialize(or_index *ix) {
  ix->part_bytes = (uint8_t **)calloc((size_t)ix->R, sizeof(uint8_t *));
  ix->part_len = (size_t *)calloc((size_t)ix->R, sizeof(size_t));
  for (int t = 0; t < ix->nterms; t++) {
    term_rec *tr = &ix->terms[t];
    ix->part_len[tr->part] += 8 + key_bytes(tr) + val_bytes(tr);
  }
  uint8_t **cur = (uint8_t **)calloc((size_t)ix->R, sizeof(uint8_t *));
  for (int r = 0; r < ix->R; r++) cur[r] = ix->part_bytes[r] = (uint8_t *)malloc(ix->part_len[r] + 1);
  for (int t = 0; t < ix->nterms; t++) {
    term_rec *tr = &ix->terms[t];
    uint8_t **p = &cur[tr->part];
    size_t kb = key_bytes(tr), vb = val_bytes(tr);
    put_i32(p, (int32_t)(kb + vb));
    put_i32(p, (int32_t)kb);
    put_i32(p, tr->k);
    for (int i = 0; i < tr->k; i++) {
      int l = mutf8_len(tr->gram[i].p, tr->gram[i].n);
      (*p)[0] = (uint8_t)(l >> 8);
      (*p)[1] = (uint8_t)l;
      *p += 2;
      *p += mutf8_encode(tr->gram[i].p, tr->gram[i].n, *p);
    }
    put_i32(p, tr->df_field);
    put_i32(p, tr->npost);
    if (tr->npost > 0) {
      size_t cl = strlen(CLASSNAME);
      (*p)[0] = (uint8_t)(cl >> 8);
      (*p)[1] = (uint8_t)cl;
      *p += 2;
      memcpy(*p, CLASSNAME, cl);
      *p += cl;
      for (int i = 0; i < tr->npost; i++) {
        put_i32(p, tr->post[i].docno);
        put_i32(p, tr->post[i].tf);
      }
    }
  }
  free(cur);
}

void or_index_free(or_index *ix) {
  if (!ix) return;
  for (int t = 0; t < ix->nterms; t++) {
    for (int i = 0; i < ix->terms[t].k; i++) js_free(&ix->terms[t].gram[i]);
    free(ix->terms[t].gram);
    free(ix->terms[t].post);
  }
  free(ix->terms);
  if (ix->part_bytes)
    for (int r = 0; r < ix->R; r++) free(ix->part_bytes[r]);
  free(ix->part_bytes);
  free(ix->part_len);
  free(ix->lk);
  free(ix);
}

/*
 * Build the index.  splits: n_splits+1 byte offsets (split i = [s[i], s[i+1]));
 * NULL means one split over the whole corpus (Hadoop local mode, one map task).
 */
or_index *or_build_index(const uint8_t *corpus, size_t n, const uint8_t *map_bytes, size_t map_len,
                         int K, int R, const uint64_t *splits, int n_splits) {
  g_err[0] = 0;
  if (K < 1 || R < 1) {
    snprintf(g_err, sizeof g_err, "bad K/R");
    return NULL;
  }
  mapping mp;
  if (load_mapping(map_bytes, map_len, &mp) < 0) return NULL;
  js_init(&SPACE_KEY);
  js_set_ascii(&SPACE_KEY, " ");
  g_K = K;

  uint64_t one_split[2] = {0, (uint64_t)n};
  if (!splits) {
    splits = one_split;
    n_splits = 1;
  }

  size_t mcap = 1024, mn = 0;
  mrec *m = (mrec *)malloc(sizeof(mrec) * mcap);
  size_t dcap = 64, dn = 0;
  docbuf *docs = (docbuf *)malloc(sizeof(docbuf) * dcap);
  int N = 0;
  jstr text, id;
  js_init(&text);
  js_init(&id);
  int fail = 0;

  for (int s = 0; s < n_splits && !fail; s++) {
    rec *recs;
    int nrec;
    split_records(corpus, n, (size_t)splits[s], (size_t)splits[s + 1], &recs, &nrec);
    posting shared = {0, 0}; /* MyMapper.posting, fresh per map task */
    for (int r = 0; r < nrec; r++) {
      utf8_to_utf16(corpus + recs[r].off, recs[r].len, &text);
      if (get_docid(&text, &id) < 0) {
        fail = 1;
        break;
      }
      int docno = get_docno(&mp, id.p, id.n);
      N++;
      if (mn + 2 > mcap) {
        mcap *= 2;
        m = (mrec *)realloc(m, sizeof(mrec) * mcap);
      }
      m[mn].gram = NULL;
      m[mn].docno = shared.docno;
      m[mn].tf = shared.tf;
      mn++;
      if (dn == dcap) {
        dcap *= 2;
        docs = (docbuf *)realloc(docs, sizeof(docbuf) * dcap);
      }
      jl_init(&docs[dn].toks);
      or_process_content(text.p, text.n, &docs[dn].toks);
      shared.docno = docno;
      shared.tf = 1;
      int T = docs[dn].toks.n;
      for (int i = 0; i + K <= T; i++) {
        if (mn + 1 > mcap) {
          mcap *= 2;
          m = (mrec *)realloc(m, sizeof(mrec) * mcap);
        }
        m[mn].gram = &docs[dn].toks.v[i]; /* toks.v is final once processContent returned */
        m[mn].docno = docno;
        m[mn].tf = 1;
        mn++;
      }
      dn++;
    }
    free(recs);
  }
  js_free(&text);
  js_free(&id);
  if (fail) {
    for (size_t d = 0; d < dn; d++) jl_free(&docs[d].toks);
    free(docs);
    free(m);
    free(mp.ids);
    return NULL;
  }
  for (size_t i = 0; i < mn; i++) m[i].part = partition_of(&m[i], R);

  mrec *tmp = (mrec *)malloc(sizeof(mrec) * (mn ? mn : 1));
  msort(m, tmp, mn);
  free(tmp);

  or_index *ix = (or_index *)calloc(1, sizeof(or_index));
  ix->K = K;
  ix->R = R;
  ix->N = N;
  /* reduce, per partition, groups of equal keys */
  size_t tcap = 1024;
  ix->terms = (term_rec *)malloc(sizeof(term_rec) * tcap);
  for (size_t i = 0; i < mn;) {
    size_t j = i + 1;
    while (j < mn && m[j].part == m[i].part && key_cmp(&m[j], &m[i]) == 0) j++;
    if ((size_t)ix->nterms == tcap) {
      tcap *= 2;
      ix->terms = (term_rec *)realloc(ix->terms, sizeof(term_rec) * tcap);
    }
    term_rec *tr = &ix->terms[ix->nterms++];
    tr->k = gram_len(&m[i]);
    tr->gram = (jstr *)calloc((size_t)tr->k, sizeof(jstr));
    for (int g = 0; g < tr->k; g++) js_set(&tr->gram[g], gram_at(&m[i], g)->p, gram_at(&m[i], g)->n);
    tr->part = m[i].part;
    int cnt = (int)(j - i);
    posting *res = (posting *)malloc(sizeof(posting) * (size_t)cnt);
    for (int q = 0; q < cnt; q++) {
      res[q].docno = m[i + q].docno;
      res[q].tf = m[i + q].tf;
    }
    if (m[i].gram == NULL) { /* doc counter: term.getK_gram()[0].equals(" ") */
      tr->df_field = cnt;
      tr->post = res;
      tr->npost = cnt;
    } else {
      posting *tmpp = (posting *)malloc(sizeof(posting) * (size_t)cnt);
      stable_sort_postings(res, tmpp, cnt, 0);
      int w = 0;
      for (int q = 0; q < cnt; q++) {
        int sum = res[q].tf;
        int r = q + 1;
        while (r < cnt && res[r].docno == res[q].docno) sum += res[r++].tf;
        res[w].docno = res[q].docno;
        res[w].tf = sum;
        w++;
        q = r - 1;
      }
      stable_sort_postings(res, tmpp, w, 1);
      free(tmpp);
      tr->df_field = 1; /* T1: reducer never updates df of real terms */
      tr->post = res;
      tr->npost = w;
    }
    i = j;
  }
  free(m);
  for (size_t d = 0; d < dn; d++) jl_free(&docs[d].toks);
  free(docs);
  for (int i = 0; i < mp.n; i++) js_free(&mp.ids[i]);
  free(mp.ids);
  serialize(ix);
  return ix;
}

/* ---- accessors (ctypes) ---- */
int or_index_nterms(const or_index *ix) { return ix->nterms; }
int or_index_N(const or_index *ix) { return ix->N; }
size_t or_index_part_len(const or_index *ix, int part) { return ix->part_len[part]; }
const uint8_t *or_index_part_bytes(const or_index *ix, int part) { return ix->part_bytes[part]; }
int or_index_term_part(const or_index *ix, int t) { return ix->terms[t].part; }
int or_index_term_npost(const or_index *ix, int t) { return ix->terms[t].npost; }
int or_index_term_df_field(const or_index *ix, int t) { return ix->terms[t].df_field; }
int or_index_term_k(const or_index *ix, int t) { return ix->terms[t].k; }
/* modified-UTF-8 bytes of gram element g into buf (cap bytes); returns length */
int or_index_term_gram(const or_index *ix, int t, int g, uint8_t *buf, int cap) {
  const jstr *s = &ix->terms[t].gram[g];
  int l = mutf8_len(s->p, s->n);
  if (l > cap) return -l;
  mutf8_encode(s->p, s->n, buf);
  return l;
}
void or_index_term_postings(const or_index *ix, int t, int32_t *docno, int32_t *tf) {
  for (int i = 0; i < ix->terms[t].npost; i++) {
    docno[i] = ix->terms[t].post[i].docno;
    tf[i] = ix->terms[t].post[i].tf;
  }
}

/* ------------------------------------------------------------------ */
/* query: rank()                                                        */

/* TermDF.compareTo on two index terms (TermDF.java:64-70) */
static int term_key_cmp(const term_rec *a, const term_rec *b) {
  int m = a->k < b->k ? a->k : b->k;
  for (int i = 0; i < m; i++) {
    int c = js_cmp(a->gram[i].p, a->gram[i].n, b->gram[i].p, b->gram[i].n);
    if (c) return c;
  }
  return a->k - b->k;
}

static int find_term_scan(const or_index *ix, const uint16_t *w, int n) {
  /* IntDocVectorsForwardIndex keys the forward index by k_gram[0] (T11): the
   * forward file lists every record in global TermDF order
   * (BuildIntDocVectorsForwardIndex.java:139-153) and the ctor's Hashtable.put
   * keeps the LAST entry per first element (IntDocVectorsForwardIndex.java:107-120). */
  int best = -1;
  for (int t = 0; t < ix->nterms; t++) {
    const jstr *g = &ix->terms[t].gram[0];
    if (g->n == n && (n == 0 || memcmp(g->p, w, (size_t)n * 2) == 0))
      if (best < 0 || term_key_cmp(&ix->terms[t], &ix->terms[best]) > 0) best = t;
  }
  return best;
}

static uint32_t js_fnv(const uint16_t *w, int n) {
  uint32_t h = 2166136261u;
  for (int i = 0; i < n; i++) h = (h ^ w[i]) * 16777619u;
  return h;
}

/* The same result as find_term_scan, through a table of the best term per
 * first element (built once per index: the scan is O(V) per query term). */
static int find_term(const or_index *cix, const uint16_t *w, int n) {
  or_index *ix = (or_index *)cix;
  if (!ix->lk) {
    int cap = 16;
    while (cap < 2 * ix->nterms + 16) cap <<= 1;
    ix->lk = (int *)malloc(sizeof(int) * (size_t)cap);
    for (int i = 0; i < cap; i++) ix->lk[i] = -1;
    ix->lk_cap = cap;
    for (int t = 0; t < ix->nterms; t++) {
      const jstr *g = &ix->terms[t].gram[0];
      uint32_t s = js_fnv(g->p, g->n) & (uint32_t)(cap - 1);
      for (;; s = (s + 1) & (uint32_t)(cap - 1)) {
        int o = ix->lk[s];
        if (o < 0) {
          ix->lk[s] = t;
          break;
        }
        const jstr *h = &ix->terms[o].gram[0];
        if (h->n == g->n && (g->n == 0 || memcmp(h->p, g->p, (size_t)g->n * 2) == 0)) {
          if (term_key_cmp(&ix->terms[t], &ix->terms[o]) > 0) ix->lk[s] = t;
          break;
        }
      }
    }
  }
  uint32_t s = js_fnv(w, n) & (uint32_t)(ix->lk_cap - 1);
  for (;; s = (s + 1) & (uint32_t)(ix->lk_cap - 1)) {
    int o = ix->lk[s];
    if (o < 0) return -1;
    const jstr *h = &ix->terms[o].gram[0];
    if (h->n == n && (n == 0 || memcmp(h->p, w, (size_t)n * 2) == 0)) return o;
  }
}

typedef struct {
  int docId;
  double score;
  int first; /* first-encounter index */
} docscore;

/* DocScore.compareTo: (int)Math.ceil(o.score - score) */
static int ds_cmp_ref(const docscore *a, const docscore *b) {
  double d = ceil(b->score - a->score);
  if (d != d) return 0;
  if (d >= 2147483647.0) return INT_MAX;
  if (d <= -2147483648.0) return INT_MIN;
  return (int)d;
}

/* Java 6 Arrays.mergeSort(Object[] src, Object[] dest, low, high, off) */
static void legacy_merge_sort(docscore *src, docscore *dest, int low, int high, int off) {
  int length = high - low;
  if (length < 7) {
    for (int i = low; i < high; i++)
      for (int j = i; j > low && ds_cmp_ref(&dest[j - 1], &dest[j]) > 0; j--) {
        docscore t = dest[j];
        dest[j] = dest[j - 1];
        dest[j - 1] = t;
      }
    return;
  }
  int destLow = low, destHigh = high;
  low += off;
  high += off;
  int mid = (int)(((unsigned)low + (unsigned)high) >> 1);
  legacy_merge_sort(dest, src, low, mid, -off);
  legacy_merge_sort(dest, src, mid, high, -off);
  if (ds_cmp_ref(&src[mid - 1], &src[mid]) <= 0) {
    memcpy(dest + destLow, src + low, (size_t)length * sizeof(docscore));
    return;
  }
  for (int i = destLow, p = low, q = mid; i < destHigh; i++) {
    if (q >= high || (p < mid && ds_cmp_ref(&src[p], &src[q]) <= 0))
      dest[i] = src[p++];
    else
      dest[i] = src[q++];
  }
}

/*
 * JDK 7 Collections.sort over the same comparator: java.util.ComparableTimSort
 * (OpenJDK 7 GA, the default since Java 7 unless -Djava.util.Arrays.
 * useLegacyMergeSort=true; not vendored in the reference -- restated from the
 * published source).  Collections.sort(List) -> Arrays.sort(Object[]) ->
 * ComparableTimSort.sort: runs (countRunAndMakeAscending, reversed when strictly
 * descending by compareTo < 0), binary insertion to minRun, the JDK 7 GA
 * mergeCollapse invariant (before the JDK-8072909 fix), gallopLeft /
 * gallopRight and mergeLo / mergeHi with MIN_GALLOP 7.  Every test is `< 0`,
 * `<= 0`, `> 0` or `>= 0` on compareTo exactly as the Java source asks it, so
 * the broken DocScore comparator (T5) is applied the way the JVM applies it.
 * A merge that finds the contract violated throws IllegalArgumentException
 * ("Comparison method violates its general contract!") in Java: returned here
 * as -1 (the reference's rank() would fail).
 */
enum { TS_MIN_MERGE = 32, TS_MIN_GALLOP = 7 };
typedef struct {
  docscore *a, *tmp;
  int tmplen, min_gallop, stack;
  int base[85], len[85];
  int err;
} tsort;

static int ts_cmp(const docscore *x, const docscore *y) { return ds_cmp_ref(x, y); } /* x.compareTo(y) */

static void ts_reverse(docscore *a, int lo, int hi) {
  hi--;
  while (lo < hi) {
    docscore t = a[lo];
    a[lo++] = a[hi];
    a[hi--] = t;
  }
}

static int ts_count_run(docscore *a, int lo, int hi) {
  int runHi = lo + 1;
  if (runHi == hi) return 1;
  if (ts_cmp(&a[runHi++], &a[lo]) < 0) {
    while (runHi < hi && ts_cmp(&a[runHi], &a[runHi - 1]) < 0) runHi++;
    ts_reverse(a, lo, runHi);
  } else {
    while (runHi < hi && ts_cmp(&a[runHi], &a[runHi - 1]) >= 0) runHi++;
  }
  return runHi - lo;
}

static void ts_binary_sort(docscore *a, int lo, int hi, int start) {
  if (start == lo) start++;
  for (; start < hi; start++) {
    docscore pivot = a[start];
    int left = lo, right = start;
    while (left < right) {
      int mid = (int)(((unsigned)left + (unsigned)right) >> 1);
      if (ts_cmp(&pivot, &a[mid]) < 0) right = mid;
      else left = mid + 1;
    }
    memmove(&a[left + 1], &a[left], (size_t)(start - left) * sizeof(docscore));
    a[left] = pivot;
  }
}

static int ts_min_run(int n) {
  int r = 0;
  while (n >= TS_MIN_MERGE) {
    r |= (n & 1);
    n >>= 1;
  }
  return n + r;
}

static int ts_gallop_left(const docscore *key, const docscore *a, int base, int len, int hint) {
  int lastOfs = 0, ofs = 1;
  if (ts_cmp(key, &a[base + hint]) > 0) {
    int maxOfs = len - hint;
    while (ofs < maxOfs && ts_cmp(key, &a[base + hint + ofs]) > 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    lastOfs += hint;
    ofs += hint;
  } else {
    int maxOfs = hint + 1;
    while (ofs < maxOfs && ts_cmp(key, &a[base + hint - ofs]) <= 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    int tmp = lastOfs;
    lastOfs = hint - ofs;
    ofs = hint - tmp;
  }
  lastOfs++;
  while (lastOfs < ofs) {
    int m = lastOfs + (int)((unsigned)(ofs - lastOfs) >> 1);
    if (ts_cmp(key, &a[base + m]) > 0) lastOfs = m + 1;
    else ofs = m;
  }
  return ofs;
}

static int ts_gallop_right(const docscore *key, const docscore *a, int base, int len, int hint) {
  int ofs = 1, lastOfs = 0;
  if (ts_cmp(key, &a[base + hint]) < 0) {
    int maxOfs = hint + 1;
    while (ofs < maxOfs && ts_cmp(key, &a[base + hint - ofs]) < 0) {
      lastOfs = ofs;
      ofs = (ofs << 1) + 1;
      if (ofs <= 0) ofs = maxOfs;
    }
    if (ofs > maxOfs) ofs = maxOfs;
    int tmp = lastOfs;
    lastOfs = hint - ofs;
    ofs = hint - tmp;
  } else {
    int maxOfs = len - hint;
    while (ofs < maxOfs && ts_cmp(key, &a[base + hint + ofs]) >= 0) {
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
    int m = lastOfs + (int)((unsigned)(ofs - lastOfs) >> 1);
    if (ts_cmp(key, &a[base + m]) < 0) ofs = m;
    else lastOfs = m + 1;
  }
  return ofs;
}

static docscore *ts_tmp(tsort *t, int n) {
  if (t->tmplen < n) {
    free(t->tmp);
    t->tmplen = n;
    t->tmp = (docscore *)malloc(sizeof(docscore) * (size_t)n);
  }
  return t->tmp;
}

static void ts_merge_lo(tsort *t, int base1, int len1, int base2, int len2) {
  docscore *a = t->a, *tmp = ts_tmp(t, len1);
  memcpy(tmp, a + base1, (size_t)len1 * sizeof(docscore));
  int cursor1 = 0, cursor2 = base2, dest = base1;
  a[dest++] = a[cursor2++];
  if (--len2 == 0) {
    memcpy(a + dest, tmp + cursor1, (size_t)len1 * sizeof(docscore));
    return;
  }
  if (len1 == 1) {
    memmove(a + dest, a + cursor2, (size_t)len2 * sizeof(docscore));
    a[dest + len2] = tmp[cursor1];
    return;
  }
  int minGallop = t->min_gallop;
  for (;;) {
    int count1 = 0, count2 = 0;
    int brk = 0;
    do {
      if (ts_cmp(&a[cursor2], &tmp[cursor1]) < 0) {
        a[dest++] = a[cursor2++];
        count2++;
        count1 = 0;
        if (--len2 == 0) { brk = 1; break; }
      } else {
        a[dest++] = tmp[cursor1++];
        count1++;
        count2 = 0;
        if (--len1 == 1) { brk = 1; break; }
      }
    } while ((count1 | count2) < minGallop);
    if (brk) break;
    do {
      count1 = ts_gallop_right(&a[cursor2], tmp, cursor1, len1, 0);
      if (count1 != 0) {
        memcpy(a + dest, tmp + cursor1, (size_t)count1 * sizeof(docscore));
        dest += count1;
        cursor1 += count1;
        len1 -= count1;
        if (len1 <= 1) { brk = 1; break; }
      }
      a[dest++] = a[cursor2++];
      if (--len2 == 0) { brk = 1; break; }
      count2 = ts_gallop_left(&tmp[cursor1], a, cursor2, len2, 0);
      if (count2 != 0) {
        memmove(a + dest, a + cursor2, (size_t)count2 * sizeof(docscore));
        dest += count2;
        cursor2 += count2;
        len2 -= count2;
        if (len2 == 0) { brk = 1; break; }
      }
      a[dest++] = tmp[cursor1++];
      if (--len1 == 1) { brk = 1; break; }
      minGallop--;
    } while (count1 >= TS_MIN_GALLOP || count2 >= TS_MIN_GALLOP);
    if (brk) break;
    if (minGallop < 0) minGallop = 0;
    minGallop += 2;
  }
  t->min_gallop = minGallop < 1 ? 1 : minGallop;
  if (len1 == 1) {
    memmove(a + dest, a + cursor2, (size_t)len2 * sizeof(docscore));
    a[dest + len2] = tmp[cursor1];
  } else if (len1 == 0) {
    t->err = 1; /* IllegalArgumentException: Comparison method violates its general contract! */
  } else {
    memcpy(a + dest, tmp + cursor1, (size_t)len1 * sizeof(docscore));
  }
}

static void ts_merge_hi(tsort *t, int base1, int len1, int base2, int len2) {
  docscore *a = t->a, *tmp = ts_tmp(t, len2);
  memcpy(tmp, a + base2, (size_t)len2 * sizeof(docscore));
  int cursor1 = base1 + len1 - 1, cursor2 = len2 - 1, dest = base2 + len2 - 1;
  a[dest--] = a[cursor1--];
  if (--len1 == 0) {
    memcpy(a + dest - (len2 - 1), tmp, (size_t)len2 * sizeof(docscore));
    return;
  }
  if (len2 == 1) {
    dest -= len1;
    cursor1 -= len1;
    memmove(a + dest + 1, a + cursor1 + 1, (size_t)len1 * sizeof(docscore));
    a[dest] = tmp[cursor2];
    return;
  }
  int minGallop = t->min_gallop;
  for (;;) {
    int count1 = 0, count2 = 0;
    int brk = 0;
    do {
      if (ts_cmp(&tmp[cursor2], &a[cursor1]) < 0) {
        a[dest--] = a[cursor1--];
        count1++;
        count2 = 0;
        if (--len1 == 0) { brk = 1; break; }
      } else {
        a[dest--] = tmp[cursor2--];
        count2++;
        count1 = 0;
        if (--len2 == 1) { brk = 1; break; }
      }
    } while ((count1 | count2) < minGallop);
    if (brk) break;
    do {
      count1 = len1 - ts_gallop_right(&tmp[cursor2], a, base1, len1, len1 - 1);
      if (count1 != 0) {
        dest -= count1;
        cursor1 -= count1;
        len1 -= count1;
        memmove(a + dest + 1, a + cursor1 + 1, (size_t)count1 * sizeof(docscore));
        if (len1 == 0) { brk = 1; break; }
      }
      a[dest--] = tmp[cursor2--];
      if (--len2 == 1) { brk = 1; break; }
      count2 = len2 - ts_gallop_left(&a[cursor1], tmp, 0, len2, len2 - 1);
      if (count2 != 0) {
        dest -= count2;
        cursor2 -= count2;
        len2 -= count2;
        memcpy(a + dest + 1, tmp + cursor2 + 1, (size_t)count2 * sizeof(docscore));
        if (len2 <= 1) { brk = 1; break; }
      }
      a[dest--] = a[cursor1--];
      if (--len1 == 0) { brk = 1; break; }
      minGallop--;
    } while (count1 >= TS_MIN_GALLOP || count2 >= TS_MIN_GALLOP);
    if (brk) break;
    if (minGallop < 0) minGallop = 0;
    minGallop += 2;
  }
  t->min_gallop = minGallop < 1 ? 1 : minGallop;
  if (len2 == 1) {
    dest -= len1;
    cursor1 -= len1;
    memmove(a + dest + 1, a + cursor1 + 1, (size_t)len1 * sizeof(docscore));
    a[dest] = tmp[cursor2];
  } else if (len2 == 0) {
    t->err = 1; /* IllegalArgumentException */
  } else {
    memcpy(a + dest - (len2 - 1), tmp, (size_t)len2 * sizeof(docscore));
  }
}

static void ts_merge_at(tsort *t, int i) {
  int base1 = t->base[i], len1 = t->len[i], base2 = t->base[i + 1], len2 = t->len[i + 1];
  t->len[i] = len1 + len2;
  if (i == t->stack - 3) {
    t->base[i + 1] = t->base[i + 2];
    t->len[i + 1] = t->len[i + 2];
  }
  t->stack--;
  int k = ts_gallop_right(&t->a[base2], t->a, base1, len1, 0);
  base1 += k;
  len1 -= k;
  if (len1 == 0) return;
  len2 = ts_gallop_left(&t->a[base1 + len1 - 1], t->a, base2, len2, len2 - 1);
  if (len2 == 0) return;
  if (len1 <= len2) ts_merge_lo(t, base1, len1, base2, len2);
  else ts_merge_hi(t, base1, len1, base2, len2);
}

static void ts_merge_collapse(tsort *t) { /* JDK 7 GA */
  while (t->stack > 1 && !t->err) {
    int n = t->stack - 2;
    if (n > 0 && t->len[n - 1] <= t->len[n] + t->len[n + 1]) {
      if (t->len[n - 1] < t->len[n + 1]) n--;
      ts_merge_at(t, n);
    } else if (t->len[n] <= t->len[n + 1]) {
      ts_merge_at(t, n);
    } else {
      break;
    }
  }
}

static void ts_merge_force_collapse(tsort *t) {
  while (t->stack > 1 && !t->err) {
    int n = t->stack - 2;
    if (n > 0 && t->len[n - 1] < t->len[n + 1]) n--;
    ts_merge_at(t, n);
  }
}

/* ComparableTimSort.sort(a, 0, n): 0, or -1 where Java throws */
static int timsort7(docscore *a, int n) {
  if (n < 2) return 0;
  int lo = 0, rem = n;
  if (rem < TS_MIN_MERGE) {
    int initRunLen = ts_count_run(a, lo, n);
    ts_binary_sort(a, lo, n, lo + initRunLen);
    return 0;
  }
  tsort t;
  memset(&t, 0, sizeof t);
  t.a = a;
  t.min_gallop = TS_MIN_GALLOP;
  int minRun = ts_min_run(rem);
  do {
    int runLen = ts_count_run(a, lo, n);
    if (runLen < minRun) {
      int force = rem <= minRun ? rem : minRun;
      ts_binary_sort(a, lo, lo + force, lo + runLen);
      runLen = force;
    }
    t.base[t.stack] = lo;
    t.len[t.stack] = runLen;
    t.stack++;
    ts_merge_collapse(&t);
    lo += runLen;
    rem -= runLen;
  } while (rem != 0 && !t.err);
  ts_merge_force_collapse(&t);
  free(t.tmp);
  return t.err ? -1 : 0;
}

static int ds_cmp_docno(const void *x, const void *y) {
  const docscore *a = (const docscore *)x, *b = (const docscore *)y;
  if (a->score > b->score) return -1;
  if (a->score < b->score) return 1;
  return (a->docId > b->docId) - (a->docId < b->docId);
}
static int ds_cmp_first(const void *x, const void *y) {
  const docscore *a = (const docscore *)x, *b = (const docscore *)y;
  if (a->score > b->score) return -1;
  if (a->score < b->score) return 1;
  return a->first - b->first;
}

/*
 * Score one query (terms as UTF-16 strings already tokenized, in token order).
 * idf_mode: 0 = reference (stored key df, T1/T2), 1 = true df (postings length), int division both.
 * order: 0 = score desc / docno asc (north-star tie-break),
 *        1 = Java 6 Collections.sort with the reference DocScore comparator,
 *        2 = score desc / first-encounter (stable exact ties),
 *        3 = Java 7 Collections.sort (ComparableTimSort) with the DocScore comparator.
 * Returns number of results written (<= k); scores/docnos out; -1 in order 3
 * where Java 7's TimSort throws IllegalArgumentException (contract violation).
 */
/* ref-faithful timing mode (bench.py cpu_baseline): the accumulator lookup is
 * the reference's linear scores.indexOf scan (T6) instead of the docno table;
 * both give the same entry, the scan is O(entries) per posting */
static int g_ref_scan = 0;
void or_set_ref_scan(int on) { g_ref_scan = on; }

int or_query(const or_index *ix, const uint16_t *const *terms, const int *lens, int nterms, int k,
             int idf_mode, int order, int32_t *out_docno, double *out_score) {
  int cap = 1024, n = 0;
  docscore *sc = (docscore *)malloc(sizeof(docscore) * cap);
  /* scores.indexOf(new DocScore(d)) (T6) finds the one entry with docId d, or
   * none: a docno -> entry table gives the same index without the O(n) scan,
   * and entries are appended in first-encounter order exactly as scores.add */
  int hcap = 1024;
  int *ht = (int *)malloc(sizeof(int) * hcap);
  for (int i = 0; i < hcap; i++) ht[i] = -1;
  int N = ix->N;
  for (int qi = 0; qi < nterms; qi++) {
    int t = find_term(ix, terms[qi], lens[qi]);
    if (t < 0) continue; /* getValue: unknown term silently skipped */
    const term_rec *tr = &ix->terms[t];
    int df = idf_mode == 0 ? tr->df_field : tr->npost;
    double idf = log10((double)(N / df));
    for (int p = 0; p < tr->npost; p++) {
      int d = tr->post[p].docno;
      uint32_t h = ((uint32_t)d * 2654435761u) & (uint32_t)(hcap - 1);
      while (ht[h] >= 0 && sc[ht[h]].docId != d) h = (h + 1) & (uint32_t)(hcap - 1);
      int idx = ht[h];
      if (g_ref_scan) { /* scores.indexOf: first entry with this docId */
        idx = -1;
        for (int s2 = 0; s2 < n; s2++)
          if (sc[s2].docId == d) {
            idx = s2;
            break;
          }
      }
      if (idx < 0) {
        if (n == cap) {
          cap *= 2;
          sc = (docscore *)realloc(sc, sizeof(docscore) * cap);
        }
        sc[n].docId = d;
        sc[n].score = 0.0;
        sc[n].first = n;
        idx = n++;
        ht[h] = idx;
        if (2 * n > hcap) { /* grow and rehash */
          free(ht);
          hcap *= 4;
          ht = (int *)malloc(sizeof(int) * hcap);
          for (int i = 0; i < hcap; i++) ht[i] = -1;
          for (int i = 0; i < n; i++) {
            uint32_t g = ((uint32_t)sc[i].docId * 2654435761u) & (uint32_t)(hcap - 1);
            while (ht[g] >= 0) g = (g + 1) & (uint32_t)(hcap - 1);
            ht[g] = i;
          }
        }
      }
      double w = (1.0 + log((double)tr->post[p].tf)) * idf;
      sc[idx].score += w;
    }
  }
  free(ht);
  if (order == 1) {
    docscore *aux = (docscore *)malloc(sizeof(docscore) * (n ? n : 1));
    memcpy(aux, sc, sizeof(docscore) * n);
    legacy_merge_sort(aux, sc, 0, n, 0);
    free(aux);
  } else if (order == 3) {
    if (timsort7(sc, n) != 0) { /* Collections.sort throws: rank() has no result */
      free(sc);
      return -1;
    }
  } else {
    qsort(sc, (size_t)n, sizeof(docscore), order == 2 ? ds_cmp_first : ds_cmp_docno);
  }
  int r = n < k ? n : k;
  for (int i = 0; i < r; i++) {
    out_docno[i] = sc[i].docId;
    out_score[i] = sc[i].score;
  }
  free(sc);
  return r;
}

/* rank()'s sort alone, for the sort tests: candidates (score[i], first-encounter
 * index i, docId i) in list order -> perm[r] = the index at rank r under `order`
 * (1 Java 6 legacy merge sort, 3 Java 7 ComparableTimSort, 0 / 2 exact orders);
 * returns n, or -1 where Java 7 throws */
int or_sort_docscores(const double *score, int n, int order, int32_t *perm) {
  docscore *sc = (docscore *)malloc(sizeof(docscore) * (size_t)(n ? n : 1));
  for (int i = 0; i < n; i++) {
    sc[i].docId = i;
    sc[i].score = score[i];
    sc[i].first = i;
  }
  int r = n;
  if (order == 1) {
    docscore *aux = (docscore *)malloc(sizeof(docscore) * (size_t)(n ? n : 1));
    memcpy(aux, sc, sizeof(docscore) * (size_t)n);
    legacy_merge_sort(aux, sc, 0, n, 0);
    free(aux);
  } else if (order == 3) {
    if (timsort7(sc, n) != 0) r = -1;
  } else {
    qsort(sc, (size_t)n, sizeof(docscore), order == 2 ? ds_cmp_first : ds_cmp_docno);
  }
  if (r >= 0)
    for (int i = 0; i < n; i++) perm[i] = sc[i].docId;
  free(sc);
  return r;
}

/* ---- tokenizer / stemmer entry points on UTF-8 (ctypes) ---- */
/* processContent on UTF-8 text; tokens written as modified UTF-8, each prefixed by u16 length. */
int or_process_content_utf8(const uint8_t *b, size_t n, uint8_t *out, size_t cap, int *ntok) {
  jstr t;
  js_init(&t);
  utf8_to_utf16(b, n, &t);
  jstr_list l;
  jl_init(&l);
  or_process_content(t.p, t.n, &l);
  size_t k = 0;
  for (int i = 0; i < l.n; i++) {
    int ml = mutf8_len(l.v[i].p, l.v[i].n);
    if (k + 2 + (size_t)ml > cap) {
      jl_free(&l);
      js_free(&t);
      return -1;
    }
    out[k] = (uint8_t)(ml >> 8);
    out[k + 1] = (uint8_t)ml;
    mutf8_encode(l.v[i].p, l.v[i].n, out + k + 2);
    k += 2 + (size_t)ml;
  }
  *ntok = l.n;
  jl_free(&l);
  js_free(&t);
  return (int)k;
}

/* TagTokenizer terms only (before stopwords/stemming). Same output format. */
int or_tag_tokenize_utf8(const uint8_t *b, size_t n, uint8_t *out, size_t cap, int *ntok) {
  jstr t;
  js_init(&t);
  utf8_to_utf16(b, n, &t);
  jstr_list l;
  jl_init(&l);
  or_tag_tokenize(t.p, t.n, &l);
  size_t k = 0;
  for (int i = 0; i < l.n; i++) {
    int ml = mutf8_len(l.v[i].p, l.v[i].n);
    if (k + 2 + (size_t)ml > cap) {
      jl_free(&l);
      js_free(&t);
      return -1;
    }
    out[k] = (uint8_t)(ml >> 8);
    out[k + 1] = (uint8_t)ml;
    mutf8_encode(l.v[i].p, l.v[i].n, out + k + 2);
    k += 2 + (size_t)ml;
  }
  *ntok = l.n;
  jl_free(&l);
  js_free(&t);
  return (int)k;
}

/* stem an ASCII/UTF-8 word; result as modified UTF-8 */
int or_stem_utf8(const uint8_t *b, size_t n, uint8_t *out, size_t cap) {
  jstr w, s;
  js_init(&w);
  js_init(&s);
  utf8_to_utf16(b, n, &w);
  or_stem_js(w.p, w.n, &s);
  int ml = mutf8_len(s.p, s.n);
  if ((size_t)ml > cap) return -1;
  mutf8_encode(s.p, s.n, out);
  js_free(&w);
  js_free(&s);
  return ml;
}

int or_is_stopword_utf8(const uint8_t *b, size_t n) {
  jstr w;
  js_init(&w);
  utf8_to_utf16(b, n, &w);
  int r = or_is_stopword(w.p, w.n);
  js_free(&w);
  return r;
}

/* query from UTF-8 strings of (already processed) terms, NUL-separated list */
int or_query_utf8(const or_index *ix, const uint8_t *terms_blob, const int *offs, int nterms, int k,
                  int idf_mode, int order, int32_t *out_docno, double *out_score) {
  uint16_t **tp = (uint16_t **)malloc(sizeof(uint16_t *) * (nterms ? nterms : 1));
  int *tl = (int *)malloc(sizeof(int) * (nterms ? nterms : 1));
  jstr *tmp = (jstr *)calloc((size_t)(nterms ? nterms : 1), sizeof(jstr));
  for (int i = 0; i < nterms; i++) {
    utf8_to_utf16(terms_blob + offs[i], (size_t)(offs[i + 1] - offs[i]), &tmp[i]);
    tp[i] = tmp[i].p;
    tl[i] = tmp[i].n;
  }
  int r = or_query(ix, (const uint16_t *const *)tp, tl, nterms, k, idf_mode, order, out_docno,
                   out_score);
  for (int i = 0; i < nterms; i++) js_free(&tmp[i]);
  free(tmp);
  free(tp);
  free(tl);
  return r;
}

/* record split only: returns count; offsets/lengths into caller arrays (cap entries) */
int or_split_records(const uint8_t *b, size_t n, uint64_t *off, uint64_t *len, int cap) {
  rec *r;
  int nr;
  split_records(b, n, 0, n, &r, &nr);
  for (int i = 0; i < nr && i < cap; i++) {
    off[i] = r[i].off;
    len[i] = r[i].len;
  }
  free(r);
  return nr;
}

/* self-check for tests: the table lookup and the O(V) scan agree on every
 * index term's first element; returns the number of disagreements */
int or_lookup_selfcheck(const or_index *ix) {
  int bad = 0;
  for (int t = 0; t < ix->nterms; t++) {
    const jstr *g = &ix->terms[t].gram[0];
    if (find_term(ix, g->p, g->n) != find_term_scan(ix, g->p, g->n)) bad++;
  }
  return bad;
}

/* number of distinct stems (processContent of each word alone) of n UTF-8 words
 * blob[offs[i] .. offs[i+1]) -- bench.py's full-size vocabulary check */
int64_t or_count_distinct_terms(const uint8_t *blob, const int64_t *offs, int64_t n) {
  int64_t cap = 1024;
  while (cap < 4 * n + 16) cap <<= 1;
  uint64_t *tab = (uint64_t *)calloc((size_t)cap, sizeof(uint64_t));
  jstr_list **keep = NULL;
  (void)keep;
  int64_t cnt = 0;
  jstr w;
  js_init(&w);
  for (int64_t i = 0; i < n; i++) {
    utf8_to_utf16(blob + offs[i], (size_t)(offs[i + 1] - offs[i]), &w);
    jstr_list out;
    jl_init(&out);
    or_process_content(w.p, w.n, &out);
    for (int t = 0; t < out.n; t++) {
      uint64_t h = 1469598103934665603ull;
      for (int c = 0; c < out.v[t].n; c++) h = (h ^ out.v[t].p[c]) * 1099511628211ull;
      h |= 1; /* 0 = empty slot; 64-bit hashes of < 2^21 strings: collisions negligible */
      int64_t s = (int64_t)(h & (uint64_t)(cap - 1));
      while (tab[s] && tab[s] != h) s = (s + 1) & (cap - 1);
      if (!tab[s]) {
        tab[s] = h;
        cnt++;
      }
    }
    jl_free(&out);
  }
  js_free(&w);
  free(tab);
  return cnt;
}
