/*
 * oracle_chargram.c -- CPU restatement of the CharKGramTermIndexer job.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for the device path.
 *
 * Reference (C/ = ABDURRAHMAN-PA2-3-code/src/):
 *   MyMapper.map     C/sa/edu/kaust/indexing/CharKGramTermIndexer.java:88-111
 *                    every token of processContent(doc) becomes '$'+token+'$'; each of its
 *                    k-unit substrings (UTF-16 units, String.substring) maps to a
 *                    HashSet<String> of the tokens containing it (in-mapper combining,
 *                    one Hashtable per map task)
 *   MyMapper.close   :114-129  emits (Text gram, ArrayListWritable<Text> of the set in
 *                    HashSet iteration order)
 *   MyReducer.reduce :136-171  with one map task every key has ONE list and the pairwise
 *                    merge loop returns it unchanged
 *   run              :228-269  R = 10 reducers, TextOutputFormat (default): the line is
 *                    key bytes '\t' value.toString() '\n'; ArrayListWritable.toString is
 *                    "[a, b, c]" (C/edu/umd/cloud9/io/array/ArrayListWritable.java:112-123)
 *
 * JDK / Hadoop behaviour restated here (parity unpinned):
 *   - HashSet iteration order is simulated with the JDK 6 HashMap algorithm: capacity
 *     16, load factor 0.75, hash(h) = h ^ (h>>>20) ^ (h>>>12); h ^ (h>>>7) ^ (h>>>4),
 *     new entries at the head of their bucket, resize when size++ >= threshold, transfer
 *     walking old buckets 0..n-1 and prepending to the new ones; iteration buckets
 *     0..cap-1, each chain from its head.  (JDK 6 is the era's runtime: the JDK's
 *     legacy merge sort is assumed for Collections.sort elsewhere in this oracle too.)
 *   - Text.set(String) / String.getBytes("UTF-8"): an unpaired surrogate (a gram may
 *     cut a surrogate pair) becomes '?'.
 *   - Grams whose UTF-16 units differ only in unpaired surrogates (a gram can cut a
 *     surrogate pair) encode to the same Text key.  The reference then emits two map
 *     outputs with one key and MyReducer.merge combines the lists in the order Hadoop's
 *     (unstable) spill sort left them; here, as on the device, one set per Text key is
 *     kept (HashSet of the union, in first-occurrence order).  Parity unpinned.
 *   - HashPartitioner on Text.hashCode (WritableComparator.hashBytes: h = 31*h + signed
 *     byte, from 1), the key order is Text's unsigned byte order (shorter prefix first).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* records of the whole corpus (oracle_index.c) */
int or_split_records(const uint8_t *b, size_t n, uint64_t *off, uint64_t *len, int cap);

/* ---------------- String.getBytes("UTF-8") ---------------- */
static int java_utf8(const uint16_t *a, int n, uint8_t *o) {
  int k = 0;
  for (int i = 0; i < n; i++) {
    unsigned c = a[i];
    if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && a[i + 1] >= 0xDC00 && a[i + 1] <= 0xDFFF) {
      unsigned cp = 0x10000 + ((c - 0xD800) << 10) + (a[i + 1] - 0xDC00);
      o[k++] = (uint8_t)(0xF0 | (cp >> 18));
      o[k++] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
      o[k++] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
      o[k++] = (uint8_t)(0x80 | (cp & 0x3F));
      i++;
    } else if (c >= 0xD800 && c <= 0xDFFF) {
      o[k++] = '?';
    } else if (c < 0x80) {
      o[k++] = (uint8_t)c;
    } else if (c < 0x800) {
      o[k++] = (uint8_t)(0xC0 | (c >> 6));
      o[k++] = (uint8_t)(0x80 | (c & 0x3F));
    } else {
      o[k++] = (uint8_t)(0xE0 | (c >> 12));
      o[k++] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
      o[k++] = (uint8_t)(0x80 | (c & 0x3F));
    }
  }
  return k;
}

/* ---------------- string dictionary (UTF-16 -> id) ---------------- */
typedef struct {
  uint16_t *chars;
  size_t nchars, cap_chars;
  size_t *off; /* [n+1] */
  int n, cap;
  int *slots; /* open addressing, -1 empty */
  size_t mask;
} dict;

static uint64_t h16(const uint16_t *a, int n) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < n; i++) h = (h ^ a[i]) * 1099511628211ull;
  return h ^ (uint64_t)n;
}
static void d_init(dict *d) {
  memset(d, 0, sizeof *d);
  d->cap = 1024;
  d->off = (size_t *)malloc(sizeof(size_t) * (d->cap + 1));
  d->off[0] = 0;
  d->cap_chars = 4096;
  d->chars = (uint16_t *)malloc(2 * d->cap_chars);
  d->mask = 4095;
  d->slots = (int *)malloc(sizeof(int) * (d->mask + 1));
  memset(d->slots, 0xFF, sizeof(int) * (d->mask + 1));
}
static void d_free(dict *d) {
  free(d->chars);
  free(d->off);
  free(d->slots);
}
static const uint16_t *d_str(const dict *d, int i, int *n) {
  *n = (int)(d->off[i + 1] - d->off[i]);
  return d->chars + d->off[i];
}
static int d_get(dict *d, const uint16_t *a, int n, int *is_new) {
  if ((size_t)(d->n + 1) * 2 > d->mask + 1) {
    size_t nm = (d->mask + 1) * 2 - 1;
    int *ns = (int *)malloc(sizeof(int) * (nm + 1));
    memset(ns, 0xFF, sizeof(int) * (nm + 1));
    for (int i = 0; i < d->n; i++) {
      int l;
      const uint16_t *s = d_str(d, i, &l);
      size_t h = (size_t)h16(s, l) & nm;
      while (ns[h] >= 0) h = (h + 1) & nm;
      ns[h] = i;
    }
    free(d->slots);
    d->slots = ns;
    d->mask = nm;
  }
  size_t h = (size_t)h16(a, n) & d->mask;
  while (d->slots[h] >= 0) {
    int l;
    const uint16_t *s = d_str(d, d->slots[h], &l);
    if (l == n && memcmp(s, a, 2 * (size_t)n) == 0) {
      *is_new = 0;
      return d->slots[h];
    }
    h = (h + 1) & d->mask;
  }
  if (d->n == d->cap) {
    d->cap *= 2;
    d->off = (size_t *)realloc(d->off, sizeof(size_t) * (d->cap + 1));
  }
  while (d->nchars + (size_t)n > d->cap_chars) {
    d->cap_chars *= 2;
    d->chars = (uint16_t *)realloc(d->chars, 2 * d->cap_chars);
  }
  memcpy(d->chars + d->nchars, a, 2 * (size_t)n);
  d->nchars += (size_t)n;
  d->off[d->n + 1] = d->nchars;
  d->slots[h] = d->n;
  *is_new = 1;
  return d->n++;
}

/* ---------------- JDK 6 HashMap<String,Object> (HashSet) ---------------- */
typedef struct {
  int term, hash, next;
} hent;
typedef struct {
  hent *e;
  int ne, cape;
  int *tab; /* bucket heads, -1 empty */
  int cap, size, thr;
} hset6;

static int spread6(int32_t h0) {
  uint32_t h = (uint32_t)h0;
  h ^= (h >> 20) ^ (h >> 12);
  return (int)(h ^ (h >> 7) ^ (h >> 4));
}
static void hs_init(hset6 *s) {
  s->cap = 16;
  s->thr = 12;
  s->size = 0;
  s->tab = (int *)malloc(sizeof(int) * 16);
  memset(s->tab, 0xFF, sizeof(int) * 16);
  s->cape = 4;
  s->ne = 0;
  s->e = (hent *)malloc(sizeof(hent) * s->cape);
}
static void hs_free(hset6 *s) {
  free(s->tab);
  free(s->e);
}
/* HashSet.add(term) with term's String.hashCode = jh (terms are unique ids) */
static void hs_add(hset6 *s, int term, int32_t jh) {
  const int hash = spread6(jh);
  int i = hash & (s->cap - 1);
  for (int x = s->tab[i]; x >= 0; x = s->e[x].next)
    if (s->e[x].hash == hash && s->e[x].term == term) return;
  if (s->ne == s->cape) {
    s->cape *= 2;
    s->e = (hent *)realloc(s->e, sizeof(hent) * s->cape);
  }
  s->e[s->ne].term = term;
  s->e[s->ne].hash = hash;
  s->e[s->ne].next = s->tab[i]; /* addEntry: new entry at the bucket head */
  s->tab[i] = s->ne++;
  if (s->size++ >= s->thr) { /* resize(2 * table.length) -> transfer */
    const int nc = 2 * s->cap;
    int *nt = (int *)malloc(sizeof(int) * nc);
    memset(nt, 0xFF, sizeof(int) * nc);
    for (int j = 0; j < s->cap; j++) {
      int x = s->tab[j];
      while (x >= 0) {
        const int nx = s->e[x].next;
        const int b = s->e[x].hash & (nc - 1);
        s->e[x].next = nt[b];
        nt[b] = x;
        x = nx;
      }
    }
    free(s->tab);
    s->tab = nt;
    s->cap = nc;
    s->thr = (int)(nc * 0.75f);
  }
}

/* ---------------- the job ---------------- */
typedef struct {
  int R;
  int ngrams;
  long long npairs;
  uint8_t **part;
  size_t *plen;
} or_chargram_t;

typedef struct {
  const uint8_t *b;
  int n, gid;
} gkey;
static int gkey_cmp(const void *x, const void *y) { /* Text order: unsigned bytes, shorter first */
  const gkey *a = (const gkey *)x, *c = (const gkey *)y;
  int m = a->n < c->n ? a->n : c->n;
  int r = memcmp(a->b, c->b, (size_t)m);
  if (r) return r;
  return (a->n > c->n) - (a->n < c->n);
}

void *or_chargram(const uint8_t *corpus, size_t n, int k, int R) {
  if (k < 1 || R < 1) return NULL;
  int cap = 1024, nrec;
  uint64_t *ro = NULL, *rl = NULL;
  for (;;) {
    ro = (uint64_t *)realloc(ro, sizeof(uint64_t) * cap);
    rl = (uint64_t *)realloc(rl, sizeof(uint64_t) * cap);
    nrec = or_split_records(corpus, n, ro, rl, cap);
    if (nrec <= cap) break;
    cap = nrec;
  }
  dict grams, terms;
  d_init(&grams);
  d_init(&terms);
  int gcap = 1024;
  hset6 *sets = (hset6 *)malloc(sizeof(hset6) * gcap);
  int32_t *thash = NULL;
  int thcap = 0;
  jstr text, tok;
  js_init(&text);
  js_init(&tok);
  jstr_list toks;
  jl_init(&toks);
  for (int r = 0; r < nrec; r++) {
    utf8_to_utf16(corpus + ro[r], (size_t)rl[r], &text);
    jl_free(&toks);
    jl_init(&toks);
    or_process_content(text.p, text.n, &toks);
    for (int t = 0; t < toks.n; t++) {
      int isnew;
      const int tid = d_get(&terms, toks.v[t].p, toks.v[t].n, &isnew);
      if (isnew) {
        if (tid >= thcap) {
          thcap = thcap ? 2 * thcap : 1024;
          thash = (int32_t *)realloc(thash, sizeof(int32_t) * thcap);
        }
        thash[tid] = js_hash(toks.v[t].p, toks.v[t].n);
      }
      tok.n = 0;
      js_push(&tok, '$');
      for (int i = 0; i < toks.v[t].n; i++) js_push(&tok, toks.v[t].p[i]);
      js_push(&tok, '$');
      for (int i = 0; i + k <= tok.n; i++) {
        /* the key is the Text (UTF-8 bytes): grams differing only in unpaired
           surrogates share one key (see the note in the header) */
        uint8_t kb8[4 * 8];
        uint16_t kb16[4 * 8];
        const int nb = java_utf8(tok.p + i, k, kb8);
        for (int j = 0; j < nb; j++) kb16[j] = kb8[j];
        const int gid = d_get(&grams, kb16, nb, &isnew);
        if (isnew) {
          if (gid == gcap) {
            gcap *= 2;
            sets = (hset6 *)realloc(sets, sizeof(hset6) * gcap);
          }
          hs_init(&sets[gid]);
        }
        hs_add(&sets[gid], tid, thash[tid]);
      }
    }
  }
  /* output: partitions of lines in Text key order */
  or_chargram_t *o = (or_chargram_t *)calloc(1, sizeof *o);
  o->R = R;
  o->ngrams = grams.n;
  o->part = (uint8_t **)calloc((size_t)R, sizeof(uint8_t *));
  o->plen = (size_t *)calloc((size_t)R, sizeof(size_t));
  gkey *keys = (gkey *)malloc(sizeof(gkey) * (grams.n + 1));
  uint8_t *kb = (uint8_t *)malloc((size_t)grams.n * 4 * (size_t)k + 8);
  size_t kbn = 0;
  for (int g = 0; g < grams.n; g++) {
    int l;
    const uint16_t *s = d_str(&grams, g, &l);
    keys[g].b = kb + kbn;
    for (int j = 0; j < l; j++) kb[kbn + j] = (uint8_t)s[j];
    keys[g].n = l;
    keys[g].gid = g;
    kbn += (size_t)keys[g].n;
  }
  qsort(keys, (size_t)grams.n, sizeof(gkey), gkey_cmp);
  size_t *pcap = (size_t *)calloc((size_t)R, sizeof(size_t));
  uint8_t *tb = (uint8_t *)malloc(1 << 16);
  size_t tbcap = 1 << 16;
  for (int x = 0; x < grams.n; x++) {
    int32_t h = 1;
    for (int i = 0; i < keys[x].n; i++) h = 31 * h + (int8_t)keys[x].b[i];
    const int p = (int)((h & 0x7fffffff) % R);
    hset6 *s = &sets[keys[x].gid];
    /* line = key '\t' '[' t1 ", " t2 ... ']' '\n' */
    size_t need = (size_t)keys[x].n + 4;
    for (int j = 0; j < s->cap; j++)
      for (int e = s->tab[j]; e >= 0; e = s->e[e].next) {
        int l;
        d_str(&terms, s->e[e].term, &l);
        need += 3 * (size_t)l + 2;
      }
    if (o->plen[p] + need > pcap[p]) {
      pcap[p] = (o->plen[p] + need) * 2;
      o->part[p] = (uint8_t *)realloc(o->part[p], pcap[p]);
    }
    uint8_t *w = o->part[p] + o->plen[p];
    memcpy(w, keys[x].b, (size_t)keys[x].n);
    w += keys[x].n;
    *w++ = '\t';
    *w++ = '[';
    int first = 1;
    for (int j = 0; j < s->cap; j++)
      for (int e = s->tab[j]; e >= 0; e = s->e[e].next) {
        int l;
        const uint16_t *ts = d_str(&terms, s->e[e].term, &l);
        if (!first) {
          *w++ = ',';
          *w++ = ' ';
        }
        first = 0;
        if ((size_t)(3 * l + 8) > tbcap) {
          tbcap = (size_t)(3 * l + 8);
          tb = (uint8_t *)realloc(tb, tbcap);
        }
        const int bl = java_utf8(ts, l, tb);
        memcpy(w, tb, (size_t)bl);
        w += bl;
        o->npairs++;
      }
    *w++ = ']';
    *w++ = '\n';
    o->plen[p] = (size_t)(w - o->part[p]);
  }
  for (int g = 0; g < grams.n; g++) hs_free(&sets[g]);
  free(sets);
  free(thash);
  free(keys);
  free(kb);
  free(pcap);
  free(tb);
  free(ro);
  free(rl);
  js_free(&text);
  js_free(&tok);
  jl_free(&toks);
  d_free(&grams);
  d_free(&terms);
  return o;
}

int or_chargram_ngrams(void *h) { return ((or_chargram_t *)h)->ngrams; }
long long or_chargram_npairs(void *h) { return ((or_chargram_t *)h)->npairs; }
size_t or_chargram_part_len(void *h, int p) { return ((or_chargram_t *)h)->plen[p]; }
const uint8_t *or_chargram_part_bytes(void *h, int p) { return ((or_chargram_t *)h)->part[p]; }
void or_chargram_free(void *h) {
  or_chargram_t *o = (or_chargram_t *)h;
  if (!o) return;
  for (int p = 0; p < o->R; p++) free(o->part[p]);
  free(o->part);
  free(o->plen);
  free(o);
}
