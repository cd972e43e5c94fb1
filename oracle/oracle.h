/*
 * oracle.h -- CPU restatement of the reference's index/query hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / the timed CPU baseline.
 *
 * Parity status: partially pinned.  The reference (Java + Hadoop 0.20) cannot
 * be compiled or run in this image (no JDK, no Hadoop jars) and ships no tests
 * or golden vectors.  This restatement is pinned by
 * the hand-derived known-answer tests of SURVEY.md Appendix B (tests/golden/)
 * and cross-checked against an independent pure-Python restatement
 * (tests/pyref.py) on fuzzed inputs.  Behaviour that comes from the JDK or
 * Hadoop rather than from the reference's own files (UTF-8 decoding with
 * replacement, String.toLowerCase for non-ASCII, Collections.sort on the
 * broken DocScore comparator) is restated from published semantics and is
 * "parity unpinned".
 *
 * Strings are held as Java does: arrays of UTF-16 code units.
 */
#ifndef SME_ORACLE_H
#define SME_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint16_t *p;
  int n;
  int cap;
} jstr;

/* ---- jstr helpers (oracle_util.c) ---- */
void js_init(jstr *s);
void js_free(jstr *s);
void js_reserve(jstr *s, int cap);
void js_set(jstr *s, const uint16_t *p, int n);
void js_set_ascii(jstr *s, const char *a);
void js_push(jstr *s, uint16_t c);
int js_cmp(const uint16_t *a, int an, const uint16_t *b, int bn); /* String.compareTo */
int32_t js_hash(const uint16_t *a, int n);                        /* String.hashCode */
/* Hadoop Text.toString: UTF-8 -> UTF-16 with U+FFFD replacement (maximal subpart). */
int utf8_to_utf16(const uint8_t *b, size_t n, jstr *out);
/* String.getBytes("UTF-8") length (unpaired surrogate -> '?'). */
int utf8_len_java(const uint16_t *a, int n);
/* DataOutput.writeUTF body (modified UTF-8), returns bytes written (no length prefix). */
int mutf8_encode(const uint16_t *a, int n, uint8_t *out);
int mutf8_len(const uint16_t *a, int n);
/* String.toLowerCase() (root/en locale), appends to out. */
void java_tolower(const uint16_t *a, int n, jstr *out);

/* ---- stemmer (oracle_stem.c): englishStemmer.stem() on word, result in out ---- */
void or_stem_js(const uint16_t *w, int n, jstr *out);

/* ---- tokenizer (oracle_tok.c) ---- */
typedef struct {
  jstr *v;
  int n, cap;
} jstr_list;
void jl_init(jstr_list *l);
void jl_free(jstr_list *l);
void jl_push(jstr_list *l, const uint16_t *p, int n);
/* TagTokenizer.tokenize(text).terms */
void or_tag_tokenize(const uint16_t *text, int n, jstr_list *terms);
/* GalagoTokenizer.processContent(text) */
void or_process_content(const uint16_t *text, int n, jstr_list *out);
int or_is_stopword(const uint16_t *w, int n);

#ifdef __cplusplus
}
#endif
#endif
