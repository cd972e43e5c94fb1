/*
 * oracle_util.c -- Java String / DataOutput / Hadoop Text semantics the
 * reference relies on (tags [J] and [H]).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  These are JDK/Hadoop behaviours
 * that are not vendored in /root/reference, so they are restated from their
 * published semantics ("parity unpinned" outside ASCII).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "unicase_tab.h"

void js_init(jstr *s) {
  s->p = NULL;
  s->n = 0;
  s->cap = 0;
}
void js_free(jstr *s) {
  free(s->p);
  js_init(s);
}
void js_reserve(jstr *s, int cap) {
  if (cap <= s->cap) return;
  int nc = s->cap ? s->cap : 16;
  while (nc < cap) nc *= 2;
  s->p = (uint16_t *)realloc(s->p, (size_t)nc * sizeof(uint16_t));
  s->cap = nc;
}
void js_set(jstr *s, const uint16_t *p, int n) {
  js_reserve(s, n + 1);
  if (n) memmove(s->p, p, (size_t)n * sizeof(uint16_t));
  s->n = n;
}
void js_set_ascii(jstr *s, const char *a) {
  int n = (int)strlen(a);
  js_reserve(s, n + 1);
  for (int i = 0; i < n; i++) s->p[i] = (unsigned char)a[i];
  s->n = n;
}
void js_push(jstr *s, uint16_t c) {
  js_reserve(s, s->n + 2);
  s->p[s->n++] = c;
}

/* String.compareTo: first differing UTF-16 unit, else length difference. */
int js_cmp(const uint16_t *a, int an, const uint16_t *b, int bn) {
  int m = an < bn ? an : bn;
  for (int i = 0; i < m; i++)
    if (a[i] != b[i]) return (int)a[i] - (int)b[i];
  return an - bn;
}

/* String.hashCode: s[0]*31^(n-1) + ... + s[n-1], int overflow. */
int32_t js_hash(const uint16_t *a, int n) {
  uint32_t h = 0;
  for (int i = 0; i < n; i++) h = 31u * h + a[i];
  return (int32_t)h;
}

/* UTF-8 decode with U+FFFD replacement of each maximal ill-formed subpart
 * (Hadoop Text.decode(..., replace=true) via the JDK UTF-8 CharsetDecoder). */
int utf8_to_utf16(const uint8_t *b, size_t n, jstr *out) {
  out->n = 0;
  js_reserve(out, (int)n + 1);
  size_t i = 0;
  while (i < n) {
    unsigned c = b[i];
    if (c < 0x80) {
      out->p[out->n++] = (uint16_t)c;
      i++;
      continue;
    }
    int need;
    unsigned lo = 0x80, hi = 0xBF, cp;
    if (c >= 0xC2 && c <= 0xDF) {
      need = 1;
      cp = c & 0x1F;
    } else if (c >= 0xE0 && c <= 0xEF) {
      need = 2;
      cp = c & 0x0F;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      need = 3;
      cp = c & 0x07;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else {
      js_push(out, 0xFFFD);
      i++;
      continue;
    }
    size_t j = i + 1;
    int k;
    for (k = 0; k < need; k++, j++) {
      if (j >= n) break;
      unsigned d = b[j];
      unsigned l = (k == 0) ? lo : 0x80, h = (k == 0) ? hi : 0xBF;
      if (d < l || d > h) break;
      cp = (cp << 6) | (d & 0x3F);
    }
    if (k < need) {
      js_push(out, 0xFFFD);
      i = j; /* consume the maximal valid prefix only */
      continue;
    }
    if (cp >= 0x10000) {
      cp -= 0x10000;
      js_push(out, (uint16_t)(0xD800 + (cp >> 10)));
      js_push(out, (uint16_t)(0xDC00 + (cp & 0x3FF)));
    } else {
      js_push(out, (uint16_t)cp);
    }
    i = j;
  }
  return out->n;
}

static int is_hi(uint16_t c) { return c >= 0xD800 && c <= 0xDBFF; }
static int is_lo(uint16_t c) { return c >= 0xDC00 && c <= 0xDFFF; }

int utf8_len_java(const uint16_t *a, int n) {
  int len = 0;
  for (int i = 0; i < n; i++) {
    uint16_t c = a[i];
    if (c < 0x80)
      len += 1;
    else if (c < 0x800)
      len += 2;
    else if (is_hi(c) && i + 1 < n && is_lo(a[i + 1])) {
      len += 4;
      i++;
    } else if (is_hi(c) || is_lo(c))
      len += 1; /* unmappable lone surrogate -> '?' */
    else
      len += 3;
  }
  return len;
}

int mutf8_len(const uint16_t *a, int n) {
  int len = 0;
  for (int i = 0; i < n; i++) {
    uint16_t c = a[i];
    if (c >= 0x0001 && c <= 0x007F)
      len += 1;
    else if (c > 0x07FF)
      len += 3;
    else
      len += 2;
  }
  return len;
}

int mutf8_encode(const uint16_t *a, int n, uint8_t *out) {
  int k = 0;
  for (int i = 0; i < n; i++) {
    uint16_t c = a[i];
    if (c >= 0x0001 && c <= 0x007F) {
      out[k++] = (uint8_t)c;
    } else if (c > 0x07FF) {
      out[k++] = (uint8_t)(0xE0 | ((c >> 12) & 0x0F));
      out[k++] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
      out[k++] = (uint8_t)(0x80 | (c & 0x3F));
    } else {
      out[k++] = (uint8_t)(0xC0 | ((c >> 6) & 0x1F));
      out[k++] = (uint8_t)(0x80 | (c & 0x3F));
    }
  }
  return k;
}

static const unicase_ent *unicase_find(unsigned cp) {
  int lo = 0, hi = UNICASE_N - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    if (UNICASE_TAB[mid].cp == cp) return &UNICASE_TAB[mid];
    if (UNICASE_TAB[mid].cp < cp)
      lo = mid + 1;
    else
      hi = mid - 1;
  }
  return NULL;
}

static void push_cp(jstr *out, unsigned cp) {
  if (cp >= 0x10000) {
    cp -= 0x10000;
    js_push(out, (uint16_t)(0xD800 + (cp >> 10)));
    js_push(out, (uint16_t)(0xDC00 + (cp & 0x3FF)));
  } else {
    js_push(out, (uint16_t)cp);
  }
}

/* String.toLowerCase(): per code point full lowercase mapping.  Final sigma is
 * mapped context-free to U+03C3 (parity unpinned, see gen_unicase.py). */
/* code point ending at / starting at unit index i (surrogate pairs joined) */
static unsigned cp_before(const uint16_t *a, int i, int *w) {
  if (i >= 2 && is_lo(a[i - 1]) && is_hi(a[i - 2])) {
    *w = 2;
    return 0x10000 + (((unsigned)a[i - 2] - 0xD800) << 10) + ((unsigned)a[i - 1] - 0xDC00);
  }
  *w = 1;
  return a[i - 1];
}
static unsigned cp_at(const uint16_t *a, int n, int i, int *w) {
  if (is_hi(a[i]) && i + 1 < n && is_lo(a[i + 1])) {
    *w = 2;
    return 0x10000 + (((unsigned)a[i] - 0xD800) << 10) + ((unsigned)a[i + 1] - 0xDC00);
  }
  *w = 1;
  return a[i];
}
static int in_ranges(const unsigned (*r)[2], int nr, unsigned cp) {
  int lo = 0, hi = nr - 1;
  while (lo <= hi) {
    int m = (lo + hi) >> 1;
    if (cp < r[m][0]) hi = m - 1;
    else if (cp > r[m][1]) lo = m + 1;
    else return 1;
  }
  return 0;
}
/* Final_Sigma context of U+03A3 at unit i of a[0..n): String.toLowerCase gives
 * U+03C2 there (ConditionalSpecialCasing; Unicode rule, see tools/gen_unicase.py):
 * a cased letter before it (case-ignorables skipped), none after it. */
static int final_sigma(const uint16_t *a, int n, int i) {
  int j = i, w;
  unsigned c = 0;
  int found = 0;
  while (j > 0) {
    c = cp_before(a, j, &w);
    j -= w;
    if (!in_ranges(UNISIGMA_CI, UNISIGMA_CI_N, c)) {
      found = 1;
      break;
    }
  }
  if (!found || !in_ranges(UNISIGMA_CASED, UNISIGMA_CASED_N, c)) return 0;
  for (j = i + 1; j < n; j += w) {
    c = cp_at(a, n, j, &w);
    if (!in_ranges(UNISIGMA_CI, UNISIGMA_CI_N, c)) return !in_ranges(UNISIGMA_CASED, UNISIGMA_CASED_N, c);
  }
  return 1;
}

void java_tolower(const uint16_t *a, int n, jstr *out) {
  for (int i = 0; i < n; i++) {
    unsigned cp = a[i];
    int w = 1;
    if (is_hi(a[i]) && i + 1 < n && is_lo(a[i + 1])) {
      cp = 0x10000 + (((unsigned)a[i] - 0xD800) << 10) + ((unsigned)a[i + 1] - 0xDC00);
      w = 2;
    }
    if (cp == 0x03A3 && final_sigma(a, n, i)) {
      js_push(out, 0x03C2);
    } else if (cp < 0x80) {
      js_push(out, (uint16_t)((cp >= 'A' && cp <= 'Z') ? cp + 32 : cp));
    } else {
      const unicase_ent *e = unicase_find(cp);
      if (!e) {
        js_push(out, a[i]);
        if (w == 2) js_push(out, a[i + 1]);
      } else {
        for (int k = 0; k < 3 && e->lo[k]; k++) push_cp(out, e->lo[k]);
      }
    }
    i += w - 1;
  }
}
