// sme_text.hpp -- device text semantics of the reference tokenizer chain.
//
//   split table            TagTokenizer.buildSplits            TagTokenizer.java:73-95
//   Character.isSpaceChar  (JDK; Zs/Zl/Zp, JDK 6/7 tables)     used at TagTokenizer.java:185,227,251,269,297
//   UTF-8 decode           Hadoop Text.toString (JDK decoder, REPLACE) TrecDocumentInputFormat.java:75
//   token normalization    onSplit/checkTokenStatus/tokenSimpleFix/tokenComplexFix/
//                          tokenAcronymProcessing/addToken     TagTokenizer.java:399-600
//   stopwords              GalagoTokenizer.java:35-133,152-156
//   sequential scan        TagTokenizer.tokenize + tag/comment/PI/entity parsing
//                          TagTokenizer.java:155-393,602-709 (slow path, one thread per record)
// (C/org/galagosearch/core/parse/ and C/ivory/tokenize/ of the reference.)
#pragma once
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "sme_stem.hpp"
#include "stopwords_tab.hpp"
#include "unicase_tab.h"

namespace sme {

// ---- character classes ---------------------------------------------------
// split set: 0..32 and ; " & / : ! # ? $ % ( ) @ ^ * + - , = > < [ ] { } | ` ~ _
__device__ __forceinline__ bool is_split_byte(uint32_t c) {
  // bitmap over 0..127 as four 32-bit words
  constexpr uint32_t w0 = 0xFFFFFFFFu;  // 0..31
  // 32..63: ' '32 !33 "34 #35 $36 %37 &38 (40 )41 *42 +43 ,44 -45 /47 :58 ;59 <60 =61 >62 ?63
  constexpr uint32_t w1 = (1u << 0) | (1u << 1) | (1u << 2) | (1u << 3) | (1u << 4) | (1u << 5) |
                          (1u << 6) | (1u << 8) | (1u << 9) | (1u << 10) | (1u << 11) | (1u << 12) |
                          (1u << 13) | (1u << 15) | (1u << 26) | (1u << 27) | (1u << 28) | (1u << 29) |
                          (1u << 30) | (1u << 31);
  // 64..95: @64 [91 ]93 ^94 _95
  constexpr uint32_t w2 = (1u << 0) | (1u << 27) | (1u << 29) | (1u << 30) | (1u << 31);
  // 96..127: `96 {123 |124 }125 ~126
  constexpr uint32_t w3 = (1u << 0) | (1u << 27) | (1u << 28) | (1u << 29) | (1u << 30);
  if (c >= 128) return false;
  uint32_t w = c < 32 ? w0 : c < 64 ? w1 : c < 96 ? w2 : w3;
  return (w >> (c & 31)) & 1u;
}

__device__ __forceinline__ bool is_space_char(uint32_t c) {
  if (c == 0x20 || c == 0xA0 || c == 0x1680 || c == 0x180E) return true;
  if (c >= 0x2000 && c <= 0x200A) return true;
  return c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

// ---- UTF-8 -> UTF-16 with U+FFFD for each maximal ill-formed subpart -------
// Decodes one code point at b[i..n); returns bytes consumed, writes 1 or 2 units.
__device__ __forceinline__ int utf8_step(const uint8_t *b, int64_t i, int64_t n, uint16_t *u,
                                         int *nu) {
  uint32_t c = b[i];
  if (c < 0x80) {
    u[0] = (uint16_t)c;
    *nu = 1;
    return 1;
  }
  int need;
  uint32_t lo = 0x80, hi = 0xBF, cp;
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
    u[0] = 0xFFFD;
    *nu = 1;
    return 1;
  }
  int k = 0;
  for (; k < need; k++) {
    int64_t j = i + 1 + k;
    if (j >= n) break;
    uint32_t d = b[j];
    uint32_t l = k == 0 ? lo : 0x80u, h = k == 0 ? hi : 0xBFu;
    if (d < l || d > h) break;
    cp = (cp << 6) | (d & 0x3F);
  }
  if (k < need) {
    u[0] = 0xFFFD;
    *nu = 1;
    return 1 + k;
  }
  if (cp >= 0x10000) {
    cp -= 0x10000;
    u[0] = (uint16_t)(0xD800 + (cp >> 10));
    u[1] = (uint16_t)(0xDC00 + (cp & 0x3FF));
    *nu = 2;
  } else {
    u[0] = (uint16_t)cp;
    *nu = 1;
  }
  return 1 + need;
}

// ---- String.toLowerCase (full mapping per code point) --------------------
__device__ __forceinline__ const unicase_ent *unicase_lookup(uint32_t cp) {
  int lo = 0, hi = UNICASE_N - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    uint32_t m = UNICASE_TAB[mid].cp;
    if (m == cp) return &UNICASE_TAB[mid];
    if (m < cp)
      lo = mid + 1;
    else
      hi = mid - 1;
  }
  return nullptr;
}

__device__ __forceinline__ bool in_cp_ranges(const unsigned int (*r)[2], int nr, uint32_t cp) {
  int lo = 0, hi = nr - 1;
  while (lo <= hi) {
    const int m = (lo + hi) >> 1;
    if (cp < r[m][0])
      hi = m - 1;
    else if (cp > r[m][1])
      lo = m + 1;
    else
      return true;
  }
  return false;
}
// Final_Sigma context of U+03A3 at unit i of a[0..n) (String.toLowerCase ->
// U+03C2, ConditionalSpecialCasing): a cased letter before it with only
// case-ignorables between, and no cased letter after it (case-ignorables
// skipped).  Tables from tools/gen_unicase.py.
__device__ inline bool final_sigma(const uint16_t *a, int n, int i) {
  int j = i;
  uint32_t c = 0;
  bool found = false;
  while (j > 0) {
    if (j >= 2 && a[j - 1] >= 0xDC00 && a[j - 1] <= 0xDFFF && a[j - 2] >= 0xD800 && a[j - 2] <= 0xDBFF) {
      c = 0x10000 + ((uint32_t)(a[j - 2] - 0xD800) << 10) + (a[j - 1] - 0xDC00u);
      j -= 2;
    } else {
      c = a[j - 1];
      j -= 1;
    }
    if (!in_cp_ranges(UNISIGMA_CI, UNISIGMA_CI_N, c)) {
      found = true;
      break;
    }
  }
  if (!found || !in_cp_ranges(UNISIGMA_CASED, UNISIGMA_CASED_N, c)) return false;
  for (j = i + 1; j < n;) {
    if (a[j] >= 0xD800 && a[j] <= 0xDBFF && j + 1 < n && a[j + 1] >= 0xDC00 && a[j + 1] <= 0xDFFF) {
      c = 0x10000 + ((uint32_t)(a[j] - 0xD800) << 10) + (a[j + 1] - 0xDC00u);
      j += 2;
    } else {
      c = a[j];
      j += 1;
    }
    if (!in_cp_ranges(UNISIGMA_CI, UNISIGMA_CI_N, c)) return !in_cp_ranges(UNISIGMA_CASED, UNISIGMA_CASED_N, c);
  }
  return true;
}

// Appends lower(a[0..n)) to out (capacity cap); returns new length or -1 on overflow.
__device__ inline int java_lower(const uint16_t *a, int n, uint16_t *out, int cap) {
  int k = 0;
  for (int i = 0; i < n; i++) {
    uint32_t cp = a[i];
    int w = 1;
    if (cp >= 0xD800 && cp <= 0xDBFF && i + 1 < n && a[i + 1] >= 0xDC00 && a[i + 1] <= 0xDFFF) {
      cp = 0x10000 + ((cp - 0xD800) << 10) + (a[i + 1] - 0xDC00u);
      w = 2;
    }
    if (cp == 0x03A3 && final_sigma(a, n, i)) {
      if (k >= cap) return -1;
      out[k++] = 0x03C2;
    } else if (cp < 0x80) {
      if (k >= cap) return -1;
      out[k++] = (uint16_t)((cp >= 'A' && cp <= 'Z') ? cp + 32 : cp);
    } else {
      const unicase_ent *e = unicase_lookup(cp);
      if (!e) {
        if (k + w > cap) return -1;
        out[k++] = a[i];
        if (w == 2) out[k++] = a[i + 1];
      } else {
        for (int t = 0; t < 3 && e->lo[t]; t++) {
          uint32_t l = e->lo[t];
          if (l >= 0x10000) {
            if (k + 2 > cap) return -1;
            l -= 0x10000;
            out[k++] = (uint16_t)(0xD800 + (l >> 10));
            out[k++] = (uint16_t)(0xDC00 + (l & 0x3FF));
          } else {
            if (k >= cap) return -1;
            out[k++] = (uint16_t)l;
          }
        }
      }
    }
    i += w - 1;
  }
  return k;
}

// String.getBytes("UTF-8").length
__device__ __forceinline__ int java_utf8_len(const uint16_t *a, int n) {
  int len = 0;
  for (int i = 0; i < n; i++) {
    uint32_t c = a[i];
    if (c < 0x80)
      len += 1;
    else if (c < 0x800)
      len += 2;
    else if (c >= 0xD800 && c <= 0xDBFF && i + 1 < n && a[i + 1] >= 0xDC00 && a[i + 1] <= 0xDFFF) {
      len += 4;
      i++;
    } else if (c >= 0xD800 && c <= 0xDFFF)
      len += 1;
    else
      len += 3;
  }
  return len;
}

__device__ __forceinline__ bool is_stopword(const uint16_t *w, int n) {
  int lo = 0, hi = SME_NSTOP - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    int b = kStopOff[mid], e = kStopOff[mid + 1];
    int sl = e - b, m = sl < n ? sl : n, c = 0;
    for (int i = 0; i < m && c == 0; i++) c = (int)(uint8_t)kStopChars[b + i] - (int)w[i];
    if (c == 0) c = sl - n;
    if (c == 0) return true;
    if (c < 0)
      lo = mid + 1;
    else
      hi = mid - 1;
  }
  return false;
}

// ---- per-raw-token normalization ---------------------------------------------
// raw: UTF-16 units of text[lastSplit+1, position).  For every token addToken
// keeps, emit(ptr, len) is called with the (not yet stopped/stemmed) token.
// work: scratch of at least 2*n+8 units (toLowerCase may expand).
template <typename Emit>
__device__ inline void normalize_raw(const uint16_t *raw, int n, uint16_t *work, int work_cap,
                                     Emit &&emit) {
  auto add_token = [&](const uint16_t *p, int l) {
    if (l <= 0) return;
    if (l > 100 / 6 && java_utf8_len(p, l) >= 100) return;
    emit(p, l);
  };
  // checkTokenStatus
  int status = 0;  // 0 clean, 1 simple, 2 complex, 3 acronym
  for (int i = 0; i < n; i++) {
    uint32_t c = raw[i];
    if ((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9')) continue;
    bool up = c >= 'A' && c <= 'Z', apo = c == '\'', per = c == '.';
    if ((up || apo) && status == 0)
      status = 1;
    else if (!per)
      status = 2;
    else {
      status = 3;
      break;
    }
  }
  if (status == 0) {
    add_token(raw, n);
    return;
  }
  // tokenSimpleFix into work[0..)
  int j = 0;
  for (int i = 0; i < n; i++) {
    uint32_t c = raw[i];
    if (c == '\'') continue;
    work[j++] = (uint16_t)((c >= 'A' && c <= 'Z') ? c + 32 : c);
  }
  if (status == 1) {
    add_token(work, j);
    return;
  }
  // tokenComplexFix: toLowerCase into work[j..)
  uint16_t *lw = work + j;
  int ln = java_lower(work, j, lw, work_cap - j);
  if (ln < 0) return;  // cannot happen with work_cap >= 2n+8 except pathological expansions
  if (status == 2) {
    add_token(lw, ln);
    return;
  }
  // tokenAcronymProcessing
  int b = 0, e = ln;
  while (b < e && lw[b] == '.') b++;
  while (e > b && lw[e - 1] == '.') e--;
  const uint16_t *s = lw + b;
  int sl = e - b;
  bool has_dot = false;
  for (int i = 0; i < sl; i++) has_dot |= (s[i] == '.');
  if (!has_dot) {
    add_token(s, sl);
    return;
  }
  bool acr = sl > 0;
  for (int pos = 1; pos < sl; pos += 2) acr &= (s[pos] == '.');
  if (acr) {
    // remove all '.' in place (target region work[0..) is free again)
    int k = 0;
    for (int i = 0; i < sl; i++)
      if (s[i] != '.') work[k++] = s[i];
    add_token(work, k);
    return;
  }
  int st = 0;
  for (int x = 0; x < sl; x++) {
    if (s[x] == '.') {
      if (x - st > 1) add_token(s + st, x - st);
      st = x + 1;
    }
  }
  if (sl - st > 1) add_token(s + st, sl - st);
}

// ---- sequential TagTokenizer over a decoded record (slow path) ---------------
// text: UTF-16 units.  For every raw token text[lastSplit+1, position) with
// position - lastSplit > 1, on_raw(unit_start, unit_end) is called.
struct TagScan {
  const uint16_t *t;
  int n;
  int pos, last;
  bool ignoring;
  uint16_t ign[8];
  int ign_len;  // ignoreUntil is only ever "script" or "style"

  __device__ int index_of(const char *s, int sl, int from) const {
    if (from < 0) from = 0;
    if (from >= n) return sl == 0 ? n : -1;
    for (int i = from; i + sl <= n; i++) {
      int k = 0;
      while (k < sl && t[i + k] == (uint16_t)(uint8_t)s[k]) k++;
      if (k == sl) return i;
    }
    return -1;
  }
  // on_raw(first unit, end unit) of text[lastSplit+1, position)
  template <typename F>
  __device__ void on_split(F &&on_raw) {
    if (pos - last > 1) on_raw(last + 1, pos);
    last = pos;
  }
  // tag name t[a, b) lowered equals "script"/"style"?
  __device__ int ignored_name(int a, int b) const {
    uint16_t buf[40];
    if (b - a > 12) return 0;  // lowering never shrinks a string by more than... it never shrinks
    int l = java_lower(t + a, b - a, buf, 40);
    if (l == 6 && buf[0] == 's' && buf[1] == 'c' && buf[2] == 'r' && buf[3] == 'i' && buf[4] == 'p' &&
        buf[5] == 't')
      return 6;
    if (l == 5 && buf[0] == 's' && buf[1] == 't' && buf[2] == 'y' && buf[3] == 'l' && buf[4] == 'e')
      return 5;
    return 0;
  }
  __device__ void parse_end_tag() {
    int i;
    for (i = pos + 2; i < n; i++) {
      uint16_t c = t[i];
      if (is_space_char(c) || c == '>') break;
    }
    if (ignoring) {
      uint16_t buf[40];
      int l = (i - (pos + 2) <= 12) ? java_lower(t + pos + 2, i - (pos + 2), buf, 40) : -1;
      if (l == ign_len) {
        bool eq = true;
        for (int k = 0; k < l; k++) eq &= buf[k] == ign[k];
        if (eq) ignoring = false;
      }
    }
    while (i < n && t[i] != '>') i++;
    pos = i;
  }
  __device__ int non_space(int s) const {
    if (s < 0) return INT_MIN;
    for (int i = s; i < n; i++)
      if (!is_space_char(t[i])) return i;
    return INT_MIN;
  }
  __device__ int end_attr(int s, int tagEnd) const {
    if (s < 0) return INT_MIN;
    bool inq = false, esc = false;
    for (int i = s; i <= tagEnd; i++) {
      uint16_t c = t[i];
      if ((c == '"' || c == '\'') && !esc) {
        inq = !inq;
        if (!inq) return i;
      } else if (!inq && (is_space_char(c) || c == '>')) {
        return i;
      } else if (c == '\\' && !esc) {
        esc = true;
      } else {
        esc = false;
      }
    }
    return INT_MIN;
  }
  __device__ int equals_at(int s, int e) const {
    if (s < 0) return INT_MIN;
    for (int i = s; i < e; i++)
      if (t[i] == '=') return i;
    return INT_MIN;
  }
  __device__ void parse_begin_tag() {
    int i;
    for (i = pos + 1; i < n; i++) {
      uint16_t c = t[i];
      if (is_space_char(c) || c == '>') break;
    }
    int ig = ignored_name(pos + 1, i);
    i = non_space(i);
    int tagEnd = index_of(">", 1, i + 1);
    bool closeIt = false;
    while (i < tagEnd && i >= 0 && tagEnd >= 0) {
      int s = non_space(i);
      if (s > 0) {
        if (t[s] == '>') {
          i = s;
          break;
        } else if (t[s] == '/' && n > s + 1 && t[s + 1] == '>') {
          i = s + 1;
          closeIt = true;
          break;
        }
      }
      int e = end_attr(s, tagEnd);
      int eq = equals_at(s, e);
      if (eq < 0 || eq == s || e == eq) {
        if (e < 0) {
          i = tagEnd;
          break;
        }
        i = e;
        continue;
      }
      int sv = eq + 1;
      if (t[sv] == '"' || t[sv] == '\'') sv++;
      if (sv >= e || s >= eq) {
        i = e;
        continue;
      }
      if (e >= n) {
        pos = n;
        break;
      }
      if (t[e] == '"' || t[e] == '\'') e++;
      i = e;
    }
    if (ig && !closeIt) {
      ignoring = true;
      ign_len = ig;
      const char *nm = ig == 6 ? "script" : "style";
      for (int k = 0; k < ig; k++) ign[k] = (uint16_t)nm[k];
    }
    pos = i;
  }
  __device__ void on_start_bracket() {
    if (pos + 1 < n) {
      uint16_t c = t[pos + 1];
      if (c == '/') {
        parse_end_tag();
      } else if (c == '!') {
        bool cm = pos + 4 <= n && t[pos + 2] == '-' && t[pos + 3] == '-';
        if (cm) {
          pos = index_of("-->", 3, pos + 1);
          if (pos >= 0) pos += 2;
        } else {
          pos = index_of(">", 1, pos + 1);
        }
        if (pos < 0) pos = n;
      } else if (c == '?') {
        pos = index_of("?>", 2, pos + 1);
        if (pos < 0) pos = n;
      } else {
        parse_begin_tag();
      }
    } else {
      pos = n;
    }
    last = pos;
  }
  template <typename F>
  __device__ void run(F &&on_raw) {
    pos = 0;
    last = -1;
    ignoring = false;
    ign_len = 0;
    for (; pos >= 0 && pos < n; pos++) {
      uint16_t c = t[pos];
      if (c == '<') {
        if (!ignoring) on_split(on_raw);
        on_start_bracket();
      } else if (ignoring) {
        continue;
      } else if (c == '&') {
        on_split(on_raw);
        for (int i = pos + 1; i < n; i++) {
          uint16_t d = t[i];
          if ((d >= 'a' && d <= 'z') || (d >= '0' && d <= '9') || d == '#') continue;
          if (d == ';') {
            pos = i;
            last = i;
          }
          break;
        }
      } else if (c < 256 && is_split_byte(c)) {
        on_split(on_raw);
      }
    }
    if (!ignoring) on_split(on_raw);
  }
};

}  // namespace sme
