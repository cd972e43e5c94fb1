// sme_stem.hpp -- device Porter2 (Snowball English, ~2010 tables) stemmer.
//
// Semantics follow C/org/tartarus/snowball/ext/englishStemmer.java (stem()
// 1149-1317, steps 178-1147) and the runtime C/org/tartarus/snowball/
// SnowballProgram.java (find_among 181, find_among_b 254, replace_s 325).
// The generated Java drives a cursor/limit/bra/ket machine over a StringBuffer;
// here the buffer is a fixed 128-unit register/scratch array (inputs are
// normalized tokens: at most 99 UTF-16 units, TagTokenizer.addToken drops
// longer ones, and a stem grows by at most 2 units).  One thread stems one
// word; this runs once per distinct raw token (vocabulary level, T13).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sme {

constexpr int kStemCap = 128;

struct AmongEnt {
  const char *s;
  int8_t len;
  int8_t substring_i;
  int8_t result;
};

#define SME_A(s, i, r) {s, (int8_t)(sizeof(s) - 1), (int8_t)(i), (int8_t)(r)}
__device__ static const AmongEnt kA0[] = {SME_A("arsen", -1, -1), SME_A("commun", -1, -1),
                                          SME_A("gener", -1, -1)};
__device__ static const AmongEnt kA1[] = {SME_A("'", -1, 1), SME_A("'s'", 0, 1), SME_A("'s", -1, 1)};
__device__ static const AmongEnt kA2[] = {SME_A("ied", -1, 2), SME_A("s", -1, 3),   SME_A("ies", 1, 2),
                                          SME_A("sses", 1, 1), SME_A("ss", 1, -1), SME_A("us", 1, -1)};
__device__ static const AmongEnt kA3[] = {SME_A("", -1, 3),  SME_A("bb", 0, 2), SME_A("dd", 0, 2),
                                          SME_A("ff", 0, 2), SME_A("gg", 0, 2), SME_A("bl", 0, 1),
                                          SME_A("mm", 0, 2), SME_A("nn", 0, 2), SME_A("pp", 0, 2),
                                          SME_A("rr", 0, 2), SME_A("at", 0, 1), SME_A("tt", 0, 2),
                                          SME_A("iz", 0, 1)};
__device__ static const AmongEnt kA4[] = {SME_A("ed", -1, 2),   SME_A("eed", 0, 1),   SME_A("ing", -1, 2),
                                          SME_A("edly", -1, 2), SME_A("eedly", 3, 1), SME_A("ingly", -1, 2)};
__device__ static const AmongEnt kA5[] = {
    SME_A("anci", -1, 3),     SME_A("enci", -1, 2),    SME_A("ogi", -1, 13),     SME_A("li", -1, 16),
    SME_A("bli", 3, 12),      SME_A("abli", 4, 4),     SME_A("alli", 3, 8),      SME_A("fulli", 3, 14),
    SME_A("lessli", 3, 15),   SME_A("ousli", 3, 10),   SME_A("entli", 3, 5),     SME_A("aliti", -1, 8),
    SME_A("biliti", -1, 12),  SME_A("iviti", -1, 11),  SME_A("tional", -1, 1),   SME_A("ational", 14, 7),
    SME_A("alism", -1, 8),    SME_A("ation", -1, 7),   SME_A("ization", 17, 6),  SME_A("izer", -1, 6),
    SME_A("ator", -1, 7),     SME_A("iveness", -1, 11), SME_A("fulness", -1, 9), SME_A("ousness", -1, 10)};
__device__ static const AmongEnt kA6[] = {SME_A("icate", -1, 4), SME_A("ative", -1, 6), SME_A("alize", -1, 3),
                                          SME_A("iciti", -1, 4), SME_A("ical", -1, 4),  SME_A("tional", -1, 1),
                                          SME_A("ational", 5, 2), SME_A("ful", -1, 5),  SME_A("ness", -1, 5)};
__device__ static const AmongEnt kA7[] = {
    SME_A("ic", -1, 1),  SME_A("ance", -1, 1), SME_A("ence", -1, 1), SME_A("able", -1, 1), SME_A("ible", -1, 1),
    SME_A("ate", -1, 1), SME_A("ive", -1, 1),  SME_A("ize", -1, 1),  SME_A("iti", -1, 1),  SME_A("al", -1, 1),
    SME_A("ism", -1, 1), SME_A("ion", -1, 2),  SME_A("er", -1, 1),   SME_A("ous", -1, 1),  SME_A("ant", -1, 1),
    SME_A("ent", -1, 1), SME_A("ment", 15, 1), SME_A("ement", 16, 1)};
__device__ static const AmongEnt kA8[] = {SME_A("e", -1, 1), SME_A("l", -1, 2)};
__device__ static const AmongEnt kA9[] = {SME_A("succeed", -1, -1), SME_A("proceed", -1, -1),
                                          SME_A("exceed", -1, -1),  SME_A("canning", -1, -1),
                                          SME_A("inning", -1, -1),  SME_A("earring", -1, -1),
                                          SME_A("herring", -1, -1), SME_A("outing", -1, -1)};
__device__ static const AmongEnt kA10[] = {
    SME_A("andes", -1, -1), SME_A("atlas", -1, -1), SME_A("bias", -1, -1),   SME_A("cosmos", -1, -1),
    SME_A("dying", -1, 3),  SME_A("early", -1, 9),  SME_A("gently", -1, 7),  SME_A("howe", -1, -1),
    SME_A("idly", -1, 6),   SME_A("lying", -1, 4),  SME_A("news", -1, -1),   SME_A("only", -1, 10),
    SME_A("singly", -1, 11), SME_A("skies", -1, 2), SME_A("skis", -1, 1),    SME_A("sky", -1, -1),
    SME_A("tying", -1, 5),  SME_A("ugly", -1, 8)};
#undef SME_A

// groupings as 32-bit masks over their [min, max] ranges
__device__ __forceinline__ bool g_v(uint32_t c) {  // a e i o u y, range 97..121
  return c >= 97 && c <= 121 && ((0x1104111u >> (c - 97)) & 1u);
}
__device__ __forceinline__ bool g_v_wxy(uint32_t c) {  // v + w x Y over 89..121
  return c >= 89 && c <= 121 && (((uint64_t)0x1D0411101ull >> (c - 89)) & 1ull);
}
__device__ __forceinline__ bool g_valid_li(uint32_t c) {  // c d e g h k m n r t over 99..116
  return c >= 99 && c <= 116 && ((0x28D37u >> (c - 99)) & 1u);
}

// b points at the word: the stemmer's own array (private, i.e. scratch
// memory, as the buffer is indexed at run time), or a caller's LDS slice
template <int CAP>
struct StemmerT {
  uint16_t own[CAP];
  uint16_t *b;
  int len;
  __device__ StemmerT() : b(own) {}
  __device__ explicit StemmerT(uint16_t *ext) : b(ext) {}
  StemmerT(const StemmerT &) = delete;
  StemmerT &operator=(const StemmerT &) = delete;
  int c, lim, lb, bra, ket;
  int p1, p2;
  bool y_found;

  template <bool (*g)(uint32_t)>
  __device__ bool in_g() {
    if (c >= lim) return false;
    if (!g(b[c])) return false;
    c++;
    return true;
  }
  template <bool (*g)(uint32_t)>
  __device__ bool in_g_b() {
    if (c <= lb) return false;
    if (!g(b[c - 1])) return false;
    c--;
    return true;
  }
  template <bool (*g)(uint32_t)>
  __device__ bool out_g() {
    if (c >= lim) return false;
    if (g(b[c])) return false;
    c++;
    return true;
  }
  template <bool (*g)(uint32_t)>
  __device__ bool out_g_b() {
    if (c <= lb) return false;
    if (g(b[c - 1])) return false;
    c--;
    return true;
  }
  __device__ bool eq1(char ch) {
    if (lim - c < 1 || b[c] != (uint16_t)ch) return false;
    c++;
    return true;
  }
  __device__ bool eq1_b(char ch) {
    if (c - lb < 1 || b[c - 1] != (uint16_t)ch) return false;
    c--;
    return true;
  }
  // forward / backward longest-match among lookups (binary search with shared prefix)
  __device__ int among_f(const AmongEnt *v, int n) {
    int i = 0, j = n, cs = c, common_i = 0, common_j = 0;
    bool first = false;
    for (;;) {
      int k = i + ((j - i) >> 1), diff = 0;
      int common = common_i < common_j ? common_i : common_j;
      const AmongEnt &w = v[k];
      for (int i2 = common; i2 < w.len; i2++) {
        if (cs + common == lim) {
          diff = -1;
          break;
        }
        diff = (int)b[cs + common] - (int)(uint8_t)w.s[i2];
        if (diff) break;
        common++;
      }
      if (diff < 0) {
        j = k;
        common_j = common;
      } else {
        i = k;
        common_i = common;
      }
      if (j - i <= 1) {
        if (i > 0 || j == i || first) break;
        first = true;
      }
    }
    for (;;) {
      const AmongEnt &w = v[i];
      if (common_i >= w.len) {
        c = cs + w.len;
        return w.result;
      }
      i = w.substring_i;
      if (i < 0) return 0;
    }
  }
  __device__ int among_b(const AmongEnt *v, int n) {
    int i = 0, j = n, cs = c, common_i = 0, common_j = 0;
    bool first = false;
    for (;;) {
      int k = i + ((j - i) >> 1), diff = 0;
      int common = common_i < common_j ? common_i : common_j;
      const AmongEnt &w = v[k];
      for (int i2 = w.len - 1 - common; i2 >= 0; i2--) {
        if (cs - common == lb) {
          diff = -1;
          break;
        }
        diff = (int)b[cs - 1 - common] - (int)(uint8_t)w.s[i2];
        if (diff) break;
        common++;
      }
      if (diff < 0) {
        j = k;
        common_j = common;
      } else {
        i = k;
        common_i = common;
      }
      if (j - i <= 1) {
        if (i > 0 || j == i || first) break;
        first = true;
      }
    }
    for (;;) {
      const AmongEnt &w = v[i];
      if (common_i >= w.len) {
        c = cs - w.len;
        return w.result;
      }
      i = w.substring_i;
      if (i < 0) return 0;
    }
  }
  // StringBuffer.replace(c_bra, c_ket, s) plus cursor/limit bookkeeping
  __device__ int replace(int c_bra, int c_ket, const char *s, int sl) {
    int adj = sl - (c_ket - c_bra);
    if (adj > 0) {
      for (int x = len - 1; x >= c_ket; x--) b[x + adj] = b[x];
    } else if (adj < 0) {
      for (int x = c_ket; x < len; x++) b[x + adj] = b[x];
    }
    for (int x = 0; x < sl; x++) b[c_bra + x] = (uint8_t)s[x];
    len += adj;
    lim += adj;
    if (c >= c_ket)
      c += adj;
    else if (c > c_bra)
      c = c_bra;
    return adj;
  }
  __device__ void slice(const char *s, int sl) { replace(bra, ket, s, sl); }
  __device__ void del() { replace(bra, ket, "", 0); }
  __device__ void ins_e() {  // <+ "e" at cursor, cursor preserved
    int cs = c;
    int adj = replace(cs, cs, "e", 1);
    if (cs <= bra) bra += adj;  // insert(): c_bra <= bra
    if (cs <= ket) ket += adj;
    c = cs;
  }

  __device__ void prelude() {
    y_found = false;
    int v = c;
    bra = c;
    if (eq1('\'')) {
      ket = c;
      del();
    }
    c = v;
    bra = c;
    if (eq1('y')) {
      ket = c;
      slice("Y", 1);
      y_found = true;
    }
    c = v;
    for (;;) {
      int v4 = c;
      bool hit = false;
      for (;;) {
        int v5 = c;
        if (in_g<g_v>()) {
          bra = c;
          if (eq1('y')) {
            ket = c;
            c = v5;
            hit = true;
            break;
          }
        }
        c = v5;
        if (c >= lim) break;
        c++;
      }
      if (!hit) {
        c = v4;
        break;
      }
      slice("Y", 1);
      y_found = true;
    }
    c = v;
  }
  __device__ bool gopast_v() {
    for (;;) {
      if (in_g<g_v>()) return true;
      if (c >= lim) return false;
      c++;
    }
  }
  __device__ bool gopast_nv() {
    for (;;) {
      if (out_g<g_v>()) return true;
      if (c >= lim) return false;
      c++;
    }
  }
  __device__ void mark_regions() {
    p1 = lim;
    p2 = lim;
    int v = c;
    do {
      int v2 = c;
      if (among_f(kA0, 3) == 0) {
        c = v2;
        if (!gopast_v() || !gopast_nv()) break;
      }
      p1 = c;
      if (!gopast_v() || !gopast_nv()) break;
      p2 = c;
    } while (0);
    c = v;
  }
  __device__ bool shortv() {
    int v = lim - c;
    if (out_g_b<g_v_wxy>() && in_g_b<g_v>() && out_g_b<g_v>()) return true;
    c = lim - v;
    if (!out_g_b<g_v>()) return false;
    if (!in_g_b<g_v>()) return false;
    return c <= lb;
  }
  __device__ void step1a() {
    int v = lim - c;
    ket = c;
    int a = among_b(kA1, 3);
    if (a == 0) {
      c = lim - v;
    } else {
      bra = c;
      del();
    }
    ket = c;
    a = among_b(kA2, 6);
    if (a == 0) return;
    bra = c;
    if (a == 1) {
      slice("ss", 2);
    } else if (a == 2) {
      int t = c - 2;
      if (lb > t || t > lim) {
        slice("ie", 2);
      } else {
        c = t;
        slice("i", 1);
      }
    } else if (a == 3) {
      if (c <= lb) return;
      c--;
      for (;;) {
        if (in_g_b<g_v>()) break;
        if (c <= lb) return;
        c--;
      }
      del();
    }
  }
  __device__ void step1b() {
    ket = c;
    int a = among_b(kA4, 6);
    if (a == 0) return;
    bra = c;
    if (a == 1) {
      if (p1 <= c) slice("ee", 2);
      return;
    }
    int v = lim - c;
    for (;;) {
      if (in_g_b<g_v>()) break;
      if (c <= lb) return;
      c--;
    }
    c = lim - v;
    del();
    int v3 = lim - c;
    a = among_b(kA3, 13);
    if (a == 0) return;
    c = lim - v3;
    if (a == 1) {
      ins_e();
    } else if (a == 2) {
      ket = c;
      if (c <= lb) return;
      c--;
      bra = c;
      del();
    } else if (a == 3) {
      if (c != p1) return;
      int v4 = lim - c;
      if (!shortv()) return;
      c = lim - v4;
      ins_e();
    }
  }
  __device__ void step1c() {
    ket = c;
    int v = lim - c;
    if (!eq1_b('y')) {
      c = lim - v;
      if (!eq1_b('Y')) return;
    }
    bra = c;
    if (!out_g_b<g_v>()) return;
    if (c <= lb) return;
    slice("i", 1);
  }
  __device__ void step2() {
    ket = c;
    int a = among_b(kA5, 24);
    if (a == 0) return;
    bra = c;
    if (!(p1 <= c)) return;
    switch (a) {
      case 1: slice("tion", 4); break;
      case 2: slice("ence", 4); break;
      case 3: slice("ance", 4); break;
      case 4: slice("able", 4); break;
      case 5: slice("ent", 3); break;
      case 6: slice("ize", 3); break;
      case 7: slice("ate", 3); break;
      case 8: slice("al", 2); break;
      case 9: slice("ful", 3); break;
      case 10: slice("ous", 3); break;
      case 11: slice("ive", 3); break;
      case 12: slice("ble", 3); break;
      case 13:
        if (eq1_b('l')) slice("og", 2);
        break;
      case 14: slice("ful", 3); break;
      case 15: slice("less", 4); break;
      case 16:
        if (in_g_b<g_valid_li>()) del();
        break;
    }
  }
  __device__ void step3() {
    ket = c;
    int a = among_b(kA6, 9);
    if (a == 0) return;
    bra = c;
    if (!(p1 <= c)) return;
    switch (a) {
      case 1: slice("tion", 4); break;
      case 2: slice("ate", 3); break;
      case 3: slice("al", 2); break;
      case 4: slice("ic", 2); break;
      case 5: del(); break;
      case 6:
        if (p2 <= c) del();
        break;
    }
  }
  __device__ void step4() {
    ket = c;
    int a = among_b(kA7, 18);
    if (a == 0) return;
    bra = c;
    if (!(p2 <= c)) return;
    if (a == 1) {
      del();
    } else if (a == 2) {
      int v = lim - c;
      if (!eq1_b('s')) {
        c = lim - v;
        if (!eq1_b('t')) return;
      }
      del();
    }
  }
  __device__ void step5() {
    ket = c;
    int a = among_b(kA8, 2);
    if (a == 0) return;
    bra = c;
    if (a == 1) {
      if (!(p2 <= c)) {
        if (!(p1 <= c)) return;
        int v = lim - c;
        if (shortv()) return;
        c = lim - v;
      }
      del();
    } else if (a == 2) {
      if (!(p2 <= c)) return;
      if (!eq1_b('l')) return;
      del();
    }
  }
  __device__ bool exception2() {
    ket = c;
    if (among_b(kA9, 8) == 0) return false;
    bra = c;
    return c <= lb;
  }
  __device__ bool exception1() {
    bra = c;
    int a = among_f(kA10, 18);
    if (a == 0) return false;
    ket = c;
    if (c < lim) return false;
    switch (a) {
      case 1: slice("ski", 3); break;
      case 2: slice("sky", 3); break;
      case 3: slice("die", 3); break;
      case 4: slice("lie", 3); break;
      case 5: slice("tie", 3); break;
      case 6: slice("idl", 3); break;
      case 7: slice("gentl", 5); break;
      case 8: slice("ugli", 4); break;
      case 9: slice("earli", 5); break;
      case 10: slice("onli", 4); break;
      case 11: slice("singl", 5); break;
    }
    return true;
  }
  __device__ void postlude() {
    if (!y_found) return;
    for (;;) {
      int v1 = c;
      bool hit = false;
      for (;;) {
        int v2 = c;
        bra = c;
        if (eq1('Y')) {
          ket = c;
          c = v2;
          hit = true;
          break;
        }
        c = v2;
        if (c >= lim) break;
        c++;
      }
      if (!hit) {
        c = v1;
        break;
      }
      slice("y", 1);
    }
  }
  // stem b[0..len) in place
  __device__ void run() {
    c = 0;
    lim = len;
    lb = 0;
    bra = 0;
    ket = len;
    if (exception1()) return;
    c = 0;
    if (3 > lim) return;  // "not hop 3": words shorter than 3 units are left alone
    prelude();
    c = 0;
    mark_regions();
    c = 0;
    lb = c;
    c = lim;
    {
      int v = lim - c;
      step1a();
      c = lim - v;
    }
    {
      int v = lim - c;
      bool ex2 = exception2();
      if (!ex2) {
        c = lim - v;
        int w;
        w = lim - c; step1b(); c = lim - w;
        w = lim - c; step1c(); c = lim - w;
        w = lim - c; step2(); c = lim - w;
        w = lim - c; step3(); c = lim - w;
        w = lim - c; step4(); c = lim - w;
        w = lim - c; step5(); c = lim - w;
      }
    }
    c = lb;
    postlude();
  }
};

using Stemmer = StemmerT<kStemCap>;

}  // namespace sme
