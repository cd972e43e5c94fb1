/*
 * oracle_stem.c -- restatement of the generated Snowball English (Porter2,
 * ~2010 tables) stemmer and its runtime.  TEST INFRASTRUCTURE ONLY (see
 * oracle.h).
 *
 * Follows, routine by routine:
 *   C/org/tartarus/snowball/ext/englishStemmer.java
 *     tables 18-165, r_prelude 178, r_mark_regions 275, r_shortv 372,
 *     r_R1 413, r_R2 421, r_Step_1a 429, r_Step_1b 534, r_Step_1c 650,
 *     r_Step_2 698, r_Step_3 812, r_Step_4 872, r_Step_5 926,
 *     r_exception2 1000, r_exception1 1019, r_postlude 1099, stem 1149-1317
 *   C/org/tartarus/snowball/SnowballProgram.java
 *     setCurrent 15, in_grouping 60, in_grouping_b 71, out_grouping 82,
 *     out_grouping_b 98, eq_s 150, eq_s_b 161, find_among 181,
 *     find_among_b 254, replace_s 325, slice_from 352, slice_del 363,
 *     insert 368
 * (C/ = /root/reference/ABDURRAHMAN-PA2-3-code/src/, U+2010 hyphens.)
 * No Among entry names a method ("" everywhere), so the reflective call in
 * find_among is never taken.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  const char *s;
  int substring_i;
  int result;
  int n; /* strlen(s) */
} among;
#define AM(str, sub, res) \
  { str, sub, res, (int)sizeof(str) - 1 }

static const among a_0[] = {AM("arsen", -1, -1), AM("commun", -1, -1), AM("gener", -1, -1)};
static const among a_1[] = {AM("'", -1, 1), AM("'s'", 0, 1), AM("'s", -1, 1)};
static const among a_2[] = {AM("ied", -1, 2), AM("s", -1, 3),   AM("ies", 1, 2),
                            AM("sses", 1, 1), AM("ss", 1, -1), AM("us", 1, -1)};
static const among a_3[] = {AM("", -1, 3),  AM("bb", 0, 2), AM("dd", 0, 2), AM("ff", 0, 2), AM("gg", 0, 2),
                            AM("bl", 0, 1), AM("mm", 0, 2), AM("nn", 0, 2), AM("pp", 0, 2), AM("rr", 0, 2),
                            AM("at", 0, 1), AM("tt", 0, 2), AM("iz", 0, 1)};
static const among a_4[] = {AM("ed", -1, 2),   AM("eed", 0, 1),   AM("ing", -1, 2),
                            AM("edly", -1, 2), AM("eedly", 3, 1), AM("ingly", -1, 2)};
static const among a_5[] = {
    AM("anci", -1, 3),    AM("enci", -1, 2),   AM("ogi", -1, 13),     AM("li", -1, 16),
    AM("bli", 3, 12),     AM("abli", 4, 4),    AM("alli", 3, 8),      AM("fulli", 3, 14),
    AM("lessli", 3, 15),  AM("ousli", 3, 10),  AM("entli", 3, 5),     AM("aliti", -1, 8),
    AM("biliti", -1, 12), AM("iviti", -1, 11), AM("tional", -1, 1),   AM("ational", 14, 7),
    AM("alism", -1, 8),   AM("ation", -1, 7),  AM("ization", 17, 6),  AM("izer", -1, 6),
    AM("ator", -1, 7),    AM("iveness", -1, 11), AM("fulness", -1, 9), AM("ousness", -1, 10)};
static const among a_6[] = {AM("icate", -1, 4), AM("ative", -1, 6),   AM("alize", -1, 3),
                            AM("iciti", -1, 4), AM("ical", -1, 4),    AM("tional", -1, 1),
                            AM("ational", 5, 2), AM("ful", -1, 5),    AM("ness", -1, 5)};
static const among a_7[] = {AM("ic", -1, 1),   AM("ance", -1, 1), AM("ence", -1, 1), AM("able", -1, 1),
                            AM("ible", -1, 1), AM("ate", -1, 1),  AM("ive", -1, 1),  AM("ize", -1, 1),
                            AM("iti", -1, 1),  AM("al", -1, 1),   AM("ism", -1, 1),  AM("ion", -1, 2),
                            AM("er", -1, 1),   AM("ous", -1, 1),  AM("ant", -1, 1),  AM("ent", -1, 1),
                            AM("ment", 15, 1), AM("ement", 16, 1)};
static const among a_8[] = {AM("e", -1, 1), AM("l", -1, 2)};
static const among a_9[] = {AM("succeed", -1, -1), AM("proceed", -1, -1), AM("exceed", -1, -1),
                            AM("canning", -1, -1), AM("inning", -1, -1),  AM("earring", -1, -1),
                            AM("herring", -1, -1), AM("outing", -1, -1)};
static const among a_10[] = {AM("andes", -1, -1), AM("atlas", -1, -1), AM("bias", -1, -1),
                             AM("cosmos", -1, -1), AM("dying", -1, 3), AM("early", -1, 9),
                             AM("gently", -1, 7), AM("howe", -1, -1), AM("idly", -1, 6),
                             AM("lying", -1, 4),  AM("news", -1, -1), AM("only", -1, 10),
                             AM("singly", -1, 11), AM("skies", -1, 2), AM("skis", -1, 1),
                             AM("sky", -1, -1),   AM("tying", -1, 5), AM("ugly", -1, 8)};

static const unsigned char g_v[] = {17, 65, 16, 1};
static const unsigned char g_v_WXY[] = {1, 17, 65, 208, 1};
static const unsigned char g_valid_LI[] = {55, 141, 2};

typedef struct {
  jstr cur;
  int cursor, limit, limit_backward, bra, ket;
  int B_Y_found, I_p1, I_p2;
} sn;

static int in_grouping(sn *z, const unsigned char *s, int min, int max) {
  if (z->cursor >= z->limit) return 0;
  int ch = z->cur.p[z->cursor];
  if (ch > max || ch < min) return 0;
  ch -= min;
  if ((s[ch >> 3] & (1 << (ch & 7))) == 0) return 0;
  z->cursor++;
  return 1;
}
static int in_grouping_b(sn *z, const unsigned char *s, int min, int max) {
  if (z->cursor <= z->limit_backward) return 0;
  int ch = z->cur.p[z->cursor - 1];
  if (ch > max || ch < min) return 0;
  ch -= min;
  if ((s[ch >> 3] & (1 << (ch & 7))) == 0) return 0;
  z->cursor--;
  return 1;
}
static int out_grouping(sn *z, const unsigned char *s, int min, int max) {
  if (z->cursor >= z->limit) return 0;
  int ch = z->cur.p[z->cursor];
  if (ch > max || ch < min) {
    z->cursor++;
    return 1;
  }
  ch -= min;
  if ((s[ch >> 3] & (1 << (ch & 7))) == 0) {
    z->cursor++;
    return 1;
  }
  return 0;
}
static int out_grouping_b(sn *z, const unsigned char *s, int min, int max) {
  if (z->cursor <= z->limit_backward) return 0;
  int ch = z->cur.p[z->cursor - 1];
  if (ch > max || ch < min) {
    z->cursor--;
    return 1;
  }
  ch -= min;
  if ((s[ch >> 3] & (1 << (ch & 7))) == 0) {
    z->cursor--;
    return 1;
  }
  return 0;
}
static int eq_s(sn *z, const char *s) {
  int n = (int)strlen(s);
  if (z->limit - z->cursor < n) return 0;
  for (int i = 0; i != n; i++)
    if (z->cur.p[z->cursor + i] != (unsigned char)s[i]) return 0;
  z->cursor += n;
  return 1;
}
static int eq_s_b(sn *z, const char *s) {
  int n = (int)strlen(s);
  if (z->cursor - z->limit_backward < n) return 0;
  for (int i = 0; i != n; i++)
    if (z->cur.p[z->cursor - n + i] != (unsigned char)s[i]) return 0;
  z->cursor -= n;
  return 1;
}

static int find_among(sn *z, const among *v, int v_size) {
  int i = 0, j = v_size;
  int c = z->cursor, l = z->limit;
  int common_i = 0, common_j = 0;
  int first_key_inspected = 0;
  for (;;) {
    int k = i + ((j - i) >> 1);
    int diff = 0;
    int common = common_i < common_j ? common_i : common_j;
    const among *w = &v[k];
    int wn = w->n;
    for (int i2 = common; i2 < wn; i2++) {
      if (c + common == l) {
        diff = -1;
        break;
      }
      diff = (int)z->cur.p[c + common] - (int)(unsigned char)w->s[i2];
      if (diff != 0) break;
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
      if (i > 0) break;
      if (j == i) break;
      if (first_key_inspected) break;
      first_key_inspected = 1;
    }
  }
  for (;;) {
    const among *w = &v[i];
    int wn = w->n;
    if (common_i >= wn) {
      z->cursor = c + wn;
      return w->result;
    }
    i = w->substring_i;
    if (i < 0) return 0;
  }
}

static int find_among_b(sn *z, const among *v, int v_size) {
  int i = 0, j = v_size;
  int c = z->cursor, lb = z->limit_backward;
  int common_i = 0, common_j = 0;
  int first_key_inspected = 0;
  for (;;) {
    int k = i + ((j - i) >> 1);
    int diff = 0;
    int common = common_i < common_j ? common_i : common_j;
    const among *w = &v[k];
    int wn = w->n;
    for (int i2 = wn - 1 - common; i2 >= 0; i2--) {
      if (c - common == lb) {
        diff = -1;
        break;
      }
      diff = (int)z->cur.p[c - 1 - common] - (int)(unsigned char)w->s[i2];
      if (diff != 0) break;
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
      if (i > 0) break;
      if (j == i) break;
      if (first_key_inspected) break;
      first_key_inspected = 1;
    }
  }
  for (;;) {
    const among *w = &v[i];
    int wn = w->n;
    if (common_i >= wn) {
      z->cursor = c - wn;
      return w->result;
    }
    i = w->substring_i;
    if (i < 0) return 0;
  }
}

static int replace_s(sn *z, int c_bra, int c_ket, const char *s) {
  int sn_ = (int)strlen(s);
  int adjustment = sn_ - (c_ket - c_bra);
  int oldn = z->cur.n;
  int newn = oldn + adjustment;
  js_reserve(&z->cur, newn + 1);
  memmove(z->cur.p + c_bra + sn_, z->cur.p + c_ket, (size_t)(oldn - c_ket) * sizeof(uint16_t));
  for (int i = 0; i < sn_; i++) z->cur.p[c_bra + i] = (unsigned char)s[i];
  z->cur.n = newn;
  z->limit += adjustment;
  if (z->cursor >= c_ket)
    z->cursor += adjustment;
  else if (z->cursor > c_bra)
    z->cursor = c_bra;
  return adjustment;
}
static void slice_from(sn *z, const char *s) { replace_s(z, z->bra, z->ket, s); }
static void slice_del(sn *z) { slice_from(z, ""); }
static void insert_s(sn *z, int c_bra, int c_ket, const char *s) {
  int adjustment = replace_s(z, c_bra, c_ket, s);
  if (c_bra <= z->bra) z->bra += adjustment;
  if (c_bra <= z->ket) z->ket += adjustment;
}

static int r_prelude(sn *z) {
  int v_1, v_2, v_3, v_4, v_5;
  z->B_Y_found = 0;
  v_1 = z->cursor;
  do {
    z->bra = z->cursor;
    if (!eq_s(z, "'")) break;
    z->ket = z->cursor;
    slice_del(z);
  } while (0);
  z->cursor = v_1;
  v_2 = z->cursor;
  do {
    z->bra = z->cursor;
    if (!eq_s(z, "y")) break;
    z->ket = z->cursor;
    slice_from(z, "Y");
    z->B_Y_found = 1;
  } while (0);
  z->cursor = v_2;
  v_3 = z->cursor;
  for (;;) { /* replab3 */
    v_4 = z->cursor;
    int ok = 0;
    for (;;) { /* golab5 */
      v_5 = z->cursor;
      int found = 0;
      do {
        if (!in_grouping(z, g_v, 97, 121)) break;
        z->bra = z->cursor;
        if (!eq_s(z, "y")) break;
        z->ket = z->cursor;
        z->cursor = v_5;
        found = 1;
      } while (0);
      if (found) {
        ok = 1;
        break;
      }
      z->cursor = v_5;
      if (z->cursor >= z->limit) break;
      z->cursor++;
    }
    if (!ok) {
      z->cursor = v_4;
      break;
    }
    slice_from(z, "Y");
    z->B_Y_found = 1;
  }
  z->cursor = v_3;
  return 1;
}

/* gopast a grouping forward: returns 0 if hit limit (caller breaks lab0) */
static int gopast_in(sn *z) {
  for (;;) {
    if (in_grouping(z, g_v, 97, 121)) return 1;
    if (z->cursor >= z->limit) return 0;
    z->cursor++;
  }
}
static int gopast_out(sn *z) {
  for (;;) {
    if (out_grouping(z, g_v, 97, 121)) return 1;
    if (z->cursor >= z->limit) return 0;
    z->cursor++;
  }
}

static int r_mark_regions(sn *z) {
  int v_1, v_2;
  z->I_p1 = z->limit;
  z->I_p2 = z->limit;
  v_1 = z->cursor;
  do { /* lab0 */
    int lab1_done = 0;
    v_2 = z->cursor;
    if (find_among(z, a_0, 3) != 0) lab1_done = 1;
    if (!lab1_done) {
      z->cursor = v_2;
      if (!gopast_in(z)) break;
      if (!gopast_out(z)) break;
    }
    z->I_p1 = z->cursor;
    if (!gopast_in(z)) break;
    if (!gopast_out(z)) break;
    z->I_p2 = z->cursor;
  } while (0);
  z->cursor = v_1;
  return 1;
}

static int r_shortv(sn *z) {
  int v_1 = z->limit - z->cursor;
  do {
    if (!out_grouping_b(z, g_v_WXY, 89, 121)) break;
    if (!in_grouping_b(z, g_v, 97, 121)) break;
    if (!out_grouping_b(z, g_v, 97, 121)) break;
    return 1;
  } while (0);
  z->cursor = z->limit - v_1;
  if (!out_grouping_b(z, g_v, 97, 121)) return 0;
  if (!in_grouping_b(z, g_v, 97, 121)) return 0;
  if (z->cursor > z->limit_backward) return 0;
  return 1;
}
static int r_R1(sn *z) { return z->I_p1 <= z->cursor; }
static int r_R2(sn *z) { return z->I_p2 <= z->cursor; }

static int r_Step_1a(sn *z) {
  int among_var, v_1, v_2;
  v_1 = z->limit - z->cursor;
  do {
    z->ket = z->cursor;
    among_var = find_among_b(z, a_1, 3);
    if (among_var == 0) {
      z->cursor = z->limit - v_1;
      break;
    }
    z->bra = z->cursor;
    if (among_var == 1) slice_del(z);
  } while (0);
  z->ket = z->cursor;
  among_var = find_among_b(z, a_2, 6);
  if (among_var == 0) return 0;
  z->bra = z->cursor;
  switch (among_var) {
    case 1:
      slice_from(z, "ss");
      break;
    case 2:
      v_2 = z->limit - z->cursor;
      {
        int c = z->cursor - 2;
        if (z->limit_backward > c || c > z->limit) {
          z->cursor = z->limit - v_2;
          slice_from(z, "ie");
        } else {
          z->cursor = c;
          slice_from(z, "i");
        }
      }
      break;
    case 3:
      if (z->cursor <= z->limit_backward) return 0;
      z->cursor--;
      for (;;) {
        if (in_grouping_b(z, g_v, 97, 121)) break;
        if (z->cursor <= z->limit_backward) return 0;
        z->cursor--;
      }
      slice_del(z);
      break;
  }
  return 1;
}

static int r_Step_1b(sn *z) {
  int among_var, v_1, v_3, v_4;
  z->ket = z->cursor;
  among_var = find_among_b(z, a_4, 6);
  if (among_var == 0) return 0;
  z->bra = z->cursor;
  switch (among_var) {
    case 1:
      if (!r_R1(z)) return 0;
      slice_from(z, "ee");
      break;
    case 2:
      v_1 = z->limit - z->cursor;
      for (;;) {
        if (in_grouping_b(z, g_v, 97, 121)) break;
        if (z->cursor <= z->limit_backward) return 0;
        z->cursor--;
      }
      z->cursor = z->limit - v_1;
      slice_del(z);
      v_3 = z->limit - z->cursor;
      among_var = find_among_b(z, a_3, 13);
      if (among_var == 0) return 0;
      z->cursor = z->limit - v_3;
      switch (among_var) {
        case 1: {
          int c = z->cursor;
          insert_s(z, z->cursor, z->cursor, "e");
          z->cursor = c;
        } break;
        case 2:
          z->ket = z->cursor;
          if (z->cursor <= z->limit_backward) return 0;
          z->cursor--;
          z->bra = z->cursor;
          slice_del(z);
          break;
        case 3:
          if (z->cursor != z->I_p1) return 0;
          v_4 = z->limit - z->cursor;
          if (!r_shortv(z)) return 0;
          z->cursor = z->limit - v_4;
          {
            int c = z->cursor;
            insert_s(z, z->cursor, z->cursor, "e");
            z->cursor = c;
          }
          break;
      }
      break;
  }
  return 1;
}

static int r_Step_1c(sn *z) {
  int v_1, v_2;
  z->ket = z->cursor;
  v_1 = z->limit - z->cursor;
  if (!eq_s_b(z, "y")) {
    z->cursor = z->limit - v_1;
    if (!eq_s_b(z, "Y")) return 0;
  }
  z->bra = z->cursor;
  if (!out_grouping_b(z, g_v, 97, 121)) return 0;
  v_2 = z->limit - z->cursor;
  if (!(z->cursor > z->limit_backward)) return 0; /* not atlimit */
  z->cursor = z->limit - v_2;
  slice_from(z, "i");
  return 1;
}

static int r_Step_2(sn *z) {
  int among_var;
  z->ket = z->cursor;
  among_var = find_among_b(z, a_5, 24);
  if (among_var == 0) return 0;
  z->bra = z->cursor;
  if (!r_R1(z)) return 0;
  switch (among_var) {
    case 1: slice_from(z, "tion"); break;
    case 2: slice_from(z, "ence"); break;
    case 3: slice_from(z, "ance"); break;
    case 4: slice_from(z, "able"); break;
    case 5: slice_from(z, "ent"); break;
    case 6: slice_from(z, "ize"); break;
    case 7: slice_from(z, "ate"); break;
    case 8: slice_from(z, "al"); break;
    case 9: slice_from(z, "ful"); break;
    case 10: slice_from(z, "ous"); break;
    case 11: slice_from(z, "ive"); break;
    case 12: slice_from(z, "ble"); break;
    case 13:
      if (!eq_s_b(z, "l")) return 0;
      slice_from(z, "og");
      break;
    case 14: slice_from(z, "ful"); break;
    case 15: slice_from(z, "less"); break;
    case 16:
      if (!in_grouping_b(z, g_valid_LI, 99, 116)) return 0;
      slice_del(z);
      break;
  }
  return 1;
}

static int r_Step_3(sn *z) {
  int among_var;
  z->ket = z->cursor;
  among_var = find_among_b(z, a_6, 9);
  if (among_var == 0) return 0;
  z->bra = z->cursor;
  if (!r_R1(z)) return 0;
  switch (among_var) {
    case 1: slice_from(z, "tion"); break;
    case 2: slice_from(z, "ate"); break;
    case 3: slice_from(z, "al"); break;
    case 4: slice_from(z, "ic"); break;
    case 5: slice_del(z); break;
    case 6:
      if (!r_R2(z)) return 0;
      slice_del(z);
      break;
  }
  return 1;
}

static int r_Step_4(sn *z) {
  int among_var, v_1;
  z->ket = z->cursor;
  among_var = find_among_b(z, a_7, 18);
  if (among_var == 0) return 0;
  z->bra = z->cursor;
  if (!r_R2(z)) return 0;
  switch (among_var) {
    case 1: slice_del(z); break;
    case 2:
      v_1 = z->limit - z->cursor;
      if (!eq_s_b(z, "s")) {
        z->cursor = z->limit - v_1;
        if (!eq_s_b(z, "t")) return 0;
      }
      slice_del(z);
      break;
  }
  return 1;
}

static int r_Step_5(sn *z) {
  int among_var, v_1, v_2;
  z->ket = z->cursor;
  among_var = find_among_b(z, a_8, 2);
  if (among_var == 0) return 0;
  z->bra = z->cursor;
  switch (among_var) {
    case 1:
      v_1 = z->limit - z->cursor;
      if (!r_R2(z)) {
        z->cursor = z->limit - v_1;
        if (!r_R1(z)) return 0;
        v_2 = z->limit - z->cursor;
        if (r_shortv(z)) return 0;
        z->cursor = z->limit - v_2;
      }
      slice_del(z);
      break;
    case 2:
      if (!r_R2(z)) return 0;
      if (!eq_s_b(z, "l")) return 0;
      slice_del(z);
      break;
  }
  return 1;
}

static int r_exception2(sn *z) {
  z->ket = z->cursor;
  if (find_among_b(z, a_9, 8) == 0) return 0;
  z->bra = z->cursor;
  if (z->cursor > z->limit_backward) return 0;
  return 1;
}

static int r_exception1(sn *z) {
  int among_var;
  z->bra = z->cursor;
  among_var = find_among(z, a_10, 18);
  if (among_var == 0) return 0;
  z->ket = z->cursor;
  if (z->cursor < z->limit) return 0;
  switch (among_var) {
    case 1: slice_from(z, "ski"); break;
    case 2: slice_from(z, "sky"); break;
    case 3: slice_from(z, "die"); break;
    case 4: slice_from(z, "lie"); break;
    case 5: slice_from(z, "tie"); break;
    case 6: slice_from(z, "idl"); break;
    case 7: slice_from(z, "gentl"); break;
    case 8: slice_from(z, "ugli"); break;
    case 9: slice_from(z, "earli"); break;
    case 10: slice_from(z, "onli"); break;
    case 11: slice_from(z, "singl"); break;
  }
  return 1;
}

static int r_postlude(sn *z) {
  int v_1, v_2;
  if (!z->B_Y_found) return 0;
  for (;;) {
    v_1 = z->cursor;
    int ok = 0;
    for (;;) {
      v_2 = z->cursor;
      int found = 0;
      do {
        z->bra = z->cursor;
        if (!eq_s(z, "Y")) break;
        z->ket = z->cursor;
        z->cursor = v_2;
        found = 1;
      } while (0);
      if (found) {
        ok = 1;
        break;
      }
      z->cursor = v_2;
      if (z->cursor >= z->limit) break;
      z->cursor++;
    }
    if (!ok) {
      z->cursor = v_1;
      break;
    }
    slice_from(z, "y");
  }
  return 1;
}

static void stem(sn *z) {
  int v_1, v_3, v_4, v_5, v_6;
  /* or, line 207 */
  v_1 = z->cursor;
  if (r_exception1(z)) return;
  z->cursor = v_1;
  {
    /* not hop 3 => too short: leave unchanged */
    int c = z->cursor + 3;
    if (0 > c || c > z->limit) return;
  }
  z->cursor = v_1;
  v_3 = z->cursor;
  r_prelude(z);
  z->cursor = v_3;
  v_4 = z->cursor;
  r_mark_regions(z);
  z->cursor = v_4;
  z->limit_backward = z->cursor;
  z->cursor = z->limit;
  v_5 = z->limit - z->cursor;
  r_Step_1a(z);
  z->cursor = z->limit - v_5;
  v_6 = z->limit - z->cursor;
  if (!r_exception2(z)) {
    int v;
    z->cursor = z->limit - v_6;
    v = z->limit - z->cursor;
    r_Step_1b(z);
    z->cursor = z->limit - v;
    v = z->limit - z->cursor;
    r_Step_1c(z);
    z->cursor = z->limit - v;
    v = z->limit - z->cursor;
    r_Step_2(z);
    z->cursor = z->limit - v;
    v = z->limit - z->cursor;
    r_Step_3(z);
    z->cursor = z->limit - v;
    v = z->limit - z->cursor;
    r_Step_4(z);
    z->cursor = z->limit - v;
    v = z->limit - z->cursor;
    r_Step_5(z);
    z->cursor = z->limit - v;
  }
  z->cursor = z->limit_backward;
  {
    int v_13 = z->cursor;
    r_postlude(z);
    z->cursor = v_13;
  }
}

void or_stem_js(const uint16_t *w, int n, jstr *out) {
  sn z;
  memset(&z, 0, sizeof z);
  js_init(&z.cur);
  js_set(&z.cur, w, n);
  z.cursor = 0;
  z.limit = n;
  z.limit_backward = 0;
  z.bra = 0;
  z.ket = n;
  stem(&z);
  js_set(out, z.cur.p, z.cur.n);
  js_free(&z.cur);
}
