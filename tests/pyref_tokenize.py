"""An independent Python restatement of GalagoTokenizer.processContent -- TagTokenizer,
the Terrier stopword filter and the 2010 generated Porter2 stemmer -- written from
the Java sources, NOT from the C oracle, so that a misreading shared by the oracle
(oracle/oracle_tok.c, oracle/oracle_stem.c) and the device (sme_text.hpp,
sme_stem.hpp) would show up as a disagreement (VERDICT r2 missing #2).  Test
infrastructure only: nothing in the product imports it.

Sources restated (C/ = ABDURRAHMAN-PA2-3-code/src/ of the reference):
  C/org/galagosearch/core/parse/TagTokenizer.java:73-95 (buildSplits),
      155-202 (skipComment, skipProcessingInstruction, parseEndTag),
      221-393 (attribute scanners, parseBeginTag), 399-600 (onSplit, addToken,
      tokenComplexFix, tokenAcronymProcessing, tokenSimpleFix, checkTokenStatus),
      602-620 (onStartBracket), 644-662 (onAmpersand), 671-709 (tokenize)
  C/org/galagosearch/core/parse/Utility.java:141-147 (makeBytes: String.getBytes("UTF-8"))
  C/ivory/tokenize/GalagoTokenizer.java:35-125 (stopwords), 139-183 (processContent)
  C/org/tartarus/snowball/SnowballProgram.java (the cursor machine, find_among[_b],
      replace_s / slice_from / insert), C/org/tartarus/snowball/ext/englishStemmer.java
      (tables 18-165, routines 178-1317)

Strings are lists of UTF-16 code units (ints), as Java's String / StringBuffer.
JDK behaviour the sources rely on (parity unpinned) is taken
from Python: Character.isSpaceChar = Unicode categories Zs/Zl/Zp,
String.toLowerCase = str.lower(), Text.toString = UTF-8 decode with U+FFFD
replacement.  Tag bookkeeping (openTags / closedTags) is left out: it never
changes the token stream.
"""
import unicodedata

from pyref_stopwords import TERRIER_STOP_WORDS

STOPWORDS = frozenset(TERRIER_STOP_WORDS)
MIN_INT = -(1 << 31)


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def units(s):
    """Python str -> UTF-16 code units."""
    b = s.encode("utf-16-le", "surrogatepass")
    return [b[i] | (b[i + 1] << 8) for i in range(0, len(b), 2)]


def ustr(u):
    """UTF-16 code units -> Python str (lone surrogates kept)."""
    return b"".join(x.to_bytes(2, "little") for x in u).decode("utf-16-le", "surrogatepass")


def decode_record(raw):
    """Hadoop Text.toString of the record bytes: UTF-8 with replacement."""
    return units(raw.decode("utf-8", "replace"))


def _is_space_char(c):
    return unicodedata.category(chr(c)) in ("Zs", "Zl", "Zp")


def _to_lower(u):
    return units(ustr(u).lower())


def _utf8_len(u):
    """String.getBytes("UTF-8") length: pairs 4 bytes, an unpaired surrogate '?'."""
    n, i = 0, 0
    while i < len(u):
        c = u[i]
        if 0xD800 <= c <= 0xDBFF and i + 1 < len(u) and 0xDC00 <= u[i + 1] <= 0xDFFF:
            n += 4
            i += 2
            continue
        n += 1 if c < 0x80 else 2 if c < 0x800 else 1 if 0xD800 <= c <= 0xDFFF else 3
        i += 1
    return n


_SPLITS = [False] * 257
for _c in " \t\n\r;\"&/:!#?$%()@^*+-,=><[]{}|`~_":
    _SPLITS[ord(_c)] = True
for _c in range(33):
    _SPLITS[_c] = True
_IGNORED = (units("style"), units("script"))
_LT, _GT, _SL, _BANG, _Q, _AMP, _SEMI, _EQ, _DQ, _SQ, _BS, _DOT, _APOS = (ord(c) for c in "<>/!?&;=\"'\\.'")
_CLEAN, _SIMPLE, _COMPLEX, _ACRONYM = range(4)


class TagTokenizer:
    """TagTokenizer.tokenize(String) -> the token strings (TagTokenizer.java:671-709)."""

    def __init__(self, text):
        self.text = text
        self.n = len(text)
        self.position = 0
        self.last_split = -1
        self.ignore_until = None
        self.tokens = []

    # --- java.lang.String helpers over code units
    def _index_of(self, pat, frm):
        frm = max(frm, 0)
        t, m = self.text, len(pat)
        for i in range(frm, self.n - m + 1):
            if t[i:i + m] == pat:
                return i
        return -1

    def _index_of_non_space(self, start):
        if start < 0:
            return MIN_INT
        for i in range(start, self.n):
            if not _is_space_char(self.text[i]):
                return i
        return MIN_INT

    def _index_of_end_attribute(self, start, tag_end):
        if start < 0:
            return MIN_INT
        in_quote, last_escape = False, False
        for i in range(start, tag_end + 1):
            c = self.text[i]
            if (c == _DQ or c == _SQ) and not last_escape:
                in_quote = not in_quote
                if not in_quote:
                    return i
            elif not in_quote and (_is_space_char(c) or c == _GT):
                return i
            elif c == _BS and not last_escape:
                last_escape = True
            else:
                last_escape = False
        return MIN_INT

    def _index_of_equals(self, start, end):
        if start < 0:
            return MIN_INT
        for i in range(start, end):
            if self.text[i] == _EQ:
                return i
        return MIN_INT

    # --- markup
    def _skip_comment(self):
        if self.text[self.position:self.position + 4] == units("<!--"):
            self.position = self._index_of(units("-->"), self.position + 1)
            if self.position >= 0:
                self.position += 2
        else:
            self.position = self._index_of([_GT], self.position + 1)
        if self.position < 0:
            self.position = self.n

    def _skip_processing_instruction(self):
        self.position = self._index_of(units("?>"), self.position + 1)
        if self.position < 0:
            self.position = self.n

    def _parse_end_tag(self):
        t = self.text
        i = self.position + 2
        while i < self.n and not (_is_space_char(t[i]) or t[i] == _GT):
            i += 1
        name = _to_lower(t[self.position + 2:i])
        if self.ignore_until is not None and self.ignore_until == name:
            self.ignore_until = None
        while i < self.n and t[i] != _GT:
            i += 1
        self.position = i

    def _parse_begin_tag(self):
        t, n = self.text, self.n
        i = self.position + 1
        while i < n and not (_is_space_char(t[i]) or t[i] == _GT):
            i += 1
        name = _to_lower(t[self.position + 1:i])
        i = self._index_of_non_space(i)
        tag_end = self._index_of([_GT], _i32(i + 1))
        close_it = False
        while i < tag_end and i >= 0 and tag_end >= 0:
            start = self._index_of_non_space(i)
            if start > 0:
                if t[start] == _GT:
                    i = start
                    break
                elif t[start] == _SL and n > start + 1 and t[start + 1] == _GT:
                    i = start + 1
                    close_it = True
                    break
            end = self._index_of_end_attribute(start, tag_end)
            equals = self._index_of_equals(start, end)
            if equals < 0 or equals == start or end == equals:
                if end < 0:
                    i = tag_end
                    break
                i = end
                continue
            start_key, end_key, start_value, end_value = start, equals, equals + 1, end
            if t[start_value] == _DQ or t[start_value] == _SQ:
                start_value += 1
            if start_value >= end_value or start_key >= end_key:
                i = end
                continue
            if end >= n:  # endParsing(); break -- position is then overwritten with i below
                self.position = n
                break
            if t[end] == _DQ or t[end] == _SQ:
                end += 1
            i = end
        if name not in _IGNORED:
            pass  # BeginTag bookkeeping only
        elif not close_it:
            self.ignore_until = name
        self.position = i

    def _on_start_bracket(self):
        if self.position + 1 < self.n:
            c = self.text[self.position + 1]
            if c == _SL:
                self._parse_end_tag()
            elif c == _BANG:
                self._skip_comment()
            elif c == _Q:
                self._skip_processing_instruction()
            else:
                self._parse_begin_tag()
        else:
            self.position = self.n
        self.last_split = self.position

    def _on_ampersand(self):
        self._on_split()
        for i in range(self.position + 1, self.n):
            c = self.text[i]
            if 97 <= c <= 122 or 48 <= c <= 57 or c == ord("#"):
                continue
            if c == _SEMI:
                self.position = i
                self.last_split = i
                return
            break

    # --- tokens
    @staticmethod
    def _status(tok):
        st = _CLEAN
        for c in tok:
            if 97 <= c <= 122 or 48 <= c <= 57:
                continue
            if (65 <= c <= 90 or c == _APOS) and st == _CLEAN:
                st = _SIMPLE
            elif c != _DOT:
                st = _COMPLEX
            else:
                st = _ACRONYM
                break
        return st

    @staticmethod
    def _simple_fix(tok):
        return [c + 32 if 65 <= c <= 90 else c for c in tok if c != _APOS]

    def _complex_fix(self, tok):
        return _to_lower(self._simple_fix(tok))

    def _add_token(self, tok):
        if len(tok) <= 0:
            return
        if len(tok) > 100 // 6 and _utf8_len(tok) >= 100:
            return
        self.tokens.append(tok)

    def _acronym(self, tok):
        tok = self._complex_fix(tok)
        while tok[:1] == [_DOT]:
            tok = tok[1:]
        while tok[-1:] == [_DOT]:
            tok = tok[:-1]
        if _DOT in tok:
            is_acronym = len(tok) > 0
            for p in range(1, len(tok), 2):
                if tok[p] != _DOT:
                    is_acronym = False
            if is_acronym:
                self._add_token([c for c in tok if c != _DOT])
            else:
                s = 0
                for e in range(len(tok)):
                    if tok[e] == _DOT:
                        if e - s > 1:
                            self._add_token(tok[s:e])
                        s = e + 1
                if len(tok) - s > 1:
                    self._add_token(tok[s:])
        else:
            self._add_token(tok)

    def _on_split(self):
        if _i32(self.position - self.last_split) > 1:
            start = self.last_split + 1
            tok = self.text[start:self.position]
            st = self._status(tok)
            if st == _SIMPLE:
                tok = self._simple_fix(tok)
            elif st == _COMPLEX:
                tok = self._complex_fix(tok)
            elif st == _ACRONYM:
                self._acronym(tok)
            if st != _ACRONYM:
                self._add_token(tok)
        self.last_split = self.position

    def tokenize(self):
        t = self.text
        while 0 <= self.position < self.n:
            c = t[self.position]
            if c == _LT:
                if self.ignore_until is None:
                    self._on_split()
                self._on_start_bracket()
            elif self.ignore_until is not None:
                pass
            elif c == _AMP:
                self._on_ampersand()
            elif c < 256 and _SPLITS[c]:
                self._on_split()
            self.position += 1
        if self.ignore_until is None:
            self._on_split()
        return self.tokens


# ---------------------------------------------------------------------------
# Porter2 (the 2010 generated englishStemmer + SnowballProgram)
# ---------------------------------------------------------------------------
def _among(rows):
    return [(units(s), si, r) for s, si, r in rows]


A_0 = _among([("arsen", -1, -1), ("commun", -1, -1), ("gener", -1, -1)])
A_1 = _among([("'", -1, 1), ("'s'", 0, 1), ("'s", -1, 1)])
A_2 = _among([("ied", -1, 2), ("s", -1, 3), ("ies", 1, 2), ("sses", 1, 1), ("ss", 1, -1), ("us", 1, -1)])
A_3 = _among([("", -1, 3), ("bb", 0, 2), ("dd", 0, 2), ("ff", 0, 2), ("gg", 0, 2), ("bl", 0, 1), ("mm", 0, 2),
              ("nn", 0, 2), ("pp", 0, 2), ("rr", 0, 2), ("at", 0, 1), ("tt", 0, 2), ("iz", 0, 1)])
A_4 = _among([("ed", -1, 2), ("eed", 0, 1), ("ing", -1, 2), ("edly", -1, 2), ("eedly", 3, 1), ("ingly", -1, 2)])
A_5 = _among([("anci", -1, 3), ("enci", -1, 2), ("ogi", -1, 13), ("li", -1, 16), ("bli", 3, 12), ("abli", 4, 4),
              ("alli", 3, 8), ("fulli", 3, 14), ("lessli", 3, 15), ("ousli", 3, 10), ("entli", 3, 5),
              ("aliti", -1, 8), ("biliti", -1, 12), ("iviti", -1, 11), ("tional", -1, 1), ("ational", 14, 7),
              ("alism", -1, 8), ("ation", -1, 7), ("ization", 17, 6), ("izer", -1, 6), ("ator", -1, 7),
              ("iveness", -1, 11), ("fulness", -1, 9), ("ousness", -1, 10)])
A_6 = _among([("icate", -1, 4), ("ative", -1, 6), ("alize", -1, 3), ("iciti", -1, 4), ("ical", -1, 4),
              ("tional", -1, 1), ("ational", 5, 2), ("ful", -1, 5), ("ness", -1, 5)])
A_7 = _among([("ic", -1, 1), ("ance", -1, 1), ("ence", -1, 1), ("able", -1, 1), ("ible", -1, 1), ("ate", -1, 1),
              ("ive", -1, 1), ("ize", -1, 1), ("iti", -1, 1), ("al", -1, 1), ("ism", -1, 1), ("ion", -1, 2),
              ("er", -1, 1), ("ous", -1, 1), ("ant", -1, 1), ("ent", -1, 1), ("ment", 15, 1), ("ement", 16, 1)])
A_8 = _among([("e", -1, 1), ("l", -1, 2)])
A_9 = _among([("succeed", -1, -1), ("proceed", -1, -1), ("exceed", -1, -1), ("canning", -1, -1),
              ("inning", -1, -1), ("earring", -1, -1), ("herring", -1, -1), ("outing", -1, -1)])
A_10 = _among([("andes", -1, -1), ("atlas", -1, -1), ("bias", -1, -1), ("cosmos", -1, -1), ("dying", -1, 3),
               ("early", -1, 9), ("gently", -1, 7), ("howe", -1, -1), ("idly", -1, 6), ("lying", -1, 4),
               ("news", -1, -1), ("only", -1, 10), ("singly", -1, 11), ("skies", -1, 2), ("skis", -1, 1),
               ("sky", -1, -1), ("tying", -1, 5), ("ugly", -1, 8)])
G_V = [17, 65, 16, 1]
G_V_WXY = [1, 17, 65, 208, 1]
G_VALID_LI = [55, 141, 2]


class EnglishStemmer:
    def stem(self, word):
        """englishStemmer.setCurrent(word); stem(); getCurrent() -- word as code units."""
        self.cur = list(word)
        self.cursor, self.limit, self.limit_backward = 0, len(self.cur), 0
        self.bra, self.ket = 0, len(self.cur)
        self.y_found, self.p1, self.p2 = False, 0, 0
        self._stem()
        return self.cur

    # ---- SnowballProgram
    def in_grouping(self, s, mn, mx):
        if self.cursor >= self.limit:
            return False
        ch = self.cur[self.cursor]
        if ch > mx or ch < mn:
            return False
        ch -= mn
        if (s[ch >> 3] & (1 << (ch & 7))) == 0:
            return False
        self.cursor += 1
        return True

    def in_grouping_b(self, s, mn, mx):
        if self.cursor <= self.limit_backward:
            return False
        ch = self.cur[self.cursor - 1]
        if ch > mx or ch < mn:
            return False
        ch -= mn
        if (s[ch >> 3] & (1 << (ch & 7))) == 0:
            return False
        self.cursor -= 1
        return True

    def out_grouping(self, s, mn, mx):
        if self.cursor >= self.limit:
            return False
        ch = self.cur[self.cursor]
        if ch > mx or ch < mn or (s[(ch - mn) >> 3] & (1 << ((ch - mn) & 7))) == 0:
            self.cursor += 1
            return True
        return False

    def out_grouping_b(self, s, mn, mx):
        if self.cursor <= self.limit_backward:
            return False
        ch = self.cur[self.cursor - 1]
        if ch > mx or ch < mn or (s[(ch - mn) >> 3] & (1 << ((ch - mn) & 7))) == 0:
            self.cursor -= 1
            return True
        return False

    def eq_s(self, s):
        s = units(s)
        if self.limit - self.cursor < len(s):
            return False
        if self.cur[self.cursor:self.cursor + len(s)] != s:
            return False
        self.cursor += len(s)
        return True

    def eq_s_b(self, s):
        s = units(s)
        if self.cursor - self.limit_backward < len(s):
            return False
        if self.cur[self.cursor - len(s):self.cursor] != s:
            return False
        self.cursor -= len(s)
        return True

    def find_among(self, v):
        i, j, c, l = 0, len(v), self.cursor, self.limit
        common_i = common_j = 0
        first_key_inspected = False
        while True:
            k = i + ((j - i) >> 1)
            diff = 0
            common = min(common_i, common_j)
            w = v[k][0]
            for i2 in range(common, len(w)):
                if c + common == l:
                    diff = -1
                    break
                diff = self.cur[c + common] - w[i2]
                if diff != 0:
                    break
                common += 1
            if diff < 0:
                j, common_j = k, common
            else:
                i, common_i = k, common
            if j - i <= 1:
                if i > 0 or j == i or first_key_inspected:
                    break
                first_key_inspected = True
        while True:
            w, si, res = v[i]
            if common_i >= len(w):
                self.cursor = c + len(w)
                return res
            i = si
            if i < 0:
                return 0

    def find_among_b(self, v):
        i, j, c, lb = 0, len(v), self.cursor, self.limit_backward
        common_i = common_j = 0
        first_key_inspected = False
        while True:
            k = i + ((j - i) >> 1)
            diff = 0
            common = min(common_i, common_j)
            w = v[k][0]
            for i2 in range(len(w) - 1 - common, -1, -1):
                if c - common == lb:
                    diff = -1
                    break
                diff = self.cur[c - 1 - common] - w[i2]
                if diff != 0:
                    break
                common += 1
            if diff < 0:
                j, common_j = k, common
            else:
                i, common_i = k, common
            if j - i <= 1:
                if i > 0 or j == i or first_key_inspected:
                    break
                first_key_inspected = True
        while True:
            w, si, res = v[i]
            if common_i >= len(w):
                self.cursor = c - len(w)
                return res
            i = si
            if i < 0:
                return 0

    def replace_s(self, c_bra, c_ket, s):
        s = units(s)
        adj = len(s) - (c_ket - c_bra)
        self.cur[c_bra:c_ket] = s
        self.limit += adj
        if self.cursor >= c_ket:
            self.cursor += adj
        elif self.cursor > c_bra:
            self.cursor = c_bra
        return adj

    def slice_from(self, s):
        self.replace_s(self.bra, self.ket, s)

    def slice_del(self):
        self.slice_from("")

    def insert(self, c_bra, c_ket, s):
        adj = self.replace_s(c_bra, c_ket, s)
        if c_bra <= self.bra:
            self.bra += adj
        if c_bra <= self.ket:
            self.ket += adj

    # ---- englishStemmer routines
    def r_prelude(self):
        self.y_found = False
        v1 = self.cursor
        self.bra = self.cursor
        if self.eq_s("'"):
            self.ket = self.cursor
            self.slice_del()
        self.cursor = v1
        v2 = self.cursor
        self.bra = self.cursor
        if self.eq_s("y"):
            self.ket = self.cursor
            self.slice_from("Y")
            self.y_found = True
        self.cursor = v2
        v3 = self.cursor
        while True:  # repeat (goto (v [ 'y' ]) <- 'Y')
            v4 = self.cursor
            found = False
            while True:
                v5 = self.cursor
                if self.in_grouping(G_V, 97, 121):
                    self.bra = self.cursor
                    if self.eq_s("y"):
                        self.ket = self.cursor
                        self.cursor = v5
                        found = True
                        break
                self.cursor = v5
                if self.cursor >= self.limit:
                    break
                self.cursor += 1
            if not found:
                self.cursor = v4
                break
            self.slice_from("Y")
            self.y_found = True
        self.cursor = v3
        return True

    def _gopast_v(self):
        while not self.in_grouping(G_V, 97, 121):
            if self.cursor >= self.limit:
                return False
            self.cursor += 1
        return True

    def _gopast_nonv(self):
        while not self.out_grouping(G_V, 97, 121):
            if self.cursor >= self.limit:
                return False
            self.cursor += 1
        return True

    def r_mark_regions(self):
        self.p1 = self.limit
        self.p2 = self.limit
        v1 = self.cursor
        ok = True
        v2 = self.cursor
        if self.find_among(A_0) == 0:
            self.cursor = v2
            ok = self._gopast_v() and self._gopast_nonv()
        if ok:
            self.p1 = self.cursor
            if self._gopast_v() and self._gopast_nonv():
                self.p2 = self.cursor
        self.cursor = v1
        return True

    def r_shortv(self):
        v1 = self.limit - self.cursor
        if (self.out_grouping_b(G_V_WXY, 89, 121) and self.in_grouping_b(G_V, 97, 121)
                and self.out_grouping_b(G_V, 97, 121)):
            return True
        self.cursor = self.limit - v1
        if not self.out_grouping_b(G_V, 97, 121):
            return False
        if not self.in_grouping_b(G_V, 97, 121):
            return False
        if self.cursor > self.limit_backward:
            return False
        return True

    def r_R1(self):
        return self.p1 <= self.cursor

    def r_R2(self):
        return self.p2 <= self.cursor

    def r_step_1a(self):
        v1 = self.limit - self.cursor
        self.ket = self.cursor
        av = self.find_among_b(A_1)
        if av == 0:
            self.cursor = self.limit - v1
        else:
            self.bra = self.cursor
            if av == 1:
                self.slice_del()
        self.ket = self.cursor
        av = self.find_among_b(A_2)
        if av == 0:
            return False
        self.bra = self.cursor
        if av == 1:
            self.slice_from("ss")
        elif av == 2:
            v2 = self.limit - self.cursor
            c = self.cursor - 2
            if not (self.limit_backward > c or c > self.limit):
                self.cursor = c
                self.slice_from("i")
            else:
                self.cursor = self.limit - v2
                self.slice_from("ie")
        elif av == 3:
            if self.cursor <= self.limit_backward:
                return False
            self.cursor -= 1
            while not self.in_grouping_b(G_V, 97, 121):
                if self.cursor <= self.limit_backward:
                    return False
                self.cursor -= 1
            self.slice_del()
        return True

    def r_step_1b(self):
        self.ket = self.cursor
        av = self.find_among_b(A_4)
        if av == 0:
            return False
        self.bra = self.cursor
        if av == 1:
            if not self.r_R1():
                return False
            self.slice_from("ee")
        elif av == 2:
            v1 = self.limit - self.cursor
            while not self.in_grouping_b(G_V, 97, 121):
                if self.cursor <= self.limit_backward:
                    return False
                self.cursor -= 1
            self.cursor = self.limit - v1
            self.slice_del()
            v3 = self.limit - self.cursor
            av = self.find_among_b(A_3)
            if av == 0:
                return False
            self.cursor = self.limit - v3
            if av == 1:
                c = self.cursor
                self.insert(self.cursor, self.cursor, "e")
                self.cursor = c
            elif av == 2:
                self.ket = self.cursor
                if self.cursor <= self.limit_backward:
                    return False
                self.cursor -= 1
                self.bra = self.cursor
                self.slice_del()
            elif av == 3:
                if self.cursor != self.p1:
                    return False
                v4 = self.limit - self.cursor
                if not self.r_shortv():
                    return False
                self.cursor = self.limit - v4
                c = self.cursor
                self.insert(self.cursor, self.cursor, "e")
                self.cursor = c
        return True

    def r_step_1c(self):
        self.ket = self.cursor
        v1 = self.limit - self.cursor
        if not self.eq_s_b("y"):
            self.cursor = self.limit - v1
            if not self.eq_s_b("Y"):
                return False
        self.bra = self.cursor
        if not self.out_grouping_b(G_V, 97, 121):
            return False
        v2 = self.limit - self.cursor
        if not self.cursor > self.limit_backward:  # not atlimit
            return False
        self.cursor = self.limit - v2
        self.slice_from("i")
        return True

    _STEP2 = {1: "tion", 2: "ence", 3: "ance", 4: "able", 5: "ent", 6: "ize", 7: "ate", 8: "al", 9: "ful",
              10: "ous", 11: "ive", 12: "ble", 14: "ful", 15: "less"}

    def r_step_2(self):
        self.ket = self.cursor
        av = self.find_among_b(A_5)
        if av == 0:
            return False
        self.bra = self.cursor
        if not self.r_R1():
            return False
        if av in self._STEP2:
            self.slice_from(self._STEP2[av])
        elif av == 13:
            if not self.eq_s_b("l"):
                return False
            self.slice_from("og")
        elif av == 16:
            if not self.in_grouping_b(G_VALID_LI, 99, 116):
                return False
            self.slice_del()
        return True

    def r_step_3(self):
        self.ket = self.cursor
        av = self.find_among_b(A_6)
        if av == 0:
            return False
        self.bra = self.cursor
        if not self.r_R1():
            return False
        if av in (1, 2, 3, 4):
            self.slice_from({1: "tion", 2: "ate", 3: "al", 4: "ic"}[av])
        elif av == 5:
            self.slice_del()
        elif av == 6:
            if not self.r_R2():
                return False
            self.slice_del()
        return True

    def r_step_4(self):
        self.ket = self.cursor
        av = self.find_among_b(A_7)
        if av == 0:
            return False
        self.bra = self.cursor
        if not self.r_R2():
            return False
        if av == 1:
            self.slice_del()
        elif av == 2:
            v1 = self.limit - self.cursor
            if not self.eq_s_b("s"):
                self.cursor = self.limit - v1
                if not self.eq_s_b("t"):
                    return False
            self.slice_del()
        return True

    def r_step_5(self):
        self.ket = self.cursor
        av = self.find_among_b(A_8)
        if av == 0:
            return False
        self.bra = self.cursor
        if av == 1:
            v1 = self.limit - self.cursor
            if not self.r_R2():
                self.cursor = self.limit - v1
                if not self.r_R1():
                    return False
                v2 = self.limit - self.cursor
                if self.r_shortv():
                    return False
                self.cursor = self.limit - v2
            self.slice_del()
        elif av == 2:
            if not self.r_R2():
                return False
            if not self.eq_s_b("l"):
                return False
            self.slice_del()
        return True

    def r_exception2(self):
        self.ket = self.cursor
        if self.find_among_b(A_9) == 0:
            return False
        self.bra = self.cursor
        if self.cursor > self.limit_backward:
            return False
        return True

    _EXC1 = {1: "ski", 2: "sky", 3: "die", 4: "lie", 5: "tie", 6: "idl", 7: "gentl", 8: "ugli", 9: "earli",
             10: "onli", 11: "singl"}

    def r_exception1(self):
        self.bra = self.cursor
        av = self.find_among(A_10)
        if av == 0:
            return False
        self.ket = self.cursor
        if self.cursor < self.limit:
            return False
        if av in self._EXC1:
            self.slice_from(self._EXC1[av])
        return True

    def r_postlude(self):
        if not self.y_found:
            return False
        while True:
            v1 = self.cursor
            found = False
            while True:
                v2 = self.cursor
                self.bra = self.cursor
                if self.eq_s("Y"):
                    self.ket = self.cursor
                    self.cursor = v2
                    found = True
                    break
                self.cursor = v2
                if self.cursor >= self.limit:
                    break
                self.cursor += 1
            if not found:
                self.cursor = v1
                break
            self.slice_from("y")
        return True

    def _stem(self):
        v1 = self.cursor
        if self.r_exception1():
            return True
        self.cursor = v1
        c = self.cursor + 3  # hop 3: words shorter than 3 are left as they are
        if 0 > c or c > self.limit:
            return True
        self.cursor = v1
        v3 = self.cursor
        self.r_prelude()
        self.cursor = v3
        v4 = self.cursor
        self.r_mark_regions()
        self.cursor = v4
        self.limit_backward = self.cursor
        self.cursor = self.limit
        v5 = self.limit - self.cursor
        self.r_step_1a()
        self.cursor = self.limit - v5
        v6 = self.limit - self.cursor
        if not self.r_exception2():
            self.cursor = self.limit - v6
            for step in (self.r_step_1b, self.r_step_1c, self.r_step_2, self.r_step_3, self.r_step_4,
                         self.r_step_5):
                v = self.limit - self.cursor
                step()
                self.cursor = self.limit - v
        self.cursor = self.limit_backward
        v13 = self.cursor
        self.r_postlude()
        self.cursor = v13
        return True


_STEMMER = EnglishStemmer()


def stem(word):
    """englishStemmer on one word (str) -> str."""
    return ustr(_STEMMER.stem(units(word)))


def tag_tokenize(text):
    """TagTokenizer.tokenize: str or record bytes -> raw normalized tokens (str)."""
    u = decode_record(text) if isinstance(text, (bytes, bytearray)) else units(text)
    return [ustr(t) for t in TagTokenizer(u).tokenize()]


def process_content(text):
    """GalagoTokenizer.processContent: tokenize, drop stopwords (exact match,
    before stemming), stem every remaining token (the per-instance cache only
    memoizes the same function)."""
    u = decode_record(text) if isinstance(text, (bytes, bytearray)) else units(text)
    out = []
    for tok in TagTokenizer(u).tokenize():
        s = ustr(tok)
        if s in STOPWORDS:
            continue
        out.append(ustr(_STEMMER.stem(tok)))
    return out
