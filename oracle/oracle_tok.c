/*
 * oracle_tok.c -- restatement of the reference tokenizer chain:
 *   GalagoTokenizer.processContent   C/ivory/tokenize/GalagoTokenizer.java:139-183
 *     stopwords (Terrier list)        GalagoTokenizer.java:35-133, filter 152-156
 *     stem loop                       GalagoTokenizer.java:158-179 (cache is pure memoization)
 *   TagTokenizer                      C/org/galagosearch/core/parse/TagTokenizer.java
 *     buildSplits 73-95, skipComment 155-169, skipProcessingInstruction 171-177,
 *     parseEndTag 179-202, indexOfNonSpace 221-233, indexOfEndAttribute 235-261,
 *     indexOfEquals 277-289, parseBeginTag 291-393, onSplit 399-429,
 *     addToken 439-453, tokenComplexFix 455-460, tokenAcronymProcessing 479-527,
 *     tokenSimpleFix 536-559, checkTokenStatus 573-600, onStartBracket 602-620,
 *     onAmpersand 644-662, tokenize 671-709
 *   Utility.makeBytes                 C/org/galagosearch/core/parse/Utility.java:141-147
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Strings are UTF-16 like Java's.
 */
#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

void jl_init(jstr_list *l) {
  l->v = NULL;
  l->n = 0;
  l->cap = 0;
}
void jl_free(jstr_list *l) {
  for (int i = 0; i < l->n; i++) js_free(&l->v[i]);
  free(l->v);
  jl_init(l);
}
void jl_push(jstr_list *l, const uint16_t *p, int n) {
  if (l->n == l->cap) {
    l->cap = l->cap ? 2 * l->cap : 16;
    l->v = (jstr *)realloc(l->v, (size_t)l->cap * sizeof(jstr));
  }
  js_init(&l->v[l->n]);
  js_set(&l->v[l->n], p, n);
  l->n++;
}

/* Character.isSpaceChar: categories Zs, Zl, Zp (JDK 6/7 tables: U+180E is Zs). */
static int is_space_char(uint16_t c) {
  if (c == 0x20 || c == 0xA0 || c == 0x1680 || c == 0x180E) return 1;
  if (c >= 0x2000 && c <= 0x200A) return 1;
  return c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

/* buildSplits: 0..32 plus the listed punctuation. */
static int is_split(uint16_t c) {
  if (c >= 256) return 0;
  if (c <= 32) return 1;
  switch (c) {
    case ';': case '"': case '&': case '/': case ':': case '!': case '#':
    case '?': case '$': case '%': case '(': case ')': case '@': case '^':
    case '*': case '+': case '-': case ',': case '=': case '>': case '<':
    case '[': case ']': case '{': case '}': case '|': case '`': case '~':
    case '_':
      return 1;
  }
  return 0;
}

typedef struct {
  const uint16_t *text;
  int len;
  int position;
  int lastSplit;
  int ignoring;     /* ignoreUntil != null */
  jstr ignoreUntil; /* lowercased tag name */
  jstr_list *tokens;
} tt;

/* String.indexOf(String, fromIndex) */
static int index_of(const tt *t, const char *s, int from) {
  int sn = (int)strlen(s);
  if (from < 0) from = 0;
  if (from >= t->len) return sn == 0 ? t->len : -1;
  for (int i = from; i + sn <= t->len; i++) {
    int k = 0;
    while (k < sn && t->text[i + k] == (unsigned char)s[k]) k++;
    if (k == sn) return i;
  }
  return -1;
}

static void add_token(tt *t, const uint16_t *p, int n) {
  if (n <= 0) return;
  if (n > 100 / 6 && utf8_len_java(p, n) >= 100) return;
  jl_push(t->tokens, p, n);
}

static void simple_fix(const uint16_t *p, int n, jstr *out) {
  js_reserve(out, n + 1);
  int j = 0;
  for (int i = 0; i < n; i++) {
    uint16_t c = p[i];
    if (c >= 'A' && c <= 'Z')
      out->p[j] = (uint16_t)(c + 'a' - 'A');
    else if (c == '\'')
      j--;
    else
      out->p[j] = c;
    j++;
  }
  out->n = j;
}

static void complex_fix(const uint16_t *p, int n, jstr *out) {
  jstr tmp;
  js_init(&tmp);
  simple_fix(p, n, &tmp);
  out->n = 0;
  java_tolower(tmp.p, tmp.n, out);
  js_free(&tmp);
}

enum { CLEAN, SIMPLE, COMPLEX, ACRONYM };

static int check_status(const uint16_t *p, int n) {
  int status = CLEAN;
  for (int i = 0; i < n; i++) {
    uint16_t c = p[i];
    if ((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9')) continue;
    int up = (c >= 'A' && c <= 'Z');
    int per = (c == '.');
    int apo = (c == '\'');
    if ((up || apo) && status == CLEAN)
      status = SIMPLE;
    else if (!per)
      status = COMPLEX;
    else {
      status = ACRONYM;
      break;
    }
  }
  return status;
}

static void acronym(tt *t, const uint16_t *p, int n) {
  jstr tok;
  js_init(&tok);
  complex_fix(p, n, &tok);
  int b = 0, e = tok.n;
  while (b < e && tok.p[b] == '.') b++;
  while (e > b && tok.p[e - 1] == '.') e--;
  const uint16_t *s = tok.p + b;
  int sl = e - b;
  int has_dot = 0;
  for (int i = 0; i < sl; i++)
    if (s[i] == '.') has_dot = 1;
  if (has_dot) {
    int is_acr = sl > 0;
    for (int pos = 1; pos < sl; pos += 2)
      if (s[pos] != '.') is_acr = 0;
    if (is_acr) {
      jstr r;
      js_init(&r);
      for (int i = 0; i < sl; i++)
        if (s[i] != '.') js_push(&r, s[i]);
      add_token(t, r.p, r.n);
      js_free(&r);
    } else {
      int st = 0;
      for (int x = 0; x < sl; x++) {
        if (s[x] == '.') {
          if (x - st > 1) add_token(t, s + st, x - st);
          st = x + 1;
        }
      }
      if (sl - st > 1) add_token(t, s + st, sl - st);
    }
  } else {
    add_token(t, s, sl);
  }
  js_free(&tok);
}

static void on_split(tt *t) {
  if (t->position - t->lastSplit > 1) {
    int start = t->lastSplit + 1;
    const uint16_t *p = t->text + start;
    int n = t->position - start;
    int st = check_status(p, n);
    jstr tok;
    js_init(&tok);
    switch (st) {
      case SIMPLE:
        simple_fix(p, n, &tok);
        add_token(t, tok.p, tok.n);
        break;
      case COMPLEX:
        complex_fix(p, n, &tok);
        add_token(t, tok.p, tok.n);
        break;
      case ACRONYM:
        acronym(t, p, n);
        break;
      default:
        add_token(t, p, n);
        break;
    }
    js_free(&tok);
  }
  t->lastSplit = t->position;
}

static void end_parsing(tt *t) { t->position = t->len; }

static void skip_comment(tt *t) {
  int pos = t->position;
  int starts = (pos + 4 <= t->len && t->text[pos] == '<' && t->text[pos + 1] == '!' &&
                t->text[pos + 2] == '-' && t->text[pos + 3] == '-');
  if (starts) {
    t->position = index_of(t, "-->", pos + 1);
    if (t->position >= 0) t->position += 2;
  } else {
    t->position = index_of(t, ">", pos + 1);
  }
  if (t->position < 0) t->position = t->len;
}

static void skip_pi(tt *t) {
  t->position = index_of(t, "?>", t->position + 1);
  if (t->position < 0) t->position = t->len;
}

static int name_is(const jstr *a, const jstr *b) {
  return a->n == b->n && (a->n == 0 || memcmp(a->p, b->p, (size_t)a->n * 2) == 0);
}

static void parse_end_tag(tt *t) {
  int i;
  for (i = t->position + 2; i < t->len; i++) {
    uint16_t c = t->text[i];
    if (is_space_char(c) || c == '>') break;
  }
  jstr name;
  js_init(&name);
  java_tolower(t->text + t->position + 2, i - (t->position + 2), &name);
  if (t->ignoring && name_is(&t->ignoreUntil, &name)) t->ignoring = 0;
  while (i < t->len && t->text[i] != '>') i++;
  t->position = i;
  js_free(&name);
}

static int index_of_non_space(tt *t, int start) {
  if (start < 0) return INT_MIN;
  for (int i = start; i < t->len; i++)
    if (!is_space_char(t->text[i])) return i;
  return INT_MIN;
}

static int index_of_end_attribute(tt *t, int start, int tagEnd) {
  if (start < 0) return INT_MIN;
  int inQuote = 0, lastEscape = 0;
  for (int i = start; i <= tagEnd; i++) {
    uint16_t c = t->text[i];
    if ((c == '"' || c == '\'') && !lastEscape) {
      inQuote = !inQuote;
      if (!inQuote) return i;
    } else if (!inQuote && (is_space_char(c) || c == '>')) {
      return i;
    } else if (c == '\\' && !lastEscape) {
      lastEscape = 1;
    } else {
      lastEscape = 0;
    }
  }
  return INT_MIN;
}

static int index_of_equals(tt *t, int start, int end) {
  if (start < 0) return INT_MIN;
  for (int i = start; i < end; i++)
    if (t->text[i] == '=') return i;
  return INT_MIN;
}

static void parse_begin_tag(tt *t) {
  int i;
  for (i = t->position + 1; i < t->len; i++) {
    uint16_t c = t->text[i];
    if (is_space_char(c) || c == '>') break;
  }
  jstr name;
  js_init(&name);
  java_tolower(t->text + t->position + 1, i - (t->position + 1), &name);

  i = index_of_non_space(t, i);
  int tagEnd = index_of(t, ">", i + 1); /* i may be INT_MIN: Java treats negative fromIndex as 0 */
  int closeIt = 0;
  while (i < tagEnd && i >= 0 && tagEnd >= 0) {
    int start = index_of_non_space(t, i);
    if (start > 0) {
      if (t->text[start] == '>') {
        i = start;
        break;
      } else if (t->text[start] == '/' && t->len > start + 1 && t->text[start + 1] == '>') {
        i = start + 1;
        closeIt = 1;
        break;
      }
    }
    int end = index_of_end_attribute(t, start, tagEnd);
    int equals = index_of_equals(t, start, end);
    if (equals < 0 || equals == start || end == equals) {
      if (end < 0) {
        i = tagEnd;
        break;
      } else {
        i = end;
        continue;
      }
    }
    int startKey = start, endKey = equals;
    int startValue = equals + 1, endValue = end;
    if (t->text[startValue] == '"' || t->text[startValue] == '\'') startValue++;
    if (startValue >= endValue || startKey >= endKey) {
      i = end;
      continue;
    }
    if (end >= t->len) {
      end_parsing(t);
      break;
    }
    if (t->text[end] == '"' || t->text[end] == '\'') end++;
    i = end;
  }
  int ignored = (name.n == 6 && name.p[0] == 's' && name.p[1] == 'c' && name.p[2] == 'r' &&
                 name.p[3] == 'i' && name.p[4] == 'p' && name.p[5] == 't') ||
                (name.n == 5 && name.p[0] == 's' && name.p[1] == 't' && name.p[2] == 'y' &&
                 name.p[3] == 'l' && name.p[4] == 'e');
  if (ignored && !closeIt) {
    t->ignoring = 1;
    js_set(&t->ignoreUntil, name.p, name.n);
  }
  t->position = i;
  js_free(&name);
}

static void on_start_bracket(tt *t) {
  if (t->position + 1 < t->len) {
    uint16_t c = t->text[t->position + 1];
    if (c == '/')
      parse_end_tag(t);
    else if (c == '!')
      skip_comment(t);
    else if (c == '?')
      skip_pi(t);
    else
      parse_begin_tag(t);
  } else {
    end_parsing(t);
  }
  t->lastSplit = t->position;
}

static void on_ampersand(tt *t) {
  on_split(t);
  for (int i = t->position + 1; i < t->len; i++) {
    uint16_t c = t->text[i];
    if ((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '#') continue;
    if (c == ';') {
      t->position = i;
      t->lastSplit = i;
      return;
    }
    break;
  }
}

void or_tag_tokenize(const uint16_t *text, int n, jstr_list *terms) {
  tt t;
  t.text = text;
  t.len = n;
  t.position = 0;
  t.lastSplit = -1;
  t.ignoring = 0;
  js_init(&t.ignoreUntil);
  t.tokens = terms;
  for (; t.position >= 0 && t.position < t.len; t.position++) {
    uint16_t c = t.text[t.position];
    if (c == '<') {
      if (!t.ignoring) on_split(&t);
      on_start_bracket(&t);
    } else if (t.ignoring) {
      continue;
    } else if (c == '&') {
      on_ampersand(&t);
    } else if (is_split(c)) {
      on_split(&t);
    }
  }
  if (!t.ignoring) on_split(&t);
  js_free(&t.ignoreUntil);
}

/* Terrier stop list, GalagoTokenizer.java:35-125 (733 literals). */
static const char *STOP[] = {
    "x", "y", "your", "yours", "yourself", "yourselves", "you", "yond", "yonder", "yon", "ye",
    "yet", "z", "zillion", "j", "u", "umpteen", "usually", "us", "username", "uponed", "upons",
    "uponing", "upon", "ups", "upping", "upped", "up", "unto", "until", "unless", "unlike",
    "unliker", "unlikest", "under", "underneath", "use", "used", "usedest", "r", "rath", "rather",
    "rathest", "rathe", "re", "relate", "related", "relatively", "regarding", "really", "res",
    "respecting", "respectively", "q", "quite", "que", "qua", "n", "neither", "neaths", "neath",
    "nethe", "nethermost", "necessary", "necessariest", "necessarier", "never", "nevertheless",
    "nigh", "nighest", "nigher", "nine", "noone", "nobody", "nobodies", "nowhere", "nowheres",
    "no", "noes", "nor", "nos", "no-one", "none", "not", "notwithstanding", "nothings", "nothing",
    "nathless", "natheless", "t", "ten", "tills", "till", "tilled", "tilling", "to", "towards",
    "toward", "towardest", "towarder", "together", "too", "thy", "thyself", "thus", "than", "that",
    "those", "thou", "though", "thous", "thouses", "thoroughest", "thorougher", "thorough",
    "thoroughly", "thru", "thruer", "thruest", "thro", "through", "throughout", "throughest",
    "througher", "thine", "this", "thises", "they", "thee", "the", "then", "thence", "thenest",
    "thener", "them", "themselves", "these", "therer", "there", "thereby", "therest",
    "thereafter", "therein", "thereupon", "therefore", "their", "theirs", "thing", "things",
    "three", "two", "o", "oh", "owt", "owning", "owned", "own", "owns", "others", "other",
    "otherwise", "otherwisest", "otherwiser", "of", "often", "oftener", "oftenest", "off", "offs",
    "offest", "one", "ought", "oughts", "our", "ours", "ourselves", "ourself", "out", "outest",
    "outed", "outwith", "outs", "outside", "over", "overallest", "overaller", "overalls",
    "overall", "overs", "or", "orer", "orest", "on", "oneself", "onest", "ons", "onto", "a",
    "atween", "at", "athwart", "atop", "afore", "afterward", "afterwards", "after", "afterest",
    "afterer", "ain", "an", "any", "anything", "anybody", "anyone", "anyhow", "anywhere",
    "anent", "anear", "and", "andor", "another", "around", "ares", "are", "aest", "aer",
    "against", "again", "accordingly", "abaft", "abafter", "abaftest", "abovest", "above",
    "abover", "abouter", "aboutest", "about", "aid", "amidst", "amid", "among", "amongst",
    "apartest", "aparter", "apart", "appeared", "appears", "appear", "appearing", "appropriating",
    "appropriate", "appropriatest", "appropriates", "appropriater", "appropriated", "already",
    "always", "also", "along", "alongside", "although", "almost", "all", "allest", "aller",
    "allyou", "alls", "albeit", "awfully", "as", "aside", "asides", "aslant", "ases", "astrider",
    "astride", "astridest", "astraddlest", "astraddler", "astraddle", "availablest",
    "availabler", "available", "aughts", "aught", "vs", "v", "variousest", "variouser",
    "various", "via", "vis-a-vis", "vis-a-viser", "vis-a-visest", "viz", "very", "veriest",
    "verier", "versus", "k", "g", "go", "gone", "good", "got", "gotta", "gotten", "get", "gets",
    "getting", "b", "by", "byandby", "by-and-by", "bist", "both", "but", "buts", "be", "beyond",
    "because", "became", "becomes", "become", "becoming", "becomings", "becominger",
    "becomingest", "behind", "behinds", "before", "beforehand", "beforehandest", "beforehander",
    "bettered", "betters", "better", "bettering", "betwixt", "between", "beneath", "been",
    "below", "besides", "beside", "m", "my", "myself", "mucher", "muchest", "much", "must",
    "musts", "musths", "musth", "main", "make", "mayest", "many", "mauger", "maugre", "me",
    "meanwhiles", "meanwhile", "mostly", "most", "moreover", "more", "might", "mights", "midst",
    "midsts", "h", "huh", "humph", "he", "hers", "herself", "her", "hereby", "herein",
    "hereafters", "hereafter", "hereupon", "hence", "hadst", "had", "having", "haves", "have",
    "has", "hast", "hardly", "hae", "hath", "him", "himself", "hither", "hitherest", "hitherer",
    "his", "how-do-you-do", "however", "how", "howbeit", "howdoyoudo", "hoos", "hoo", "w",
    "woulded", "woulding", "would", "woulds", "was", "wast", "we", "wert", "were", "with",
    "withal", "without", "within", "why", "what", "whatever", "whateverer", "whateverest",
    "whatsoeverer", "whatsoeverest", "whatsoever", "whence", "whencesoever", "whenever",
    "whensoever", "when", "whenas", "whether", "wheen", "whereto", "whereupon", "wherever",
    "whereon", "whereof", "where", "whereby", "wherewithal", "wherewith", "whereinto",
    "wherein", "whereafter", "whereas", "wheresoever", "wherefrom", "which", "whichever",
    "whichsoever", "whilst", "while", "whiles", "whithersoever", "whither", "whoever",
    "whosoever", "whoso", "whose", "whomever", "s", "syne", "syn", "shalling", "shall", "shalled",
    "shalls", "shoulding", "should", "shoulded", "shoulds", "she", "sayyid", "sayid", "said",
    "saider", "saidest", "same", "samest", "sames", "samer", "saved", "sans", "sanses",
    "sanserifs", "sanserif", "so", "soer", "soest", "sobeit", "someone", "somebody", "somehow",
    "some", "somewhere", "somewhat", "something", "sometimest", "sometimes", "sometimer",
    "sometime", "several", "severaler", "severalest", "serious", "seriousest", "seriouser",
    "senza", "send", "sent", "seem", "seems", "seemed", "seemingest", "seeminger", "seemings",
    "seven", "summat", "sups", "sup", "supping", "supped", "such", "since", "sine", "sines",
    "sith", "six", "stop", "stopped", "p", "plaintiff", "plenty", "plenties", "please",
    "pleased", "pleases", "per", "perhaps", "particulars", "particularly", "particular",
    "particularest", "particularer", "pro", "providing", "provides", "provided", "provide",
    "probably", "l", "layabout", "layabouts", "latter", "latterest", "latterer", "latterly",
    "latters", "lots", "lotting", "lotted", "lot", "lest", "less", "ie", "ifs", "if", "i",
    "info", "information", "itself", "its", "it", "is", "idem", "idemer", "idemest",
    "immediate", "immediately", "immediatest", "immediater", "in", "inwards", "inwardest",
    "inwarder", "inward", "inasmuch", "into", "instead", "insofar", "indicates", "indicated",
    "indicate", "indicating", "indeed", "inc", "f", "fact", "facts", "fs", "figupon",
    "figupons", "figuponing", "figuponed", "few", "fewer", "fewest", "frae", "from", "failing",
    "failings", "five", "furthers", "furtherer", "furthered", "furtherest", "further",
    "furthering", "furthermore", "fourscore", "followthrough", "for", "forwhy", "fornenst",
    "formerly", "former", "formerer", "formerest", "formers", "forbye", "forby", "fore",
    "forever", "forer", "fores", "four", "d", "ddays", "dday", "do", "doing", "doings", "doe",
    "does", "doth", "downwarder", "downwardest", "downward", "downwards", "downs", "done",
    "doner", "dones", "donest", "dos", "dost", "did", "differentest", "differenter",
    "different", "describing", "describe", "describes", "described", "despiting", "despites",
    "despited", "despite", "during", "c", "cum", "circa", "chez", "cer", "certain",
    "certainest", "certainer", "cest", "canst", "cannot", "cant", "cants", "canting", "cantest",
    "canted", "co", "could", "couldst", "comeon", "comeons", "come-ons", "come-on", "concerning",
    "concerninger", "concerningest", "consequently", "considering", "e", "eg", "eight",
    "either", "even", "evens", "evenser", "evensest", "evened", "evenest", "ever", "everyone",
    "everything", "everybody", "everywhere", "every", "ere", "each", "et", "etc", "elsewhere",
    "else", "ex", "excepted", "excepts", "except", "excepting", "exes", "enough"};

int or_stopword_count(void) { return (int)(sizeof STOP / sizeof STOP[0]); }

int or_is_stopword(const uint16_t *w, int n) {
  for (size_t i = 0; i < sizeof STOP / sizeof STOP[0]; i++) {
    const char *s = STOP[i];
    int sl = (int)strlen(s);
    if (sl != n) continue;
    int k = 0;
    while (k < n && w[k] == (unsigned char)s[k]) k++;
    if (k == n) return 1;
  }
  return 0;
}

void or_process_content(const uint16_t *text, int n, jstr_list *out) {
  jstr_list toks;
  jl_init(&toks);
  or_tag_tokenize(text, n, &toks);
  jstr st;
  js_init(&st);
  for (int i = 0; i < toks.n; i++) {
    if (or_is_stopword(toks.v[i].p, toks.v[i].n)) continue;
    or_stem_js(toks.v[i].p, toks.v[i].n, &st);
    jl_push(out, st.p, st.n);
  }
  js_free(&st);
  jl_free(&toks);
}
const char *or_stopword(int i) { return STOP[i]; }
