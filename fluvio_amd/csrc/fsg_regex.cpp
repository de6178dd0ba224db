// fsg_regex.cpp — chain-build-time compiler: Rust-regex pattern -> UTF-8 byte DFA.
//
// The reference compiles `Regex::new(param "regex")` inside the guest's init()
// (smartmodule/regex-filter/src/lib.rs:13-22) and calls `Regex::is_match` per
// record (lib.rs:24-28; filter_regex: examples/filter_regex/src/lib.rs).  The
// regex crate (1.6.0 / 1.8.1) is a third-party dependency that is not in the
// reference tree; we restate its published semantics for the supported subset:
// unanchored is_match over valid UTF-8, Unicode-aware `.` (any scalar but \n),
// `\d` (Unicode Nd), `\s` (White_Space), `\w` (Alphabetic + M + Nd + Pc +
// Join_Control), `\p{..}` / `\P{..}` (General_Category values and groups, Any,
// ASCII, Assigned, regex-syntax's binary properties, Script and
// Script_Extensions values; fsg_unicode.h, generated from this image's Unicode
// tables), `^`/`$` at value start/end or, under the m flag, at line
// boundaries (DFA states that remember whether the previous byte was \n),
// `\A` / `\z`, `[[:name:]]` ASCII classes, inline flags i (simple case folding:
// the CaseFolding C + S orbits, on literals, ranges and Unicode classes), s, U, m, x (whitespace and #
// comments ignored) and u (off: ASCII \d \s \w; a negated class, `.` or \W that
// could match invalid UTF-8 is the crate's init error).  `\b`, `\B`: word
// boundaries are DFA states that remember whether the previous byte was a word
// byte (ASCII values); for values with non-ASCII bytes the full DFA is built
// over the bytes with a marker before each code point carrying its Unicode \w
// class (determinize's marker mode); a (?-u) \b keeps non-ASCII values
// FSG_E_UNSUPPORTED.  Nested classes and the class set operations && -- ~~, escapes
// \x \u \U (fixed digits or braces).  Other enumerated properties in \p{..}
// (Age, the break properties, ...) are rejected at init (FSG_E_UNSUPPORTED).
//
// Output: a DFA over bytes with unanchored restart folded in, byte classes,
// sticky acceptance, an end-of-value acceptance bit and the longest possible
// match length (used by the kernel's chunk-parallel scan).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "fsg_regex.h"
#include "fsg_unicode.h"

namespace fsg {
namespace {

struct Range {
  uint32_t lo, hi;
};

const Range kNd[] = {
    {0x30, 0x39},       {0x660, 0x669},     {0x6F0, 0x6F9},     {0x7C0, 0x7C9},     {0x966, 0x96F},
    {0x9E6, 0x9EF},     {0xA66, 0xA6F},     {0xAE6, 0xAEF},     {0xB66, 0xB6F},     {0xBE6, 0xBEF},
    {0xC66, 0xC6F},     {0xCE6, 0xCEF},     {0xD66, 0xD6F},     {0xDE6, 0xDEF},     {0xE50, 0xE59},
    {0xED0, 0xED9},     {0xF20, 0xF29},     {0x1040, 0x1049},   {0x1090, 0x1099},   {0x17E0, 0x17E9},
    {0x1810, 0x1819},   {0x1946, 0x194F},   {0x19D0, 0x19D9},   {0x1A80, 0x1A89},   {0x1A90, 0x1A99},
    {0x1B50, 0x1B59},   {0x1BB0, 0x1BB9},   {0x1C40, 0x1C49},   {0x1C50, 0x1C59},   {0xA620, 0xA629},
    {0xA8D0, 0xA8D9},   {0xA900, 0xA909},   {0xA9D0, 0xA9D9},   {0xA9F0, 0xA9F9},   {0xAA50, 0xAA59},
    {0xABF0, 0xABF9},   {0xFF10, 0xFF19},   {0x104A0, 0x104A9}, {0x10D30, 0x10D39}, {0x11066, 0x1106F},
    {0x110F0, 0x110F9}, {0x11136, 0x1113F}, {0x111D0, 0x111D9}, {0x112F0, 0x112F9}, {0x11450, 0x11459},
    {0x114D0, 0x114D9}, {0x11650, 0x11659}, {0x116C0, 0x116C9}, {0x11730, 0x11739}, {0x118E0, 0x118E9},
    {0x11950, 0x11959}, {0x11C50, 0x11C59}, {0x11D50, 0x11D59}, {0x11DA0, 0x11DA9}, {0x11F50, 0x11F59},
    {0x16A60, 0x16A69}, {0x16AC0, 0x16AC9}, {0x16B50, 0x16B59}, {0x1D7CE, 0x1D7FF}, {0x1E140, 0x1E149},
    {0x1E2F0, 0x1E2F9}, {0x1E4F0, 0x1E4F9}, {0x1E950, 0x1E959}, {0x1FBF0, 0x1FBF9}};
const Range kWs[] = {{0x09, 0x0D}, {0x20, 0x20},     {0x85, 0x85},     {0xA0, 0xA0},     {0x1680, 0x1680},
                     {0x2000, 0x200A}, {0x2028, 0x2029}, {0x202F, 0x202F}, {0x205F, 0x205F}, {0x3000, 0x3000}};
const Range kWordAscii[] = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
const Range kDigitAscii[] = {{'0', '9'}};
const Range kSpaceAscii[] = {{'\t', '\r'}, {' ', ' '}};  // (?-u)\s: [\t\n\v\f\r ]

using Set = std::vector<Range>;

Set norm(Set s) {
  std::sort(s.begin(), s.end(), [](const Range& a, const Range& b) { return a.lo < b.lo; });
  Set o;
  for (auto& r : s) {
    if (!o.empty() && r.lo <= o.back().hi + 1)
      o.back().hi = std::max(o.back().hi, r.hi);
    else
      o.push_back(r);
  }
  return o;
}
Set negate(const Set& s0) {
  Set s = norm(s0), o;
  uint32_t next = 0;
  for (auto& r : s) {
    if (r.lo > next) o.push_back({next, r.lo - 1});
    next = r.hi + 1;
  }
  if (next <= 0x10FFFF) o.push_back({next, 0x10FFFF});
  return o;
}
// class set operations (regex-syntax ClassSetBinaryOpKind): &&, --, ~~
Set set_union(Set a, const Set& b) {
  a.insert(a.end(), b.begin(), b.end());
  return norm(a);
}
Set set_inter(const Set& a, const Set& b) { return negate(set_union(negate(a), negate(b))); }
Set set_diff(const Set& a, const Set& b) { return set_inter(a, negate(b)); }
Set set_symdiff(const Set& a, const Set& b) { return set_union(set_diff(a, b), set_diff(b, a)); }
template <size_t N>
Set table(const Range (&t)[N], bool neg) {
  Set s(t, t + N);
  return neg ? negate(s) : s;
}

Set urange(const fsg_urange* r, uint32_t n) {
  Set o;
  for (uint32_t k = 0; k < n; k++) o.push_back({r[k].lo, r[k].hi});
  return o;
}

// ---------------- AST
// N_MBOL / N_MEOL: ^ / $ under the m flag (after / before a \n, or at the ends)
enum NodeT { N_EMPTY, N_SET, N_CAT, N_ALT, N_REP, N_BOL, N_EOL, N_WB, N_NWB, N_MBOL, N_MEOL };
struct Node {
  NodeT t = N_EMPTY;
  Set set;
  std::vector<std::unique_ptr<Node>> kids;
  std::unique_ptr<Node> sub;
  int mn = 0, mx = 0;  // mx < 0: unbounded
};
using NodeP = std::unique_ptr<Node>;

struct Parser {
  std::vector<uint32_t> p;
  size_t i = 0;
  bool err = false, unsup = false, word = false, wb = false, ml = false;
  bool wbu = false, wba = false;  // \b / \B seen in Unicode mode / under (?-u)
  bool fi = false, fs = false;  // inline flags i, s
  bool fm = false, fx = false, fu = true;  // m (multi-line), x (verbose), u (Unicode, on by default)
  // utab: a class built from version-dependent Unicode tables (\d \w, \p, (?i)
  // folding, Unicode \b) — values holding a fsg_u_newer code point are
  // FSG_E_UNSUPPORTED; perr: the first \p name regex-syntax rejects at
  // Regex::new (fsg_u_unresolved 2 / 3) and its span [perr_lo, perr_hi)
  bool utab = false;
  int perr = 0;
  size_t perr_lo = 0, perr_hi = 0;

  // x: whitespace (char::is_whitespace) and # comments between tokens are ignored
  static bool uspace(uint32_t c) {
    for (const Range& r : kWs)
      if (c >= r.lo && c <= r.hi) return true;
    return false;
  }
  void skip_x() {
    while (fx && i < p.size()) {
      if (uspace(p[i])) {
        i++;
      } else if (p[i] == '#') {
        while (i < p.size() && p[i] != '\n') i++;
      } else {
        break;
      }
    }
  }
  // \p{..} / \pX after the 'p' / 'P' (regex-syntax: names compared without case,
  // spaces, '_' and '-'); 2 = a set, 0 = failure (err / unsup set)
  int property(bool neg, Set* out) {
    if (!fu) {  // Unicode classes need the u flag
      err = true;
      return 0;
    }
    const size_t at0 = i - 2;  // the escape's '\'
    std::string name;
    if (at('{')) {
      i++;
      if (at('^')) {
        neg = !neg;
        i++;
      }
      // the raw text splits at its first ':' / '=' and each part is normalized
      // on its own (symbolic_name_normalize, UAX44-LM3): an "is" prefix of the
      // raw part dropped ("isc" kept), then ' ', '_', '-' removed, lowercased
      std::string part;
      bool is_pfx = false, start = true, split = false;
      auto finish = [&]() {
        if (is_pfx && part == "c") part = "isc";
        name += part;
        part.clear();
      };
      while (i < p.size() && p[i] != '}') {
        const uint32_t c = p[i++];
        if (c >= 0x80) {
          unsup = true;
          return 0;
        }
        if (!split && (c == ':' || c == '=')) {
          finish();
          name += '=';
          split = true;
          start = true;
          continue;
        }
        if (start) {
          start = false;
          const uint32_t c2 = i < p.size() ? p[i] : 0;
          if ((c | 0x20) == 'i' && (c2 | 0x20) == 's') {
            is_pfx = true;
            i++;
            continue;
          }
          is_pfx = false;
        }
        if (c == ' ' || c == '_' || c == '-') continue;
        part += (char)(c >= 'A' && c <= 'Z' ? c + 32 : c);
      }
      finish();
      if (!at('}')) {
        err = true;
        return 0;
      }
      i++;
    } else {
      if (i >= p.size()) {
        err = true;
        return 0;
      }
      const uint32_t c = p[i++];
      if (c >= 0x80) {
        err = true;
        return 0;
      }
      name += (char)(c >= 'A' && c <= 'Z' ? c + 32 : c);
    }
    const long m = fsg_u_property(name.c_str());
    Set st;
    if (m == FSG_UPROP_ASCII) {
      st.push_back({0, 0x7F});
    } else if (m == FSG_UPROP_WSPACE) {
      st.assign(std::begin(kWs), std::end(kWs));
    } else if (m >= 0) {
      for (uint32_t k = 0; k < fsg_u_ncats; k++)
        if (m & (1L << k)) {
          Set t = urange(fsg_u_cats[k].r, fsg_u_cats[k].n);
          st.insert(st.end(), t.begin(), t.end());
        }
    } else {
      // binary properties, Script / Script_Extensions values (sc= / scx=)
      const fsg_urange* pr = nullptr;
      uint32_t pn = 0;
      if (!fsg_u_lookup(name.c_str(), &pr, &pn)) {
        const int k = fsg_u_unresolved(name.c_str());
        if (k == 1) {
          unsup = true;  // Age values, CWKCF: regex-syntax has them, not restated here
          return 0;
        }
        if (!perr) {  // rejected at Regex::new: reported once the whole pattern parsed
          perr = k;
          perr_lo = at0;
          perr_hi = i;
        }
        *out = Set{};
        return 2;
      }
      st = urange(pr, pn);
    }
    if (m != FSG_UPROP_ASCII && m != FSG_UPROP_WSPACE) utab = true;
    if (fi) fold_set(st);  // (?i): simple case folding, before the negation
    *out = neg ? negate(st) : norm(st);
    return 2;
  }
  int depth = 0;

  // (?i): regex-syntax's simple case folding (CaseFolding.txt C + S orbits,
  // fsg_unicode.h) in Unicode mode; (?-u) folds ASCII letters only (its byte
  // classes)
  static void fold_add(void* ctx, uint32_t c) { static_cast<Set*>(ctx)->push_back({c, c}); }
  void fold_set(Set& st) {
    utab = true;
    const Set base = st;
    for (const auto& r : base) fsg_u_fold_range(r.lo, r.hi, fold_add, &st);
  }
  void add_folded(Set& st, uint32_t lo, uint32_t hi) {
    st.push_back({lo, hi});
    if (!fi) return;
    if (fu) {
      utab = true;
      fsg_u_fold_range(lo, hi, fold_add, &st);
      return;
    }
    if (hi >= 0x80) {
      unsup = true;
      return;
    }
    uint32_t a = std::max<uint32_t>(lo, 'a'), b = std::min<uint32_t>(hi, 'z');
    if (a <= b) st.push_back({a - 32, b - 32});
    a = std::max<uint32_t>(lo, 'A');
    b = std::min<uint32_t>(hi, 'Z');
    if (a <= b) st.push_back({a + 32, b + 32});
  }
  // [:name:] ASCII classes (regex-syntax ClassAsciiKind)
  static bool posix(const std::vector<uint32_t>& name, Set& st) {
    static const struct {
      const char* n;
      Range r[4];
      int k;
    } T[] = {{"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}, 3},
             {"alpha", {{'A', 'Z'}, {'a', 'z'}}, 2},
             {"ascii", {{0, 0x7F}}, 1},
             {"blank", {{'\t', '\t'}, {' ', ' '}}, 2},
             {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}, 2},
             {"digit", {{'0', '9'}}, 1},
             {"graph", {{'!', '~'}}, 1},
             {"lower", {{'a', 'z'}}, 1},
             {"print", {{' ', '~'}}, 1},
             {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}, 4},
             {"space", {{'\t', '\r'}, {' ', ' '}}, 2},
             {"upper", {{'A', 'Z'}}, 1},
             {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}, 4},
             {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}, 3}};
    for (auto& t : T) {
      if (strlen(t.n) != name.size() || !std::equal(name.begin(), name.end(), t.n)) continue;
      for (int q = 0; q < t.k; q++) st.push_back(t.r[q]);
      return true;
    }
    return false;
  }

  bool at(uint32_t c) const { return i < p.size() && p[i] == c; }
  static bool hex(uint32_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
  static uint32_t hv(uint32_t c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }

  // 1: single code point in *c; 2: set in *s; 3 \b, 4 \B, 5 \A, 6 \z;
  // 0: failure (err/unsup set)
  int escape(uint32_t* c, Set* s, bool in_class = false) {
    if (i >= p.size()) {
      err = true;
      return 0;
    }
    uint32_t e = p[i++];
    switch (e) {
      case 'd': case 'D': case 's': case 'S': case 'w': case 'W': {
        const bool neg = e < 'a';
        if (!fu && neg) {  // (?-u)\D \S \W can match invalid UTF-8 (Regex on &str)
          err = true;
          return 0;
        }
        if (fu && (e | 0x20) != 's') utab = true;  // White_Space is the same in every version
        Set t = (e | 0x20) == 'd' ? (fu ? table(kNd, false) : table(kDigitAscii, false))
                : (e | 0x20) == 's' ? (fu ? table(kWs, false) : table(kSpaceAscii, false))
                : (fu ? urange(fsg_u_word, fsg_u_word_n) : table(kWordAscii, false));
        *s = neg ? negate(t) : norm(t);
        return 2;
      }
      case 'p': case 'P': return property(e == 'P', s);
      case 'n': *c = '\n'; return 1;
      case 't': *c = '\t'; return 1;
      case 'r': *c = '\r'; return 1;
      case 'f': *c = '\f'; return 1;
      case 'v': *c = '\v'; return 1;
      case 'a': *c = 7; return 1;
      case 'x': case 'u': case 'U': {  // \x7F \x{..}, \u007F \u{..}, \U0000007F \U{..} (regex-syntax parse_hex)
        const int fixed = e == 'x' ? 2 : e == 'u' ? 4 : 8;
        uint32_t v = 0;
        if (at('{')) {
          i++;
          int nd = 0;
          while (i < p.size() && hex(p[i]) && nd <= 8) {
            v = v * 16 + hv(p[i++]);
            nd++;
          }
          if (!at('}') || nd == 0 || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) {
            err = true;
            return 0;
          }
          i++;
        } else {
          for (int k = 0; k < fixed; k++) {
            if (i >= p.size() || !hex(p[i])) {
              err = true;
              return 0;
            }
            v = v * 16 + hv(p[i++]);
          }
          if (v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) {
            err = true;
            return 0;
          }
        }
        *c = v;
        return 1;
      }
      case 'b': case 'B': case 'A': case 'z':
        if (in_class) {
          err = true;
          return 0;
        }
        if (e == 'b' || e == 'B') {
          word = wb = true;
          (fu ? wbu : wba) = true;
        }
        return e == 'b' ? 3 : e == 'B' ? 4 : e == 'A' ? 5 : 6;
      default:
        if (e < 0x80 && !((e >= '0' && e <= '9') || (e >= 'a' && e <= 'z') || (e >= 'A' && e <= 'Z'))) {
          *c = e;
          return 1;
        }
        err = true;
        return 0;
    }
  }

  // a bracketed class after its '[' through the matching ']' (regex-syntax
  // parse_set_class): items are unions; nested brackets are items; the binary
  // operators && (intersection), -- (difference) and ~~ (symmetric difference)
  // are left-associative and bind looser than the union; a leading ']' and
  // leading '-'s are literals; negation applies to the whole result
  Set bracket() {
    bool neg = false;
    if (at('^')) {
      neg = true;
      i++;
    }
    Set uni, lhs;
    int op = 0;  // 0 none, 1 &&, 2 --, 3 ~~
    bool first = true;
    auto literal = [&](uint32_t lo, uint32_t hi) {
      if (!fu && hi >= 0x80) {  // class_literal_byte: UnicodeNotAllowed in a (?-u) class
        err = true;
        return;
      }
      add_folded(uni, lo, hi);
    };
    for (;;) {
      skip_x();
      if (i >= p.size()) {
        err = true;
        return uni;
      }
      uint32_t c = p[i];
      if (first) {  // parse_set_class_open: a leading ']' and any leading '-' are literals
        first = false;
        if (c == ']') {
          i++;
          literal(']', ']');
          continue;
        }
        if (c == '-') {
          while (at('-')) {
            i++;
            literal('-', '-');
          }
          continue;
        }
      }
      if (c == ']') {
        i++;
        break;
      }
      if (c == '[' && i + 1 < p.size() && p[i + 1] == ':') {  // [:name:] / [:^name:]
        size_t j = i + 2;
        bool pneg = false;
        if (j < p.size() && p[j] == '^') {
          pneg = true;
          j++;
        }
        size_t k = j;
        while (k + 1 < p.size() && !(p[k] == ':' && p[k + 1] == ']')) k++;
        Set ps;
        if (k + 1 < p.size() && posix(std::vector<uint32_t>(p.begin() + j, p.begin() + k), ps)) {
          if (pneg) ps = negate(ps);
          for (auto& r : ps) add_folded(uni, r.lo, r.hi);
          i = k + 2;
          continue;
        }
      }
      if (c == '[') {  // a nested class: one item of the union
        i++;
        if (++depth > 64) {
          unsup = true;
          return uni;
        }
        Set in = bracket();
        depth--;
        if (err || unsup) return uni;
        uni.insert(uni.end(), in.begin(), in.end());
        continue;
      }
      if ((c == '&' || c == '-' || c == '~') && i + 1 < p.size() && p[i + 1] == c) {
        i += 2;
        lhs = op == 0 ? norm(uni) : op == 1 ? set_inter(lhs, uni) : op == 2 ? set_diff(lhs, uni) : set_symdiff(lhs, uni);
        uni.clear();
        op = c == '&' ? 1 : c == '-' ? 2 : 3;
        continue;
      }
      i++;
      uint32_t lo;
      if (c == '\\') {
        Set s;
        int k = escape(&lo, &s, true);
        if (k == 2) {
          uni.insert(uni.end(), s.begin(), s.end());
          continue;
        }
        if (k == 0) return uni;
      } else {
        lo = c;
      }
      uint32_t hi = lo;
      // parse_set_class_range: bump_space after the first item; a '-' makes a
      // range unless the next non-space char is ']' or '-' (a difference)
      skip_x();
      size_t j = i + 1;
      if (fx && i < p.size()) {
        const size_t at_dash = i;
        i = j;
        skip_x();
        j = i;
        i = at_dash;
      }
      if (i < p.size() && p[i] == '-' && j < p.size() && p[j] != ']' && p[j] != '-') {
        i = j;
        uint32_t c2 = p[i++];
        if (c2 == '\\') {
          Set s;
          int k = escape(&hi, &s);
          if (k != 1) {
            if (k == 2) err = true;
            return uni;
          }
        } else {
          hi = c2;
        }
        if (hi < lo) {
          err = true;
          return uni;
        }
      }
      literal(lo, hi);
      if (err) return uni;
    }
    Set r = op == 0 ? norm(uni) : op == 1 ? set_inter(lhs, uni) : op == 2 ? set_diff(lhs, uni) : set_symdiff(lhs, uni);
    return neg ? negate(r) : r;  // case folding applies before the negation
  }
  NodeP cls() {
    auto n = std::make_unique<Node>();
    n->t = N_SET;
    n->set = bracket();
    // (?-u): a class that can match a byte >= 0x80 can match invalid UTF-8 (Regex on &str)
    if (!fu && !err && !unsup && !n->set.empty() && n->set.back().hi >= 0x80) err = true;
    return n;
  }

  bool num(int* v) {
    int nd = 0;
    long x = 0;
    while (i < p.size() && p[i] >= '0' && p[i] <= '9') {
      x = std::min(100000L, x * 10 + (long)(p[i++] - '0'));
      nd++;
    }
    *v = (int)x;
    return nd > 0;
  }

  NodeP atom() {
    uint32_t c = p[i++];
    auto n = std::make_unique<Node>();
    if (c == '(') {
      if (at('?')) {
        i++;
        if (at(':')) {
          i++;
        } else if (at('P') || at('<')) {
          if (at('P')) i++;
          if (!at('<')) {
            err = true;
            return n;
          }
          while (i < p.size() && p[i] != '>') i++;
          if (i >= p.size()) {
            err = true;
            return n;
          }
          i++;
        } else {  // inline flags (?flags) / (?flags:re): i, s, U; m, x, u, R unsupported
          int neg = 0, nflags = 0;
          bool nfi = fi, nfs = fs, nfm = fm, nfx = fx, nfu = fu;
          for (;;) {
            if (i >= p.size()) {
              err = true;
              return n;
            }
            const uint32_t f = p[i++];
            if (f == ':' || f == ')') {
              if (!nflags || neg == 1) {
                err = true;
                return n;
              }
              if (f == ')') {  // until the end of the enclosing group
                fi = nfi;
                fs = nfs;
                fm = nfm;
                fx = nfx;
                fu = nfu;
                return n;  // N_EMPTY
              }
              break;
            }
            if (f == '-') {
              if (neg) {
                err = true;
                return n;
              }
              neg = 1;
              continue;
            }
            if (f == 'i') {
              nfi = !neg;
            } else if (f == 's') {
              nfs = !neg;
            } else if (f == 'U') {  // greed only: same language for is_match
            } else if (f == 'm') {
              nfm = !neg;
            } else if (f == 'x') {
              nfx = !neg;
            } else if (f == 'u') {
              nfu = !neg;
            } else if (f == 'R') {  // CRLF mode (regex 1.8): not restated
              unsup = true;
              return n;
            } else {
              err = true;
              return n;
            }
            nflags++;
            if (neg) neg = 2;
          }
          const bool sfi = fi, sfs = fs, sfm = fm, sfx = fx, sfu = fu;
          fi = nfi;
          fs = nfs;
          fm = nfm;
          fx = nfx;
          fu = nfu;
          if (++depth > 200) {
            err = true;
            return n;
          }
          NodeP g = alt();
          depth--;
          fi = sfi;
          fs = sfs;
          fm = sfm;
          fx = sfx;
          fu = sfu;
          if (!at(')')) {
            err = true;
            return g;
          }
          i++;
          return g;
        }
      }
      if (++depth > 200) {
        err = true;
        return n;
      }
      const bool sfi = fi, sfs = fs, sfm = fm, sfx = fx, sfu = fu;  // flags set inside a group end with it
      NodeP g = alt();
      depth--;
      fi = sfi;
      fs = sfs;
      fm = sfm;
      fx = sfx;
      fu = sfu;
      if (!at(')')) {
        err = true;
        return g;
      }
      i++;
      return g;
    }
    if (c == '[') return cls();
    if (c == '.') {
      if (!fu) {  // (?-u:.) can match invalid UTF-8 (Regex on &str)
        err = true;
        return n;
      }
      n->t = N_SET;
      if (fs)
        n->set = {{0, 0x10FFFF}};
      else
        n->set = {{0, '\n' - 1}, {'\n' + 1, 0x10FFFF}};
      return n;
    }
    if (c == '^') {
      n->t = fm ? N_MBOL : N_BOL;
      ml |= fm;
      return n;
    }
    if (c == '$') {
      n->t = fm ? N_MEOL : N_EOL;
      ml |= fm;
      return n;
    }
    if (c == '\\') {
      uint32_t cp = 0;
      Set s;
      int k = escape(&cp, &s);
      n->t = N_SET;
      if (k == 2) {
        n->set = norm(s);
      } else if (k == 1) {
        add_folded(n->set, cp, cp);
        n->set = norm(n->set);
      } else if (k >= 3) {
        n->t = k == 3 ? N_WB : k == 4 ? N_NWB : k == 5 ? N_BOL : N_EOL;
      }
      return n;
    }
    if (c == '*' || c == '+' || c == '?' || c == ')' || c == '|' || c == '{') {
      err = true;
      return n;
    }
    n->t = N_SET;
    add_folded(n->set, c, c);
    n->set = norm(n->set);
    return n;
  }

  NodeP cat() {
    auto n = std::make_unique<Node>();
    n->t = N_CAT;
    for (;;) {
      skip_x();
      if (!(i < p.size() && p[i] != '|' && p[i] != ')' && !err && !unsup)) break;
      NodeP a = atom();
      for (;;) {
        skip_x();
        if (i >= p.size()) break;
        uint32_t q = p[i];
        int mn, mx;
        if (q == '*') {
          mn = 0;
          mx = -1;
          i++;
        } else if (q == '+') {
          mn = 1;
          mx = -1;
          i++;
        } else if (q == '?') {
          mn = 0;
          mx = 1;
          i++;
        } else if (q == '{') {
          i++;
          if (!num(&mn)) {
            err = true;
            break;
          }
          mx = mn;
          if (at(',')) {
            i++;
            if (!num(&mx)) mx = -1;
          }
          if (!at('}') || (mx >= 0 && mx < mn)) {
            err = true;
            break;
          }
          i++;
          if (mn > 1000 || mx > 1000) {
            unsup = true;
            break;
          }
        } else {
          break;
        }
        if (at('?')) i++;  // lazy: same language for is_match
        auto r = std::make_unique<Node>();
        r->t = N_REP;
        r->mn = mn;
        r->mx = mx;
        r->sub = std::move(a);
        a = std::move(r);
      }
      n->kids.push_back(std::move(a));
    }
    return n;
  }

  NodeP alt() {
    auto n = std::make_unique<Node>();
    n->t = N_ALT;
    n->kids.push_back(cat());
    while (at('|') && !err && !unsup) {
      i++;
      n->kids.push_back(cat());
    }
    return n;
  }
};

// ---------------- max match length in bytes (-1 unbounded)
int utf8_len(uint32_t c) { return c < 0x80 ? 1 : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4; }
int64_t max_len(const Node* n, bool ascii) {
  switch (n->t) {
    case N_EMPTY: case N_BOL: case N_EOL: case N_WB: case N_NWB: case N_MBOL: case N_MEOL: return 0;
    case N_SET: {
      int m = 0;
      for (auto& r : n->set) {
        if (ascii && r.lo > 0x7F) continue;
        m = std::max(m, ascii ? 1 : utf8_len(r.hi));
      }
      return m;
    }
    case N_CAT: {
      int64_t s = 0;
      for (auto& k : n->kids) {
        int64_t v = max_len(k.get(), ascii);
        if (v < 0) return -1;
        s += v;
      }
      return s;
    }
    case N_ALT: {
      int64_t m = 0;
      for (auto& k : n->kids) {
        int64_t v = max_len(k.get(), ascii);
        if (v < 0) return -1;
        m = std::max(m, v);
      }
      return m;
    }
    case N_REP: {
      int64_t v = max_len(n->sub.get(), ascii);
      if (v < 0) return -1;
      if (n->mx < 0) return v == 0 ? 0 : -1;
      return v * n->mx;
    }
  }
  return -1;
}

// ---------------- byte NFA
enum NfaT { F_BYTE, F_SPLIT, F_EPS, F_BOT, F_EOT, F_MATCH, F_WB, F_NWB, F_MBOT, F_MEOT };
struct NState {
  NfaT t;
  uint8_t lo, hi;
  int a, b;  // next states
};
struct Nfa {
  std::vector<NState> st;
  int add(NfaT t, uint8_t lo = 0, uint8_t hi = 0) {
    st.push_back({t, lo, hi, -1, -1});
    return (int)st.size() - 1;
  }
};
// fragment: start state + list of dangling out-pointers (state index, which: 0 a / 1 b)
struct Frag {
  int start;
  std::vector<std::pair<int, int>> outs;
};
void patch(Nfa& g, const Frag& f, int to) {
  for (auto& o : f.outs) (o.second ? g.st[o.first].b : g.st[o.first].a) = to;
}
Frag eps(Nfa& g) {
  int s = g.add(F_EPS);
  return {s, {{s, 0}}};
}
Frag cat2(Nfa& g, Frag a, Frag b) {
  patch(g, a, b.start);
  return {a.start, b.outs};
}
Frag alt2(Nfa& g, Frag a, Frag b) {
  int s = g.add(F_SPLIT);
  g.st[s].a = a.start;
  g.st[s].b = b.start;
  Frag f{s, a.outs};
  f.outs.insert(f.outs.end(), b.outs.begin(), b.outs.end());
  return f;
}
Frag bytes_seq(Nfa& g, const std::vector<std::pair<uint8_t, uint8_t>>& seq) {
  Frag f{-1, {}};
  int prev = -1;
  for (auto& br : seq) {
    int s = g.add(F_BYTE, br.first, br.second);
    if (prev < 0)
      f.start = s;
    else
      g.st[prev].a = s;
    prev = s;
  }
  f.outs = {{prev, 0}};
  return f;
}
// UTF-8 byte-range sequences of a code point range (surrogates excluded)
void utf8_seqs(uint32_t lo, uint32_t hi, std::vector<std::vector<std::pair<uint8_t, uint8_t>>>& out) {
  if (lo > hi) return;
  if (lo <= 0xDFFF && hi >= 0xD800) {
    if (lo < 0xD800) utf8_seqs(lo, 0xD7FF, out);
    if (hi > 0xDFFF) utf8_seqs(0xE000, hi, out);
    return;
  }
  static const uint32_t bounds[] = {0x7F, 0x7FF, 0xFFFF};
  for (uint32_t bd : bounds)
    if (lo <= bd && hi > bd) {
      utf8_seqs(lo, bd, out);
      utf8_seqs(bd + 1, hi, out);
      return;
    }
  if (hi <= 0x7F) {
    out.push_back({{(uint8_t)lo, (uint8_t)hi}});
    return;
  }
  int n = utf8_len(lo);
  for (int k = 1; k < n; k++) {
    uint32_t m = (1u << (6 * k)) - 1;
    if ((lo & ~m) != (hi & ~m)) {
      if ((lo & m) != 0) {
        utf8_seqs(lo, lo | m, out);
        utf8_seqs((lo | m) + 1, hi, out);
        return;
      }
      if ((hi & m) != m) {
        utf8_seqs(lo, (hi & ~m) - 1, out);
        utf8_seqs(hi & ~m, hi, out);
        return;
      }
    }
  }
  auto enc = [](uint32_t c, uint8_t* b) {
    int n = utf8_len(c);
    if (n == 1) {
      b[0] = (uint8_t)c;
    } else if (n == 2) {
      b[0] = 0xC0 | (c >> 6);
      b[1] = 0x80 | (c & 0x3F);
    } else if (n == 3) {
      b[0] = 0xE0 | (c >> 12);
      b[1] = 0x80 | ((c >> 6) & 0x3F);
      b[2] = 0x80 | (c & 0x3F);
    } else {
      b[0] = 0xF0 | (c >> 18);
      b[1] = 0x80 | ((c >> 12) & 0x3F);
      b[2] = 0x80 | ((c >> 6) & 0x3F);
      b[3] = 0x80 | (c & 0x3F);
    }
    return n;
  };
  uint8_t a[4], b[4];
  enc(lo, a);
  enc(hi, b);
  std::vector<std::pair<uint8_t, uint8_t>> seq;
  for (int k = 0; k < n; k++) seq.push_back({a[k], b[k]});
  out.push_back(seq);
}

Frag build(Nfa& g, const Node* n, bool ascii) {
  switch (n->t) {
    case N_EMPTY: return eps(g);
    case N_BOL: {
      int s = g.add(F_BOT);
      return {s, {{s, 0}}};
    }
    case N_EOL: {
      int s = g.add(F_EOT);
      return {s, {{s, 0}}};
    }
    case N_WB:
    case N_NWB: {
      int s = g.add(n->t == N_WB ? F_WB : F_NWB);
      return {s, {{s, 0}}};
    }
    case N_MBOL:
    case N_MEOL: {
      int s = g.add(n->t == N_MBOL ? F_MBOT : F_MEOT);
      return {s, {{s, 0}}};
    }
    case N_SET: {
      std::vector<std::vector<std::pair<uint8_t, uint8_t>>> seqs;
      for (auto& r : n->set) {
        if (ascii && r.lo > 0x7F) continue;
        utf8_seqs(r.lo, ascii ? std::min<uint32_t>(r.hi, 0x7F) : r.hi, seqs);
      }
      if (seqs.empty()) {
        // empty class: matches nothing — a byte range that is never taken
        int s = g.add(F_SPLIT);  // dead: both edges unset -> no progress
        g.st[s].a = -2;
        g.st[s].b = -2;
        return {s, {}};
      }
      // The sequences of a normalized set have, under a common prefix, byte
      // ranges that are equal or disjoint: they form a deterministic trie.
      // Equal subtrees are shared (hash-consed from the leaves), giving the
      // minimal acyclic automaton of the class: \w is ~60 lead-byte edges
      // into a handful of shared continuation chains, not ~700 alternatives.
      struct TNode {
        std::vector<std::pair<std::pair<uint8_t, uint8_t>, int>> kids;  // (range, child); leaf: none
      };
      std::vector<TNode> trie(1);
      for (auto& sq : seqs) {
        int at = 0;
        for (auto& r : sq) {
          int nx = -1;
          for (auto& kd : trie[at].kids)
            if (kd.first == r) nx = kd.second;
          if (nx < 0) {
            nx = (int)trie.size();
            trie[at].kids.push_back({r, nx});
            trie.emplace_back();
          }
          at = nx;
        }
      }
      // canonical ids bottom-up (children have larger indices than parents)
      std::vector<int> canon(trie.size());
      std::map<std::vector<int>, int> sig;
      for (size_t k = trie.size(); k-- > 0;) {
        std::vector<int> key;
        auto kids = trie[k].kids;
        std::sort(kids.begin(), kids.end());
        for (auto& kd : kids) {
          key.push_back(kd.first.first);
          key.push_back(kd.first.second);
          key.push_back(canon[kd.second]);
        }
        canon[k] = sig.emplace(key, (int)sig.size()).first->second;
      }
      // emit each canonical node once: a balanced split tree over its edges
      Frag f{-1, {}};
      std::vector<int> entry(sig.size(), -1);
      std::function<int(int)> emit = [&](int k) -> int {
        if (entry[canon[k]] >= 0) return entry[canon[k]];
        std::vector<int> edges;
        for (auto& kd : trie[k].kids) {
          int s = g.add(F_BYTE, kd.first.first, kd.first.second);
          if (trie[kd.second].kids.empty())
            f.outs.push_back({s, 0});
          else
            g.st[s].a = emit(kd.second);
          edges.push_back(s);
        }
        std::function<int(size_t, size_t)> tree = [&](size_t a, size_t b) -> int {
          if (b - a == 1) return edges[a];
          int sp = g.add(F_SPLIT);
          const size_t mid = (a + b) / 2;
          const int l = tree(a, mid), r = tree(mid, b);
          g.st[sp].a = l;
          g.st[sp].b = r;
          return sp;
        };
        return entry[canon[k]] = tree(0, edges.size());
      };
      f.start = emit(0);
      return f;
    }
    case N_CAT: {
      Frag f = eps(g);
      for (auto& k : n->kids) f = cat2(g, f, build(g, k.get(), ascii));
      return f;
    }
    case N_ALT: {
      Frag f = build(g, n->kids[0].get(), ascii);
      for (size_t k = 1; k < n->kids.size(); k++) f = alt2(g, f, build(g, n->kids[k].get(), ascii));
      return f;
    }
    case N_REP: {
      Frag f = eps(g);
      for (int k = 0; k < n->mn; k++) f = cat2(g, f, build(g, n->sub.get(), ascii));
      if (n->mx < 0) {
        int s = g.add(F_SPLIT);
        Frag body = build(g, n->sub.get(), ascii);
        g.st[s].a = body.start;
        patch(g, body, s);
        patch(g, f, s);
        return {f.start, {{s, 1}}};
      }
      for (int k = n->mn; k < n->mx; k++) {
        int s = g.add(F_SPLIT);
        Frag body = build(g, n->sub.get(), ascii);
        g.st[s].a = body.start;
        patch(g, f, s);
        Frag nf{f.start, body.outs};
        nf.outs.push_back({s, 1});
        f = nf;
      }
      return f;
    }
  }
  return eps(g);
}

struct Closure {
  const Nfa& g;
  std::vector<int> mark;
  int gen = 0;
  int64_t work = 0;  // NFA states visited (the compile-time budget)
  explicit Closure(const Nfa& n) : g(n), mark(n.st.size(), 0) {}
  // closure of `seeds`; keeps BYTE, MATCH and (unfollowed) EOT states; word
  // boundaries are kept pending (resolve = false) or decided from the previous
  // and next byte's word-ness (resolve = true)
  // multi-line anchors: ^ passes at the start or after a \n (pnl), $ at the
  // end or before a \n (nnl); kept pending unless resolved like the boundaries
  std::vector<int> run(const std::vector<int>& seeds, bool bot, bool eot, bool resolve = false, bool pw = false,
                       bool nw = false, bool pnl = false, bool nnl = false) {
    gen++;
    std::vector<int> out, stack(seeds.rbegin(), seeds.rend());
    while (!stack.empty()) {
      int s = stack.back();
      stack.pop_back();
      if (s < 0 || mark[s] == gen) continue;
      mark[s] = gen;
      work++;
      const NState& x = g.st[s];
      switch (x.t) {
        case F_BYTE: case F_MATCH: out.push_back(s); break;
        case F_EPS: stack.push_back(x.a); break;
        case F_SPLIT:
          stack.push_back(x.b);
          stack.push_back(x.a);
          break;
        case F_BOT:
          if (bot) stack.push_back(x.a);
          break;
        case F_EOT:
          if (eot)
            stack.push_back(x.a);
          else
            out.push_back(s);
          break;
        case F_WB:
        case F_NWB:
          if (!resolve)
            out.push_back(s);
          else if ((pw != nw) == (x.t == F_WB))
            stack.push_back(x.a);
          break;
        case F_MBOT:
          if (bot || (resolve && pnl))
            stack.push_back(x.a);
          else if (!resolve)
            out.push_back(s);
          break;
        case F_MEOT:
          if (eot || (resolve && nnl))
            stack.push_back(x.a);
          else if (!resolve)
            out.push_back(s);
          break;
      }
    }
    std::sort(out.begin(), out.end());
    return out;
  }
};

}  // namespace

static int determinize(const Node* rootp, bool ascii, bool word, bool wb, bool mlm, Dfa& out, std::string& msg,
                       bool marker = false);

int compile_regex(const std::string& pattern, Dfa& out, Dfa& full, std::string& msg) {
  // pattern -> code points (must be valid UTF-8; Rust &str)
  Parser P;
  {
    const uint8_t* s = (const uint8_t*)pattern.data();
    size_t n = pattern.size(), i = 0;
    while (i < n) {
      uint32_t c = s[i];
      int w = c < 0x80 ? 1 : c < 0xE0 ? 2 : c < 0xF0 ? 3 : 4;
      if (i + w > n) {
        msg = "regex parse error";
        return -2;
      }
      uint32_t cp = w == 1 ? c : w == 2 ? (c & 0x1F) : w == 3 ? (c & 0x0F) : (c & 0x07);
      for (int k = 1; k < w; k++) cp = (cp << 6) | (s[i + k] & 0x3F);
      P.p.push_back(cp);
      i += w;
    }
  }
  NodeP root = P.alt();
  if (P.perr && !P.err && P.i == P.p.size()) {
    msg = syntax_error_text(P.p, P.perr_lo, P.perr_hi,
                            P.perr == 2 ? "Unicode property value not found" : "Unicode property not found");
    return -2;
  }
  if (P.unsup) {
    msg = "unsupported regex syntax";
    return -103;
  }
  if (P.err || P.i != P.p.size()) {
    msg = "regex parse error";
    return -2;
  }
  if (int rc = determinize(root.get(), true, P.word, P.wb, P.ml, out, msg)) return rc;
  // Unicode word boundaries: the full DFA is the marked one (a (?-u) \b among
  // them keeps non-ASCII values FSG_E_UNSUPPORTED: bytes inside a code point)
  const int rc = determinize(root.get(), false, P.word, P.wb, P.ml, full, msg, P.wbu && !P.wba);
  out.utab = full.utab = P.utab || P.wbu;
  return rc;
}

// regex-syntax's error Display (error.rs Formatter / Spans::notate, the same in
// 0.6.27 and 0.7.1): "regex parse error:", the pattern's lines (4 spaces in
// front, or a right-aligned line number and ": " when the pattern has a '\n',
// between two lines of 79 '~'), a line of '^' under a one-line span, "on line
// .. through line .." for a span over lines, then "error: <kind>".  Columns
// count code points; [lo, hi) are code-point offsets into the pattern.
static void put_utf8(std::string& s, uint32_t c) {
  if (c < 0x80) {
    s += (char)c;
  } else if (c < 0x800) {
    s += (char)(0xC0 | (c >> 6));
    s += (char)(0x80 | (c & 0x3F));
  } else if (c < 0x10000) {
    s += (char)(0xE0 | (c >> 12));
    s += (char)(0x80 | ((c >> 6) & 0x3F));
    s += (char)(0x80 | (c & 0x3F));
  } else {
    s += (char)(0xF0 | (c >> 18));
    s += (char)(0x80 | ((c >> 12) & 0x3F));
    s += (char)(0x80 | ((c >> 6) & 0x3F));
    s += (char)(0x80 | (c & 0x3F));
  }
}

std::string syntax_error_text(const std::vector<uint32_t>& p, size_t lo, size_t hi, const char* kind) {
  // str::lines: split at '\n', one trailing '\r' dropped per line, no empty last line
  std::vector<std::pair<size_t, size_t>> lines;
  for (size_t s = 0, k = 0; k <= p.size(); k++)
    if (k == p.size() || p[k] == '\n') {
      if (k < p.size() || k > s) lines.push_back({s, k < p.size() && k > s && p[k - 1] == '\r' ? k - 1 : k});
      s = k + 1;
    }
  const bool multi = std::find(p.begin(), p.end(), (uint32_t)'\n') != p.end();
  size_t line_count = lines.size() + (!p.empty() && p.back() == '\n' ? 1 : 0);
  const size_t lnw = line_count <= 1 ? 0 : std::to_string(line_count).size();
  auto pos = [&](size_t off, size_t& line, size_t& col) {  // 1-based line / column of offset off
    line = 1;
    size_t ls = 0;
    for (size_t k = 0; k < off; k++)
      if (p[k] == '\n') {
        line++;
        ls = k + 1;
      }
    col = off - ls + 1;
  };
  size_t l0, c0, l1, c1;
  pos(lo, l0, c0);
  pos(hi, l1, c1);
  std::string notated;
  for (size_t n = 0; n < lines.size(); n++) {
    if (lnw) {
      const std::string num = std::to_string(n + 1);
      notated += std::string(lnw - num.size(), ' ') + num + ": ";
    } else {
      notated += "    ";
    }
    for (size_t k = lines[n].first; k < lines[n].second; k++) put_utf8(notated, p[k]);
    notated += '\n';
    if (l0 == l1 && l0 == n + 1) {
      notated += std::string(lnw ? 2 + lnw : 4, ' ');
      notated += std::string(c0 - 1, ' ');
      notated += std::string(std::max<size_t>(1, c1 > c0 ? c1 - c0 : 0), '^');
      notated += '\n';
    }
  }
  std::string out = "regex parse error:\n";
  if (!multi) return out + notated + "error: " + kind;
  const std::string div(79, '~');
  out += div + "\n" + notated + div + "\n";
  if (l0 != l1)
    out += "on line " + std::to_string(l0) + " (column " + std::to_string(c0) + ") through line " +
           std::to_string(l1) + " (column " + std::to_string(c1 - 1) + ")\n";
  return out + "error: " + kind;
}

static bool word_cp(uint32_t c) {
  uint32_t a = 0, b = fsg_u_word_n;
  while (a < b) {
    const uint32_t m = (a + b) / 2;
    if (fsg_u_word[m].hi < c) a = m + 1; else b = m;
  }
  return a < fsg_u_word_n && fsg_u_word[a].lo <= c;
}

// ~0.5 s of subset construction on one core: a pattern whose DFA needs more is
// one the GPU subset does not take (FSG_E_UNSUPPORTED), not a stalled chain build
static const int64_t kCompileBudget = 60000000;

static bool word_byte(int b) { return (b >= '0' && b <= '9') || (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == '_'; }

int determinize(const Node* rootp, bool ascii, bool word, bool wb, bool mlm, Dfa& out, std::string& msg, bool marker) {
  // word boundaries and multi-line anchors need the previous byte: no
  // chunk-parallel restarts (max_len -1)
  const int64_t ml = (wb || mlm) ? -1 : max_len(rootp, ascii);
  const bool resolve = wb || mlm;  // assertions decided at each transition from the previous / next byte
  // marker mode (Unicode \b): the assertions are decided at the marker before
  // each code point (its word-ness / \n), the unanchored restart added there;
  // the code point's bytes only move the NFA (pending assertions wait)
  Nfa g;
  Frag f = build(g, rootp, ascii);
  int m = g.add(F_MATCH);
  patch(g, f, m);
  const int start = f.start;
  // byte classes from all byte-range boundaries
  std::vector<int> cut(257, 0);
  cut[0] = cut[256] = 1;
  for (auto& s : g.st)
    if (s.t == F_BYTE) {
      cut[s.lo] = 1;
      cut[s.hi + 1] = 1;
    }
  if (wb)  // word bytes form their own classes
    for (int b = 0; b < 256; b++)
      if (word_byte(b) != (b > 0 && word_byte(b - 1))) cut[b] = 1;
  if (mlm) cut['\n'] = cut['\n' + 1] = 1;  // \n is its own class
  if (marker)  // each marker its own class
    for (int b = kMarkWord; b <= kMarkNl + 1; b++) cut[b] = 1;
  std::vector<uint8_t> cls(256);
  std::vector<int> rep;
  int nc = -1;
  for (int b = 0; b < 256; b++) {
    if (cut[b]) {
      nc++;
      rep.push_back(b);
    }
    cls[b] = (uint8_t)nc;
  }
  const int ncls = nc + 1;
  Closure C(g);
  std::map<std::vector<int>, int> ids;
  std::vector<std::vector<int>> sets;
  std::vector<uint8_t> bot_flag, pw_flag, nl_flag;
  auto intern = [&](const std::vector<int>& s, bool is_bot, bool pw, bool pnl = false) {
    auto key = s;
    if (is_bot) key.push_back(-7);  // the BOT state is distinct (EOT acceptance with ^ satisfied)
    if (pw) key.push_back(-8);      // the previous byte was a word byte (word boundaries)
    if (pnl) key.push_back(-9);     // the previous byte was \n (multi-line anchors)
    auto it = ids.find(key);
    if (it != ids.end()) return it->second;
    int id = (int)sets.size();
    ids[key] = id;
    sets.push_back(s);
    bot_flag.push_back(is_bot);
    pw_flag.push_back(pw);
    nl_flag.push_back(pnl);
    return id;
  };
  auto has_match = [&](const std::vector<int>& v) {
    return std::find_if(v.begin(), v.end(), [&](int s) { return g.st[s].t == F_MATCH; }) != v.end();
  };
  auto by_class = [&](const std::vector<int>& v, std::vector<std::vector<int>>& bucket) {
    for (auto& b : bucket) b.clear();
    for (int s : v) {
      const NState& x = g.st[s];
      if (x.t != F_BYTE) continue;
      for (int c = cls[x.lo]; c <= cls[x.hi]; c++) bucket[c].push_back(x.a);
    }
  };
  // Without assertions to resolve, every subset holds the restart closure S
  // (the pattern started again at each position); a subset is kept as its
  // members outside S, and S's successors per class are computed once.
  const bool fast = !resolve;
  std::vector<uint8_t> in_s(g.st.size(), 0);
  std::vector<std::vector<int>> es(ncls), bucket(ncls);
  bool s_has = false, s_eot = false;
  auto strip = [&](std::vector<int> v) {
    if (fast) v.erase(std::remove_if(v.begin(), v.end(), [&](int s) { return in_s[s] != 0; }), v.end());
    return v;
  };
  std::vector<int> S;
  if (fast) {
    S = C.run({start}, false, false);
    for (int s : S) in_s[s] = 1;
    s_has = has_match(S);
    s_eot = has_match(C.run(S, false, true));
    by_class(S, es);
    for (auto& e : es) e = strip(C.run(e, false, false));
  }
  const int s_bot = intern(strip(C.run({start}, true, false)), true, false);
  const int s_mid = intern(strip(C.run({start}, false, false)), false, false);
  int s_acc = -1;  // sticky accept reached through a word boundary decided at a transition
  std::vector<std::vector<int>> trans;
  std::vector<uint8_t> acc;
  for (size_t k = 0; k < sets.size(); k++) {
    // bounded chain-build cost: subsets before minimization and closure work
    if (sets.size() > (ascii ? 1024u : 32768u) || C.work > kCompileBudget) {
      msg = "regex too large for the GPU DFA";
      return -103;
    }
    const auto cur = sets[k];
    const bool pw = pw_flag[k], pnl = nl_flag[k];
    const bool is_acc = has_match(cur) || s_has;
    uint8_t a = is_acc ? 1 : 0;
    if (!is_acc) {  // at the end: no next byte
      std::vector<int> full = cur;
      if (fast && bot_flag[k]) {
        full.insert(full.end(), S.begin(), S.end());
        std::sort(full.begin(), full.end());
      }
      if (marker) full.push_back(start);  // a match may start at the end position
      auto ce = C.run(full, bot_flag[k], true, resolve, pw, false, pnl, false);
      if (has_match(ce) || (fast && !bot_flag[k] && s_eot)) a |= 2;
    } else {
      a |= 2;
    }
    acc.push_back(a);
    std::vector<int> row(ncls);
    if (fast && !is_acc) by_class(cur, bucket);  // targets of each byte state, by class (one pass)
    for (int c = 0; c < ncls; c++) {
      if (is_acc) {
        row[c] = (int)k;  // sticky: is_match is decided
        continue;
      }
      const int byte = rep[c];
      if (marker && byte < kMarkWord) {  // a byte of the code point: no assertion decided, no restart
        std::vector<int> nxt;
        for (int s : cur) {
          const NState& x = g.st[s];
          if (x.t == F_BYTE && byte >= x.lo && byte <= x.hi) nxt.push_back(x.a);
        }
        row[c] = intern(C.run(nxt, false, false), false, pw, pnl);
        continue;
      }
      if (marker && byte > kMarkNl) {  // never fed
        row[c] = (int)k;
        continue;
      }
      const bool nw = marker ? byte == kMarkWord : wb && word_byte(byte);
      const bool nnl = marker ? (mlm && byte == kMarkNl) : mlm && byte == '\n';
      std::vector<int> seeds = cur;
      if (marker) seeds.push_back(start);  // the unanchored restart at this code point
      const std::vector<int> res = resolve ? C.run(seeds, bot_flag[k], false, true, pw, nw, pnl, nnl) : cur;
      if (marker) {  // the marker consumes nothing: the resolved set waits for the code point's bytes
        if (has_match(res)) {
          if (s_acc < 0) s_acc = intern({m}, false, false);
          row[c] = s_acc;
        } else {
          row[c] = intern(res, false, nw, nnl);
        }
        continue;
      }
      if (resolve && has_match(res)) {  // an assertion before this byte completed the match
        if (s_acc < 0) s_acc = intern({m}, false, false);
        row[c] = s_acc;
        continue;
      }
      std::vector<int> nxt;
      if (resolve) {
        for (int s : res) {
          const NState& x = g.st[s];
          if (x.t == F_BYTE && byte >= x.lo && byte <= x.hi) nxt.push_back(x.a);
        }
        nxt.push_back(start);  // unanchored restart at the next position
        row[c] = intern(C.run(nxt, false, false), false, nw, nnl);
      } else {
        nxt.swap(bucket[c]);
        nxt.insert(nxt.end(), es[c].begin(), es[c].end());  // S is implied
        row[c] = intern(strip(C.run(nxt, false, false)), false, false, false);
      }
    }
    trans.push_back(row);
  }
  // Moore minimization: states with the same acceptance whose transitions
  // lead to the same blocks are merged (suffix-equivalent subsets, the many
  // sticky accepts); block ids renumbered in first-reached order from s_bot
  const int n0 = (int)sets.size();
  std::vector<int> blk(n0);
  for (int k = 0; k < n0; k++) blk[k] = acc[k];
  for (int nb = -1;;) {
    std::map<std::vector<int>, int> sig;
    std::vector<int> nblk(n0);
    for (int k = 0; k < n0; k++) {
      std::vector<int> key(ncls + 1);
      key[0] = blk[k];
      for (int c = 0; c < ncls; c++) key[c + 1] = blk[trans[k][c]];
      nblk[k] = sig.emplace(std::move(key), (int)sig.size()).first->second;
    }
    blk.swap(nblk);
    if ((int)sig.size() == nb) break;
    nb = (int)sig.size();
  }
  std::vector<int> ren(n0, -1), rep_of;
  {
    std::vector<int> order{s_bot, s_mid};
    for (size_t q = 0; q < order.size(); q++) {
      const int k = order[q];
      if (ren[blk[k]] >= 0) continue;
      ren[blk[k]] = (int)rep_of.size();
      rep_of.push_back(k);
      for (int c = 0; c < ncls; c++)
        if (ren[blk[trans[k][c]]] < 0) order.push_back(trans[k][c]);
    }
  }
  {
    std::vector<std::vector<int>> mt(rep_of.size(), std::vector<int>(ncls));
    std::vector<uint8_t> ma(rep_of.size());
    for (size_t q = 0; q < rep_of.size(); q++) {
      ma[q] = acc[rep_of[q]];
      for (int c = 0; c < ncls; c++) mt[q][c] = ren[blk[trans[rep_of[q]][c]]];
    }
    trans.swap(mt);
    acc.swap(ma);
  }
  if (trans.size() > (ascii ? 255u : 65535u)) {
    msg = "regex too large for the GPU DFA";
    return -103;
  }
  out.nstates = (uint32_t)trans.size();
  out.nclasses = (uint32_t)ncls;
  out.s_bot = (uint32_t)ren[blk[s_bot]];
  out.s_mid = (uint32_t)ren[blk[s_mid]];
  out.max_len = ml < 0 || ml > (1 << 20) ? -1 : (int32_t)ml;
  out.unicode_word = word;
  out.marked = marker;
  out.classmap = cls;
  out.classmap_up.resize(256);
  for (int b = 0; b < 256; b++) out.classmap_up[b] = cls[(b >= 'a' && b <= 'z') ? b - 32 : b];
  out.trans.resize(out.nstates * out.nclasses);
  for (uint32_t s = 0; s < out.nstates; s++)
    for (uint32_t c = 0; c < out.nclasses; c++) out.trans[s * out.nclasses + c] = (uint16_t)trans[s][c];
  out.accept = acc;
  return 0;
}

std::vector<uint32_t> unicode_newer_ranges() {
  std::vector<uint32_t> v;
  for (uint32_t q = 0; q < fsg_u_newer_n; q++) {
    v.push_back(fsg_u_newer[q].lo);
    v.push_back(fsg_u_newer[q].hi);
  }
  return v;
}

bool utf8_has_newer(const uint8_t* s, size_t n) {
  for (size_t i = 0; i < n;) {
    const uint32_t c0 = s[i];
    const size_t w = c0 < 0x80 ? 1 : c0 < 0xE0 ? 2 : c0 < 0xF0 ? 3 : 4;
    uint32_t cp = w == 1 ? c0 : w == 2 ? (c0 & 0x1F) : w == 3 ? (c0 & 0x0F) : (c0 & 0x07);
    for (size_t k = 1; k < w && i + k < n; k++) cp = (cp << 6) | (s[i + k] & 0x3F);
    if (cp >= 0x80 && fsg_u_is_newer(cp)) return true;
    i += w;
  }
  return false;
}

std::vector<uint32_t> unicode_word_ranges() {
  std::vector<uint32_t> v;
  for (uint32_t q = 0; q < fsg_u_word_n; q++) {
    v.push_back(fsg_u_word[q].lo);
    v.push_back(fsg_u_word[q].hi);
  }
  return v;
}

bool dfa_is_match_marked(const Dfa& d, const uint8_t* s, size_t n) {
  uint32_t st = d.s_bot;
  if (d.accept[st] & 1) return true;
  auto step = [&](uint8_t b) {
    st = d.trans[st * d.nclasses + d.classmap[b]];
    return (d.accept[st] & 1) != 0;
  };
  for (size_t i = 0; i < n;) {
    const uint32_t c0 = s[i];
    const size_t w = c0 < 0x80 ? 1 : c0 < 0xE0 ? 2 : c0 < 0xF0 ? 3 : 4;
    uint32_t cp = w == 1 ? c0 : w == 2 ? (c0 & 0x1F) : w == 3 ? (c0 & 0x0F) : (c0 & 0x07);
    for (size_t k = 1; k < w && i + k < n; k++) cp = (cp << 6) | (s[i + k] & 0x3F);
    if (step(cp == '\n' ? kMarkNl : word_cp(cp) ? kMarkWord : kMarkOther)) return true;
    for (size_t k = 0; k < w && i + k < n; k++)
      if (step(s[i + k])) return true;
    i += w;
  }
  return (d.accept[st] & 2) != 0;
}

bool dfa_is_match(const Dfa& d, const uint8_t* s, size_t n) {
  uint32_t st = d.s_bot;
  if (d.accept[st] & 1) return true;
  for (size_t i = 0; i < n; i++) {
    st = d.trans[st * d.nclasses + d.classmap[s[i]]];
    if (d.accept[st] & 1) return true;
  }
  return (d.accept[st] & 2) != 0;
}

bool rust_str_debug(const std::string& raw, std::string& out) {
  out += '"';
  for (size_t i = 0; i < raw.size();) {
    const uint8_t c = (uint8_t)raw[i];
    uint32_t cp = c;
    size_t len = 1;
    if (c >= 0x80) {
      len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
      if (c < 0xC2 || c > 0xF4 || i + len > raw.size()) return false;
      cp = c & (0x7Fu >> len);
      for (size_t k = 1; k < len; k++) {
        const uint8_t t = (uint8_t)raw[i + k];
        if ((t & 0xC0) != 0x80) return false;
        cp = (cp << 6) | (t & 0x3Fu);
      }
    }
    switch (cp) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case 0: out += "\\0"; break;
      default:
        if (fsg_u_dbg_escaped(cp)) {
          char u[16];
          snprintf(u, sizeof u, "\\u{%x}", cp);
          out += u;
        } else {
          out.append(raw, i, len);
        }
    }
    i += len;
  }
  out += '"';
  return true;
}

}  // namespace fsg
