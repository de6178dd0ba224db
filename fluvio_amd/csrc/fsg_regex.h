// fsg_regex.h — Rust-regex subset -> UTF-8 byte DFA (chain-build time)
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fsg {

struct Dfa {
  uint32_t nstates = 0, nclasses = 0, s_bot = 0, s_mid = 0;
  int32_t max_len = -1;  // longest match in bytes, -1 unbounded
  bool unicode_word = false;
  // the full DFA of a pattern with Unicode \b / \B runs over the value's bytes
  // with a marker before every code point (kMarkWord / kMarkOther / kMarkNl:
  // bytes that never occur in UTF-8) carrying that code point's word-ness, so
  // the boundaries are decided between code points (dfa_is_match_marked)
  bool marked = false;
  // utab: the pattern uses version-dependent Unicode tables (\d \w \p, (?i)
  // folding, Unicode \b): a value holding a fsg_u_newer code point is FSG_E_UNSUPPORTED
  bool utab = false;
  std::vector<uint8_t> classmap, classmap_up, accept;
  std::vector<uint16_t> trans;
};

// Two DFAs of one pattern: `ascii` with every class restricted to ASCII (exact
// on ASCII-only values; <= 255 states, staged in LDS) and `full` over all of
// Unicode (<= 65535 states, read through L1/L2 for values with non-ASCII bytes).
// 0 ok; -2 (FSG_E_INIT) syntax error; -103 (FSG_E_UNSUPPORTED) outside the supported subset
int compile_regex(const std::string& pattern, Dfa& ascii, Dfa& full, std::string& msg);
// regex-syntax's error Display for a span [lo, hi) of code points of the pattern
std::string syntax_error_text(const std::vector<uint32_t>& p, size_t lo, size_t hi, const char* kind);
constexpr uint8_t kMarkWord = 0xFC, kMarkOther = 0xFD, kMarkNl = 0xFE;
// host walk of the compiled DFA — used only by the compiler's unit tests
bool dfa_is_match(const Dfa& d, const uint8_t* s, size_t n);
// the marked walk over valid UTF-8 (isword: regex-syntax's Unicode \w)
bool dfa_is_match_marked(const Dfa& d, const uint8_t* s, size_t n);
// regex-syntax's Unicode \w as (lo, hi) pairs (the marked walk's table on the device)
std::vector<uint32_t> unicode_word_ranges();
// the version-uncertain code points (fsg_unicode.h fsg_u_newer) as (lo, hi) pairs
std::vector<uint32_t> unicode_newer_ranges();
// a code point of the valid UTF-8 text in those ranges
bool utf8_has_newer(const uint8_t* s, size_t n);
// <str as Debug>::fmt of Rust 1.75 (serde's "invalid type: string \"..\""):
// \0 \t \r \n \\ \" escaped, Grapheme_Extend and non-printable chars as
// \u{hex} (this image's Unicode 13 categories; parity unpinned for code points
// assigned later); false when `raw` is not UTF-8
bool rust_str_debug(const std::string& raw, std::string& out);

}  // namespace fsg
