// fsg_debug.cpp — host-only hooks for unit-testing on machines without a GPU:
// the chain-build-time regex -> DFA compiler and the JSON float arithmetic the
// kernels share with the host (fsg_float.h).  Not part of the data path: no
// record of a process call ever goes through these.
#include <algorithm>
#include <cstring>
#include <string>

#include "fsg_float.h"
#include "fsg_regex.h"

extern "C" int fsg_debug_regex_match(const char* pattern, const uint8_t* text, size_t n, int* is_match,
                                     int* max_len, int* nstates) {
  fsg::Dfa a, d;
  std::string msg;
  int rc = fsg::compile_regex(pattern, a, d, msg);
  if (rc) return rc;
  bool ascii = true;
  for (size_t i = 0; i < n; i++) ascii &= text[i] < 0x80;
  // the kernel's choice: ASCII DFA for ASCII-only values, full DFA otherwise
  // (the marked walk for Unicode word boundaries)
  if (!ascii && a.unicode_word && !d.marked) return -103;
  if (!ascii && d.utab && fsg::utf8_has_newer(text, n)) return -103;  // k_eval's version check
  *is_match = (ascii ? fsg::dfa_is_match(a, text, n) : d.marked ? fsg::dfa_is_match_marked(d, text, n)
                                                                : fsg::dfa_is_match(d, text, n)) ? 1 : 0;
  if (max_len) *max_len = a.max_len;
  if (nstates) *nstates = (int)d.nstates;
  return 0;
}

// the chain-build message of a pattern (compile_regex's msg: the init error
// text for FSG_E_INIT); returns compile_regex's code, msg NUL-terminated in cap
extern "C" int fsg_debug_regex_error(const char* pattern, char* msg, size_t cap) {
  fsg::Dfa a, d;
  std::string m;
  const int rc = fsg::compile_regex(pattern, a, d, m);
  if (cap) {
    const size_t k = std::min(cap - 1, m.size());
    memcpy(msg, m.data(), k);
    msg[k] = 0;
  }
  return rc;
}

// serde_json's reading of the JSON number text[0..n) (fsg_float.h num_value):
// returns kind (0 integer, 1 f64, 2 out of range); *bits = the f64's bits;
// ryu[0..*ryu_len) = Value::to_string of it, disp[0..*disp_len) = Rust Display
// with serde's WithDecimalPoint (buffers of 400 bytes); *err = range error index
extern "C" int fsg_debug_json_number(const uint8_t* text, uint32_t n, uint64_t* bits, uint8_t* ryu, uint32_t* ryu_len,
                                     uint8_t* disp, uint32_t* disp_len, uint32_t* err) {
  auto at = [&](uint32_t k) -> int { return k < n ? text[k] : -1; };
  const fsg::flt::NumVal v = fsg::flt::num_value(at, 0, n);
  *err = v.err;
  if (v.kind == 1) {
    memcpy(bits, &v.f, 8);
    *ryu_len = fsg::flt::ryu_format(v.f, ryu);
    *disp_len = fsg::flt::display_with_point(v.f, disp);
  }
  return v.kind;
}
