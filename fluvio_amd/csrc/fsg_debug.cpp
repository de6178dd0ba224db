// fsg_debug.cpp — host-only hooks for unit-testing chain-build-time compilers
// on machines without a GPU (the regex -> DFA compiler).  Not part of the data
// path: no record of a process call ever goes through these.
#include <cstring>
#include <string>

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
  *is_match = fsg::dfa_is_match(ascii ? a : d, text, n) ? 1 : 0;
  if (!ascii && a.unicode_word) return -103;
  if (max_len) *max_len = a.max_len;
  if (nstates) *nstates = (int)d.nstates;
  return 0;
}
