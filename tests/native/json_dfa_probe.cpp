// Host restatement of the lean filter_json decision (fsg_kernels.hip
// lean_json_stage) for one value, over the same token DFA (fsg_json_dfa.h).
// TEST INFRASTRUCTURE: lets the CPU suite check that whatever the DFA accepts,
// the serde_json restatement (oracle) accepts with the same level.
#include <cstddef>
#include <cstdint>
#include <vector>

#include "fsg_json_dfa.h"

using namespace fsg;

static uint32_t str_class(const uint8_t* s, uint32_t a, uint32_t n) {
  auto eq = [&](const char* t, uint32_t tn) {
    if (n != tn) return false;
    for (uint32_t k = 0; k < n; k++)
      if (s[a + k] != (uint8_t)t[k]) return false;
    return true;
  };
  return eq("level", 5) ? JC_Q_LEVEL : eq("message", 7) ? JC_Q_MSG : eq("debug", 5) ? JC_Q_DEBUG
       : eq("info", 4) ? JC_Q_INFO : eq("warn", 4) ? JC_Q_WARN : eq("error", 5) ? JC_Q_ERROR : JC_Q_OTHER;
}

// 1 accepted (*level), 0 not decided by the fast path
extern "C" int json_dfa_probe(const uint8_t* s, size_t n, int* level) {
  struct Tok { uint32_t pos, cls; };
  std::vector<Tok> toks;
  bool instr = false;
  for (uint32_t p = 0; p < n; p++) {
    const uint8_t b = s[p];
    const bool special = b < 0x20 || b == '\\' || b >= 0x80;
    if (b == '"') {
      toks.push_back({p, instr ? (uint32_t)JC_Q_CLOSE : (uint32_t)JC_Q_OTHER});
      instr = !instr;
    } else if (special || (!instr && b != ' ')) {
      toks.push_back({p, kJsonDfa.bcls[b]});
    }
  }
  if (instr) return 0;  // the record ends inside a string
  for (size_t t = 0; t + 1 < toks.size(); t++)
    if (toks[t].cls == JC_Q_OTHER && toks[t + 1].cls == JC_Q_CLOSE)
      toks[t].cls = str_class(s, toks[t].pos + 1, toks[t + 1].pos - toks[t].pos - 1);
  uint32_t st = JS_OBJ, prev = 0xFFFFFFFFu, flags = 0;
  int lvl = -1;
  for (const Tok& tk : toks) {
    const uint32_t adj = tk.pos == prev + 1 ? 1u : 0u;
    prev = tk.pos;
    if (st >= JS_INV_D && st <= JS_INV_E) lvl = (int)(st - JS_INV_D);
    st = kJsonDfa.t[st * kJsonCls2 + tk.cls * 2 + adj];
    const uint32_t fb = st == JS_INKEY_LV ? 1u : st == JS_INKEY_MSG ? 2u : 0u;
    if (flags & fb) st = JS_FAIL;
    flags |= fb;
  }
  if (st != JS_END || flags != 3u) return 0;
  *level = lvl;
  return 1;
}
