// Device restatement of serde_json 1.0.96 `from_slice::<StructuredLog>` — the
// filter of smartmodule/examples/filter_json/src/lib.rs:54-70 (LogLevel enum
// debug < info < warn < error, rename_all lowercase; `message: String`; other
// keys ignored).  One thread parses one record value.
//
// The routine structure follows serde_json (deserialize_struct, MapAccess,
// SeqAccess, deserialize_enum, deserialize_str, peek_invalid_type,
// ignore_value, SliceRead::parse_str / ignore_str) because the error position
// ("at line L column C") depends on which routine detects an error and how far
// the reader has advanced at that moment.  Strings are scanned four bytes per
// step while they hold no '"', '\\', control byte or non-ASCII byte.
//
// Output: JRes {ok, level} or an error descriptor {code, sub, pos, a, b}; the
// host renders the Display text from it (fsg_runtime.cpp json_hint).
#pragma once
#include <cstdint>

#include "fsg_device.h"
#include "fsg_float.h"

namespace fsg {

// serde_json ErrorCode (syntax errors carry a reader position)
enum JsonErr : uint8_t {
  JE_NONE = 0,
  JE_EOF_LIST, JE_EOF_OBJECT, JE_EOF_STRING, JE_EOF_VALUE, JE_COLON, JE_LIST_COMMA, JE_OBJ_COMMA, JE_IDENT,
  JE_VALUE, JE_ESCAPE, JE_NUMBER, JE_CODEPOINT, JE_CONTROL, JE_KEY, JE_SURROGATE, JE_TRAILING_COMMA,
  JE_TRAILING, JE_HEX_END, JE_RECURSION,
  // serde custom errors (position fixed by serde_json's fix_position)
  JE_DUP_FIELD,        // a = field index
  JE_MISSING_FIELD,    // a = field index
  JE_INVALID_LENGTH,   // a = elements seen
  JE_UNKNOWN_VARIANT,  // [a, b) = raw string content (between the quotes)
  JE_INVALID_TYPE,     // sub = unexpected kind | expected kind << 4; a, b = span (number digits / string)
  JE_DEEP,             // ignored value nested deeper than the device frame stack (outside the restatement)
  JE_UNSUP,            // valid input outside the device restatement (array_map: floats, unsorted keys)
  JE_INVALID_VALUE,    // u32 visitor: sub = JU_UINT / JU_NINT, [a, b) = the digits ("invalid value: integer `N`, expected u32")
  JE_RANGE,            // "number out of range" (f64_from_parts / parse_exponent_overflow), at pos
};
enum JsonUnexp : uint8_t { JU_UNIT = 0, JU_TRUE, JU_FALSE, JU_UINT, JU_NINT, JU_FLOAT, JU_STR, JU_SEQ, JU_MAP };
enum JsonExp : uint8_t { JX_STRUCT = 0, JX_STRING, JX_VARIANT, JX_UNIT, JX_SEQ, JX_MAP, JX_U32 };

struct JRes {
  uint8_t ok;
  uint8_t level;
  uint8_t code;
  uint8_t sub;
  uint32_t pos;  // reader index the position is computed from
  uint32_t a, b;
};

// serde_json::to_string of a validated JSON value (Value: objects are
// BTreeMap<String, Value>), from its source text s[0..n): whitespace dropped,
// strings re-escaped (ser.rs format_escaped_str: \" \\ \b \t \n \f \r, other
// control bytes \u00xx, the rest raw), numbers as serde_json reads them (u64 /
// i64 keep their text, f64 through ryu), object members in key-byte order with
// a repeated key keeping its last value (Map::insert).  Members are picked by
// selection — the smallest key above the one emitted last — so no member list
// is stored; one frame per open container.  o == nullptr counts only.
// Returns the length, or ~0u past kCanonFrames nesting levels.  One lane; the
// rare path (elements whose canonical text differs from their source text).
constexpr uint32_t kCanonFrames = 128;  // serde_json's recursion limit bounds the depth
template <typename P>
struct JsonCanon {
  P s;
  uint32_t n;
  bool upper;
  uint8_t* o;
  uint32_t w;
  __device__ __forceinline__ uint32_t at(uint32_t k) const {
    uint8_t c = s[k];
    if (upper && c >= 'a' && c <= 'z') c -= 32;
    return c;
  }
  __device__ __forceinline__ void put(uint32_t c) {
    if (o) o[w] = (uint8_t)c;
    w++;
  }
  static __device__ __forceinline__ uint32_t hexv(uint32_t c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }
  __device__ __forceinline__ uint32_t ws(uint32_t p) const {
    while (p < n) {
      const uint32_t c = at(p);
      if (c != ' ' && c != '\n' && c != '\t' && c != '\r') break;
      p++;
    }
    return p;
  }
  // one decoded code point of a validated string at p (p past the escape / bytes)
  __device__ __forceinline__ uint32_t str_cp(uint32_t& p, uint32_t* nb) const {
    uint32_t c = at(p++);
    if (c != '\\') {
      *nb = 1;  // raw byte (UTF-8 passes through byte by byte)
      return c;
    }
    const uint32_t e = at(p++);
    *nb = 0;
    switch (e) {
      case 'b': return 0x08;
      case 'f': return 0x0C;
      case 'n': return 0x0A;
      case 'r': return 0x0D;
      case 't': return 0x09;
      case 'u': {
        uint32_t cp = (hexv(at(p)) << 12) | (hexv(at(p + 1)) << 8) | (hexv(at(p + 2)) << 4) | hexv(at(p + 3));
        p += 4;
        if (cp >= 0xD800 && cp <= 0xDBFF) {  // validated pair
          const uint32_t c2 = (hexv(at(p + 2)) << 12) | (hexv(at(p + 3)) << 8) | (hexv(at(p + 4)) << 4) | hexv(at(p + 5));
          p += 6;
          cp = (((cp - 0xD800) << 10) | (c2 - 0xDC00)) + 0x10000;
        }
        return cp;
      }
      default: return e;  // " \ /
    }
  }
  // decoded key bytes one at a time (for the BTreeMap order)
  struct KeyIt {
    uint32_t p;
    uint8_t b[4];
    uint32_t nb, k;
  };
  __device__ __forceinline__ int key_next(KeyIt& it) const {  // -1 at the closing quote
    if (it.k < it.nb) return it.b[it.k++];
    if (at(it.p) == '"') return -1;
    uint32_t raw;
    const uint32_t cp = str_cp(it.p, &raw);
    if (raw || cp < 0x80) return (int)cp;
    it.k = 1;
    if (cp < 0x800) {
      it.nb = 2;
      it.b[0] = (uint8_t)(0xC0 | (cp >> 6));
      it.b[1] = (uint8_t)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      it.nb = 3;
      it.b[0] = (uint8_t)(0xE0 | (cp >> 12));
      it.b[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
      it.b[2] = (uint8_t)(0x80 | (cp & 0x3F));
    } else {
      it.nb = 4;
      it.b[0] = (uint8_t)(0xF0 | (cp >> 18));
      it.b[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
      it.b[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
      it.b[3] = (uint8_t)(0x80 | (cp & 0x3F));
    }
    return it.b[0];
  }
  // keys at a and b (positions after their opening quotes): <0, 0, >0
  __device__ int key_cmp(uint32_t a, uint32_t b) const {
    KeyIt x{a, {0, 0, 0, 0}, 0, 0}, y{b, {0, 0, 0, 0}, 0, 0};
    for (;;) {
      const int u = key_next(x), v = key_next(y);
      if (u != v) return u < v ? -1 : 1;  // -1 (end) sorts first
      if (u < 0) return 0;
    }
  }
  __device__ __forceinline__ uint32_t skip_str(uint32_t p) const {  // p after the opening quote -> past the closing one
    for (;;) {
      const uint32_t c = at(p++);
      if (c == '"') return p;
      if (c == '\\') p++;
    }
  }
  __device__ uint32_t skip_value(uint32_t p) const {  // validated value at p -> past it
    const uint32_t c = at(p);
    if (c == '"') return skip_str(p + 1);
    if (c == '[' || c == '{') {
      uint32_t d = 0;
      for (;;) {
        const uint32_t x = at(p++);
        if (x == '"') {
          p = skip_str(p);
        } else if (x == '[' || x == '{') {
          d++;
        } else if (x == ']' || x == '}') {
          if (--d == 0) return p;
        }
      }
    }
    while (p < n) {
      const uint32_t x = at(p);
      if (x == ',' || x == ']' || x == '}' || x == ' ' || x == '\n' || x == '\t' || x == '\r') break;
      p++;
    }
    return p;
  }
  __device__ void emit_str(uint32_t p) {  // p after the opening quote
    put('"');
    for (;;) {
      if (at(p) == '"') break;
      uint32_t raw;
      const uint32_t cp = str_cp(p, &raw);
      if (raw && cp >= 0x80) {
        put(cp);
        continue;
      }
      if (cp < 0x80) {
        switch (cp) {
          case '"': put('\\'); put('"'); break;
          case '\\': put('\\'); put('\\'); break;
          case 0x08: put('\\'); put('b'); break;
          case 0x09: put('\\'); put('t'); break;
          case 0x0A: put('\\'); put('n'); break;
          case 0x0C: put('\\'); put('f'); break;
          case 0x0D: put('\\'); put('r'); break;
          default:
            if (cp < 0x20) {
              const char* hx = "0123456789abcdef";
              put('\\'); put('u'); put('0'); put('0');
              put((uint8_t)hx[cp >> 4]);
              put((uint8_t)hx[cp & 15]);
            } else {
              put(cp);
            }
        }
      } else if (cp < 0x800) {
        put(0xC0 | (cp >> 6));
        put(0x80 | (cp & 0x3F));
      } else if (cp < 0x10000) {
        put(0xE0 | (cp >> 12));
        put(0x80 | ((cp >> 6) & 0x3F));
        put(0x80 | (cp & 0x3F));
      } else {
        put(0xF0 | (cp >> 18));
        put(0x80 | ((cp >> 12) & 0x3F));
        put(0x80 | ((cp >> 6) & 0x3F));
        put(0x80 | (cp & 0x3F));
      }
    }
    put('"');
  }
  // a scalar at p -> past it
  __device__ uint32_t emit_scalar(uint32_t p) {
    const uint32_t c = at(p);
    if (c == '"') {
      emit_str(p + 1);
      return skip_str(p + 1);
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
      auto acc = [&](uint32_t k) -> int { return k < n ? (int)at(k) : -1; };
      const flt::NumVal v = flt::num_value(acc, p, n);
      if (v.kind == 1) {
        w += flt::ryu_format(v.f, o ? o + w : nullptr);
      } else {
        for (uint32_t k = p; k < v.end; k++) put(at(k));
      }
      return v.end;
    }
    const uint32_t e = skip_value(p);  // true / false / null
    for (uint32_t k = p; k < e; k++) put(at(k));
    return e;
  }
  // the smallest member key above `last` (~0u: none yet) of the object whose
  // members start at p; *kp = key position, *vp = its last value; false: none left
  __device__ bool next_member(uint32_t p, uint32_t last, uint32_t* kp, uint32_t* vp) const {
    bool any = false;
    p = ws(p);
    while (at(p) != '}') {
      if (at(p) == ',') p = ws(p + 1);
      const uint32_t k = p + 1;
      p = ws(skip_str(k));  // ':'
      const uint32_t v = ws(p + 1);
      p = ws(skip_value(v));
      if (last != ~0u && key_cmp(k, last) <= 0) continue;
      const int c = any ? key_cmp(k, *kp) : -1;
      if (c <= 0) {  // smaller, or the same key again (a later insert replaces the value)
        *kp = k;
        *vp = v;
        any = true;
      }
    }
    return any;
  }
  __device__ uint32_t run() {
    uint32_t fpos[kCanonFrames], flast[kCanonFrames];  // '[': next element / 0|1 emitted; '{': first member / last key
    uint64_t fkind[kCanonFrames / 64] = {};            // bit = 1: '['
    uint32_t sn = 0;
    w = 0;
    uint32_t p = ws(0), vend = 0;
    bool value = true;  // a value at p is to be emitted
    for (;;) {
      if (value) {
        const uint32_t c = at(p);
        if (c == '[' || c == '{') {
          if (sn >= kCanonFrames) return ~0u;
          put(c);
          const uint64_t bit = 1ull << (sn & 63);
          if (c == '[') fkind[sn >> 6] |= bit; else fkind[sn >> 6] &= ~bit;
          fpos[sn] = p + 1;
          flast[sn] = c == '[' ? 0u : ~0u;
          sn++;
        } else {
          vend = emit_scalar(p);
          if (sn == 0) return w;
          if ((fkind[(sn - 1) >> 6] >> ((sn - 1) & 63)) & 1) fpos[sn - 1] = vend;
        }
        value = false;
        continue;
      }
      const uint32_t f = sn - 1;
      if ((fkind[f >> 6] >> (f & 63)) & 1) {  // '['
        uint32_t q = ws(fpos[f]);
        if (at(q) == ',') q = ws(q + 1);
        if (at(q) == ']') {
          put(']');
          vend = q + 1;
          sn--;
          if (sn == 0) return w;
          if ((fkind[(sn - 1) >> 6] >> ((sn - 1) & 63)) & 1) fpos[sn - 1] = vend;
          continue;
        }
        if (flast[f]) put(',');
        flast[f] = 1;
        p = q;
        value = true;
      } else {  // '{'
        uint32_t kp = 0, vp = 0;
        if (!next_member(fpos[f], flast[f], &kp, &vp)) {
          put('}');
          sn--;
          if (sn == 0) return w;
          if ((fkind[(sn - 1) >> 6] >> ((sn - 1) & 63)) & 1) fpos[sn - 1] = skip_value(fpos[f] - 1);
          continue;
        }
        if (flast[f] != ~0u) put(',');
        flast[f] = kp;
        emit_str(kp);
        put(':');
        p = vp;
        value = true;
      }
    }
  }
};
template <typename P>
__device__ __noinline__ uint32_t json_canon(P s, uint32_t n, bool upper, uint8_t* o) {
  JsonCanon<P> c;
  c.s = s;
  c.n = n;
  c.upper = upper;
  c.o = o;
  c.w = 0;
  return c.run();
}

constexpr uint32_t kJsonFrames = 256;  // ignore_value frame stack: four u64 words of bits ('[' = 1, '{' = 0)

template <typename P>
struct JsonDev {
  P s;
  uint32_t n;
  uint32_t i;
  bool upper;  // the stage input is the ASCII-uppercased value (a `map` ran before)
  int depth;
  bool failed;
  bool has_pos;
  JRes r;

  __device__ __forceinline__ int at(uint32_t k) const {
    uint8_t c = s[k];
    if (upper && c >= 'a' && c <= 'z') c -= 32;
    return c;
  }
  __device__ __forceinline__ int peek() const { return i < n ? at(i) : -1; }
  __device__ __forceinline__ void eat() { i++; }
  __device__ __forceinline__ int next() { return i < n ? at(i++) : -1; }

  __device__ __forceinline__ int fail_at(uint32_t idx, uint8_t code) {
    failed = true;
    has_pos = true;
    r.code = code;
    r.pos = idx;
    return -1;
  }
  __device__ __forceinline__ int error(uint8_t code) { return fail_at(i, code); }
  __device__ __forceinline__ int peek_error(uint8_t code) { return fail_at(i + 1 < n ? i + 1 : n, code); }
  __device__ __forceinline__ int custom(uint8_t code, uint32_t a, uint32_t b, uint8_t sub) {
    failed = true;
    has_pos = false;
    r.code = code;
    r.a = a;
    r.b = b;
    r.sub = sub;
    return -1;
  }
  __device__ __forceinline__ void fix_position() {
    if (failed && !has_pos) {
      has_pos = true;
      r.pos = i;
    }
  }

  __device__ __forceinline__ int ws() {
    for (;;) {
      const int c = peek();
      if (c == ' ' || c == '\n' || c == '\t' || c == '\r')
        eat();
      else
        return c;
    }
  }
  __device__ __forceinline__ int ident(const char* id, int len) {
    for (int k = 0; k < len; k++) {
      const int c = next();
      if (c < 0) return error(JE_EOF_VALUE);
      if (c != id[k]) return error(JE_IDENT);
    }
    return 0;
  }

  // ---- strings
  static __device__ __forceinline__ bool esc(int c) { return c == '"' || c == '\\' || (c >= 0 && c < 0x20); }
  static __device__ __forceinline__ int hexv(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  __device__ __forceinline__ int hex4(uint32_t* out) {
    if (i + 4 > n) {
      i = n;
      return error(JE_EOF_STRING);
    }
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      const int h = hexv(at(i));
      i++;
      if (h < 0) return error(JE_ESCAPE);
      v = (v << 4) + (uint32_t)h;
    }
    *out = v;
    return 0;
  }
  // skip a run of plain bytes: 4 at a time while no escape/control/quote and
  // (when `ascii`) no byte >= 0x80; returns with i at the first byte that needs
  // individual treatment (or n)
  __device__ __forceinline__ void skip_plain(bool ascii) {
    while (i + 4 <= n) {
      const uint32_t w = (uint32_t)at(i) | ((uint32_t)at(i + 1) << 8) | ((uint32_t)at(i + 2) << 16) |
                         ((uint32_t)at(i + 3) << 24);
      // bytes == '"' (0x22), '\\' (0x5C), < 0x20, or >= 0x80 (when ascii)
      const uint32_t q = w ^ 0x22222222u, bs = w ^ 0x5C5C5C5Cu;
      const uint32_t zq = (q - 0x01010101u) & ~q, zb = (bs - 0x01010101u) & ~bs;
      const uint32_t ctl = (w - 0x20202020u) & ~w;
      uint32_t hit = (zq | zb | ctl) & 0x80808080u;
      if (ascii) hit |= w & 0x80808080u;
      if (hit) break;
      i += 4;
    }
  }

  // incremental UTF-8 validation of decoded string bytes
  struct U8 {
    uint8_t need, lo, hi;
    bool bad;
  };
  static __device__ __forceinline__ void u8_feed(U8& u, uint32_t c) {
    if (u.bad) return;
    if (u.need) {
      if (c < u.lo || c > u.hi) {
        u.bad = true;
        return;
      }
      u.need--;
      u.lo = 0x80;
      u.hi = 0xBF;
      return;
    }
    if (c < 0x80) return;
    u.lo = 0x80;
    u.hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) {
      u.need = 1;
    } else if (c >= 0xE0 && c <= 0xEF) {
      u.need = 2;
      if (c == 0xE0) u.lo = 0xA0;
      if (c == 0xED) u.hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      u.need = 3;
      if (c == 0xF0) u.lo = 0x90;
      if (c == 0xF4) u.hi = 0x8F;
    } else {
      u.bad = true;
    }
  }
  // candidate-string matcher over the decoded bytes (keys / enum variants):
  // up to 4 candidates of <= 8 bytes packed little-endian in u64 registers
  struct Match {
    uint64_t c[4];
    uint32_t l[4];
    uint32_t alive;  // bit per candidate
    uint32_t len;    // decoded length so far
  };
  static __device__ __forceinline__ void m_feed(Match& m, uint32_t c) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const bool ok = m.len < m.l[k] && ((m.c[k] >> (8 * (m.len & 7))) & 0xFF) == c;
      if (!ok) m.alive &= ~(1u << k);
    }
    m.len++;
  }
  __device__ __forceinline__ int m_hit(const Match& m) const {
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (((m.alive >> k) & 1) && m.l[k] == m.len) return k;
    return -1;
  }
  static __device__ __forceinline__ void feed(U8& u, Match* m, uint32_t c) {
    u8_feed(u, c);
    if (m) m_feed(*m, c);
  }
  static __device__ __forceinline__ void feed_cp(U8& u, Match* m, uint32_t c) {
    if (c < 0x80) {
      feed(u, m, c);
    } else if (c < 0x800) {
      feed(u, m, 0xC0 | (c >> 6));
      feed(u, m, 0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      feed(u, m, 0xE0 | (c >> 12));
      feed(u, m, 0x80 | ((c >> 6) & 0x3F));
      feed(u, m, 0x80 | (c & 0x3F));
    } else {
      feed(u, m, 0xF0 | (c >> 18));
      feed(u, m, 0x80 | ((c >> 12) & 0x3F));
      feed(u, m, 0x80 | ((c >> 6) & 0x3F));
      feed(u, m, 0x80 | (c & 0x3F));
    }
  }
  // read.rs parse_escape (validate = true)
  __device__ __forceinline__ int escape(U8& u, Match* m) {
    const int ch = next();
    if (ch < 0) return error(JE_EOF_STRING);
    switch (ch) {
      case '"': feed(u, m, '"'); return 0;
      case '\\': feed(u, m, '\\'); return 0;
      case '/': feed(u, m, '/'); return 0;
      case 'b': feed(u, m, 0x08); return 0;
      case 'f': feed(u, m, 0x0c); return 0;
      case 'n': feed(u, m, '\n'); return 0;
      case 'r': feed(u, m, '\r'); return 0;
      case 't': feed(u, m, '\t'); return 0;
      case 'u': {
        uint32_t n1;
        if (hex4(&n1)) return -1;
        if (n1 >= 0xDC00 && n1 <= 0xDFFF) return error(JE_SURROGATE);
        if (n1 >= 0xD800 && n1 <= 0xDBFF) {
          int p = peek();
          if (p < 0) return error(JE_EOF_STRING);
          if (p != '\\') {
            eat();
            return error(JE_HEX_END);
          }
          eat();
          p = peek();
          if (p < 0) return error(JE_EOF_STRING);
          if (p != 'u') {
            eat();
            return error(JE_HEX_END);
          }
          eat();
          uint32_t n2;
          if (hex4(&n2)) return -1;
          if (n2 < 0xDC00 || n2 > 0xDFFF) return error(JE_SURROGATE);
          feed_cp(u, m, (((n1 - 0xD800) << 10) | (n2 - 0xDC00)) + 0x10000);
          return 0;
        }
        feed_cp(u, m, n1);
        return 0;
      }
      default: return error(JE_ESCAPE);
    }
  }
  // SliceRead::parse_str after the opening quote; [*b0, *b1) = raw content span
  __device__ __forceinline__ int parse_str(Match* m, uint32_t* b0, uint32_t* b1) {
    U8 u = {0, 0x80, 0xBF, false};
    *b0 = i;
    for (;;) {
      if (!m || !m->alive) skip_plain(true);
      if (i >= n) return error(JE_EOF_STRING);
      const int c = at(i);
      if (c == '"') {
        *b1 = i;
        i++;
        if (u.bad || u.need) return error(JE_CODEPOINT);
        return 0;
      } else if (c == '\\') {
        i++;
        if (escape(u, m)) return -1;
      } else if (c < 0x20) {
        i++;
        return error(JE_CONTROL);
      } else {
        i++;
        feed(u, m, (uint32_t)c);
      }
    }
  }
  __device__ __forceinline__ int ignore_escape() {
    const int ch = next();
    if (ch < 0) return error(JE_EOF_STRING);
    switch (ch) {
      case '"': case '\\': case '/': case 'b': case 'f': case 'n': case 'r': case 't': return 0;
      case 'u': {
        uint32_t v;
        return hex4(&v);
      }
      default: return error(JE_ESCAPE);
    }
  }
  __device__ __forceinline__ int ignore_str() {
    for (;;) {
      skip_plain(false);
      if (i >= n) return error(JE_EOF_STRING);
      const int c = at(i);
      if (c == '"') {
        i++;
        return 0;
      } else if (c == '\\') {
        i++;
        if (ignore_escape()) return -1;
      } else if (c < 0x20) {
        return error(JE_CONTROL);
      } else {
        i++;
      }
    }
  }

  // ---- numbers
  __device__ __forceinline__ int pnull() const { const int c = peek(); return c < 0 ? 0 : c; }
  static __device__ __forceinline__ bool dig(int c) { return c >= '0' && c <= '9'; }
  __device__ __forceinline__ int ignore_exponent() {
    eat();
    const int c = pnull();
    if (c == '+' || c == '-') eat();
    if (!dig(next())) return error(JE_NUMBER);
    while (dig(pnull())) eat();
    return 0;
  }
  __device__ __forceinline__ int ignore_decimal() {
    eat();
    bool any = false;
    while (dig(pnull())) {
      eat();
      any = true;
    }
    if (!any) return peek_error(JE_NUMBER);
    const int c = pnull();
    if (c == 'e' || c == 'E') return ignore_exponent();
    return 0;
  }
  __device__ __forceinline__ int ignore_integer() {
    const int c = next();
    if (c == '0') {
      if (dig(pnull())) return peek_error(JE_NUMBER);
    } else if (c >= '1' && c <= '9') {
      while (dig(pnull())) eat();
    } else {
      return error(JE_NUMBER);
    }
    const int d = pnull();
    if (d == '.') return ignore_decimal();
    if (d == 'e' || d == 'E') return ignore_exponent();
    return 0;
  }
  __device__ __forceinline__ int exponent_syn() {
    eat();
    const int c = pnull();
    if (c == '+' || c == '-') eat();
    const int nx = next();
    if (nx < 0) return error(JE_EOF_VALUE);
    if (!dig(nx)) return error(JE_NUMBER);
    while (dig(pnull())) eat();
    return 0;
  }
  __device__ __forceinline__ int decimal_syn() {
    eat();
    bool any = false;
    while (dig(pnull())) {
      eat();
      any = true;
    }
    if (!any) return peek() >= 0 ? peek_error(JE_NUMBER) : peek_error(JE_EOF_VALUE);
    const int c = pnull();
    if (c == 'e' || c == 'E') return exponent_syn();
    return 0;
  }
  // parse_integer + parse_number syntax; *kind = JU_UINT / JU_NINT / JU_FLOAT.
  // A float's value is read as serde_json reads it (fsg_float.h num_value):
  // where f64_from_parts / parse_exponent_overflow fail, "number out of range".
  __device__ __forceinline__ int parse_integer(bool positive, uint8_t* kind) {
    const uint32_t st = positive ? i : i - 1;  // the '-' was eaten by the caller
    const int c = next();
    if (c < 0) return error(JE_EOF_VALUE);
    uint64_t sig = 0;
    bool flt = false, longi = false;
    if (c == '0') {
      if (dig(pnull())) return peek_error(JE_NUMBER);
    } else if (c >= '1' && c <= '9') {
      sig = (uint64_t)(c - '0');
      for (;;) {
        const int p = pnull();
        if (!dig(p)) break;
        const uint64_t dg = (uint64_t)(p - '0');
        if (sig > (~0ull - dg) / 10) {  // parse_long_integer
          while (dig(pnull())) eat();
          flt = longi = true;
          break;
        }
        eat();
        sig = sig * 10 + dg;
      }
    } else {
      return error(JE_NUMBER);
    }
    const int t = pnull();
    if (t == '.') {
      flt = true;
      if (decimal_syn()) return -1;
    } else if (t == 'e' || t == 'E') {
      flt = true;
      if (exponent_syn()) return -1;
    }
    if (!longi && !positive && (sig == 0 || sig > 0x8000000000000000ull)) flt = true;  // -0 / below i64::MIN -> f64
    *kind = flt ? JU_FLOAT : (positive ? JU_UINT : JU_NINT);
    if (flt) {
      auto acc = [&](uint32_t k) -> int { return k < n ? at(k) : -1; };
      const flt::NumVal v = flt::num_value(acc, st, n);
      if (v.kind == 2) return fail_at(v.err, JE_RANGE);
    }
    return 0;
  }

  // de.rs peek_invalid_type (expected kind `ex`)
  __device__ __forceinline__ int invalid_type(uint8_t ex) {
    int c = peek();
    if (c < 0) c = 0;
    uint8_t un;
    uint32_t a = 0, b = 0;
    switch (c) {
      case 'n':
        eat();
        if (ident("ull", 3)) return -1;
        un = JU_UNIT;
        break;
      case 't':
        eat();
        if (ident("rue", 3)) return -1;
        un = JU_TRUE;
        break;
      case 'f':
        eat();
        if (ident("alse", 4)) return -1;
        un = JU_FALSE;
        break;
      case '-':
      case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8': case '9': {
        const bool pos = c != '-';
        if (!pos) eat();
        a = i;
        if (parse_integer(pos, &un)) return -1;
        b = i;
        break;
      }
      case '"': {
        eat();
        if (parse_str(nullptr, &a, &b)) return -1;
        un = JU_STR;
        break;
      }
      case '[': un = JU_SEQ; break;
      case '{': un = JU_MAP; break;
      default: return peek_error(JE_VALUE);
    }
    custom(JE_INVALID_TYPE, a, b, (uint8_t)(un | (ex << 4)));
    fix_position();
    return -1;
  }

  // de.rs ignore_value (frames as a bit stack: 1 = '[', 0 = '{'; serde keeps
  // them in a Vec with no limit, here 256 levels in four words selected by
  // value, not by an indexed array, so they stay in registers)
  __device__ __forceinline__ int ignore_value() {
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    uint32_t sn = 0;
    auto top = [&](uint32_t n) -> int {
      const uint32_t w = n >> 6;
      const uint64_t x = w == 0 ? s0 : w == 1 ? s1 : w == 2 ? s2 : s3;
      return ((x >> (n & 63)) & 1) ? '[' : '{';
    };
    int enclosing = 0;
    for (;;) {
      const int peek_c = ws();
      if (peek_c < 0) return peek_error(JE_EOF_VALUE);
      int frame = 0;
      switch (peek_c) {
        case 'n': eat(); if (ident("ull", 3)) return -1; break;
        case 't': eat(); if (ident("rue", 3)) return -1; break;
        case 'f': eat(); if (ident("alse", 4)) return -1; break;
        case '-': eat(); if (ignore_integer()) return -1; break;
        case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8': case '9':
          if (ignore_integer()) return -1;
          break;
        case '"': eat(); if (ignore_str()) return -1; break;
        case '[':
        case '{':
          if (enclosing) {
            if (sn >= kJsonFrames) return fail_at(i, JE_DEEP);
            const uint64_t bit = 1ull << (sn & 63), set = enclosing == '[' ? bit : 0ull;
            const uint32_t w = sn >> 6;
            s0 = w == 0 ? (s0 & ~bit) | set : s0;
            s1 = w == 1 ? (s1 & ~bit) | set : s1;
            s2 = w == 2 ? (s2 & ~bit) | set : s2;
            s3 = w == 3 ? (s3 & ~bit) | set : s3;
            sn++;
          }
          enclosing = 0;
          eat();
          frame = peek_c;
          break;
        default: return peek_error(JE_VALUE);
      }
      bool accept_comma;
      if (frame) {
        accept_comma = false;
      } else if (enclosing) {
        frame = enclosing;
        enclosing = 0;
        accept_comma = true;
      } else if (sn) {
        sn--;
        frame = top(sn);
        accept_comma = true;
      } else {
        return 0;
      }
      for (;;) {
        const int c = ws();
        if (c == ',' && accept_comma) {
          eat();
          break;
        } else if ((c == ']' && frame == '[') || (c == '}' && frame == '{')) {
          // close the frame below
        } else if (c >= 0) {
          if (accept_comma) return peek_error(frame == '[' ? JE_LIST_COMMA : JE_OBJ_COMMA);
          break;
        } else {
          return peek_error(frame == '[' ? JE_EOF_LIST : JE_EOF_OBJECT);
        }
        eat();
        if (!sn) return 0;
        sn--;
        frame = top(sn);
        accept_comma = true;
      }
      if (frame == '{') {
        int c = ws();
        if (c == '"')
          eat();
        else if (c >= 0)
          return peek_error(JE_KEY);
        else
          return peek_error(JE_EOF_OBJECT);
        if (ignore_str()) return -1;
        c = ws();
        if (c == ':')
          eat();
        else if (c >= 0)
          return peek_error(JE_COLON);
        else
          return peek_error(JE_EOF_OBJECT);
      }
      enclosing = frame;
    }
  }

  // deserialize_str for the `message: String` field (expected "a string")
  __device__ __forceinline__ int de_string() {
    const int p = ws();
    if (p < 0) return peek_error(JE_EOF_VALUE);
    if (p == '"') {
      eat();
      uint32_t a, b;
      return parse_str(nullptr, &a, &b);
    }
    invalid_type(JX_STRING);
    fix_position();
    return -1;
  }
  // variant identifier of LogLevel (deserialize_identifier -> deserialize_str)
  __device__ __forceinline__ int variant(int* var) {
    const int p = ws();
    if (p < 0) return peek_error(JE_EOF_VALUE);
    if (p != '"') {
      invalid_type(JX_VARIANT);
      fix_position();
      return -1;
    }
    eat();
    // "debug", "info", "warn", "error" (little-endian packed)
    Match m = {{0x6775626564ull, 0x6f666e69ull, 0x6e726177ull, 0x726f727265ull}, {5, 4, 4, 5}, 0xFu, 0};
    uint32_t a, b;
    if (parse_str(&m, &a, &b)) return -1;
    const int k = m_hit(m);
    if (k >= 0) {
      *var = k;
      return 0;
    }
    custom(JE_UNKNOWN_VARIANT, a, b, 0);
    fix_position();
    return -1;
  }
  __device__ __forceinline__ int de_unit() {
    const int p = ws();
    if (p < 0) return peek_error(JE_EOF_VALUE);
    if (p == 'n') {
      eat();
      return ident("ull", 3);
    }
    invalid_type(JX_UNIT);
    fix_position();
    return -1;
  }
  __device__ __forceinline__ int de_enum(int* var) {
    const int p = ws();
    if (p == '{') {
      if (--depth == 0) return peek_error(JE_RECURSION);
      eat();
      if (variant(var)) return -1;
      int c = ws();
      if (c == ':')
        eat();
      else if (c >= 0)
        return peek_error(JE_COLON);
      else
        return peek_error(JE_EOF_OBJECT);
      if (de_unit()) return -1;
      depth++;
      c = ws();
      if (c == '}') {
        eat();
        return 0;
      }
      if (c >= 0) return error(JE_VALUE);
      return error(JE_EOF_OBJECT);
    }
    if (p == '"') return variant(var);
    if (p >= 0) return peek_error(JE_VALUE);
    return peek_error(JE_EOF_VALUE);
  }
  __device__ __forceinline__ int field_value(int f, int* level) { return f == 0 ? de_enum(level) : de_string(); }

  __device__ __forceinline__ int visit_map(int* level) {
    bool seen0 = false, seen1 = false, first = true;
    for (;;) {
      int p = ws();
      if (p == '}') break;
      if (p == ',' && !first) {
        eat();
        p = ws();
      } else if (p >= 0) {
        if (first)
          first = false;
        else
          return peek_error(JE_OBJ_COMMA);
      } else {
        return peek_error(JE_EOF_OBJECT);
      }
      if (p == '}') return peek_error(JE_TRAILING_COMMA);
      if (p < 0) return peek_error(JE_EOF_VALUE);
      if (p != '"') return peek_error(JE_KEY);
      eat();
      // "level", "message"
      Match m = {{0x6c6576656cull, 0x6567617373656dull, 0, 0}, {5, 7, 0, 0}, 3u, 0};
      uint32_t a, b;
      if (parse_str(&m, &a, &b)) return -1;
      const int f = m_hit(m);
      if (f == 0 && seen0) return custom(JE_DUP_FIELD, 0, 0, 0);
      if (f == 1 && seen1) return custom(JE_DUP_FIELD, 1, 0, 0);
      const int c = ws();
      if (c == ':')
        eat();
      else if (c >= 0)
        return peek_error(JE_COLON);
      else
        return peek_error(JE_EOF_OBJECT);
      if (f < 0) {
        if (ignore_value()) return -1;
      } else {
        if (field_value(f, level)) return -1;
        if (f == 0)
          seen0 = true;
        else
          seen1 = true;
      }
    }
    if (!seen0) return custom(JE_MISSING_FIELD, 0, 0, 0);
    if (!seen1) return custom(JE_MISSING_FIELD, 1, 0, 0);
    return 0;
  }
  __device__ __forceinline__ int visit_seq(int* level) {
    bool first = true;
    for (int k = 0; k < 2; k++) {
      int p = ws();
      if (p == ']') return custom(JE_INVALID_LENGTH, (uint32_t)k, 0, 0);
      if (p == ',' && !first) {
        eat();
        p = ws();
      } else if (p >= 0) {
        if (first)
          first = false;
        else
          return peek_error(JE_LIST_COMMA);
      } else {
        return peek_error(JE_EOF_LIST);
      }
      if (p == ']') return peek_error(JE_TRAILING_COMMA);
      if (p < 0) return peek_error(JE_EOF_VALUE);
      if (field_value(k, level)) return -1;
    }
    return 0;
  }
  __device__ __forceinline__ int end_map() {
    const int c = ws();
    if (c == '}') {
      eat();
      return 0;
    }
    if (c == ',') return peek_error(JE_TRAILING_COMMA);
    if (c >= 0) return peek_error(JE_TRAILING);
    return peek_error(JE_EOF_OBJECT);
  }
  __device__ __forceinline__ int end_seq() {
    const int c = ws();
    if (c == ']') {
      eat();
      return 0;
    }
    if (c == ',') {
      eat();
      const int p = ws();
      if (p == ']') return peek_error(JE_TRAILING_COMMA);
      return peek_error(JE_TRAILING);
    }
    if (c >= 0) return peek_error(JE_TRAILING);
    return peek_error(JE_EOF_LIST);
  }
  // the end check after a failed visitor only moves the reader
  __device__ __forceinline__ void end_probe(bool seq) {
    const bool f0 = failed, h0 = has_pos;
    const JRes r0 = r;
    failed = false;
    if (seq)
      end_seq();
    else
      end_map();
    failed = f0;
    has_pos = h0;
    r = r0;
  }
  __device__ __forceinline__ int de_struct(int* level) {
    const int p = ws();
    if (p < 0) return peek_error(JE_EOF_VALUE);
    int rc;
    if (p == '[' || p == '{') {
      if (--depth == 0) return peek_error(JE_RECURSION);
      eat();
      rc = p == '[' ? visit_seq(level) : visit_map(level);
      depth++;
      if (rc)
        end_probe(p == '[');
      else
        rc = p == '[' ? end_seq() : end_map();
    } else {
      invalid_type(JX_STRUCT);
      rc = -1;
    }
    if (rc) fix_position();
    return rc;
  }
  // ------------------------------------------------------------------------
  // array_map_json_array (smartmodule/examples/array_map_json_array/src/lib.rs:
  // 38-55): from_slice::<Vec<Value>> then to_string of every element.  The
  // parse follows de.rs deserialize_seq / SeqAccess / deserialize_any /
  // MapAccess / parse_object_colon; instead of building Values it records,
  // per element, its source span and the length of its canonical
  // serialization (ser.rs: compact, format_escaped_str, itoa, ryu).  An
  // element holding a float (serde_json reads fractions, exponents, -0 and
  // integers beyond u64/i64 as f64) or an object whose keys are not already
  // in BTreeMap order, and one whose text differs from its canonical text
  // (whitespace, escapes), is measured and written by json_canon in their own
  // kernels (k_canon_len, k_write_canon: the canonicalizer's frame stack and
  // bignums stay out of k_eval / k_write); a verbatim one is copied by k_write.
  // ------------------------------------------------------------------------
  uint32_t vcanon;  // canonical bytes of the element being parsed
  bool vhas_u;      // a \u escape was decoded (canonical form may differ in bytes)
  bool vhas_bs;     // the last string held a backslash
  bool vunsup;      // outside the device restatement: unsupported unless a later syntax error decides
  bool vcomplex;    // a float or an object out of key order: the canonical text comes from json_canon
  static __device__ __forceinline__ uint32_t canon_byte_len(uint32_t c) {
    if (c == '"' || c == '\\' || c == 0x08 || c == 0x09 || c == 0x0A || c == 0x0C || c == 0x0D) return 2;
    return c < 0x20 ? 6 : 1;
  }
  __device__ __forceinline__ void vfeed_cp(U8& u, uint32_t c) {
    feed_cp(u, nullptr, c);
    vcanon += c < 0x80 ? canon_byte_len(c) : c < 0x800 ? 2 : c < 0x10000 ? 3 : 4;
  }
  // read.rs parse_escape (validate = true) adding the canonical length
  __device__ __forceinline__ int vescape(U8& u) {
    const int ch = next();
    if (ch < 0) return error(JE_EOF_STRING);
    switch (ch) {
      case '"': vfeed_cp(u, '"'); return 0;
      case '\\': vfeed_cp(u, '\\'); return 0;
      case '/': vfeed_cp(u, '/'); return 0;
      case 'b': vfeed_cp(u, 0x08); return 0;
      case 'f': vfeed_cp(u, 0x0c); return 0;
      case 'n': vfeed_cp(u, '\n'); return 0;
      case 'r': vfeed_cp(u, '\r'); return 0;
      case 't': vfeed_cp(u, '\t'); return 0;
      case 'u': {
        vhas_u = true;
        uint32_t n1;
        if (hex4(&n1)) return -1;
        if (n1 >= 0xDC00 && n1 <= 0xDFFF) return error(JE_SURROGATE);
        if (n1 >= 0xD800 && n1 <= 0xDBFF) {
          int p = peek();
          if (p < 0) return error(JE_EOF_STRING);
          if (p != '\\') {
            eat();
            return error(JE_HEX_END);
          }
          eat();
          p = peek();
          if (p < 0) return error(JE_EOF_STRING);
          if (p != 'u') {
            eat();
            return error(JE_HEX_END);
          }
          eat();
          uint32_t n2;
          if (hex4(&n2)) return -1;
          if (n2 < 0xDC00 || n2 > 0xDFFF) return error(JE_SURROGATE);
          vfeed_cp(u, (((n1 - 0xD800) << 10) | (n2 - 0xDC00)) + 0x10000);
          return 0;
        }
        vfeed_cp(u, n1);
        return 0;
      }
      default: return error(JE_ESCAPE);
    }
  }
  // SliceRead::parse_str after the opening quote (validating), adding the
  // canonical length of the string (quotes included) to vcanon
  __device__ __forceinline__ int vstr() {
    U8 u = {0, 0x80, 0xBF, false};
    vcanon += 2;
    vhas_bs = false;
    for (;;) {
      const uint32_t i0 = i;
      skip_plain(true);
      vcanon += i - i0;
      if (i >= n) return error(JE_EOF_STRING);
      const int c = at(i);
      if (c == '"') {
        i++;
        if (u.bad || u.need) return error(JE_CODEPOINT);
        return 0;
      } else if (c == '\\') {
        i++;
        vhas_bs = true;
        if (vescape(u)) return -1;
      } else if (c < 0x20) {
        i++;
        return error(JE_CONTROL);
      } else {
        i++;
        feed(u, nullptr, (uint32_t)c);
        vcanon += 1;
      }
    }
  }
  // raw key compare (keys without escapes): <0, 0, >0
  __device__ __forceinline__ int key_cmp(uint32_t a0, uint32_t a1, uint32_t b0, uint32_t b1) const {
    const uint32_t la = a1 - a0, lb = b1 - b0, m = la < lb ? la : lb;
    for (uint32_t k = 0; k < m; k++) {
      const int x = at(a0 + k), y = at(b0 + k);
      if (x != y) return x - y;
    }
    return (int)la - (int)lb;
  }
  static constexpr int kKeyFrames = 8;  // objects checked for key order at these nesting levels
  // one Value (deserialize_any), iteratively over a 128-level frame bit stack
  __device__ int any_value() {
    uint64_t stk[2] = {0, 0};  // bit = 1: '[' frame, 0: '{' frame
    uint32_t sn = 0;
    uint32_t pk0[kKeyFrames], pk1[kKeyFrames];  // previous key (raw content span) per object level; pk1 = ~0: none
    bool first = false;
    int frame = 0;
    for (;;) {
      // ---- VALUE
      int c = ws();
      if (c < 0) return peek_error(JE_EOF_VALUE);
      switch (c) {
        case 'n': eat(); if (ident("ull", 3)) return -1; vcanon += 4; break;
        case 't': eat(); if (ident("rue", 3)) return -1; vcanon += 4; break;
        case 'f': eat(); if (ident("alse", 4)) return -1; vcanon += 5; break;
        case '-':
        case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8': case '9': {
          const uint32_t i0 = i;
          if (c == '-') eat();
          uint8_t kind;
          if (parse_integer(c != '-', &kind)) return -1;
          if (kind == JU_FLOAT) vcomplex = true;  // ryu's text
          vcanon += i - i0;  // an integer's canonical text is its source text (JSON has no + / leading 0)
          break;
        }
        case '"': eat(); if (vstr()) return -1; break;
        case '[':
        case '{': {
          if (--depth == 0) return peek_error(JE_RECURSION);
          eat();
          const uint64_t bit = 1ull << (sn & 63);
          if (c == '[') stk[sn >> 6] |= bit; else stk[sn >> 6] &= ~bit;
          if (c == '{' && sn < (uint32_t)kKeyFrames) pk1[sn] = 0xFFFFFFFFu;
          sn++;
          vcanon += 1;
          first = true;
          frame = c;
          goto next_member;
        }
        default: return peek_error(JE_VALUE);
      }
    after_value:
      if (sn == 0) return 0;
      frame = ((stk[(sn - 1) >> 6] >> ((sn - 1) & 63)) & 1) ? '[' : '{';
      first = false;
    next_member:
      c = ws();
      if ((frame == '[' && c == ']') || (frame == '{' && c == '}')) {
        eat();  // end_seq / end_map after the visitor saw the close
        depth++;
        vcanon += 1;
        sn--;
        goto after_value;
      }
      if (c == ',' && !first) {
        eat();
        c = ws();
        vcanon += 1;
      } else if (c >= 0) {
        if (!first) return peek_error(frame == '[' ? JE_LIST_COMMA : JE_OBJ_COMMA);
      } else {
        return peek_error(frame == '[' ? JE_EOF_LIST : JE_EOF_OBJECT);
      }
      const bool first_member = first;
      first = false;
      if (frame == '[') {
        if (c == ']') return peek_error(JE_TRAILING_COMMA);
        if (c < 0) return peek_error(JE_EOF_VALUE);
        continue;  // element value
      }
      if (c == '}') return peek_error(JE_TRAILING_COMMA);
      if (c < 0) return peek_error(JE_EOF_VALUE);
      if (c != '"') return peek_error(JE_KEY);
      eat();
      const uint32_t k0 = i;
      if (vstr()) return -1;
      const uint32_t k1 = i - 1;
      {  // BTreeMap order: keys must arrive strictly increasing (else re-sorting / dedup needed)
        const uint32_t lv = sn - 1;
        if (lv >= (uint32_t)kKeyFrames) {
          // deeper objects: only a single-member object is known to be in order
          if (!first_member) vcomplex = true;
        } else {
          if (pk1[lv] != 0xFFFFFFFFu) {
            const bool esc_prev = (pk0[lv] >> 31) != 0;
            if (esc_prev || vhas_bs || key_cmp(pk0[lv] & 0x7FFFFFFFu, pk1[lv], k0, k1) >= 0) vcomplex = true;
          }
          pk0[lv] = k0 | (vhas_bs ? 0x80000000u : 0u);
          pk1[lv] = k1;
        }
      }
      c = ws();  // parse_object_colon
      if (c == ':') {
        eat();
      } else if (c >= 0) {
        return peek_error(JE_COLON);
      } else {
        return peek_error(JE_EOF_OBJECT);
      }
      vcanon += 1;
    }
  }
  // from_slice::<Vec<Value>>: elements -> out[0..*count) (pos absolute, canonical
  // length, bit 31 = canonical bytes equal the source bytes)
  __device__ __forceinline__ JRes run_array(ElemRec* out, uint64_t abs0, uint32_t* count) {
    r = JRes{0, 0, 0, 0, 0, 0, 0};
    failed = false;
    has_pos = false;
    depth = 128;
    i = 0;
    vunsup = false;
    uint32_t k = 0;
    int rc = 0;
    int c = ws();
    if (c < 0) {
      rc = peek_error(JE_EOF_VALUE);
    } else if (c == '[') {
      --depth;  // 127: cannot reach 0
      eat();
      bool first = true;
      for (;;) {  // SeqAccess::next_element_seed
        int p = ws();
        if (p == ']') break;
        if (p == ',' && !first) {
          eat();
          p = ws();
        } else if (p >= 0) {
          if (!first) {
            rc = peek_error(JE_LIST_COMMA);
            break;
          }
          first = false;
        } else {
          rc = peek_error(JE_EOF_LIST);
          break;
        }
        if (p == ']') {
          rc = peek_error(JE_TRAILING_COMMA);
          break;
        }
        if (p < 0) {
          rc = peek_error(JE_EOF_VALUE);
          break;
        }
        const uint32_t e0 = i;
        vcanon = 0;
        vhas_u = false;
        vcomplex = false;
        if (any_value()) {
          rc = -1;
          break;
        }
        const uint32_t span = i - e0;
        if (vcomplex) vcanon = 0;  // floats / members out of key order: k_canon_len measures it
        const bool verb = span == vcanon && !vhas_u && !vcomplex;
        if (!verb) r.sub = 1;  // the batch has elements for k_canon_len / k_write_canon
        out[k].pos = abs0 + e0;
        out[k].src_len = span;
        out[k].out_len = vcanon | (verb ? 0x80000000u : 0u);
        k++;
      }
      depth++;
      if (!rc) rc = end_seq();
    } else {
      invalid_type(JX_SEQ);
      rc = -1;
    }
    if (rc) fix_position();
    if (!rc && ws() >= 0) rc = peek_error(JE_TRAILING);  // Deserializer::end
    // a valid document whose objects need re-ordering: outside the restatement
    if (!rc && vunsup) rc = fail_at(i, JE_UNSUP);
    *count = k;
    if (!rc) r.ok = 1;  // (r.sub on success: some element is not verbatim)
    return r;
  }

  // aggregate-json (examples/aggregate-json/src/lib.rs:22-36):
  // from_slice::<HashMap<String, u32>> (de.rs deserialize_map / MapAccess,
  // keys deserialize_string, values deserialize_number with the u32 visitor).
  // Entries (key content span, value) -> out[0..*count) in text order,
  // duplicates included (the aggregation keeps the last value of a key).
  // Keys with escapes and float values are JE_UNSUP.
  __device__ __forceinline__ JRes run_map_u32(ElemRec* out, uint64_t abs0, uint32_t* count) {
    r = JRes{0, 0, 0, 0, 0, 0, 0};
    failed = false;
    has_pos = false;
    depth = 128;
    i = 0;
    vunsup = false;
    uint32_t k = 0;
    int rc = 0;
    int c = ws();
    if (c < 0) {
      rc = peek_error(JE_EOF_VALUE);
    } else if (c == '{') {
      --depth;
      eat();
      bool first = true;
      for (;;) {
        int p = ws();
        if (p == '}') break;
        if (p == ',' && !first) {
          eat();
          p = ws();
        } else if (p >= 0) {
          if (!first) {
            rc = peek_error(JE_OBJ_COMMA);
            break;
          }
          first = false;
        } else {
          rc = peek_error(JE_EOF_OBJECT);
          break;
        }
        if (p == '}') {
          rc = peek_error(JE_TRAILING_COMMA);
          break;
        }
        if (p < 0) {
          rc = peek_error(JE_EOF_VALUE);
          break;
        }
        if (p != '"') {
          rc = peek_error(JE_KEY);
          break;
        }
        eat();
        const uint32_t k0 = i;
        vcanon = 0;
        if (vstr()) {
          rc = -1;
          break;
        }
        const uint32_t k1 = i - 1;
        if (vhas_bs) vunsup = true;  // the decoded key differs from its source bytes
        c = ws();  // parse_object_colon
        if (c == ':') {
          eat();
        } else if (c >= 0) {
          rc = peek_error(JE_COLON);
          break;
        } else {
          rc = peek_error(JE_EOF_OBJECT);
          break;
        }
        // deserialize_number -> PrimitiveVisitor<u32>
        const int q = ws();
        if (q < 0) {
          rc = peek_error(JE_EOF_VALUE);
          break;
        }
        uint32_t v = 0;
        if (q == '-' || dig(q)) {
          const bool pos = q != '-';
          if (!pos) eat();
          const uint32_t a = i;
          uint8_t kind;
          if (parse_integer(pos, &kind)) {
            rc = -1;
            break;
          }
          const uint32_t b = i;
          if (kind == JU_FLOAT) {  // visit_f64: the u32 visitor's default, invalid_type(Unexpected::Float)
            custom(JE_INVALID_TYPE, a, b, (uint8_t)(JU_FLOAT | (JX_U32 << 4)));
            fix_position();
            rc = -1;
            break;
          }
          uint64_t mag = 0;
          const bool big = b - a > 10;
          for (uint32_t t = a; !big && t < b; t++) mag = mag * 10 + (uint64_t)(at(t) - '0');
          if (!pos || big || mag > 0xFFFFFFFFull) {  // visit_i64 / visit_u64 out of range
            custom(JE_INVALID_VALUE, a, b, kind);
            fix_position();
            rc = -1;
            break;
          }
          v = (uint32_t)mag;
        } else {
          invalid_type(JX_U32);
          rc = -1;
          break;
        }
        out[k].pos = abs0 + k0;
        out[k].src_len = k1 - k0;
        out[k].out_len = v;
        k++;
      }
      depth++;
      if (!rc) rc = end_map();
    } else {
      invalid_type(JX_MAP);
      rc = -1;
    }
    if (rc) fix_position();
    if (!rc && ws() >= 0) rc = peek_error(JE_TRAILING);  // Deserializer::end
    if (!rc && vunsup) rc = fail_at(i, JE_UNSUP);
    *count = k;
    if (!rc) r.ok = 1;
    return r;
  }

  // map_json_project (C3 field projection; defined by the oracle, parity
  // unpinned): from_slice::<Map<String, Value>> (de.rs deserialize_map /
  // MapAccess), the last member whose key equals `field`.  *ps / *pl = its
  // value's span, *found, *verb = the span is already serde_json::to_string's
  // text (else the projection is JE_UNSUP: the output is a span of the input).
  // Keys with escapes, floats and unsorted objects inside the projected value
  // are JE_UNSUP.
  __device__ __forceinline__ JRes run_project(const uint8_t* field, uint32_t fl, uint32_t* ps, uint32_t* pl,
                                              bool* found) {
    r = JRes{0, 0, 0, 0, 0, 0, 0};
    failed = false;
    has_pos = false;
    depth = 128;
    i = 0;
    vunsup = false;
    *found = false;
    bool fverb = true, funsup = false;
    int rc = 0;
    int c = ws();
    if (c < 0) {
      rc = peek_error(JE_EOF_VALUE);
    } else if (c == '{') {
      --depth;  // 127: cannot reach 0
      eat();
      bool first = true;
      for (;;) {
        int p = ws();
        if (p == '}') break;
        if (p == ',' && !first) {
          eat();
          p = ws();
        } else if (p >= 0) {
          if (!first) {
            rc = peek_error(JE_OBJ_COMMA);
            break;
          }
          first = false;
        } else {
          rc = peek_error(JE_EOF_OBJECT);
          break;
        }
        if (p == '}') {
          rc = peek_error(JE_TRAILING_COMMA);
          break;
        }
        if (p < 0) {
          rc = peek_error(JE_EOF_VALUE);
          break;
        }
        if (p != '"') {
          rc = peek_error(JE_KEY);
          break;
        }
        eat();
        const uint32_t k0 = i;
        vcanon = 0;
        if (vstr()) {
          rc = -1;
          break;
        }
        const uint32_t k1 = i - 1;
        bool hit = !vhas_bs && k1 - k0 == fl;
        for (uint32_t k = 0; hit && k < fl; k++) hit = at(k0 + k) == field[k];
        const bool maybe = vhas_bs;  // an escaped key could decode to the field name
        c = ws();  // parse_object_colon
        if (c == ':') {
          eat();
        } else if (c >= 0) {
          rc = peek_error(JE_COLON);
          break;
        } else {
          rc = peek_error(JE_EOF_OBJECT);
          break;
        }
        const bool un0 = vunsup;
        vunsup = false;
        vcomplex = false;
        vcanon = 0;
        vhas_u = false;
        ws();
        const uint32_t e0 = i;
        if (any_value()) {
          rc = -1;
          break;
        }
        if (hit) {
          *found = true;
          *ps = e0;
          *pl = i - e0;
          fverb = i - e0 == vcanon && !vhas_u;
          funsup = vunsup || vcomplex;  // a projection is a span of its source: no generated text
        }
        vunsup = un0 || maybe;
      }
      depth++;
      if (!rc) rc = end_map();
    } else {
      invalid_type(JX_MAP);
      rc = -1;
    }
    if (rc) fix_position();
    if (!rc && ws() >= 0) rc = peek_error(JE_TRAILING);  // Deserializer::end
    if (!rc && (vunsup || (*found && (funsup || !fverb)))) rc = fail_at(i, JE_UNSUP);
    if (!rc) r.ok = 1;
    return r;
  }

  __device__ __forceinline__ JRes run() {
    int level = 0;
    r = JRes{0, 0, 0, 0, 0, 0, 0};
    failed = false;
    has_pos = false;
    depth = 128;
    i = 0;
    int rc = de_struct(&level);
    if (!rc && ws() >= 0) rc = peek_error(JE_TRAILING);  // Deserializer::end
    if (!rc) {
      r.ok = 1;
      r.level = (uint8_t)level;
    }
    return r;
  }
};

// one out-of-line copy over a generic pointer (LDS window, global slice or a
// private i32 text buffer); the parser's helpers inline into it so its state
// stays in registers, and k_eval keeps one call site per variant
__device__ __noinline__ JRes json_structured_log(const uint8_t* s, uint32_t n, bool upper) {
  JsonDev<const uint8_t*> d;
  d.s = s;
  d.n = n;
  d.upper = upper;
  return d.run();
}
// map_json_project over one value
__device__ __noinline__ JRes json_project(const uint8_t* s, uint32_t n, bool upper, const uint8_t* field, uint32_t fl,
                                          uint32_t* ps, uint32_t* pl, bool* found) {
  JsonDev<const uint8_t*> d;
  d.s = s;
  d.n = n;
  d.upper = upper;
  return d.run_project(field, fl, ps, pl, found);
}
// array_map_json_array over one value: element descriptors to out[0..*count)
__device__ __noinline__ JRes json_map_u32(const uint8_t* s, uint32_t n, bool upper, ElemRec* out, uint64_t abs0,
                                          uint32_t* count) {
  JsonDev<const uint8_t*> d;
  d.s = s;
  d.n = n;
  d.upper = upper;
  return d.run_map_u32(out, abs0, count);
}
__device__ __noinline__ JRes json_array_explode(const uint8_t* s, uint32_t n, bool upper, ElemRec* out, uint64_t abs0,
                                               uint32_t* count) {
  JsonDev<const uint8_t*> d;
  d.s = s;
  d.n = n;
  d.upper = upper;
  return d.run_array(out, abs0, count);
}

}  // namespace fsg
