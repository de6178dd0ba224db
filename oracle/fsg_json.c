/* TEST INFRASTRUCTURE — CPU oracle (never linked into or called by the product path).
 *
 * Scalar restatement of serde_json 1.0.96 (crates.io; pinned in
 * smartmodule/examples/Cargo.lock, absent from the reference tree) as used by
 * smartmodule/examples/filter_json/src/lib.rs:54-70:
 *     serde_json::from_slice::<StructuredLog>(record.value.as_ref())?
 * with `#[derive(Deserialize)] struct StructuredLog { level: LogLevel,
 * #[serde(rename = "message")] _message: String }` and the unit enum
 * `LogLevel { Debug, Info, Warn, Error }` (rename_all = "lowercase").
 *
 * The functions below follow serde_json's call structure one to one, because
 * the error text (and its "at line L column C" position) depends on which
 * routine detects an error and how far the reader has advanced:
 *   from_trait + Deserializer::end            (de.rs)
 *   deserialize_struct / visit_map / visit_seq (de.rs + serde_derive output)
 *   MapAccess::next_key_seed / next_value_seed, parse_object_colon, end_map
 *   SeqAccess::next_element_seed, end_seq
 *   deserialize_enum, UnitVariantAccess, VariantAccess, deserialize_unit
 *   deserialize_str (fix_position), peek_invalid_type, parse_integer/number
 *   ignore_value / ignore_integer / ignore_decimal / ignore_exponent
 *   SliceRead::parse_str_bytes / ignore_str / decode_hex_escape, parse_escape
 *   position_of_index (line = 1 + #'\n' before i, column = bytes since it)
 * Error Display = "<msg> at line L column C" (line 0: "<msg>").  serde's
 * messages: invalid type / invalid length / unknown variant / duplicate field /
 * missing field (serde/src/de/mod.rs).
 *
 * Floats: serde_json's f64 reading (f64_from_parts, no float_roundtrip) and
 * Rust's shortest Display behind serde's WithDecimalPoint for "invalid type:
 * floating point `..`"; ryu's format for Value::to_string.
 * "invalid type: string ..." renders the string with Rust's str Debug
 * (str_debug: Unicode escapes from this image's Unicode 13 categories and
 * Grapheme_Extend, parity unpinned for code points assigned later).
 * Outside the restatement (status ORC_E_UNSUPPORTED, mirrored by the GPU path):
 * an ignored value nested more than 256 levels below its first bracket.  (An
 * error text holding a NUL byte, from "unknown variant" of StructuredLog, is
 * carried with its length.)
 */
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fsg_oracle.h"

enum { JF_IGNORED = 0, JF_ENUM = 1, JF_STRING = 2 };

typedef struct {
  const char *name;
  int type;                  /* JF_ENUM / JF_STRING */
  const char *const *variants; /* JF_ENUM */
  int nvariants;
} jfield;

typedef struct {
  const char *name; /* struct name for "expected struct X" */
  const jfield *fields;
  int nfields;
} jstruct;

typedef struct {
  const uint8_t *s;
  size_t n;
  size_t i;
  int depth; /* remaining_depth */
  /* error state */
  int failed;
  int unsupported;
  int has_pos;
  size_t err_index; /* reader index the position is computed from */
  char *msg;        /* heap, msg_len bytes (may hold any byte) */
  size_t msg_len;
} jde;

/* ---- reader primitives (SliceRead) */
static int jpeek(jde *d) { return d->i < d->n ? d->s[d->i] : -1; }
static void jeat(jde *d) { d->i++; }
static int jnext(jde *d) { return d->i < d->n ? d->s[d->i++] : -1; }

/* ---- errors */
static void jset_msg(jde *d, const char *m, size_t n) {
  free(d->msg);
  d->msg = (char *)malloc(n + 1);
  memcpy(d->msg, m, n);
  d->msg[n] = 0;
  d->msg_len = n;
}
static int jfail_at(jde *d, size_t idx, const char *msg) {
  d->failed = 1;
  d->has_pos = 1;
  d->err_index = idx;
  jset_msg(d, msg, strlen(msg));
  return -1;
}
static int jerror(jde *d, const char *msg) { return jfail_at(d, d->i, msg); }
static int jpeek_error(jde *d, const char *msg) { return jfail_at(d, d->i + 1 < d->n ? d->i + 1 : d->n, msg); }
static int jcustom(jde *d, const char *fmt, ...) {
  d->failed = 1;
  d->has_pos = 0;
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(NULL, 0, fmt, ap);
  va_end(ap);
  char *m = (char *)malloc((size_t)n + 1);
  va_start(ap, fmt);
  vsnprintf(m, (size_t)n + 1, fmt, ap);
  va_end(ap);
  free(d->msg);
  d->msg = m;
  d->msg_len = (size_t)n;
  return -1;
}
/* custom message from binary pieces (strings may hold NUL or any byte) */
static int jcustom_parts(jde *d, const char *a, const uint8_t *b, size_t bn, const char *c) {
  size_t an = strlen(a), cn = strlen(c);
  char *m = (char *)malloc(an + bn + cn + 1);
  memcpy(m, a, an);
  memcpy(m + an, b, bn);
  memcpy(m + an + bn, c, cn);
  m[an + bn + cn] = 0;
  d->failed = 1;
  d->has_pos = 0;
  free(d->msg);
  d->msg = m;
  d->msg_len = an + bn + cn;
  return -1;
}
static int junsupported(jde *d) {
  d->failed = 1;
  d->unsupported = 1;
  return -1;
}
/* Error::fix_position: give a position-less (custom) error the current one */
static void jfix_position(jde *d) {
  if (d->failed && !d->has_pos && !d->unsupported) {
    d->has_pos = 1;
    d->err_index = d->i;
  }
}

#define E_EOF_LIST "EOF while parsing a list"
#define E_EOF_OBJECT "EOF while parsing an object"
#define E_EOF_STRING "EOF while parsing a string"
#define E_EOF_VALUE "EOF while parsing a value"
#define E_COLON "expected `:`"
#define E_LIST_COMMA "expected `,` or `]`"
#define E_OBJ_COMMA "expected `,` or `}`"
#define E_IDENT "expected ident"
#define E_VALUE "expected value"
#define E_ESCAPE "invalid escape"
#define E_NUMBER "invalid number"
#define E_CODEPOINT "invalid unicode code point"
#define E_CONTROL "control character (\\u0000-\\u001F) found while parsing a string"
#define E_KEY "key must be a string"
#define E_SURROGATE "lone leading surrogate in hex escape"
#define E_TRAILING_COMMA "trailing comma"
#define E_TRAILING "trailing characters"
#define E_HEX_END "unexpected end of hex escape"
#define E_RECURSION "recursion limit exceeded"

static int parse_whitespace(jde *d) {
  for (;;) {
    int c = jpeek(d);
    if (c == ' ' || c == '\n' || c == '\t' || c == '\r')
      jeat(d);
    else
      return c;
  }
}

static int parse_ident(jde *d, const char *ident) {
  for (const char *p = ident; *p; p++) {
    int c = jnext(d);
    if (c < 0) return jerror(d, E_EOF_VALUE);
    if (c != (uint8_t)*p) return jerror(d, E_IDENT);
  }
  return 0;
}

/* ---- strings */
static int ESC(int c) { return c == '"' || c == '\\' || (c >= 0 && c < 0x20); }

static int hexval(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

static int decode_hex_escape(jde *d, uint32_t *out) {
  if (d->i + 4 > d->n) {
    d->i = d->n;
    return jerror(d, E_EOF_STRING);
  }
  uint32_t v = 0;
  for (int k = 0; k < 4; k++) {
    int h = hexval(d->s[d->i]);
    d->i++;
    if (h < 0) return jerror(d, E_ESCAPE);
    v = (v << 4) + (uint32_t)h;
  }
  *out = v;
  return 0;
}

typedef struct {
  uint8_t *b;
  size_t n, cap;
} jbuf;
static void jb_push(jbuf *b, const uint8_t *p, size_t n) {
  if (b->n + n > b->cap) {
    b->cap = (b->n + n) * 2 + 16;
    b->b = (uint8_t *)realloc(b->b, b->cap);
  }
  memcpy(b->b + b->n, p, n);
  b->n += n;
}
static void jb_byte(jbuf *b, uint8_t c) { jb_push(b, &c, 1); }

static void push_utf8(jbuf *b, uint32_t c) {
  uint8_t t[4];
  size_t k;
  if (c < 0x80) {
    t[0] = (uint8_t)c;
    k = 1;
  } else if (c < 0x800) {
    t[0] = (uint8_t)(0xC0 | (c >> 6));
    t[1] = (uint8_t)(0x80 | (c & 0x3F));
    k = 2;
  } else if (c < 0x10000) {
    t[0] = (uint8_t)(0xE0 | (c >> 12));
    t[1] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
    t[2] = (uint8_t)(0x80 | (c & 0x3F));
    k = 3;
  } else {
    t[0] = (uint8_t)(0xF0 | (c >> 18));
    t[1] = (uint8_t)(0x80 | ((c >> 12) & 0x3F));
    t[2] = (uint8_t)(0x80 | ((c >> 6) & 0x3F));
    t[3] = (uint8_t)(0x80 | (c & 0x3F));
    k = 4;
  }
  jb_push(b, t, k);
}

/* read.rs parse_escape (validate = true: deserializing a str) */
static int parse_escape(jde *d, jbuf *scratch) {
  int ch = jnext(d);
  if (ch < 0) return jerror(d, E_EOF_STRING);
  switch (ch) {
    case '"': jb_byte(scratch, '"'); return 0;
    case '\\': jb_byte(scratch, '\\'); return 0;
    case '/': jb_byte(scratch, '/'); return 0;
    case 'b': jb_byte(scratch, 0x08); return 0;
    case 'f': jb_byte(scratch, 0x0c); return 0;
    case 'n': jb_byte(scratch, '\n'); return 0;
    case 'r': jb_byte(scratch, '\r'); return 0;
    case 't': jb_byte(scratch, '\t'); return 0;
    case 'u': {
      uint32_t n1;
      if (decode_hex_escape(d, &n1)) return -1;
      if (n1 >= 0xDC00 && n1 <= 0xDFFF) return jerror(d, E_SURROGATE);
      if (n1 >= 0xD800 && n1 <= 0xDBFF) {
        int p = jpeek(d);
        if (p < 0) return jerror(d, E_EOF_STRING);
        if (p != '\\') {
          jeat(d);
          return jerror(d, E_HEX_END);
        }
        jeat(d);
        p = jpeek(d);
        if (p < 0) return jerror(d, E_EOF_STRING);
        if (p != 'u') {
          jeat(d);
          return jerror(d, E_HEX_END);
        }
        jeat(d);
        uint32_t n2;
        if (decode_hex_escape(d, &n2)) return -1;
        if (n2 < 0xDC00 || n2 > 0xDFFF) return jerror(d, E_SURROGATE);
        push_utf8(scratch, (((n1 - 0xD800) << 10) | (n2 - 0xDC00)) + 0x10000);
        return 0;
      }
      push_utf8(scratch, n1);
      return 0;
    }
    default: return jerror(d, E_ESCAPE);
  }
}

static int utf8_valid(const uint8_t *s, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    size_t w;
    uint32_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF)
      w = 2;
    else if (c >= 0xE0 && c <= 0xEF) {
      w = 3;
      if (c == 0xE0) lo = 0xA0;
      if (c == 0xED) hi = 0x9F;
    } else if (c >= 0xF0 && c <= 0xF4) {
      w = 4;
      if (c == 0xF0) lo = 0x90;
      if (c == 0xF4) hi = 0x8F;
    } else
      return 0;
    if (i + w > n) return 0;
    if (s[i + 1] < lo || s[i + 1] > hi) return 0;
    for (size_t k = 2; k < w; k++)
      if (s[i + k] < 0x80 || s[i + k] > 0xBF) return 0;
    i += w;
  }
  return 1;
}

/* SliceRead::parse_str (after the opening quote was eaten): decoded UTF-8 string
 * in *out (scratch or borrowed copy), caller frees out->b */
static int parse_str(jde *d, jbuf *out) {
  memset(out, 0, sizeof *out);
  size_t start = d->i;
  for (;;) {
    while (d->i < d->n && !ESC(d->s[d->i])) d->i++;
    if (d->i == d->n) return jerror(d, E_EOF_STRING);
    int c = d->s[d->i];
    if (c == '"') {
      jb_push(out, d->s + start, d->i - start);
      d->i++;
      if (!utf8_valid(out->b, out->n)) return jerror(d, E_CODEPOINT);
      return 0;
    } else if (c == '\\') {
      jb_push(out, d->s + start, d->i - start);
      d->i++;
      if (parse_escape(d, out)) return -1;
      start = d->i;
    } else {
      d->i++;
      return jerror(d, E_CONTROL);
    }
  }
}

/* read.rs ignore_escape / SliceRead::ignore_str (no UTF-8 validation) */
static int ignore_escape(jde *d) {
  int ch = jnext(d);
  if (ch < 0) return jerror(d, E_EOF_STRING);
  switch (ch) {
    case '"': case '\\': case '/': case 'b': case 'f': case 'n': case 'r': case 't': return 0;
    case 'u': {
      uint32_t v;
      return decode_hex_escape(d, &v);
    }
    default: return jerror(d, E_ESCAPE);
  }
}
static int ignore_str(jde *d) {
  for (;;) {
    while (d->i < d->n && !ESC(d->s[d->i])) d->i++;
    if (d->i == d->n) return jerror(d, E_EOF_STRING);
    int c = d->s[d->i];
    if (c == '"') {
      d->i++;
      return 0;
    } else if (c == '\\') {
      d->i++;
      if (ignore_escape(d)) return -1;
    } else {
      return jerror(d, E_CONTROL);
    }
  }
}

/* ---- numbers */
static int peek_or_null(jde *d) { int c = jpeek(d); return c < 0 ? 0 : c; }
static int isdig(int c) { return c >= '0' && c <= '9'; }

static int ignore_exponent(jde *d) {
  jeat(d);
  int c = peek_or_null(d);
  if (c == '+' || c == '-') jeat(d);
  c = jnext(d);
  if (!isdig(c)) return jerror(d, E_NUMBER);
  while (isdig(peek_or_null(d))) jeat(d);
  return 0;
}
static int ignore_decimal(jde *d) {
  jeat(d);
  int any = 0;
  while (isdig(peek_or_null(d))) {
    jeat(d);
    any = 1;
  }
  if (!any) return jpeek_error(d, E_NUMBER);
  int c = peek_or_null(d);
  if (c == 'e' || c == 'E') return ignore_exponent(d);
  return 0;
}
static int ignore_integer(jde *d) {
  int c = jnext(d);
  if (c == '0') {
    if (isdig(peek_or_null(d))) return jpeek_error(d, E_NUMBER);
  } else if (c >= '1' && c <= '9') {
    while (isdig(peek_or_null(d))) jeat(d);
  } else {
    return jerror(d, E_NUMBER);
  }
  c = peek_or_null(d);
  if (c == '.') return ignore_decimal(d);
  if (c == 'e' || c == 'E') return ignore_exponent(d);
  return 0;
}

/* parse_integer / parse_number / parse_long_integer / parse_decimal(_overflow) /
 * parse_exponent(_overflow) / f64_from_parts (de.rs, the default build without
 * the float_roundtrip feature): the syntax, the reader movement and the value.
 * A u64 significand collects the digits (past u64 they only move the decimal
 * exponent); the f64 is significand * or / POW10[|exponent|] (1e0 ..= 1e308),
 * "number out of range" where that overflows. */
typedef struct {
  int is_float;
  int neg;
  uint64_t mag;
  double f; /* is_float */
} jnum;

#define E_RANGE "number out of range"
static const double ORC_POW10[309] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22, 1e23, 1e24, 1e25, 1e26, 1e27, 1e28, 1e29, 1e30, 1e31, 1e32, 1e33, 1e34, 1e35, 1e36, 1e37, 1e38, 1e39, 1e40, 1e41, 1e42, 1e43, 1e44, 1e45, 1e46, 1e47, 1e48, 1e49, 1e50, 1e51, 1e52, 1e53, 1e54, 1e55, 1e56, 1e57, 1e58, 1e59, 1e60, 1e61, 1e62, 1e63, 1e64, 1e65, 1e66, 1e67, 1e68, 1e69, 1e70, 1e71, 1e72, 1e73, 1e74, 1e75, 1e76, 1e77, 1e78, 1e79, 1e80, 1e81, 1e82, 1e83, 1e84, 1e85, 1e86, 1e87, 1e88, 1e89, 1e90, 1e91, 1e92, 1e93, 1e94, 1e95, 1e96, 1e97, 1e98, 1e99, 1e100, 1e101, 1e102, 1e103, 1e104, 1e105, 1e106, 1e107, 1e108, 1e109, 1e110, 1e111, 1e112, 1e113, 1e114, 1e115, 1e116, 1e117, 1e118, 1e119, 1e120, 1e121, 1e122, 1e123, 1e124, 1e125, 1e126, 1e127, 1e128, 1e129, 1e130, 1e131, 1e132, 1e133, 1e134, 1e135, 1e136, 1e137, 1e138, 1e139, 1e140, 1e141, 1e142, 1e143, 1e144, 1e145, 1e146, 1e147, 1e148, 1e149, 1e150, 1e151, 1e152, 1e153, 1e154, 1e155, 1e156, 1e157, 1e158, 1e159, 1e160, 1e161, 1e162, 1e163, 1e164, 1e165, 1e166, 1e167, 1e168, 1e169, 1e170, 1e171, 1e172, 1e173, 1e174, 1e175, 1e176, 1e177, 1e178, 1e179, 1e180, 1e181, 1e182, 1e183, 1e184, 1e185, 1e186, 1e187, 1e188, 1e189, 1e190, 1e191, 1e192, 1e193, 1e194, 1e195, 1e196, 1e197, 1e198, 1e199, 1e200, 1e201, 1e202, 1e203, 1e204, 1e205, 1e206, 1e207, 1e208, 1e209, 1e210, 1e211, 1e212, 1e213, 1e214, 1e215, 1e216, 1e217, 1e218, 1e219, 1e220, 1e221, 1e222, 1e223, 1e224, 1e225, 1e226, 1e227, 1e228, 1e229, 1e230, 1e231, 1e232, 1e233, 1e234, 1e235, 1e236, 1e237, 1e238, 1e239, 1e240, 1e241, 1e242, 1e243, 1e244, 1e245, 1e246, 1e247, 1e248, 1e249, 1e250, 1e251, 1e252, 1e253, 1e254, 1e255, 1e256, 1e257, 1e258, 1e259, 1e260, 1e261, 1e262, 1e263, 1e264, 1e265, 1e266, 1e267, 1e268, 1e269, 1e270, 1e271, 1e272, 1e273, 1e274, 1e275, 1e276, 1e277, 1e278, 1e279, 1e280, 1e281, 1e282, 1e283, 1e284, 1e285, 1e286, 1e287, 1e288, 1e289, 1e290, 1e291, 1e292, 1e293, 1e294, 1e295, 1e296, 1e297, 1e298, 1e299, 1e300, 1e301, 1e302, 1e303, 1e304, 1e305, 1e306, 1e307, 1e308};

static int f64_from_parts(jde *d, int positive, uint64_t significand, int32_t exponent, jnum *o) {
  double f = (double)significand;
  for (;;) {
    uint32_t ae = exponent < 0 ? 0u - (uint32_t)exponent : (uint32_t)exponent; /* wrapping_abs as usize */
    if (exponent != INT32_MIN && ae <= 308) {
      if (exponent >= 0) {
        f *= ORC_POW10[ae];
        if (isinf(f)) return jerror(d, E_RANGE);
      } else {
        f /= ORC_POW10[ae];
      }
      break;
    }
    if (f == 0.0) break;
    if (exponent >= 0) return jerror(d, E_RANGE);
    f /= 1e308;
    exponent += 308;
  }
  o->is_float = 1;
  o->f = positive ? f : -f;
  return 0;
}
static int sig_overflows(uint64_t sig, uint64_t dg) { return sig > UINT64_MAX / 10 || (sig == UINT64_MAX / 10 && dg > UINT64_MAX % 10); }

static int parse_exponent(jde *d, int positive, uint64_t significand, int32_t starting_exp, jnum *o) {
  jeat(d);
  int positive_exp = 1;
  int c = peek_or_null(d);
  if (c == '+') {
    jeat(d);
  } else if (c == '-') {
    jeat(d);
    positive_exp = 0;
  }
  int nx = jnext(d);
  if (nx < 0) return jerror(d, E_EOF_VALUE);
  if (!isdig(nx)) return jerror(d, E_NUMBER);
  int32_t exp = nx - '0';
  while (isdig(peek_or_null(d))) {
    int dg = jnext(d) - '0';
    if (exp > INT32_MAX / 10 || (exp == INT32_MAX / 10 && dg > INT32_MAX % 10)) {
      /* parse_exponent_overflow: error instead of +/- infinity */
      if (significand != 0 && positive_exp) return jerror(d, E_RANGE);
      while (isdig(peek_or_null(d))) jeat(d);
      o->is_float = 1;
      o->f = positive ? 0.0 : -0.0;
      return 0;
    }
    exp = exp * 10 + dg;
  }
  int64_t fe = positive_exp ? (int64_t)starting_exp + exp : (int64_t)starting_exp - exp; /* saturating */
  if (fe > INT32_MAX) fe = INT32_MAX;
  if (fe < INT32_MIN) fe = INT32_MIN;
  return f64_from_parts(d, positive, significand, (int32_t)fe, o);
}
static int parse_decimal(jde *d, int positive, uint64_t significand, int32_t exponent_before, jnum *o) {
  jeat(d);
  int32_t after = 0;
  int overflow = 0;
  while (isdig(peek_or_null(d))) {
    uint64_t dg = (uint64_t)(peek_or_null(d) - '0');
    if (sig_overflows(significand, dg)) { /* parse_decimal_overflow: further digits ignored */
      overflow = 1;
      while (isdig(peek_or_null(d))) jeat(d);
      break;
    }
    jeat(d);
    significand = significand * 10 + dg;
    after--;
  }
  if (!overflow && after == 0) {
    if (jpeek(d) >= 0) return jpeek_error(d, E_NUMBER);
    return jpeek_error(d, E_EOF_VALUE);
  }
  int c = peek_or_null(d);
  if (c == 'e' || c == 'E') return parse_exponent(d, positive, significand, exponent_before + after, o);
  return f64_from_parts(d, positive, significand, exponent_before + after, o);
}
static int parse_number_tail(jde *d, int positive, uint64_t significand, jnum *o) {
  int c = peek_or_null(d);
  if (c == '.') return parse_decimal(d, positive, significand, 0, o);
  if (c == 'e' || c == 'E') return parse_exponent(d, positive, significand, 0, o);
  o->mag = significand;
  if (!positive) {
    int64_t neg = (int64_t)(0 - significand); /* (significand as i64).wrapping_neg() */
    if (neg >= 0) {                           /* -0 / below i64::MIN: -(significand as f64) */
      o->is_float = 1;
      o->f = -(double)significand;
    }
  }
  return 0;
}
static int parse_integer(jde *d, int positive, jnum *o) {
  memset(o, 0, sizeof *o);
  o->neg = !positive;
  int c = jnext(d);
  if (c < 0) return jerror(d, E_EOF_VALUE);
  if (c == '0') {
    if (isdig(peek_or_null(d))) return jpeek_error(d, E_NUMBER);
    return parse_number_tail(d, positive, 0, o);
  }
  if (c >= '1' && c <= '9') {
    uint64_t sig = (uint64_t)(c - '0');
    for (;;) {
      int p = peek_or_null(d);
      if (!isdig(p)) break;
      uint64_t dg = (uint64_t)(p - '0');
      if (sig_overflows(sig, dg)) {
        /* parse_long_integer: every further integer digit raises the exponent */
        int32_t exponent = 0;
        while (isdig(peek_or_null(d))) {
          jeat(d);
          exponent++;
        }
        int q = peek_or_null(d);
        if (q == '.') return parse_decimal(d, positive, sig, exponent, o);
        if (q == 'e' || q == 'E') return parse_exponent(d, positive, sig, exponent, o);
        return f64_from_parts(d, positive, sig, exponent, o);
      }
      jeat(d);
      sig = sig * 10 + dg;
    }
    return parse_number_tail(d, positive, sig, o);
  }
  return jerror(d, E_NUMBER);
}

/* Shortest round-trip digits of |v| > 0, found independently of the product's
 * bignum generator: for p = 1..17 the correctly rounded p-digit decimal
 * (glibc printf, exact, ties to even) and its two p-digit neighbours, the
 * first that reads back (glibc strtod, correctly rounded) as v.  Among valid
 * p-digit candidates the rounded one is the closest; when v lies exactly
 * halfway and both round-trip, ryu keeps the even digit and Rust's Display
 * (flt2dec dragon format_shortest) rounds up.  dig[0..n), v ~ 0.dig x 10^k. */
static int orc_shortest(double v, int tie_up, char *dig, int *k) {
  v = fabs(v);
  char buf[64];
  for (int p = 1; p <= 17; p++) {
    snprintf(buf, sizeof buf, "%.*e", p - 1, v);
    char ds[24];
    int nd = 0;
    const char *q = buf;
    for (; *q && *q != 'e'; q++)
      if (*q >= '0' && *q <= '9') ds[nd++] = *q;
    int e10 = atoi(q + 1);
    /* candidates: the rounded value, one unit above, one unit below (same length) */
    for (int cand = 0; cand < 3; cand++) {
      char cd[24];
      memcpy(cd, ds, (size_t)nd);
      int ce = e10, cn = nd;
      if (cand) {
        int j = nd - 1;
        if (cand == 1) {
          while (j >= 0 && cd[j] == '9') cd[j--] = '0';
          if (j < 0) { /* 99..9 + 1 = 100..0: one more digit position */
            cd[0] = '1';
            for (int t = 1; t < nd; t++) cd[t] = '0';
            ce++;
          } else {
            cd[j]++;
          }
        } else {
          while (j >= 0 && cd[j] == '0') cd[j--] = '9';
          if (j < 0 || (j == 0 && cd[0] == '1' && nd == 1)) continue;
          cd[j]--;
          if (cd[0] == '0') continue; /* would drop a digit: a shorter length covers it */
        }
      }
      char t[48];
      snprintf(t, sizeof t, "%c.%.*se%d", cd[0], cn - 1, cd + 1, ce);
      if (cn == 1) snprintf(t, sizeof t, "%ce%d", cd[0], ce);
      if (strtod(t, NULL) != v) continue;
      if (cand == 0 && tie_up) {
        /* exactly halfway (the exact expansion continues 5000..): take the upper one if valid */
        char ex[1200];
        snprintf(ex, sizeof ex, "%.*e", 800, v);
        char xd[900];
        int xn = 0;
        for (const char *r = ex; *r && *r != 'e'; r++)
          if (*r >= '0' && *r <= '9') xd[xn++] = *r;
        int xe = atoi(strchr(ex, 'e') + 1);
        int tie = 0;
        /* the digits of v past the first p (relative to the rounded candidate's exponent) */
        int off = p + (xe - e10);
        if (xe == e10 && off < xn && xd[off] == '5') {
          tie = 1;
          for (int r = off + 1; r < xn; r++)
            if (xd[r] != '0') tie = 0;
        }
        if (tie && memcmp(xd, cd, (size_t)p) == 0) { /* the rounded one went down: try up */
          char ud[24];
          memcpy(ud, cd, (size_t)cn);
          int j = cn - 1, ue = ce;
          while (j >= 0 && ud[j] == '9') ud[j--] = '0';
          if (j < 0) {
            ud[0] = '1';
            ue++;
          } else {
            ud[j]++;
          }
          char u[48];
          if (cn == 1)
            snprintf(u, sizeof u, "%ce%d", ud[0], ue);
          else
            snprintf(u, sizeof u, "%c.%.*se%d", ud[0], cn - 1, ud + 1, ue);
          if (strtod(u, NULL) == v) {
            memcpy(cd, ud, (size_t)cn);
            ce = ue;
          }
        }
      }
      memcpy(dig, cd, (size_t)cn);
      *k = ce + 1;
      return cn;
    }
  }
  return 0; /* unreachable: 17 digits always round-trip */
}

/* ryu 1.0.13 Buffer::format_finite (pretty/mod.rs format64) */
static void orc_ryu(double v, jbuf *out) {
  if (signbit(v)) jb_byte(out, '-');
  if (v == 0.0) {
    jb_push(out, (const uint8_t *)"0.0", 3);
    return;
  }
  char dig[24];
  int kk;
  int len = orc_shortest(v, 0, dig, &kk);
  int e = kk - len;
  char t[64];
  if (e >= 0 && kk <= 16) { /* 1234e7 -> 12340000000.0 */
    jb_push(out, (const uint8_t *)dig, (size_t)len);
    for (int j = len; j < kk; j++) jb_byte(out, '0');
    jb_push(out, (const uint8_t *)".0", 2);
  } else if (kk > 0 && kk <= 16) { /* 1234e-2 -> 12.34 */
    jb_push(out, (const uint8_t *)dig, (size_t)kk);
    jb_byte(out, '.');
    jb_push(out, (const uint8_t *)dig + kk, (size_t)(len - kk));
  } else if (kk > -5 && kk <= 0) { /* 1234e-6 -> 0.001234 */
    jb_push(out, (const uint8_t *)"0.", 2);
    for (int j = kk; j < 0; j++) jb_byte(out, '0');
    jb_push(out, (const uint8_t *)dig, (size_t)len);
  } else if (len == 1) { /* 1e30 */
    int m = snprintf(t, sizeof t, "%ce%d", dig[0], kk - 1);
    jb_push(out, (const uint8_t *)t, (size_t)m);
  } else { /* 1234e30 -> 1.234e33 */
    jb_byte(out, (uint8_t)dig[0]);
    jb_byte(out, '.');
    jb_push(out, (const uint8_t *)dig + 1, (size_t)(len - 1));
    int m = snprintf(t, sizeof t, "e%d", kk - 1);
    jb_push(out, (const uint8_t *)t, (size_t)m);
  }
}

/* serde 1.0.160 Unexpected::Float: `{}` of WithDecimalPoint(f) — Rust's f64
 * Display (shortest digits, no exponent, "-0" for negative zero), ".0" added
 * when it printed no '.' */
static void orc_display_point(double v, char *o, size_t cap) {
  jbuf b = {0};
  if (signbit(v)) jb_byte(&b, '-');
  if (v == 0.0) {
    jb_byte(&b, '0');
  } else {
    char dig[24];
    int kk;
    int len = orc_shortest(v, 1, dig, &kk);
    if (kk <= 0) {
      jb_push(&b, (const uint8_t *)"0.", 2);
      for (int j = kk; j < 0; j++) jb_byte(&b, '0');
      jb_push(&b, (const uint8_t *)dig, (size_t)len);
    } else if (kk < len) {
      jb_push(&b, (const uint8_t *)dig, (size_t)kk);
      jb_byte(&b, '.');
      jb_push(&b, (const uint8_t *)dig + kk, (size_t)(len - kk));
    } else {
      jb_push(&b, (const uint8_t *)dig, (size_t)len);
      for (int j = len; j < kk; j++) jb_byte(&b, '0');
    }
  }
  if (!memchr(b.b, '.', b.n)) jb_push(&b, (const uint8_t *)".0", 2);
  size_t m = b.n < cap - 1 ? b.n : cap - 1;
  memcpy(o, b.b, m);
  o[m] = 0;
  free(b.b);
}

/* Rust `{:?}` of a str, restricted to printable ASCII plus the escapes Rust
 * uses for \t \r \n \" \\ and \0 (anything else: unsupported) */
/* <str as Debug>::fmt (core/src/fmt/mod.rs, Rust 1.75): each char through
 * char::escape_debug_ext with escape_grapheme_extended and escape_double_quote
 * (not the single quote): \0 \t \r \n \\ \" as backslash escapes, a
 * Grapheme_Extend or non-printable char (core/src/unicode/printable.rs) as
 * \u{hex}, lowercase hex without leading zeros; anything else as is */
static int str_debug(jde *d, const jbuf *s, jbuf *out) {
  memset(out, 0, sizeof *out);
  jb_byte(out, '"');
  for (size_t i = 0; i < s->n;) {
    uint8_t c = s->b[i];
    uint32_t cp;
    size_t len;
    if (c < 0x80) {
      cp = c;
      len = 1;
    } else {  /* the string is valid UTF-8 (parse_str checked it) */
      len = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
      if (c < 0xC2 || c > 0xF4 || i + len > s->n) return junsupported(d);
      cp = c & (0x7F >> len);
      for (size_t k = 1; k < len; k++) {
        if ((s->b[i + k] & 0xC0) != 0x80) return junsupported(d);
        cp = (cp << 6) | (s->b[i + k] & 0x3F);
      }
    }
    const char *e = NULL;
    if (cp == '"') e = "\\\"";
    else if (cp == '\\') e = "\\\\";
    else if (cp == '\n') e = "\\n";
    else if (cp == '\r') e = "\\r";
    else if (cp == '\t') e = "\\t";
    else if (cp == 0) e = "\\0";
    if (e) {
      jb_push(out, (const uint8_t *)e, strlen(e));
    } else if (orc_u_dbg_escaped(cp)) {
      char u[16];
      int k = snprintf(u, sizeof u, "\\u{%x}", cp);
      jb_push(out, (const uint8_t *)u, (size_t)k);
    } else {
      jb_push(out, s->b + i, len);
    }
    i += len;
  }
  jb_byte(out, '"');
  return 0;
}

/* de.rs peek_invalid_type */
static int peek_invalid_type(jde *d, const char *expected) {
  int c = jpeek(d);
  if (c < 0) c = 0;
  char unexp[400];
  jbuf dbg = {0};
  switch (c) {
    case 'n':
      jeat(d);
      if (parse_ident(d, "ull")) return -1;
      snprintf(unexp, sizeof unexp, "unit value");
      break;
    case 't':
      jeat(d);
      if (parse_ident(d, "rue")) return -1;
      snprintf(unexp, sizeof unexp, "boolean `true`");
      break;
    case 'f':
      jeat(d);
      if (parse_ident(d, "alse")) return -1;
      snprintf(unexp, sizeof unexp, "boolean `false`");
      break;
    case '-':
    case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8': case '9': {
      int pos = c != '-';
      if (!pos) jeat(d);
      jnum num;
      if (parse_integer(d, pos, &num)) return -1;
      if (num.is_float) {
        char fl[360];
        orc_display_point(num.f, fl, sizeof fl);
        snprintf(unexp, sizeof unexp, "floating point `%s`", fl);
      } else if (num.neg)
        snprintf(unexp, sizeof unexp, "integer `-%llu`", (unsigned long long)num.mag);
      else
        snprintf(unexp, sizeof unexp, "integer `%llu`", (unsigned long long)num.mag);
      break;
    }
    case '"': {
      jeat(d);
      jbuf sb;
      if (parse_str(d, &sb)) {
        free(sb.b);
        return -1;
      }
      int r = str_debug(d, &sb, &dbg);
      free(sb.b);
      if (r) {
        free(dbg.b);
        return -1;
      }
      snprintf(unexp, sizeof unexp, "string ");
      break;
    }
    case '[': snprintf(unexp, sizeof unexp, "sequence"); break;
    case '{': snprintf(unexp, sizeof unexp, "map"); break;
    default: return jpeek_error(d, E_VALUE);
  }
  char tail[160];
  snprintf(tail, sizeof tail, ", expected %s", expected);
  char head[440];
  snprintf(head, sizeof head, "invalid type: %s", unexp);
  jcustom_parts(d, head, dbg.b, dbg.n, tail);
  free(dbg.b);
  jfix_position(d);
  return -1;
}

/* de.rs ignore_value (explicit frame stack, no recursion limit) */
static int ignore_value(jde *d) {
  char *stack = NULL;
  size_t sn = 0, scap = 0;
  int enclosing = 0; /* 0 none */
  int rc = -1;
#define PUSH(f)                                          \
  do {                                                   \
    if (sn == scap) {                                    \
      scap = scap * 2 + 16;                              \
      stack = (char *)realloc(stack, scap);              \
    }                                                    \
    stack[sn++] = (char)(f);                             \
  } while (0)
  for (;;) {
    int peek = parse_whitespace(d);
    if (peek < 0) {
      jpeek_error(d, E_EOF_VALUE);
      goto out;
    }
    int frame = 0; /* 0: scalar consumed */
    switch (peek) {
      case 'n': jeat(d); if (parse_ident(d, "ull")) goto out; break;
      case 't': jeat(d); if (parse_ident(d, "rue")) goto out; break;
      case 'f': jeat(d); if (parse_ident(d, "alse")) goto out; break;
      case '-': jeat(d); if (ignore_integer(d)) goto out; break;
      case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8': case '9':
        if (ignore_integer(d)) goto out;
        break;
      case '"': jeat(d); if (ignore_str(d)) goto out; break;
      case '[':
      case '{':
        /* the device path keeps ignore_value's frames in a 256-entry bit stack
         * (serde's Vec has no limit): deeper nesting is outside both restatements */
        if (enclosing && sn >= 256) {
          junsupported(d);
          goto out;
        }
        if (enclosing) PUSH(enclosing);
        enclosing = 0;
        jeat(d);
        frame = peek;
        break;
      default: jpeek_error(d, E_VALUE); goto out;
    }
    int accept_comma;
    if (frame) {
      accept_comma = 0;
    } else if (enclosing) {
      frame = enclosing;
      enclosing = 0;
      accept_comma = 1;
    } else if (sn) {
      frame = stack[--sn];
      accept_comma = 1;
    } else {
      rc = 0;
      goto out;
    }
    for (;;) {
      int c = parse_whitespace(d);
      if (c == ',' && accept_comma) {
        jeat(d);
        break;
      } else if ((c == ']' && frame == '[') || (c == '}' && frame == '{')) {
        /* fallthrough to close */
      } else if (c >= 0) {
        if (accept_comma) {
          jpeek_error(d, frame == '[' ? E_LIST_COMMA : E_OBJ_COMMA);
          goto out;
        }
        break;
      } else {
        jpeek_error(d, frame == '[' ? E_EOF_LIST : E_EOF_OBJECT);
        goto out;
      }
      jeat(d);
      if (!sn) {
        rc = 0;
        goto out;
      }
      frame = stack[--sn];
      accept_comma = 1;
    }
    if (frame == '{') {
      int c = parse_whitespace(d);
      if (c == '"')
        jeat(d);
      else if (c >= 0) {
        jpeek_error(d, E_KEY);
        goto out;
      } else {
        jpeek_error(d, E_EOF_OBJECT);
        goto out;
      }
      if (ignore_str(d)) goto out;
      c = parse_whitespace(d);
      if (c == ':')
        jeat(d);
      else if (c >= 0) {
        jpeek_error(d, E_COLON);
        goto out;
      } else {
        jpeek_error(d, E_EOF_OBJECT);
        goto out;
      }
    }
    enclosing = frame;
  }
out:
#undef PUSH
  free(stack);
  return rc;
}

/* deserialize_str with a visitor: parses a string; returns it in *out */
static int deserialize_str(jde *d, const char *expected, jbuf *out) {
  memset(out, 0, sizeof *out);
  int peek = parse_whitespace(d);
  if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
  if (peek == '"') {
    jeat(d);
    if (parse_str(d, out)) return -1;
    return 0;
  }
  peek_invalid_type(d, expected);
  jfix_position(d);
  return -1;
}

static void one_of(char *o, size_t cap, const char *const *names, int n) {
  size_t k = 0;
  if (n == 1) {
    snprintf(o, cap, "`%s`", names[0]);
    return;
  }
  if (n == 2) {
    snprintf(o, cap, "`%s` or `%s`", names[0], names[1]);
    return;
  }
  k += (size_t)snprintf(o + k, cap - k, "one of ");
  for (int i = 0; i < n; i++) k += (size_t)snprintf(o + k, cap - k, "%s`%s`", i ? ", " : "", names[i]);
}

/* the variant identifier (deserialize_identifier -> deserialize_str, visitor
 * "variant identifier"; unknown -> serde unknown_variant, fixed at the
 * position after the string) */
static int variant_ident(jde *d, const jfield *f, int *var) {
  jbuf s;
  if (deserialize_str(d, "variant identifier", &s)) {
    free(s.b);
    return -1;
  }
  for (int v = 0; v < f->nvariants; v++)
    if (strlen(f->variants[v]) == s.n && !memcmp(f->variants[v], s.b, s.n)) {
      *var = v;
      free(s.b);
      return 0;
    }
  /* the unknown value is displayed as-is (Display of a str) */
  char names[512];
  one_of(names, sizeof names, f->variants, f->nvariants);
  char tail[560];
  snprintf(tail, sizeof tail, "`, expected %s", names);
  jcustom_parts(d, "unknown variant `", s.b, s.n, tail);
  free(s.b);
  jfix_position(d);
  return -1;
}

/* de.rs deserialize_unit (the `()` of VariantAccess::unit_variant) */
static int deserialize_unit(jde *d) {
  int peek = parse_whitespace(d);
  if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
  if (peek == 'n') {
    jeat(d);
    return parse_ident(d, "ull");
  }
  peek_invalid_type(d, "unit");
  jfix_position(d);
  return -1;
}

/* de.rs deserialize_enum for a unit-variant enum */
static int deserialize_enum(jde *d, const jfield *f, int *var) {
  int peek = parse_whitespace(d);
  if (peek == '{') {
    if (--d->depth == 0) return jpeek_error(d, E_RECURSION);
    jeat(d);
    /* VariantAccess::variant_seed: identifier, then parse_object_colon */
    if (variant_ident(d, f, var)) return -1;
    int c = parse_whitespace(d);
    if (c == ':')
      jeat(d);
    else if (c >= 0)
      return jpeek_error(d, E_COLON);
    else
      return jpeek_error(d, E_EOF_OBJECT);
    /* unit_variant: Deserialize for () */
    if (deserialize_unit(d)) return -1;
    d->depth++;
    c = parse_whitespace(d);
    if (c == '}') {
      jeat(d);
      return 0;
    }
    if (c >= 0) return jerror(d, E_VALUE);
    return jerror(d, E_EOF_OBJECT);
  }
  if (peek == '"') return variant_ident(d, f, var); /* UnitVariantAccess */
  if (peek >= 0) return jpeek_error(d, E_VALUE);
  return jpeek_error(d, E_EOF_VALUE);
}

/* one field value (next_value_seed after parse_object_colon, or a seq element) */
static int field_value(jde *d, const jfield *f, int *enum_out) {
  if (f->type == JF_ENUM) return deserialize_enum(d, f, enum_out);
  jbuf s;
  int r = deserialize_str(d, "a string", &s);
  free(s.b);
  return r;
}

static int end_map(jde *d) {
  int c = parse_whitespace(d);
  if (c == '}') {
    jeat(d);
    return 0;
  }
  if (c == ',') return jpeek_error(d, E_TRAILING_COMMA);
  if (c >= 0) return jpeek_error(d, E_TRAILING);
  return jpeek_error(d, E_EOF_OBJECT);
}
static int end_seq(jde *d) {
  int c = parse_whitespace(d);
  if (c == ']') {
    jeat(d);
    return 0;
  }
  if (c == ',') {
    jeat(d);
    int p = parse_whitespace(d);
    if (p == ']') return jpeek_error(d, E_TRAILING_COMMA);
    return jpeek_error(d, E_TRAILING);
  }
  if (c >= 0) return jpeek_error(d, E_TRAILING);
  return jpeek_error(d, E_EOF_LIST);
}

/* the derive's visit_map: fields by name, duplicates and missing fields are
 * errors in declaration order, unknown keys are IgnoredAny */
static int visit_map(jde *d, const jstruct *st, int *vals) {
  int seen[8] = {0};
  int first = 1;
  for (;;) {
    /* MapAccess::next_key_seed */
    int peek = parse_whitespace(d);
    if (peek == '}') break;
    if (peek == ',' && !first) {
      jeat(d);
      peek = parse_whitespace(d);
    } else if (peek >= 0) {
      if (first)
        first = 0;
      else
        return jpeek_error(d, E_OBJ_COMMA);
    } else {
      return jpeek_error(d, E_EOF_OBJECT);
    }
    if (peek == '}') return jpeek_error(d, E_TRAILING_COMMA);
    if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
    if (peek != '"') return jpeek_error(d, E_KEY);
    jeat(d); /* MapKey::deserialize_any */
    jbuf key;
    if (parse_str(d, &key)) {
      free(key.b);
      return -1;
    }
    int fi = -1;
    for (int k = 0; k < st->nfields; k++)
      if (strlen(st->fields[k].name) == key.n && !memcmp(st->fields[k].name, key.b, key.n)) fi = k;
    free(key.b);
    if (fi >= 0 && seen[fi]) return jcustom(d, "duplicate field `%s`", st->fields[fi].name);
    /* MapAccess::next_value_seed */
    int c = parse_whitespace(d);
    if (c == ':')
      jeat(d);
    else if (c >= 0)
      return jpeek_error(d, E_COLON);
    else
      return jpeek_error(d, E_EOF_OBJECT);
    if (fi < 0) {
      if (ignore_value(d)) return -1;
    } else {
      if (field_value(d, &st->fields[fi], &vals[fi])) return -1;
      seen[fi] = 1;
    }
  }
  for (int k = 0; k < st->nfields; k++)
    if (!seen[k]) return jcustom(d, "missing field `%s`", st->fields[k].name);
  return 0;
}

/* the derive's visit_seq: fields in order, a missing element is invalid_length */
static int visit_seq(jde *d, const jstruct *st, int *vals) {
  int first = 1;
  for (int k = 0; k < st->nfields; k++) {
    int peek = parse_whitespace(d);
    int none = 0;
    if (peek == ']')
      none = 1;
    else if (peek == ',' && !first) {
      jeat(d);
      peek = parse_whitespace(d);
    } else if (peek >= 0) {
      if (first)
        first = 0;
      else
        return jpeek_error(d, E_LIST_COMMA);
    } else {
      return jpeek_error(d, E_EOF_LIST);
    }
    if (!none) {
      if (peek == ']') return jpeek_error(d, E_TRAILING_COMMA);
      if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
      if (field_value(d, &st->fields[k], &vals[k])) return -1;
    } else {
      return jcustom(d, "invalid length %d, expected struct %s with %d elements", k, st->name, st->nfields);
    }
  }
  return 0;
}

static int deserialize_struct(jde *d, const jstruct *st, int *vals) {
  int peek = parse_whitespace(d);
  if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
  int r;
  if (peek == '[' || peek == '{') {
    if (--d->depth == 0) return jpeek_error(d, E_RECURSION);
    jeat(d);
    r = peek == '[' ? visit_seq(d, st, vals) : visit_map(d, st, vals);
    d->depth++;
    /* match (ret, self.end_seq()/end_map()): the end check runs either way;
     * the visitor's error wins */
    if (r) {
      /* keep the visitor's error, but let the end check move the reader */
      jde probe = *d;
      probe.msg = NULL;
      probe.msg_len = 0;
      probe.failed = 0;
      (void)(peek == '[' ? end_seq(&probe) : end_map(&probe));
      free(probe.msg);
      d->i = probe.i;
    } else {
      r = peek == '[' ? end_seq(d) : end_map(d);
    }
  } else {
    char exp[128];
    snprintf(exp, sizeof exp, "struct %s", st->name);
    peek_invalid_type(d, exp);
    r = -1;
  }
  if (r) jfix_position(d);
  return r;
}

static char *render(jde *d, size_t *len) {
  size_t line = 1, col = 0;
  for (size_t i = 0; i < d->err_index && i < d->n; i++) {
    if (d->s[i] == '\n') {
      line++;
      col = 0;
    } else {
      col++;
    }
  }
  char *m = (char *)malloc(d->msg_len + 64);
  memcpy(m, d->msg, d->msg_len);
  size_t k = d->msg_len;
  if (d->has_pos) k += (size_t)sprintf(m + k, " at line %zu column %zu", line, col);
  m[k] = 0;
  *len = k;
  return m;
}

/* serde_json::from_slice::<struct>: 0 ok, 1 error (*msg), ORC_E_UNSUPPORTED */
static int from_slice_struct(const uint8_t *s, size_t n, const jstruct *st, int *vals, char **msg,
                             size_t *msg_len) {
  jde d;
  memset(&d, 0, sizeof d);
  d.s = s;
  d.n = n;
  d.depth = 128;
  *msg = NULL;
  int r = deserialize_struct(&d, st, vals);
  if (!r) {
    /* Deserializer::end */
    if (parse_whitespace(&d) >= 0) r = jpeek_error(&d, E_TRAILING);
  }
  if (!r) {
    free(d.msg);
    return 0;
  }
  if (d.unsupported) {
    free(d.msg);
    return ORC_E_UNSUPPORTED;
  }
  *msg = render(&d, msg_len); /* may hold a NUL ("unknown variant" of a raw string): *msg_len carries it */
  free(d.msg);
  return 1;
}

static const char *const LOG_LEVELS[] = {"debug", "info", "warn", "error"};
static const jfield STRUCTURED_LOG_FIELDS[] = {
    {"level", JF_ENUM, LOG_LEVELS, 4},
    {"message", JF_STRING, NULL, 0},
};
static const jstruct STRUCTURED_LOG = {"StructuredLog", STRUCTURED_LOG_FIELDS, 2};

int orc_json_structured_log(const uint8_t *s, size_t n, int *level, char **msg, size_t *msg_len) {
  int vals[2] = {0, 0};
  int r = from_slice_struct(s, n, &STRUCTURED_LOG, vals, msg, msg_len);
  if (r == 0) *level = vals[0];
  return r;
}

/* ------------------------------------------------------------------ */
/* smartmodule/examples/array_map_json_array/src/lib.rs:38-55:           */
/*   let array: Vec<serde_json::Value> = serde_json::from_slice(value)?; */
/*   array.map(|v| serde_json::to_string(&v))                            */
/* serde_json 1.0.96 without preserve_order (examples/Cargo.lock: deps   */
/* itoa, ryu, serde only): objects are BTreeMap<String, Value>, so       */
/* to_string emits members sorted by key bytes, a repeated key keeps its */
/* last value (Map::insert).  Value parse = Deserializer::deserialize_any */
/* (de.rs), serialization = ser.rs format_escaped_str + itoa; floats    */
/* (and -0 / integers beyond u64/i64, which serde_json parses as f64)    */
/* through ryu's shortest round-trip format (orc_ryu).                   */
/* ------------------------------------------------------------------ */

/* ser.rs format_escaped_str_contents: ESCAPE table — '"' '\\', the short
 * escapes \b \t \n \f \r, every other byte < 0x20 as \u00XX (lowercase hex) */
static void canon_str(jbuf *out, const uint8_t *s, size_t n) {
  static const char HEX[] = "0123456789abcdef";
  jb_byte(out, '"');
  for (size_t i = 0; i < n; i++) {
    uint8_t c = s[i];
    switch (c) {
      case '"': jb_push(out, (const uint8_t *)"\\\"", 2); break;
      case '\\': jb_push(out, (const uint8_t *)"\\\\", 2); break;
      case 0x08: jb_push(out, (const uint8_t *)"\\b", 2); break;
      case 0x09: jb_push(out, (const uint8_t *)"\\t", 2); break;
      case 0x0A: jb_push(out, (const uint8_t *)"\\n", 2); break;
      case 0x0C: jb_push(out, (const uint8_t *)"\\f", 2); break;
      case 0x0D: jb_push(out, (const uint8_t *)"\\r", 2); break;
      default:
        if (c < 0x20) {
          uint8_t u[6] = {'\\', 'u', '0', '0', (uint8_t)HEX[c >> 4], (uint8_t)HEX[c & 15]};
          jb_push(out, u, 6);
        } else {
          jb_byte(out, c);
        }
    }
  }
  jb_byte(out, '"');
}

typedef struct {
  jbuf key; /* decoded key bytes */
  jbuf val; /* canonical serialization of the value */
} jmember;

static int member_cmp(const void *a, const void *b) {
  const jmember *x = (const jmember *)a, *y = (const jmember *)b;
  size_t m = x->key.n < y->key.n ? x->key.n : y->key.n;
  int c = m ? memcmp(x->key.b, y->key.b, m) : 0;
  if (c) return c;
  return x->key.n < y->key.n ? -1 : x->key.n > y->key.n ? 1 : 0;
}

static int value_canon(jde *d, jbuf *out);

/* ValueVisitor::visit_seq via SeqAccess::next_element_seed (de.rs) */
static int visit_seq_values(jde *d, jbuf *out, size_t *count) {
  int first = 1;
  size_t k = 0;
  for (;;) {
    int peek = parse_whitespace(d);
    if (peek == ']') break;
    if (peek == ',' && !first) {
      jeat(d);
      peek = parse_whitespace(d);
    } else if (peek >= 0) {
      if (first)
        first = 0;
      else
        return jpeek_error(d, E_LIST_COMMA);
    } else {
      return jpeek_error(d, E_EOF_LIST);
    }
    if (peek == ']') return jpeek_error(d, E_TRAILING_COMMA);
    if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
    if (out && k) jb_byte(out, ',');
    if (value_canon(d, out)) return -1;
    k++;
  }
  if (count) *count = k;
  return 0;
}

/* ValueVisitor::visit_map via MapAccess (KeyClassifier keys, Map::insert) */
static int visit_map_values(jde *d, jbuf *out) {
  jmember *m = NULL;
  size_t nm = 0, cap = 0;
  int first = 1, rc = -1;
  for (;;) {
    int peek = parse_whitespace(d);
    if (peek == '}') break;
    if (peek == ',' && !first) {
      jeat(d);
      peek = parse_whitespace(d);
    } else if (peek >= 0) {
      if (first)
        first = 0;
      else {
        jpeek_error(d, E_OBJ_COMMA);
        goto out;
      }
    } else {
      jpeek_error(d, E_EOF_OBJECT);
      goto out;
    }
    if (peek == '}') { jpeek_error(d, E_TRAILING_COMMA); goto out; }
    if (peek < 0) { jpeek_error(d, E_EOF_VALUE); goto out; }
    if (peek != '"') { jpeek_error(d, E_KEY); goto out; }
    jeat(d);
    if (nm == cap) {
      cap = cap * 2 + 8;
      m = (jmember *)realloc(m, cap * sizeof(jmember));
    }
    memset(&m[nm], 0, sizeof(jmember));
    nm++;
    if (parse_str(d, &m[nm - 1].key)) goto out;
    int c = parse_whitespace(d);
    if (c == ':')
      jeat(d);
    else if (c >= 0) {
      jpeek_error(d, E_COLON);
      goto out;
    } else {
      jpeek_error(d, E_EOF_OBJECT);
      goto out;
    }
    if (value_canon(d, &m[nm - 1].val)) goto out;
  }
  rc = 0;
  if (out) {
    /* BTreeMap: a later insert of the same key replaces the value -> keep the
     * last occurrence of every key, then emit in key order */
    size_t w = 0;
    for (size_t i = 0; i < nm; i++) {
      int dup = 0;
      for (size_t j = i + 1; j < nm && !dup; j++)
        dup = m[i].key.n == m[j].key.n && (!m[i].key.n || !memcmp(m[i].key.b, m[j].key.b, m[i].key.n));
      if (dup) {
        free(m[i].key.b);
        free(m[i].val.b);
      } else {
        m[w++] = m[i];
      }
    }
    nm = w;
    qsort(m, nm, sizeof(jmember), member_cmp);
    jb_byte(out, '{');
    for (size_t i = 0; i < nm; i++) {
      if (i) jb_byte(out, ',');
      canon_str(out, m[i].key.b, m[i].key.n);
      jb_byte(out, ':');
      jb_push(out, m[i].val.b, m[i].val.n);
    }
    jb_byte(out, '}');
  }
out:
  for (size_t i = 0; i < nm; i++) {
    free(m[i].key.b);
    free(m[i].val.b);
  }
  free(m);
  return rc;
}

/* Deserializer::deserialize_any for Value, serialized with to_string */
static int value_canon(jde *d, jbuf *out) {
  int peek = parse_whitespace(d);
  if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
  int r = 0;
  switch (peek) {
    case 'n':
      jeat(d);
      if (parse_ident(d, "ull")) return -1;
      jb_push(out, (const uint8_t *)"null", 4);
      break;
    case 't':
      jeat(d);
      if (parse_ident(d, "rue")) return -1;
      jb_push(out, (const uint8_t *)"true", 4);
      break;
    case 'f':
      jeat(d);
      if (parse_ident(d, "alse")) return -1;
      jb_push(out, (const uint8_t *)"false", 5);
      break;
    case '-':
    case '0': case '1': case '2': case '3': case '4': case '5': case '6': case '7': case '8': case '9': {
      int pos = peek != '-';
      if (!pos) jeat(d);
      jnum num;
      if (parse_integer(d, pos, &num)) return -1;
      if (num.is_float) { /* ser.rs serialize_f64 -> ryu format_finite (a parsed f64 is finite) */
        orc_ryu(num.f, out);
        break;
      }
      char t[32];
      int k = snprintf(t, sizeof t, "%s%llu", num.neg ? "-" : "", (unsigned long long)num.mag);
      jb_push(out, (const uint8_t *)t, (size_t)k);
      break;
    }
    case '"': {
      jeat(d);
      jbuf s;
      if (parse_str(d, &s)) {
        free(s.b);
        return -1;
      }
      canon_str(out, s.b, s.n);
      free(s.b);
      break;
    }
    case '[':
    case '{': {
      /* check_recursion! */
      if (--d->depth == 0) return jpeek_error(d, E_RECURSION);
      jeat(d);
      if (peek == '[') {
        jb_byte(out, '[');
        r = visit_seq_values(d, out, NULL);
        if (!r) jb_byte(out, ']');
      } else {
        r = visit_map_values(d, out);
      }
      d->depth++;
      if (r) {
        jde probe = *d; /* (Err, _): the end check still moves the reader */
        probe.msg = NULL;
        probe.msg_len = 0;
        probe.failed = 0;
        (void)(peek == '[' ? end_seq(&probe) : end_map(&probe));
        free(probe.msg);
        d->i = probe.i;
      } else {
        r = peek == '[' ? end_seq(d) : end_map(d);
      }
      break;
    }
    default: return jpeek_error(d, E_VALUE);
  }
  if (r) jfix_position(d);
  return r;
}

/* from_slice::<Vec<Value>> + to_string of each element.  0 ok (*elems: count
 * malloc'd canonical strings), 1 error (*msg), ORC_E_UNSUPPORTED */
int orc_json_array_map(const uint8_t *s, size_t n, uint8_t ***elems, size_t **lens, size_t *count, char **msg,
                       size_t *msg_len) {
  jde d;
  memset(&d, 0, sizeof d);
  d.s = s;
  d.n = n;
  d.depth = 128;
  *msg = NULL;
  *elems = NULL;
  *lens = NULL;
  *count = 0;
  int r;
  int peek = parse_whitespace(&d);
  if (peek < 0) {
    r = jpeek_error(&d, E_EOF_VALUE);
  } else if (peek == '[') { /* deserialize_seq */
    if (--d.depth == 0) {
      r = jpeek_error(&d, E_RECURSION);
    } else {
      jeat(&d);
      /* VecVisitor::visit_seq: each element parsed into its own buffer */
      size_t cap = 0;
      int first = 1;
      r = 0;
      for (;;) {
        int p = parse_whitespace(&d);
        if (p == ']') break;
        if (p == ',' && !first) {
          jeat(&d);
          p = parse_whitespace(&d);
        } else if (p >= 0) {
          if (first)
            first = 0;
          else {
            r = jpeek_error(&d, E_LIST_COMMA);
            break;
          }
        } else {
          r = jpeek_error(&d, E_EOF_LIST);
          break;
        }
        if (p == ']') { r = jpeek_error(&d, E_TRAILING_COMMA); break; }
        if (p < 0) { r = jpeek_error(&d, E_EOF_VALUE); break; }
        jbuf v = {0};
        if (value_canon(&d, &v)) {
          free(v.b);
          r = -1;
          break;
        }
        if (*count == cap) {
          cap = cap * 2 + 8;
          *elems = (uint8_t **)realloc(*elems, cap * sizeof(uint8_t *));
          *lens = (size_t *)realloc(*lens, cap * sizeof(size_t));
        }
        (*elems)[*count] = v.b ? v.b : (uint8_t *)malloc(1);
        (*lens)[*count] = v.n;
        (*count)++;
      }
      d.depth++;
      if (r) {
        jde probe = d;
        probe.msg = NULL;
        probe.msg_len = 0;
        probe.failed = 0;
        (void)end_seq(&probe);
        free(probe.msg);
        d.i = probe.i;
      } else {
        r = end_seq(&d);
      }
    }
    if (r) jfix_position(&d);
  } else {
    r = peek_invalid_type(&d, "a sequence");
    jfix_position(&d);
  }
  if (!r && parse_whitespace(&d) >= 0) r = jpeek_error(&d, E_TRAILING); /* Deserializer::end */
  if (!r) {
    free(d.msg);
    return 0;
  }
  for (size_t i = 0; i < *count; i++) free((*elems)[i]);
  free(*elems);
  free(*lens);
  *elems = NULL;
  *lens = NULL;
  *count = 0;
  if (d.unsupported) {
    free(d.msg);
    return ORC_E_UNSUPPORTED;
  }
  *msg = render(&d, msg_len);
  free(d.msg);
  if (memchr(*msg, 0, *msg_len)) {
    free(*msg);
    *msg = NULL;
    return ORC_E_UNSUPPORTED;
  }
  return 1;
}

/* ------------------------------------------------------------------ */
/* map_json_project (C3 "field projection"; no reference module exists —  */
/* BASELINE configs[2] names the transform, the reference ships it only   */
/* as the hub's Jolt module, so this restatement DEFINES it: parity       */
/* unpinned).  FilterMap semantics in serde_json terms:                   */
/*   let m: Map<String, Value> = serde_json::from_slice(value)?;          */
/*   m.get(field).map(|v| serde_json::to_string(v))                      */
/* a missing field drops the record.  Map::insert: a repeated key keeps   */
/* its last value.                                                        */
/* ------------------------------------------------------------------ */
int orc_json_project(const uint8_t *s, size_t n, const char *field, uint8_t **out, size_t *out_len, int *found,
                     char **msg, size_t *msg_len) {
  jde d;
  memset(&d, 0, sizeof d);
  d.s = s;
  d.n = n;
  d.depth = 128;
  *msg = NULL;
  *out = NULL;
  *out_len = 0;
  *found = 0;
  const size_t fl = strlen(field);
  jbuf val = {0};
  int r = 0;
  int peek = parse_whitespace(&d);
  if (peek < 0) {
    r = jpeek_error(&d, E_EOF_VALUE);
  } else if (peek == '{') { /* deserialize_map */
    --d.depth;
    jeat(&d);
    int first = 1;
    for (;;) { /* MapAccess::next_key_seed / next_value_seed */
      int p = parse_whitespace(&d);
      if (p == '}') break;
      if (p == ',' && !first) {
        jeat(&d);
        p = parse_whitespace(&d);
      } else if (p >= 0) {
        if (first)
          first = 0;
        else {
          r = jpeek_error(&d, E_OBJ_COMMA);
          break;
        }
      } else {
        r = jpeek_error(&d, E_EOF_OBJECT);
        break;
      }
      if (p == '}') { r = jpeek_error(&d, E_TRAILING_COMMA); break; }
      if (p < 0) { r = jpeek_error(&d, E_EOF_VALUE); break; }
      if (p != '"') { r = jpeek_error(&d, E_KEY); break; }
      jeat(&d);
      jbuf key;
      if (parse_str(&d, &key)) {
        free(key.b);
        r = -1;
        break;
      }
      const int hit = key.n == fl && (!fl || !memcmp(key.b, field, fl));
      free(key.b);
      int c = parse_whitespace(&d);
      if (c == ':')
        jeat(&d);
      else if (c >= 0) {
        r = jpeek_error(&d, E_COLON);
        break;
      } else {
        r = jpeek_error(&d, E_EOF_OBJECT);
        break;
      }
      jbuf v = {0};
      if (value_canon(&d, &v)) {
        free(v.b);
        r = -1;
        break;
      }
      if (hit) {
        free(val.b);
        val = v;
        *found = 1;
      } else {
        free(v.b);
      }
    }
    d.depth++;
    if (r) {
      jde probe = d;
      probe.msg = NULL;
      probe.msg_len = 0;
      probe.failed = 0;
      (void)end_map(&probe);
      free(probe.msg);
      d.i = probe.i;
    } else {
      r = end_map(&d);
    }
    if (r) jfix_position(&d);
  } else {
    r = peek_invalid_type(&d, "a map");
    jfix_position(&d);
  }
  if (!r && parse_whitespace(&d) >= 0) r = jpeek_error(&d, E_TRAILING); /* Deserializer::end */
  if (!r) {
    free(d.msg);
    if (*found) {
      *out = val.b ? val.b : (uint8_t *)malloc(1);
      *out_len = val.n;
    } else {
      free(val.b);
    }
    return 0;
  }
  free(val.b);
  *found = 0;
  if (d.unsupported) {
    free(d.msg);
    return ORC_E_UNSUPPORTED;
  }
  *msg = render(&d, msg_len);
  free(d.msg);
  if (memchr(*msg, 0, *msg_len)) {
    free(*msg);
    *msg = NULL;
    return ORC_E_UNSUPPORTED;
  }
  return 1;
}

/* generic entry for pinning against other serde_json fixtures of the reference:
 * fields as "name" (string) or "name=v1|v2|.." (unit enum) */
int orc_json_struct(const uint8_t *s, size_t n, const char *name, const char **fields, int nfields, int *vals,
                    char **msg, size_t *msg_len) {
  jfield f[8];
  char *vbuf[8] = {0};
  const char *vars[8][16];
  if (nfields > 8) return ORC_E_INVALID_ARG;
  char *names[8];
  for (int k = 0; k < nfields; k++) {
    const char *eq = strchr(fields[k], '=');
    if (!eq) {
      names[k] = strdup(fields[k]);
      f[k].name = names[k];
      f[k].type = JF_STRING;
      f[k].variants = NULL;
      f[k].nvariants = 0;
      continue;
    }
    names[k] = strndup(fields[k], (size_t)(eq - fields[k]));
    f[k].name = names[k];
    f[k].type = JF_ENUM;
    vbuf[k] = strdup(eq + 1);
    int nv = 0;
    for (char *p = strtok(vbuf[k], "|"); p && nv < 16; p = strtok(NULL, "|")) vars[k][nv++] = p;
    f[k].variants = vars[k];
    f[k].nvariants = nv;
  }
  jstruct st = {name, f, nfields};
  int r = from_slice_struct(s, n, &st, vals, msg, msg_len);
  for (int k = 0; k < nfields; k++) {
    free(names[k]);
    free(vbuf[k]);
  }
  return r;
}

/* ------------------------------------------------------------------------
 * aggregate-json (smartmodule/examples/aggregate-json/src/lib.rs:1-36):
 * serde_json::from_slice::<HashMap<String, u32>> of one value (de.rs
 * deserialize_map + MapAccess, keys deserialize_string, values through the
 * u32 PrimitiveVisitor of deserialize_number: visit_u64 / visit_i64 out of
 * range -> "invalid value: integer `N`, expected u32", anything else ->
 * "invalid type: ..., expected u32"; a float is outside the restatement).
 * Entries come back in text order, duplicates included (HashMap::insert:
 * the last value of a key wins).  0 = ok, ORC_E_UNSUPPORTED, or -1 with *msg.
 * ---------------------------------------------------------------------- */
static int deserialize_u32(jde *d, uint32_t *out) {
  int peek = parse_whitespace(d);
  if (peek < 0) return jpeek_error(d, E_EOF_VALUE);
  if (peek == '-' || isdig(peek)) {
    const int pos = peek != '-';
    if (!pos) jeat(d);
    jnum num;
    if (parse_integer(d, pos, &num)) return -1;
    if (num.is_float) { /* visit_f64: the u32 visitor's default, invalid_type(Unexpected::Float) */
      char fl[360];
      orc_display_point(num.f, fl, sizeof fl);
      jcustom(d, "invalid type: floating point `%s`, expected u32", fl);
      jfix_position(d);
      return -1;
    }
    if (num.neg || num.mag > 0xFFFFFFFFull) {
      if (num.neg)
        jcustom(d, "invalid value: integer `-%llu`, expected u32", (unsigned long long)num.mag);
      else
        jcustom(d, "invalid value: integer `%llu`, expected u32", (unsigned long long)num.mag);
      jfix_position(d);
      return -1;
    }
    *out = (uint32_t)num.mag;
    return 0;
  }
  return peek_invalid_type(d, "u32");
}

int orc_json_map_u32(const uint8_t *s, size_t n, uint8_t ***keys, size_t **klens, uint32_t **vals, size_t *count,
                     char **msg, size_t *msg_len) {
  jde d;
  memset(&d, 0, sizeof d);
  d.s = s;
  d.n = n;
  d.depth = 128;
  *msg = NULL;
  *keys = NULL;
  *klens = NULL;
  *vals = NULL;
  *count = 0;
  size_t cap = 0;
  int r = 0;
  int peek = parse_whitespace(&d);
  if (peek < 0) {
    r = jpeek_error(&d, E_EOF_VALUE);
  } else if (peek == '{') { /* deserialize_map */
    --d.depth;
    jeat(&d);
    int first = 1;
    for (;;) {
      int p = parse_whitespace(&d);
      if (p == '}') break;
      if (p == ',' && !first) {
        jeat(&d);
        p = parse_whitespace(&d);
      } else if (p >= 0) {
        if (first)
          first = 0;
        else {
          r = jpeek_error(&d, E_OBJ_COMMA);
          break;
        }
      } else {
        r = jpeek_error(&d, E_EOF_OBJECT);
        break;
      }
      if (p == '}') { r = jpeek_error(&d, E_TRAILING_COMMA); break; }
      if (p < 0) { r = jpeek_error(&d, E_EOF_VALUE); break; }
      if (p != '"') { r = jpeek_error(&d, E_KEY); break; }
      jeat(&d);
      jbuf key;
      if (parse_str(&d, &key)) {
        free(key.b);
        r = -1;
        break;
      }
      int c = parse_whitespace(&d);
      if (c == ':')
        jeat(&d);
      else if (c >= 0) {
        free(key.b);
        r = jpeek_error(&d, E_COLON);
        break;
      } else {
        free(key.b);
        r = jpeek_error(&d, E_EOF_OBJECT);
        break;
      }
      uint32_t v = 0;
      if (deserialize_u32(&d, &v)) {
        free(key.b);
        r = -1;
        break;
      }
      if (*count == cap) {
        cap = cap * 2 + 8;
        *keys = (uint8_t **)realloc(*keys, cap * sizeof(uint8_t *));
        *klens = (size_t *)realloc(*klens, cap * sizeof(size_t));
        *vals = (uint32_t *)realloc(*vals, cap * sizeof(uint32_t));
      }
      (*keys)[*count] = key.b ? key.b : (uint8_t *)malloc(1);
      (*klens)[*count] = key.n;
      (*vals)[*count] = v;
      (*count)++;
    }
    d.depth++;
    if (r) {
      jde probe = d;
      probe.msg = NULL;
      probe.msg_len = 0;
      probe.failed = 0;
      (void)end_map(&probe);
      free(probe.msg);
      d.i = probe.i;
    } else {
      r = end_map(&d);
    }
    if (r) jfix_position(&d);
  } else {
    r = peek_invalid_type(&d, "a map");
    jfix_position(&d);
  }
  if (!r && parse_whitespace(&d) >= 0) r = jpeek_error(&d, E_TRAILING); /* Deserializer::end */
  if (!r) {
    free(d.msg);
    return 0;
  }
  for (size_t k = 0; k < *count; k++) free((*keys)[k]);
  free(*keys);
  free(*klens);
  free(*vals);
  *keys = NULL;
  *klens = NULL;
  *vals = NULL;
  *count = 0;
  if (d.unsupported) {
    free(d.msg);
    return ORC_E_UNSUPPORTED;
  }
  *msg = render(&d, msg_len);
  free(d.msg);
  if (memchr(*msg, 0, *msg_len)) {
    free(*msg);
    *msg = NULL;
    return ORC_E_UNSUPPORTED;
  }
  return -1;
}

/* serde_json::to_vec_pretty of a map (ser.rs PrettyFormatter, two-space
 * indent): "{}" when empty, else "{\n  \"k\": v,\n  ...\n}" */
void orc_json_pretty_map(uint8_t *const *keys, const size_t *klens, const uint32_t *vals, size_t n, uint8_t **out,
                         size_t *out_len) {
  jbuf o = {0};
  jb_byte(&o, '{');
  for (size_t k = 0; k < n; k++) {
    jb_push(&o, (const uint8_t *)(k ? ",\n  " : "\n  "), k ? 4 : 3);
    canon_str(&o, keys[k], klens[k]);
    char num[16];
    int nl = snprintf(num, sizeof num, ": %u", vals[k]);
    jb_push(&o, (const uint8_t *)num, (size_t)nl);
  }
  if (n) jb_push(&o, (const uint8_t *)"\n}", 2);
  else jb_byte(&o, '}');
  *out = o.b;
  *out_len = o.n;
}
