/*
 * fsg_oracle.c — CPU ORACLE (test infrastructure, NOT the product).
 *
 * A scalar plain-C restatement of the reference SmartModule record-transform
 * path, written to be read side by side with the reference sources
 * (paths relative to /root/reference, deem0n/fluvio @ 2025-02-17):
 *
 *   varint          crates/fluvio-protocol/src/core/varint.rs:13-80
 *   Vec/Option/bool crates/fluvio-protocol/src/core/decoder.rs:39-97
 *   RecordData      crates/fluvio-protocol/src/record/data.rs:186-227
 *   Record          crates/fluvio-protocol/src/record/data.rs:375-562
 *   Batch + CRC32C  crates/fluvio-protocol/src/record/batch.rs:398-430, 444-508
 *   file framing    crates/fluvio-storage/src/iterators.rs:55-160
 *   chain process   crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:135-185
 *   guest loops     crates/fluvio-smartmodule-derive/src/generator/{filter,map,filter_map,
 *                   array_map,aggregate}.rs
 *   runtime error   crates/fluvio-protocol/src/link/smartmodule.rs:12-43
 *   process_batch   crates/fluvio-spu/src/smartengine/batch.rs:41-142
 *   modules         smartmodule/regex-filter/src/lib.rs, smartmodule/examples/<name>/src/lib.rs
 *
 * It is deliberately naive: it re-encodes and re-decodes between chain stages
 * exactly as engine.rs:163-166 does, allocates per record like the guest does,
 * and is single-threaded.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 */
#include "fsg_oracle.h"
#include "fsg_unicode.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int orc_u_dbg_escaped(uint32_t cp) { return fsg_u_dbg_escaped(cp); }

/* ------------------------------------------------------------------ */
/* growable byte buffer                                                 */
/* ------------------------------------------------------------------ */
typedef struct {
  uint8_t *p;
  size_t n, cap;
} obuf;

static void ob_reserve(obuf *b, size_t extra) {
  if (b->n + extra <= b->cap) return;
  size_t nc = b->cap ? b->cap : 64;
  while (nc < b->n + extra) nc *= 2;
  b->p = (uint8_t *)realloc(b->p, nc);
  b->cap = nc;
}
static void ob_put(obuf *b, const void *d, size_t n) {
  ob_reserve(b, n);
  if (n) memcpy(b->p + b->n, d, n);
  b->n += n;
}
static void ob_u8(obuf *b, uint8_t v) { ob_put(b, &v, 1); }
static void ob_be(obuf *b, uint64_t v, int nbytes) {
  uint8_t t[8];
  for (int i = 0; i < nbytes; i++) t[i] = (uint8_t)(v >> (8 * (nbytes - 1 - i)));
  ob_put(b, t, nbytes);
}
static void ob_free(obuf *b) {
  free(b->p);
  b->p = NULL;
  b->n = b->cap = 0;
}
static uint8_t *dup_bytes(const uint8_t *p, size_t n) {
  uint8_t *r = (uint8_t *)malloc(n ? n : 1);
  if (n) memcpy(r, p, n);
  return r;
}
static char *dup_str(const char *s) {
  size_t n = strlen(s);
  char *r = (char *)malloc(n + 1);
  memcpy(r, s, n + 1);
  return r;
}
static char *fmt_str(const char *f, ...) {
  va_list ap;
  va_start(ap, f);
  char tmp[512];
  vsnprintf(tmp, sizeof tmp, f, ap);
  va_end(ap);
  return dup_str(tmp);
}
void orc_free(void *p) { free(p); }

/* ------------------------------------------------------------------ */
/* CRC32C (Castagnoli, reflected 0x82F63B78), crc32c 0.6.4 semantics:  */
/* init 0xFFFFFFFF, final xor 0xFFFFFFFF.  batch.rs:425                 */
/* ------------------------------------------------------------------ */
static uint32_t crc_tab[256];
static int crc_init_done;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc_tab[i] = c;
  }
  crc_init_done = 1;
}
uint32_t orc_crc32c(const uint8_t *p, size_t n) {
  if (!crc_init_done) crc_init();
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

/* ------------------------------------------------------------------ */
/* varint (varint.rs:13-80).  Encoder quirk: zigzag with >>31 and loop  */
/* mask 0xffffff80 on an i64 (exact only for -2^31 <= n < 2^31).        */
/* ------------------------------------------------------------------ */
size_t orc_varint_encode(int64_t num, uint8_t *out) {
  int64_t v = (int64_t)(((uint64_t)num << 1) ^ (uint64_t)(num >> 31));
  size_t k = 0;
  while ((v & (int64_t)0xffffff80) != 0) {
    out[k++] = (uint8_t)((v & 0x7f) | 0x80);
    v >>= 7; /* arithmetic shift, as Rust i64 >>= */
  }
  out[k++] = (uint8_t)v;
  return k;
}
size_t orc_varint_size(int64_t num) {
  int64_t v = (int64_t)(((uint64_t)num << 1) ^ (uint64_t)(num >> 31));
  size_t bytes = 1;
  while ((v & (int64_t)0xffffff80) != 0) {
    bytes++;
    v >>= 7;
  }
  return bytes;
}
/* decoder: standard i64 zigzag; shift amount wraps mod 64 like release Rust */
int orc_varint_decode(const uint8_t *p, size_t n, int64_t *out, size_t *used) {
  uint64_t num = 0;
  unsigned shift = 0;
  size_t i = 0;
  for (;;) {
    if (i >= n) return -1;
    uint8_t b = p[i++];
    num |= ((uint64_t)(b & 0x7f)) << (shift & 63);
    shift += 7;
    if ((b & 0x80) == 0) break;
  }
  int64_t sn = (int64_t)num;
  *out = (int64_t)((uint64_t)(sn >> 1) ^ (uint64_t)(-(sn & 1)));
  *used = i;
  return 0;
}
static void ob_varint(obuf *b, int64_t v) {
  uint8_t t[16];
  size_t k = orc_varint_encode(v, t);
  ob_put(b, t, k);
}

/* ------------------------------------------------------------------ */
/* Record model + codec (data.rs:375-562)                               */
/* ------------------------------------------------------------------ */
typedef struct {
  int8_t attributes;
  int64_t ts_delta, off_delta;
  int has_key;
  uint8_t *key;
  size_t key_len;
  uint8_t *val;
  size_t val_len;
  int64_t headers;
} rec_t;

typedef struct {
  rec_t *r;
  size_t n, cap;
} recvec;

static void rv_push(recvec *v, rec_t r) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 16;
    v->r = (rec_t *)realloc(v->r, v->cap * sizeof(rec_t));
  }
  v->r[v->n++] = r;
}
static void rec_free(rec_t *r) {
  free(r->key);
  free(r->val);
  r->key = r->val = NULL;
}
static void rv_free(recvec *v) {
  for (size_t i = 0; i < v->n; i++) rec_free(&v->r[i]);
  free(v->r);
  v->r = NULL;
  v->n = v->cap = 0;
}
static rec_t rec_clone(const rec_t *s) {
  rec_t r = *s;
  r.key = s->has_key ? dup_bytes(s->key, s->key_len) : NULL;
  r.val = dup_bytes(s->val, s->val_len);
  return r;
}

/* cursor over a byte slice, Buf semantics */
typedef struct {
  const uint8_t *p;
  size_t n, i;
} cur_t;

static int cur_varint(cur_t *c, int64_t *v) {
  size_t used;
  if (orc_varint_decode(c->p + c->i, c->n - c->i, v, &used)) return -1;
  c->i += used;
  return 0;
}
/* RecordData::decode (data.rs:207-227): varint len, then src.take(len) —
 * copies min(len, remaining) bytes without error. */
static int cur_recdata(cur_t *c, uint8_t **out, size_t *out_len) {
  int64_t len;
  if (cur_varint(c, &len)) return -1;
  uint64_t want = (uint64_t)len; /* `len as usize` */
  size_t rem = c->n - c->i;
  size_t take = want < (uint64_t)rem ? (size_t)want : rem;
  *out = dup_bytes(c->p + c->i, take);
  *out_len = take;
  c->i += take;
  return 0;
}

/* Record::decode (data.rs:534-562).  returns 0 ok / -1 io error */
static int rec_decode(cur_t *c, rec_t *r) {
  memset(r, 0, sizeof *r);
  int64_t len;
  if (cur_varint(c, &len)) return -1;
  if ((int64_t)(c->n - c->i) < len) return -1; /* "not enough for record" */
  if (c->i >= c->n) return -1;
  r->attributes = (int8_t)c->p[c->i++];
  if (cur_varint(c, &r->ts_delta)) return -1;
  if (cur_varint(c, &r->off_delta)) return -1;
  /* Option<RecordData>: bool tag (0 false, 1 true, else error) */
  if (c->i >= c->n) return -1;
  uint8_t tag = c->p[c->i++];
  if (tag > 1) return -1;
  if (tag == 1) {
    r->has_key = 1;
    if (cur_recdata(c, &r->key, &r->key_len)) {
      rec_free(r);
      return -1;
    }
  }
  if (cur_recdata(c, &r->val, &r->val_len)) {
    rec_free(r);
    return -1;
  }
  if (cur_varint(c, &r->headers)) {
    rec_free(r);
    return -1;
  }
  return 0;
}

/* Vec<Record>::decode (decoder.rs:43-63): i32 BE count; < 1 -> empty */
static int recs_decode(const uint8_t *p, size_t n, recvec *out) {
  memset(out, 0, sizeof *out);
  if (n < 4) return -1;
  int32_t cnt = (int32_t)(((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]);
  if (cnt < 1) return 0;
  cur_t c = {p, n, 4};
  for (int32_t k = 0; k < cnt; k++) {
    rec_t r;
    if (rec_decode(&c, &r)) {
      rv_free(out);
      return -1;
    }
    rv_push(out, r);
  }
  return 0;
}

/* Record::write_size / encode (data.rs:504-532) */
static size_t recdata_size(size_t len) { return orc_varint_size((int64_t)len) + len; }
static size_t rec_inner_size(const rec_t *r) {
  size_t s = 1 + orc_varint_size(r->ts_delta) + orc_varint_size(r->off_delta);
  s += 1 + (r->has_key ? recdata_size(r->key_len) : 0);
  s += recdata_size(r->val_len);
  s += orc_varint_size(r->headers);
  return s;
}
static size_t rec_size(const rec_t *r) {
  size_t in = rec_inner_size(r);
  return orc_varint_size((int64_t)in) + in;
}
static void rec_encode(obuf *b, const rec_t *r) {
  ob_varint(b, (int64_t)rec_inner_size(r));
  ob_u8(b, (uint8_t)r->attributes);
  ob_varint(b, r->ts_delta);
  ob_varint(b, r->off_delta);
  if (r->has_key) {
    ob_u8(b, 1);
    ob_varint(b, (int64_t)r->key_len);
    ob_put(b, r->key, r->key_len);
  } else {
    ob_u8(b, 0);
  }
  ob_varint(b, (int64_t)r->val_len);
  ob_put(b, r->val, r->val_len);
  ob_varint(b, r->headers);
}
static void recs_encode(obuf *b, const recvec *v) {
  ob_be(b, (uint32_t)v->n, 4);
  for (size_t i = 0; i < v->n; i++) rec_encode(b, &v->r[i]);
}
static size_t recs_size(const recvec *v) {
  size_t s = 4;
  for (size_t i = 0; i < v->n; i++) s += rec_size(&v->r[i]);
  return s;
}

/* ------------------------------------------------------------------ */
/* Rust core::str::from_utf8 (run_utf8_validation)                      */
/* returns 1 valid; else 0 with valid_up_to and error_len (0 = None)    */
/* ------------------------------------------------------------------ */
static int utf8_check(const uint8_t *s, size_t n, size_t *valid_up_to, int *error_len) {
  size_t i = 0;
  while (i < n) {
    uint8_t f = s[i];
    if (f < 0x80) {
      i++;
      continue;
    }
    int w = (f >= 0xC2 && f <= 0xDF) ? 2 : (f >= 0xE0 && f <= 0xEF) ? 3 : (f >= 0xF0 && f <= 0xF4) ? 4 : 0;
#define U8ERR(L)        \
  do {                  \
    *valid_up_to = i;   \
    *error_len = (L);   \
    return 0;           \
  } while (0)
#define U8NEXT(k) ((i + (k) < n) ? (int)s[i + (k)] : -1)
    if (w == 0) U8ERR(1);
    int b1 = U8NEXT(1);
    if (b1 < 0) U8ERR(0);
    if (w == 2) {
      if ((b1 & 0xC0) != 0x80) U8ERR(1);
      i += 2;
      continue;
    }
    int ok1;
    if (w == 3)
      ok1 = (f == 0xE0 && b1 >= 0xA0 && b1 <= 0xBF) || (f >= 0xE1 && f <= 0xEC && b1 >= 0x80 && b1 <= 0xBF) ||
            (f == 0xED && b1 >= 0x80 && b1 <= 0x9F) || (f >= 0xEE && f <= 0xEF && b1 >= 0x80 && b1 <= 0xBF);
    else
      ok1 = (f == 0xF0 && b1 >= 0x90 && b1 <= 0xBF) || (f >= 0xF1 && f <= 0xF3 && b1 >= 0x80 && b1 <= 0xBF) ||
            (f == 0xF4 && b1 >= 0x80 && b1 <= 0x8F);
    if (!ok1) U8ERR(1);
    int b2 = U8NEXT(2);
    if (b2 < 0) U8ERR(0);
    if ((b2 & 0xC0) != 0x80) U8ERR(2);
    if (w == 3) {
      i += 3;
      continue;
    }
    int b3 = U8NEXT(3);
    if (b3 < 0) U8ERR(0);
    if ((b3 & 0xC0) != 0x80) U8ERR(3);
    i += 4;
#undef U8ERR
#undef U8NEXT
  }
  return 1;
}
static char *utf8_hint(size_t vut, int elen) {
  if (elen) return fmt_str("invalid utf-8 sequence of %d bytes from index %zu", elen, vut);
  return fmt_str("incomplete utf-8 byte sequence from index %zu", vut);
}
/* decode validated UTF-8 to code points */
static uint32_t *utf8_decode(const uint8_t *s, size_t n, size_t *out_n) {
  uint32_t *cp = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
  size_t k = 0, i = 0;
  while (i < n) {
    uint8_t f = s[i];
    if (f < 0x80) {
      cp[k++] = f;
      i++;
    } else if (f < 0xE0) {
      cp[k++] = ((uint32_t)(f & 0x1F) << 6) | (s[i + 1] & 0x3F);
      i += 2;
    } else if (f < 0xF0) {
      cp[k++] = ((uint32_t)(f & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
      i += 3;
    } else {
      cp[k++] = ((uint32_t)(f & 0x07) << 18) | ((uint32_t)(s[i + 1] & 0x3F) << 12) |
                ((uint32_t)(s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
      i += 4;
    }
  }
  *out_n = k;
  return cp;
}

/* char::is_whitespace (White_Space property) */
static int cp_is_ws(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F ||
         c == 0x3000;
}

/* str::trim on validated UTF-8 -> [*b, *e) byte range */
static void utf8_trim(const uint8_t *s, size_t n, size_t *b, size_t *e) {
  size_t i = 0;
  while (i < n) {
    uint8_t f = s[i];
    size_t w = f < 0x80 ? 1 : f < 0xE0 ? 2 : f < 0xF0 ? 3 : 4;
    size_t cn;
    uint32_t *cp = utf8_decode(s + i, w, &cn);
    int ws = cp_is_ws(cp[0]);
    free(cp);
    if (!ws) break;
    i += w;
  }
  size_t j = n;
  while (j > i) {
    size_t k = j - 1;
    while (k > i && (s[k] & 0xC0) == 0x80) k--;
    size_t cn;
    uint32_t *cp = utf8_decode(s + k, j - k, &cn);
    int ws = cp_is_ws(cp[0]);
    free(cp);
    if (!ws) break;
    j = k;
  }
  *b = i;
  *e = j;
}

/* <i32 as FromStr>::from_str (core::num, radix 10).  0 ok, else kind:
 * 1 Empty, 2 InvalidDigit, 3 PosOverflow, 4 NegOverflow */
static int parse_i32(const uint8_t *s, size_t n, int32_t *out) {
  if (n == 0) return 1;
  size_t i = 0;
  int pos = 1;
  if ((s[0] == '+' || s[0] == '-') && n == 1) return 2;
  if (s[0] == '+')
    i = 1;
  else if (s[0] == '-') {
    pos = 0;
    i = 1;
  }
  int64_t acc = 0;
  for (; i < n; i++) {
    uint8_t c = s[i];
    if (c < '0' || c > '9') return 2;
    int d = c - '0';
    if (pos) {
      acc = acc * 10 + d;
      if (acc > 2147483647LL) return 3;
    } else {
      acc = acc * 10 - d;
      if (acc < -2147483648LL) return 4;
    }
  }
  *out = (int32_t)acc;
  return 0;
}
static const char *parse_int_hint(int kind) {
  switch (kind) {
    case 1: return "cannot parse integer from empty string";
    case 2: return "invalid digit found in string";
    case 3: return "number too large to fit in target type";
    default: return "number too small to fit in target type";
  }
}

/* ------------------------------------------------------------------ */
/* Regex oracle: parser for the supported Rust-regex subset + Pike VM   */
/* over Unicode scalar values.  (regex 1.6.0 / 1.8.1 is a third-party   */
/* dependency absent from /root/reference; its published semantics:     */
/* unanchored is_match, Unicode-aware '.', \d (Nd), \s (White_Space).)  */
/* ------------------------------------------------------------------ */
typedef struct {
  uint32_t lo, hi;
} cprange;

static const cprange ND_TAB[] = {
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
static const cprange WS_TAB[] = {{0x09, 0x0D}, {0x20, 0x20},     {0x85, 0x85},     {0xA0, 0xA0},
                                 {0x1680, 0x1680}, {0x2000, 0x200A}, {0x2028, 0x2029}, {0x202F, 0x202F},
                                 {0x205F, 0x205F}, {0x3000, 0x3000}};
static const cprange WORD_ASCII[] = {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}};
static const cprange DIGIT_ASCII[] = {{'0', '9'}};
static const cprange SPACE_ASCII[] = {{'\t', '\r'}, {' ', ' '}}; /* (?-u)\s */

typedef struct {
  cprange *r;
  size_t n, cap;
} cset;

static void cs_add(cset *s, uint32_t lo, uint32_t hi) {
  if (s->n == s->cap) {
    s->cap = s->cap ? s->cap * 2 : 8;
    s->r = (cprange *)realloc(s->r, s->cap * sizeof(cprange));
  }
  s->r[s->n].lo = lo;
  s->r[s->n].hi = hi;
  s->n++;
}
static int cmp_range(const void *a, const void *b) {
  const cprange *x = (const cprange *)a, *y = (const cprange *)b;
  return x->lo < y->lo ? -1 : x->lo > y->lo ? 1 : 0;
}
static void cs_norm(cset *s) {
  if (!s->n) return;
  qsort(s->r, s->n, sizeof(cprange), cmp_range);
  size_t k = 0;
  for (size_t i = 1; i < s->n; i++) {
    if (s->r[i].lo <= s->r[k].hi + 1) {
      if (s->r[i].hi > s->r[k].hi) s->r[k].hi = s->r[i].hi;
    } else
      s->r[++k] = s->r[i];
  }
  s->n = k + 1;
}
static void cs_negate(cset *s) {
  cs_norm(s);
  cset o = {0};
  uint32_t next = 0;
  for (size_t i = 0; i < s->n; i++) {
    if (s->r[i].lo > next) cs_add(&o, next, s->r[i].lo - 1);
    next = s->r[i].hi + 1;
  }
  if (next <= 0x10FFFF) cs_add(&o, next, 0x10FFFF);
  free(s->r);
  *s = o;
}
static void cs_add_tab(cset *s, const cprange *t, size_t n, int neg) {
  cset tmp = {0};
  for (size_t i = 0; i < n; i++) cs_add(&tmp, t[i].lo, t[i].hi);
  if (neg) cs_negate(&tmp);
  for (size_t i = 0; i < tmp.n; i++) cs_add(s, tmp.r[i].lo, tmp.r[i].hi);
  free(tmp.r);
}
/* class set operations (regex-syntax ClassSetBinaryOpKind): *a = *a op *b;
 * op 1 intersection (&&), 2 difference (--), 3 symmetric difference (~~) */
static void cs_copy(cset *d, const cset *s) {
  for (size_t i = 0; i < s->n; i++) cs_add(d, s->r[i].lo, s->r[i].hi);
}
static void cs_binop(cset *a, const cset *b, int op) {
  cset na = {0}, nb = {0}, t = {0};
  cs_copy(&na, a);
  cs_copy(&nb, b);
  if (op == 1) { /* a & b = ~(~a | ~b) */
    cs_negate(&na);
    cs_negate(&nb);
    cs_copy(&na, &nb);
    cs_negate(&na);
    free(a->r);
    *a = na;
    free(nb.r);
    return;
  }
  if (op == 2) { /* a - b = ~(~a | b) */
    cs_negate(&na);
    cs_copy(&na, b);
    cs_negate(&na);
    free(a->r);
    *a = na;
    free(nb.r);
    return;
  }
  /* a ^ b = (a - b) | (b - a) */
  cs_binop(&na, b, 2);
  cs_binop(&nb, a, 2);
  cs_copy(&t, &na);
  cs_copy(&t, &nb);
  cs_norm(&t);
  free(na.r);
  free(nb.r);
  free(a->r);
  *a = t;
}
static int cs_has(const cset *s, uint32_t c) {
  size_t lo = 0, hi = s->n;
  while (lo < hi) {
    size_t m = (lo + hi) / 2;
    if (c < s->r[m].lo)
      hi = m;
    else if (c > s->r[m].hi)
      lo = m + 1;
    else
      return 1;
  }
  return 0;
}

enum { RX_CHAR, RX_CLASS, RX_SPLIT, RX_JMP, RX_BOL, RX_EOL, RX_MATCH, RX_WB, RX_NWB, RX_MBOL, RX_MEOL };
typedef struct {
  int op;
  uint32_t c;
  int x, y;
} rxins;

typedef struct {
  rxins *prog;
  size_t n, cap;
  cset *classes;
  size_t ncls, ccap;
  int unicode_word; /* \b / \B used */
  int ascii_wb;     /* a (?-u) \b / \B among them: bytes inside a code point, exact only on ASCII input */
  int utab;         /* version-dependent tables: a fsg_u_newer code point in the text is unsupported */
} rxprog;

/* AST */
enum { A_EMPTY, A_CHAR, A_CLASS, A_CAT, A_ALT, A_REP, A_BOL, A_EOL, A_WB, A_NWB, A_MBOL, A_MEOL };
typedef struct anode {
  int t;
  uint32_t c;
  cset cls;
  struct anode **kids;
  size_t nk;
  int min, max; /* max -1 = inf */
  struct anode *sub;
} anode;

typedef struct {
  const uint32_t *p;
  size_t n, i;
  int err;
  int unsupported;
  int depth;
  int fi, fs;   /* inline flags i (case-insensitive), s (. matches \n); U only swaps greed */
  int fm, fx, fu; /* m: ^ $ at line boundaries; x: whitespace / # comments ignored; u: Unicode classes (on) */
  int word;     /* \b or \B used */
  int wba;      /* \b or \B under (?-u) */
  int utab;     /* a version-dependent Unicode table used (\d \w \p, (?i) folding, Unicode \b) */
  int perr;     /* the first \p name regex-syntax rejects: 2 value not found, 3 property not found */
  size_t perr_lo, perr_hi; /* its span, code-point offsets [lo, hi) */
} rxparser;

/* x: whitespace (White_Space) and # comments between tokens are skipped */
static void rx_skip_x(rxparser *P) {
  while (P->fx && P->i < P->n) {
    uint32_t c = P->p[P->i];
    int ws = 0;
    for (size_t k = 0; k < sizeof WS_TAB / sizeof WS_TAB[0]; k++) ws |= c >= WS_TAB[k].lo && c <= WS_TAB[k].hi;
    if (ws) {
      P->i++;
    } else if (c == '#') {
      while (P->i < P->n && P->p[P->i] != '\n') P->i++;
    } else {
      break;
    }
  }
}
static void cs_fold_add(void *ctx, uint32_t c) { cs_add((cset *)ctx, c, c); }
/* \p{name} / \pX (after the p / P): General_Category values and groups, Any,
 * ASCII, Assigned, White_Space, binary properties, Script / Script_Extensions
 * values; names compared without case, ' ', '_', '-' */
static int rx_property(rxparser *P, int neg, cset *set) {
  if (!P->fu) {
    P->err = 1;
    return 0;
  }
  const size_t at0 = P->i - 2; /* the escape's backslash */
  char name[64];
  size_t nl = 0;
  if (P->i < P->n && P->p[P->i] == '{') {
    P->i++;
    if (P->i < P->n && P->p[P->i] == '^') {
      neg = !neg;
      P->i++;
    }
    /* regex-syntax: the raw text splits at its first ':' / '='; each part is
     * normalized alone (symbolic_name_normalize): a raw "is" prefix dropped
     * ("isc" kept), ' ', '_', '-' removed, ASCII lowercased */
    int split = 0, start = 1, is_pfx = 0;
    size_t p0 = 0; /* where the current part starts in name */
    while (P->i < P->n && P->p[P->i] != '}') {
      uint32_t c = P->p[P->i++];
      if (c >= 0x80 || nl + 4 >= sizeof name) {
        P->unsupported = 1;
        return 0;
      }
      if (!split && (c == ':' || c == '=')) {
        if (is_pfx && nl - p0 == 1 && name[p0] == 'c') nl = p0 + (size_t)sprintf(name + p0, "isc");
        name[nl++] = '=';
        split = 1;
        start = 1;
        p0 = nl;
        continue;
      }
      if (start) {
        start = 0;
        uint32_t c2 = P->i < P->n ? P->p[P->i] : 0;
        if ((c | 0x20) == 'i' && (c2 | 0x20) == 's') {
          is_pfx = 1;
          P->i++;
          continue;
        }
        is_pfx = 0;
      }
      if (c == ' ' || c == '_' || c == '-') continue;
      name[nl++] = (char)((c >= 'A' && c <= 'Z') ? c + 32 : c);
    }
    if (is_pfx && nl - p0 == 1 && name[p0] == 'c') nl = p0 + (size_t)sprintf(name + p0, "isc");
    if (P->i >= P->n) {
      P->err = 1;
      return 0;
    }
    P->i++;
  } else {
    if (P->i >= P->n || P->p[P->i] >= 0x80) {
      P->err = 1;
      return 0;
    }
    uint32_t c = P->p[P->i++];
    name[nl++] = (char)((c >= 'A' && c <= 'Z') ? c + 32 : c);
  }
  name[nl] = 0;
  long m = fsg_u_property(name);
  cset tmp = {0};
  if (m == FSG_UPROP_ASCII) {
    cs_add(&tmp, 0, 0x7F);
  } else if (m == FSG_UPROP_WSPACE) {
    cs_add_tab(&tmp, WS_TAB, sizeof WS_TAB / sizeof WS_TAB[0], 0);
  } else if (m >= 0) {
    for (uint32_t k = 0; k < fsg_u_ncats; k++)
      if (m & (1L << k))
        for (uint32_t q = 0; q < fsg_u_cats[k].n; q++) cs_add(&tmp, fsg_u_cats[k].r[q].lo, fsg_u_cats[k].r[q].hi);
  } else { /* binary properties, Script / Script_Extensions values */
    const fsg_urange *pr = NULL;
    uint32_t pn = 0;
    if (!fsg_u_lookup(name, &pr, &pn)) {
      const int k = fsg_u_unresolved(name);
      if (k == 1) {
        P->unsupported = 1; /* Age values, CWKCF: known to regex-syntax, not restated */
        return 0;
      }
      if (!P->perr) { /* Regex::new fails; reported after the whole pattern parsed */
        P->perr = k;
        P->perr_lo = at0;
        P->perr_hi = P->i;
      }
      return 2;
    }
    for (uint32_t q = 0; q < pn; q++) cs_add(&tmp, pr[q].lo, pr[q].hi);
  }
  if (m != FSG_UPROP_ASCII && m != FSG_UPROP_WSPACE) P->utab = 1;
  if (P->fi) { /* (?i): simple case folding before the negation */
    P->utab = 1;
    size_t n0 = tmp.n;
    for (size_t q = 0; q < n0; q++) fsg_u_fold_range(tmp.r[q].lo, tmp.r[q].hi, cs_fold_add, &tmp);
  }
  cs_norm(&tmp);
  if (neg) cs_negate(&tmp);
  for (size_t q = 0; q < tmp.n; q++) cs_add(set, tmp.r[q].lo, tmp.r[q].hi);
  free(tmp.r);
  return 2;
}

/* (?i): regex-syntax's simple case folding (CaseFolding.txt C + S orbits,
 * fsg_unicode.h) in Unicode mode; (?-u) folds ASCII letters only (bytes). */
static void cs_add_folded(rxparser *P, cset *s, uint32_t lo, uint32_t hi) {
  cs_add(s, lo, hi);
  if (!P->fi) return;
  if (P->fu) {
    P->utab = 1;
    fsg_u_fold_range(lo, hi, cs_fold_add, s);
    return;
  }
  if (hi >= 0x80) {
    P->unsupported = 1;
    return;
  }
  uint32_t a = lo > 'a' ? lo : 'a', b = hi < 'z' ? hi : 'z';
  if (a <= b) cs_add(s, a - 32, b - 32);
  a = lo > 'A' ? lo : 'A';
  b = hi < 'Z' ? hi : 'Z';
  if (a <= b) cs_add(s, a + 32, b + 32);
}
/* [[:name:]] ASCII classes (regex-syntax ast ClassAsciiKind) */
static int posix_class(const uint32_t *p, size_t n, cset *s) {
  static const struct {
    const char *name;
    uint32_t r[5][2];
  } T[] = {{"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}},
           {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
           {"ascii", {{0, 0x7F}}},
           {"blank", {{'\t', '\t'}, {' ', ' '}}},
           {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
           {"digit", {{'0', '9'}}},
           {"graph", {{'!', '~'}}},
           {"lower", {{'a', 'z'}}},
           {"print", {{' ', '~'}}},
           {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}},
           {"space", {{'\t', '\r'}, {' ', ' '}}},
           {"upper", {{'A', 'Z'}}},
           {"word", {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
           {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}}};
  for (size_t k = 0; k < sizeof T / sizeof T[0]; k++) {
    size_t L = strlen(T[k].name);
    if (L != n) continue;
    size_t j = 0;
    while (j < L && p[j] == (uint32_t)T[k].name[j]) j++;
    if (j < L) continue;
    for (int q = 0; q < 5 && (q == 0 || T[k].r[q][1]); q++) cs_add(s, T[k].r[q][0], T[k].r[q][1]);
    return 1;
  }
  return 0;
}

static anode *an_new(int t) {
  anode *a = (anode *)calloc(1, sizeof(anode));
  a->t = t;
  return a;
}
static void an_push(anode *a, anode *k) {
  a->kids = (anode **)realloc(a->kids, (a->nk + 1) * sizeof(anode *));
  a->kids[a->nk++] = k;
}
static void an_free(anode *a) {
  if (!a) return;
  for (size_t i = 0; i < a->nk; i++) an_free(a->kids[i]);
  free(a->kids);
  an_free(a->sub);
  free(a->cls.r);
  free(a);
}

static anode *rx_parse_alt(rxparser *P);

static int is_hex(uint32_t c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
static uint32_t hexv(uint32_t c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }

/* parse an escape after '\'; fills either *single (returns 1) or set (returns 2) */
static int rx_escape(rxparser *P, uint32_t *single, cset *set, int in_class) {
  if (P->i >= P->n) {
    P->err = 1;
    return 0;
  }
  uint32_t c = P->p[P->i++];
  switch (c) {
    case 'd': case 'D': case 's': case 'S': case 'w': case 'W': {
      const int neg = c < 'a', k = c | 0x20;
      if (neg && !P->fu) { /* (?-u)\D \S \W can match invalid UTF-8 */
        P->err = 1;
        return 0;
      }
      if (P->fu && k != 's') P->utab = 1; /* White_Space is the same in every version */
      if (k == 'd') {
        if (P->fu) cs_add_tab(set, ND_TAB, sizeof ND_TAB / sizeof ND_TAB[0], neg);
        else cs_add_tab(set, DIGIT_ASCII, 1, 0);
      } else if (k == 's') {
        if (P->fu) cs_add_tab(set, WS_TAB, sizeof WS_TAB / sizeof WS_TAB[0], neg);
        else cs_add_tab(set, SPACE_ASCII, 2, 0);
      } else if (P->fu) {
        cs_add_tab(set, (const cprange *)fsg_u_word, fsg_u_word_n, neg); /* Alphabetic + M + Nd + Pc + Join_Control */
      } else {
        cs_add_tab(set, WORD_ASCII, 4, 0);
      }
      return 2;
    }
    case 'p': case 'P': return rx_property(P, c == 'P', set);
    case 'b': case 'B': /* word boundary assertions (Unicode \w: exact on ASCII input) */
      if (in_class) {
        P->err = 1;
        return 0;
      }
      P->word = 1;
      if (!P->fu) P->wba = 1;
      else P->utab = 1;
      return c == 'b' ? 3 : 4;
    case 'A': return in_class ? (P->err = 1, 0) : 5; /* start of text (= ^ without m) */
    case 'z': return in_class ? (P->err = 1, 0) : 6; /* end of text (= $ without m) */
    case 'n': *single = '\n'; return 1;
    case 't': *single = '\t'; return 1;
    case 'r': *single = '\r'; return 1;
    case 'f': *single = '\f'; return 1;
    case 'v': *single = '\v'; return 1;
    case 'a': *single = 7; return 1;
    case 'x': case 'u': case 'U': { /* \x7F \x{..}, \u007F \u{..}, \U0000007F \U{..} (regex-syntax parse_hex) */
      const int fixed = c == 'x' ? 2 : c == 'u' ? 4 : 8;
      uint32_t v = 0;
      if (P->i < P->n && P->p[P->i] == '{') {
        P->i++;
        int nd = 0;
        while (P->i < P->n && is_hex(P->p[P->i])) {
          v = v * 16 + hexv(P->p[P->i++]);
          nd++;
          if (nd > 8) break;
        }
        if (P->i >= P->n || P->p[P->i] != '}' || nd == 0 || v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) {
          P->err = 1;
          return 0;
        }
        P->i++;
      } else {
        for (int k = 0; k < fixed; k++) {
          if (P->i >= P->n || !is_hex(P->p[P->i])) {
            P->err = 1;
            return 0;
          }
          v = v * 16 + hexv(P->p[P->i++]);
        }
        if (v > 0x10FFFF || (v >= 0xD800 && v <= 0xDFFF)) {
          P->err = 1;
          return 0;
        }
      }
      *single = v;
      return 1;
    }
    default:
      if (c < 0x80 && !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'))) {
        *single = c; /* escaped punctuation / meta */
        return 1;
      }
      P->err = 1;
      return 0;
  }
}

/* a bracketed class after its '[' through the matching ']' (regex-syntax
 * parse_set_class): the items of a union; a nested bracket is an item; the
 * operators && -- ~~ are left-associative and bind looser than the union; a
 * leading ']' and leading '-'s are literals; the negation applies last.
 * Returns 0 ok (the set in *out), -1 on err / unsupported (flags in P). */
static int rx_parse_bracket(rxparser *P, cset *out) {
  int neg = 0;
  if (P->i < P->n && P->p[P->i] == '^') {
    neg = 1;
    P->i++;
  }
  cset uni = {0}, lhs = {0};
  int op = 0, first = 1;
#define RX_LIT(lo_, hi_)                                                                     \
  do {                                                                                       \
    if (!P->fu && (hi_) >= 0x80) { /* class_literal_byte: UnicodeNotAllowed in a (?-u) class */ \
      P->err = 1;                                                                            \
      goto fail;                                                                             \
    }                                                                                        \
    cs_add_folded(P, &uni, (lo_), (hi_));                                                    \
  } while (0)
  for (;;) {
    rx_skip_x(P);
    if (P->i >= P->n) {
      P->err = 1;
      goto fail;
    }
    uint32_t c = P->p[P->i];
    if (first) { /* parse_set_class_open: a leading ']' and any leading '-' are literals */
      first = 0;
      if (c == ']') {
        P->i++;
        RX_LIT(']', ']');
        continue;
      }
      if (c == '-') {
        while (P->i < P->n && P->p[P->i] == '-') {
          P->i++;
          RX_LIT('-', '-');
        }
        continue;
      }
    }
    if (c == ']') {
      P->i++;
      break;
    }
    if (c == '[' && P->i + 1 < P->n && P->p[P->i + 1] == ':') { /* [:name:] / [:^name:] */
      size_t j = P->i + 2;
      int pneg = 0;
      if (j < P->n && P->p[j] == '^') {
        pneg = 1;
        j++;
      }
      size_t k = j;
      while (k + 1 < P->n && !(P->p[k] == ':' && P->p[k + 1] == ']')) k++;
      cset tmp = {0};
      if (k + 1 < P->n && posix_class(P->p + j, k - j, &tmp)) {
        if (pneg) cs_negate(&tmp);
        for (size_t q = 0; q < tmp.n; q++) cs_add_folded(P, &uni, tmp.r[q].lo, tmp.r[q].hi);
        free(tmp.r);
        P->i = k + 2;
        continue;
      }
      free(tmp.r);
    }
    if (c == '[') { /* a nested class: one item of the union */
      P->i++;
      cset in = {0};
      if (++P->depth > 64) {
        P->unsupported = 1;
        goto fail;
      }
      int r = rx_parse_bracket(P, &in);
      P->depth--;
      if (r) {
        free(in.r);
        goto fail;
      }
      cs_copy(&uni, &in);
      free(in.r);
      continue;
    }
    if ((c == '&' || c == '-' || c == '~') && P->i + 1 < P->n && P->p[P->i + 1] == c) {
      P->i += 2;
      if (op == 0) {
        cs_copy(&lhs, &uni);
        cs_norm(&lhs);
      } else {
        cs_binop(&lhs, &uni, op);
      }
      free(uni.r);
      memset(&uni, 0, sizeof uni);
      op = c == '&' ? 1 : c == '-' ? 2 : 3;
      continue;
    }
    uint32_t lo;
    P->i++;
    if (c == '\\') {
      cset tmp = {0};
      int k = rx_escape(P, &lo, &tmp, 1);
      if (k == 2) {
        cs_copy(&uni, &tmp);
        free(tmp.r);
        continue;
      }
      free(tmp.r);
      if (k >= 3) P->err = 1;
      if (k != 1) goto fail;
    } else {
      lo = c;
    }
    uint32_t hi = lo;
    /* parse_set_class_range: bump_space, then '-' starts a range unless the next
     * non-space char is ']' or '-' */
    rx_skip_x(P);
    size_t nx = P->i + 1;
    if (P->fx && P->i < P->n) {
      const size_t at_dash = P->i;
      P->i = nx;
      rx_skip_x(P);
      nx = P->i;
      P->i = at_dash;
    }
    if (P->i < P->n && P->p[P->i] == '-' && nx < P->n && P->p[nx] != ']' && P->p[nx] != '-') {
      P->i = nx;
      uint32_t c2 = P->p[P->i++];
      if (c2 == '\\') {
        cset tmp = {0};
        int k = rx_escape(P, &hi, &tmp, 1);
        free(tmp.r);
        if (k != 1) {
          if (k == 2) P->err = 1;
          goto fail;
        }
      } else
        hi = c2;
      if (hi < lo) {
        P->err = 1;
        goto fail;
      }
    }
    RX_LIT(lo, hi);
  }
#undef RX_LIT
  if (op == 0) {
    cs_norm(&uni);
    *out = uni;
  } else {
    cs_binop(&lhs, &uni, op);
    free(uni.r);
    *out = lhs;
    memset(&lhs, 0, sizeof lhs);
  }
  free(lhs.r);
  if (neg) cs_negate(out); /* case folding applies before the negation */
  cs_norm(out);
  return 0;
fail:
  free(uni.r);
  free(lhs.r);
  return -1;
}
static anode *rx_parse_class(rxparser *P) {
  /* after '[' */
  anode *a = an_new(A_CLASS);
  if (rx_parse_bracket(P, &a->cls)) return a;
  /* (?-u): a class that can match a byte >= 0x80 can match invalid UTF-8 (Regex on &str) */
  if (!P->fu && a->cls.n && a->cls.r[a->cls.n - 1].hi >= 0x80) P->err = 1;
  return a;
}

static int rx_parse_int(rxparser *P, int *v) {
  int nd = 0;
  long x = 0;
  while (P->i < P->n && P->p[P->i] >= '0' && P->p[P->i] <= '9') {
    x = x * 10 + (P->p[P->i++] - '0');
    if (x > 100000) x = 100000;
    nd++;
  }
  *v = (int)x;
  return nd;
}

static anode *rx_parse_atom(rxparser *P) {
  uint32_t c = P->p[P->i++];
  if (c == '(') {
    if (P->i < P->n && P->p[P->i] == '?') {
      P->i++;
      if (P->i < P->n && P->p[P->i] == ':') {
        P->i++;
      } else if (P->i < P->n && (P->p[P->i] == 'P' || P->p[P->i] == '<')) {
        if (P->p[P->i] == 'P') P->i++;
        if (P->i >= P->n || P->p[P->i] != '<') {
          P->err = 1;
          return an_new(A_EMPTY);
        }
        while (P->i < P->n && P->p[P->i] != '>') P->i++;
        if (P->i >= P->n) {
          P->err = 1;
          return an_new(A_EMPTY);
        }
        P->i++;
      } else {
        /* inline flags (?flags) / (?flags:re): i, s, U supported; m, x, u, R not */
        int neg = 0, nflags = 0, fi = P->fi, fs = P->fs, fm = P->fm, fx = P->fx, fu = P->fu;
        for (;;) {
          if (P->i >= P->n) {
            P->err = 1;
            return an_new(A_EMPTY);
          }
          uint32_t f = P->p[P->i++];
          if (f == ':' || f == ')') {
            if (!nflags || neg == 1) { /* "(?)" / "(?-)" / "(?i-)" are errors */
              P->err = 1;
              return an_new(A_EMPTY);
            }
            if (f == ')') { /* until the end of the enclosing group */
              P->fi = fi;
              P->fs = fs;
              P->fm = fm;
              P->fx = fx;
              P->fu = fu;
              return an_new(A_EMPTY);
            }
            break;
          }
          if (f == '-') {
            if (neg) {
              P->err = 1;
              return an_new(A_EMPTY);
            }
            neg = 1;
            continue;
          }
          if (f == 'i') fi = !neg;
          else if (f == 's') fs = !neg;
          else if (f == 'U') { /* greed only: same language */ }
          else if (f == 'm') fm = !neg;
          else if (f == 'x') fx = !neg;
          else if (f == 'u') fu = !neg;
          else if (f == 'R') { /* CRLF mode (regex 1.8): not restated */
            P->unsupported = 1;
            return an_new(A_EMPTY);
          } else {
            P->err = 1;
            return an_new(A_EMPTY);
          }
          nflags++;
          if (neg) neg = 2;
        }
        int sfi = P->fi, sfs = P->fs, sfm = P->fm, sfx = P->fx, sfu = P->fu;
        P->fi = fi;
        P->fs = fs;
        P->fm = fm;
        P->fx = fx;
        P->fu = fu;
        if (++P->depth > 200) {
          P->err = 1;
          return an_new(A_EMPTY);
        }
        anode *g = rx_parse_alt(P);
        P->depth--;
        P->fi = sfi;
        P->fs = sfs;
        P->fm = sfm;
        P->fx = sfx;
        P->fu = sfu;
        if (P->i >= P->n || P->p[P->i] != ')') {
          P->err = 1;
          return g;
        }
        P->i++;
        return g;
      }
    }
    if (++P->depth > 200) {
      P->err = 1;
      return an_new(A_EMPTY);
    }
    int sfi = P->fi, sfs = P->fs, sfm = P->fm, sfx = P->fx, sfu = P->fu; /* flags set inside a group end with it */
    anode *g = rx_parse_alt(P);
    P->depth--;
    P->fi = sfi;
    P->fs = sfs;
    P->fm = sfm;
    P->fx = sfx;
    P->fu = sfu;
    if (P->i >= P->n || P->p[P->i] != ')') {
      P->err = 1;
      return g;
    }
    P->i++;
    return g;
  }
  if (c == '[') return rx_parse_class(P);
  if (c == '.') {
    if (!P->fu) { /* (?-u:.) can match invalid UTF-8 */
      P->err = 1;
      return an_new(A_EMPTY);
    }
    anode *a = an_new(A_CLASS);
    if (P->fs) {
      cs_add(&a->cls, 0, 0x10FFFF);
    } else {
      cs_add(&a->cls, 0, '\n' - 1);
      cs_add(&a->cls, '\n' + 1, 0x10FFFF);
    }
    return a;
  }
  if (c == '^') return an_new(P->fm ? A_MBOL : A_BOL);
  if (c == '$') return an_new(P->fm ? A_MEOL : A_EOL);
  if (c == '\\') {
    anode *a = an_new(A_CHAR);
    cset tmp = {0};
    uint32_t s = 0;
    int k = rx_escape(P, &s, &tmp, 0);
    if (k == 2) {
      a->t = A_CLASS;
      a->cls = tmp;
      cs_norm(&a->cls);
    } else if (k >= 3) {
      free(tmp.r);
      a->t = k == 3 ? A_WB : k == 4 ? A_NWB : k == 5 ? A_BOL : A_EOL;
    } else {
      free(tmp.r);
      a->c = s;
      if (P->fi && k == 1) {
        a->t = A_CLASS;
        cs_add_folded(P, &a->cls, s, s);
        cs_norm(&a->cls);
      }
    }
    return a;
  }
  if (c == '*' || c == '+' || c == '?' || c == ')' || c == '|') {
    P->err = 1; /* repetition operator missing expression */
    return an_new(A_EMPTY);
  }
  if (c == '{') {
    P->err = 1;
    return an_new(A_EMPTY);
  }
  anode *a = an_new(A_CHAR);
  a->c = c;
  if (P->fi) {
    a->t = A_CLASS;
    cs_add_folded(P, &a->cls, c, c);
    cs_norm(&a->cls);
  }
  return a;
}

static anode *rx_parse_cat(rxparser *P) {
  anode *cat = an_new(A_CAT);
  for (;;) {
    rx_skip_x(P);
    if (!(P->i < P->n && P->p[P->i] != '|' && P->p[P->i] != ')' && !P->err && !P->unsupported)) break;
    anode *atom = rx_parse_atom(P);
    for (;;) {
      rx_skip_x(P);
      if (P->i >= P->n) break;
      uint32_t q = P->p[P->i];
      int mn, mx;
      if (q == '*') {
        mn = 0;
        mx = -1;
        P->i++;
      } else if (q == '+') {
        mn = 1;
        mx = -1;
        P->i++;
      } else if (q == '?') {
        mn = 0;
        mx = 1;
        P->i++;
      } else if (q == '{') {
        size_t save = P->i;
        P->i++;
        if (!rx_parse_int(P, &mn)) {
          P->i = save;
          P->err = 1;
          break;
        }
        mx = mn;
        if (P->i < P->n && P->p[P->i] == ',') {
          P->i++;
          if (!rx_parse_int(P, &mx)) mx = -1;
        }
        if (P->i >= P->n || P->p[P->i] != '}' || (mx >= 0 && mx < mn)) {
          P->err = 1;
          break;
        }
        P->i++;
        if (mn > 1000 || mx > 1000) {
          P->unsupported = 1;
          break;
        }
      } else
        break;
      if (P->i < P->n && P->p[P->i] == '?') P->i++; /* lazy: same language */
      if (atom->t == A_BOL || atom->t == A_EOL || atom->t == A_EMPTY) {
        /* repetition of an empty-width item: accepted, same language */
      }
      anode *r = an_new(A_REP);
      r->min = mn;
      r->max = mx;
      r->sub = atom;
      atom = r;
    }
    an_push(cat, atom);
  }
  return cat;
}

static anode *rx_parse_alt(rxparser *P) {
  anode *alt = an_new(A_ALT);
  an_push(alt, rx_parse_cat(P));
  while (P->i < P->n && P->p[P->i] == '|' && !P->err && !P->unsupported) {
    P->i++;
    an_push(alt, rx_parse_cat(P));
  }
  return alt;
}

static int rx_emit(rxprog *g, int op, uint32_t c, int x, int y) {
  if (g->n == g->cap) {
    g->cap = g->cap ? g->cap * 2 : 64;
    g->prog = (rxins *)realloc(g->prog, g->cap * sizeof(rxins));
  }
  g->prog[g->n].op = op;
  g->prog[g->n].c = c;
  g->prog[g->n].x = x;
  g->prog[g->n].y = y;
  return (int)g->n++;
}
static int rx_addcls(rxprog *g, const cset *s) {
  if (g->ncls == g->ccap) {
    g->ccap = g->ccap ? g->ccap * 2 : 8;
    g->classes = (cset *)realloc(g->classes, g->ccap * sizeof(cset));
  }
  cset c = {0};
  for (size_t i = 0; i < s->n; i++) cs_add(&c, s->r[i].lo, s->r[i].hi);
  g->classes[g->ncls] = c;
  return (int)g->ncls++;
}
static void rx_comp(rxprog *g, const anode *a) {
  switch (a->t) {
    case A_EMPTY: break;
    case A_CHAR: rx_emit(g, RX_CHAR, a->c, 0, 0); break;
    case A_CLASS: rx_emit(g, RX_CLASS, (uint32_t)rx_addcls(g, &a->cls), 0, 0); break;
    case A_BOL: rx_emit(g, RX_BOL, 0, 0, 0); break;
    case A_EOL: rx_emit(g, RX_EOL, 0, 0, 0); break;
    case A_WB: rx_emit(g, RX_WB, 0, 0, 0); break;
    case A_MBOL: rx_emit(g, RX_MBOL, 0, 0, 0); break;
    case A_MEOL: rx_emit(g, RX_MEOL, 0, 0, 0); break;
    case A_NWB: rx_emit(g, RX_NWB, 0, 0, 0); break;
    case A_CAT:
      for (size_t i = 0; i < a->nk; i++) rx_comp(g, a->kids[i]);
      break;
    case A_ALT: {
      if (a->nk == 1) {
        rx_comp(g, a->kids[0]);
        break;
      }
      int *jmps = (int *)malloc(a->nk * sizeof(int));
      for (size_t i = 0; i < a->nk; i++) {
        if (i + 1 < a->nk) {
          int sp = rx_emit(g, RX_SPLIT, 0, 0, 0);
          g->prog[sp].x = (int)g->n;
          rx_comp(g, a->kids[i]);
          jmps[i] = rx_emit(g, RX_JMP, 0, 0, 0);
          g->prog[sp].y = (int)g->n;
        } else {
          rx_comp(g, a->kids[i]);
          jmps[i] = -1;
        }
      }
      for (size_t i = 0; i < a->nk; i++)
        if (jmps[i] >= 0) g->prog[jmps[i]].x = (int)g->n;
      free(jmps);
      break;
    }
    case A_REP: {
      for (int k = 0; k < a->min; k++) rx_comp(g, a->sub);
      if (a->max < 0) {
        int sp = rx_emit(g, RX_SPLIT, 0, 0, 0);
        g->prog[sp].x = (int)g->n;
        rx_comp(g, a->sub);
        rx_emit(g, RX_JMP, 0, sp, 0);
        g->prog[sp].y = (int)g->n;
      } else {
        int nopt = a->max - a->min;
        int *sps = (int *)malloc((nopt + 1) * sizeof(int));
        for (int k = 0; k < nopt; k++) {
          sps[k] = rx_emit(g, RX_SPLIT, 0, 0, 0);
          g->prog[sps[k]].x = (int)g->n;
          rx_comp(g, a->sub);
        }
        for (int k = 0; k < nopt; k++) g->prog[sps[k]].y = (int)g->n;
        free(sps);
      }
      break;
    }
  }
}

static void rxprog_free(rxprog *g) {
  for (size_t i = 0; i < g->ncls; i++) free(g->classes[i].r);
  free(g->classes);
  free(g->prog);
  memset(g, 0, sizeof *g);
}

/* regex-syntax's error Display (error.rs Formatter / Spans::notate, the same in
 * 0.6.27 and 0.7.1) for the span [lo, hi) of the pattern's code points cp[0..n):
 * "regex parse error:", the pattern's lines (4 spaces in front, or a
 * right-aligned line number and ": " when the pattern holds a '\n', between
 * two lines of 79 '~'), '^' under a one-line span, "on line .. through line .."
 * for a span over lines, then "error: <kind>".  Columns count code points. */
static void sb_put(char **b, size_t *len, size_t *cap, const char *s, size_t n) {
  if (*len + n + 1 > *cap) {
    *cap = (*len + n + 1) * 2;
    *b = (char *)realloc(*b, *cap);
  }
  memcpy(*b + *len, s, n);
  *len += n;
  (*b)[*len] = 0;
}
static void sb_rep(char **b, size_t *len, size_t *cap, char c, size_t n) {
  for (size_t k = 0; k < n; k++) sb_put(b, len, cap, &c, 1);
}
static void sb_cp(char **b, size_t *len, size_t *cap, uint32_t c) {
  char u[4];
  size_t w;
  if (c < 0x80) { u[0] = (char)c; w = 1; }
  else if (c < 0x800) { u[0] = (char)(0xC0 | (c >> 6)); u[1] = (char)(0x80 | (c & 0x3F)); w = 2; }
  else if (c < 0x10000) { u[0] = (char)(0xE0 | (c >> 12)); u[1] = (char)(0x80 | ((c >> 6) & 0x3F)); u[2] = (char)(0x80 | (c & 0x3F)); w = 3; }
  else { u[0] = (char)(0xF0 | (c >> 18)); u[1] = (char)(0x80 | ((c >> 12) & 0x3F)); u[2] = (char)(0x80 | ((c >> 6) & 0x3F)); u[3] = (char)(0x80 | (c & 0x3F)); w = 4; }
  sb_put(b, len, cap, u, w);
}
static void rx_pos(const uint32_t *cp, size_t off, size_t *line, size_t *col) {
  size_t ls = 0;
  *line = 1;
  for (size_t k = 0; k < off; k++)
    if (cp[k] == '\n') {
      ++*line;
      ls = k + 1;
    }
  *col = off - ls + 1;
}
static char *rx_error_text(const uint32_t *cp, size_t n, size_t lo, size_t hi, const char *kind) {
  char *b = NULL, num[32];
  size_t len = 0, cap = 0;
  int multi = 0;
  size_t nlines = 0, l0, c0, l1, c1;
  for (size_t k = 0; k < n; k++) multi |= cp[k] == '\n';
  /* str::lines: split at '\n' (a "\r\n" ending dropped whole), no empty last line */
  for (size_t s = 0, k = 0; k <= n; k++)
    if (k == n || cp[k] == '\n') {
      if (k < n || k > s) nlines++;
      s = k + 1;
    }
  size_t count = nlines + (n && cp[n - 1] == '\n' ? 1 : 0), lnw = 0;
  if (count > 1) lnw = (size_t)sprintf(num, "%zu", count);
  rx_pos(cp, lo, &l0, &c0);
  rx_pos(cp, hi, &l1, &c1);
  sb_put(&b, &len, &cap, "regex parse error:\n", 19);
  if (multi) {
    sb_rep(&b, &len, &cap, '~', 79);
    sb_put(&b, &len, &cap, "\n", 1);
  }
  size_t line = 0;
  for (size_t s = 0, k = 0; k <= n; k++) {
    if (!(k == n || cp[k] == '\n')) continue;
    if (k == n && k <= s) break; /* no empty last line */
    size_t e = (k < n && k > s && cp[k - 1] == '\r') ? k - 1 : k;
    line++;
    if (lnw) {
      int w = sprintf(num, "%zu", line);
      sb_rep(&b, &len, &cap, ' ', lnw - (size_t)w);
      sb_put(&b, &len, &cap, num, (size_t)w);
      sb_put(&b, &len, &cap, ": ", 2);
    } else {
      sb_put(&b, &len, &cap, "    ", 4);
    }
    for (size_t q = s; q < e; q++) sb_cp(&b, &len, &cap, cp[q]);
    sb_put(&b, &len, &cap, "\n", 1);
    if (l0 == l1 && l0 == line) {
      sb_rep(&b, &len, &cap, ' ', lnw ? 2 + lnw : 4);
      sb_rep(&b, &len, &cap, ' ', c0 - 1);
      sb_rep(&b, &len, &cap, '^', c1 > c0 ? c1 - c0 : 1);
      sb_put(&b, &len, &cap, "\n", 1);
    }
    s = k + 1;
  }
  if (multi) {
    sb_rep(&b, &len, &cap, '~', 79);
    sb_put(&b, &len, &cap, "\n", 1);
    if (l0 != l1) {
      char t[160];
      int w = sprintf(t, "on line %zu (column %zu) through line %zu (column %zu)\n", l0, c0, l1, c1 - 1);
      sb_put(&b, &len, &cap, t, (size_t)w);
    }
  }
  sb_put(&b, &len, &cap, "error: ", 7);
  sb_put(&b, &len, &cap, kind, strlen(kind));
  return b;
}

/* 0 ok, ORC_E_INIT on syntax error, ORC_E_UNSUPPORTED on unsupported syntax;
 * *msg (when msg is not NULL): the error text, malloc'd */
static int rx_compile(const char *pat, rxprog *g, char **msg) {
  memset(g, 0, sizeof *g);
  size_t plen = strlen(pat), vut;
  int el;
  if (!utf8_check((const uint8_t *)pat, plen, &vut, &el)) {
    if (msg) *msg = dup_str("regex parse error");
    return ORC_E_INIT;
  }
  size_t ncp;
  uint32_t *cps = utf8_decode((const uint8_t *)pat, plen, &ncp);
  rxparser P;
  memset(&P, 0, sizeof P);
  P.p = cps;
  P.n = ncp;
  P.fu = 1; /* Unicode mode is the default */
  anode *root = rx_parse_alt(&P);
  if (P.word) g->unicode_word = 1;
  if (P.wba) g->ascii_wb = 1;
  g->utab = P.utab;
  int rc = 0;
  if (P.perr && !P.err && P.i == P.n) {
    rc = ORC_E_INIT;
    if (msg)
      *msg = rx_error_text(cps, ncp, P.perr_lo, P.perr_hi,
                           P.perr == 2 ? "Unicode property value not found" : "Unicode property not found");
  } else if (P.unsupported) {
    rc = ORC_E_UNSUPPORTED;
    if (msg) *msg = dup_str("unsupported regex syntax");
  } else if (P.err || P.i != P.n) {
    rc = ORC_E_INIT;
    if (msg) *msg = dup_str("regex parse error");
  }
  if (!rc) {
    rx_comp(g, root);
    rx_emit(g, RX_MATCH, 0, 0, 0);
  }
  an_free(root);
  free(cps);
  return rc;
}

/* Pike VM.  returns 1 match, 0 no match, -1 unsupported ((?-u) \b with non-ASCII) */
typedef struct {
  int *dense, *sparse;
  int n;
} sset;
/* \b / \B on code points: regex-syntax's Unicode \w (fsg_u_word), which is
 * [0-9A-Za-z_] on ASCII */
static int rx_is_word(uint32_t c) {
  if (c < 0x80) return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
  uint32_t a = 0, b = fsg_u_word_n;
  while (a < b) {
    uint32_t m = (a + b) / 2;
    if (fsg_u_word[m].hi < c) a = m + 1; else b = m;
  }
  return a < fsg_u_word_n && fsg_u_word[a].lo <= c;
}
static void ss_add(const rxprog *g, sset *s, int pc, size_t pos, size_t n, int *match, int *stack,
                   const uint32_t *cp) {
  int sp = 0;
  stack[sp++] = pc;
  while (sp) {
    int p = stack[--sp];
    if (s->sparse[p] < s->n && s->dense[s->sparse[p]] == p) continue;
    s->sparse[p] = s->n;
    s->dense[s->n++] = p;
    const rxins *I = &g->prog[p];
    switch (I->op) {
      case RX_JMP: stack[sp++] = I->x; break;
      case RX_SPLIT:
        stack[sp++] = I->y;
        stack[sp++] = I->x;
        break;
      case RX_BOL:
        if (pos == 0) stack[sp++] = p + 1;
        break;
      case RX_EOL:
        if (pos == n) stack[sp++] = p + 1;
        break;
      case RX_MBOL: /* (?m)^ */
        if (pos == 0 || cp[pos - 1] == '\n') stack[sp++] = p + 1;
        break;
      case RX_MEOL: /* (?m)$ */
        if (pos == n || cp[pos] == '\n') stack[sp++] = p + 1;
        break;
      case RX_WB:
      case RX_NWB: {
        const int pw = pos > 0 && rx_is_word(cp[pos - 1]), nw = pos < n && rx_is_word(cp[pos]);
        if ((pw != nw) == (I->op == RX_WB)) stack[sp++] = p + 1;
        break;
      }
      case RX_MATCH: *match = 1; break;
      default: break;
    }
  }
}
static int rx_run(const rxprog *g, const uint32_t *cp, size_t n) {
  if (g->unicode_word && g->ascii_wb)
    for (size_t i = 0; i < n; i++)
      if (cp[i] >= 0x80) return -1;
  /* a code point whose class membership differs between this build's Unicode 13
   * tables and regex-syntax 0.6.27 / 0.7.1's (Unicode 14 / 15): not decided */
  if (g->utab)
    for (size_t i = 0; i < n; i++)
      if (cp[i] >= 0x80 && fsg_u_is_newer(cp[i])) return -1;
  int np = (int)g->n;
  sset a = {(int *)malloc(np * sizeof(int)), (int *)calloc(np, sizeof(int)), 0};
  sset b = {(int *)malloc(np * sizeof(int)), (int *)calloc(np, sizeof(int)), 0};
  int *stack = (int *)malloc((2 * np + 4) * sizeof(int) * 2);
  int match = 0;
  sset *cur = &a, *nxt = &b;
  for (size_t i = 0;; i++) {
    ss_add(g, cur, 0, i, n, &match, stack, cp); /* unanchored: new thread at every position */
    if (match || i == n) break;
    nxt->n = 0;
    for (int k = 0; k < cur->n; k++) {
      const rxins *I = &g->prog[cur->dense[k]];
      int ok = 0;
      if (I->op == RX_CHAR)
        ok = I->c == cp[i];
      else if (I->op == RX_CLASS)
        ok = cs_has(&g->classes[I->c], cp[i]);
      if (ok) ss_add(g, nxt, cur->dense[k] + 1, i + 1, n, &match, stack, cp);
      if (match) break;
    }
    if (match) break;
    sset *t = cur;
    cur = nxt;
    nxt = t;
  }
  free(a.dense);
  free(a.sparse);
  free(b.dense);
  free(b.sparse);
  free(stack);
  return match;
}

int orc_regex_is_match(const char *pattern, const uint8_t *text, size_t n, int *is_match) {
  rxprog g;
  int rc = rx_compile(pattern, &g, NULL);
  if (rc) return rc;
  size_t vut;
  int el;
  if (!utf8_check(text, n, &vut, &el)) {
    rxprog_free(&g);
    return ORC_E_INVALID_ARG;
  }
  size_t ncp;
  uint32_t *cp = utf8_decode(text, n, &ncp);
  int m = rx_run(&g, cp, ncp);
  free(cp);
  rxprog_free(&g);
  if (m < 0) return ORC_E_UNSUPPORTED;
  *is_match = m;
  return 0;
}

/* ------------------------------------------------------------------ */
/* SmartModules (built-in restatements of the reference modules)        */
/* ------------------------------------------------------------------ */
enum { K_FILTER = 0, K_MAP = 1, K_ARRAY_MAP = 2, K_AGGREGATE = 3, K_FILTER_MAP = 4 }; /* SmartModuleKind tags */

enum {
  M_FILTER_CONTAINS, /* filter / filter_init / filter_with_param */
  M_FILTER_REGEX,    /* regex-filter (keep match) / filter_regex (keep non-match) */
  M_FILTER_ODD,
  M_MAP_UPPER,
  M_MAP_DOUBLE,
  M_FILTER_MAP_EVEN_HALF,
  M_AGG_SUM,
  M_AGG_CONCAT,
  M_FILTER_JSON, /* examples/filter_json: StructuredLog.level > Debug */
  M_ARRAY_MAP,   /* examples/array_map_json_array: explode a JSON array */
  M_PROJECT,     /* map_json_project: the value of one JSON field (C3 projection) */
  M_AGG_JSON,    /* examples/aggregate-json: HashMap<String, u32> += per key (C5 keyed) */
  M_FILTER_LOOKBACK, /* examples/filter_look_back: keep i32 values above the last kept (look_back sets it) */
  M_FILTER_HASHSET,  /* examples/filter_hashset: dedup over a BoundedHashSet<String> (look_back inserts) */
};

/* examples/filter_hashset/src/lib.rs:46-80 BoundedHashSet<String>: BTreeMap<value,
 * seq>, seq = seq.saturating_add(1) per insert (usize = u32 on wasm32), a vacant
 * value is inserted with the current seq, and when len > limit the entry with the
 * smallest seq is removed.  Entries are only ever removed that way and keep the
 * seq of their insertion, so the min-seq entry is the oldest live insertion: the
 * restatement keeps the live entries in insertion order (a FIFO) with a chained
 * hash index for the lookups. */
typedef struct {
  uint8_t *b;
  size_t n;
  uint32_t seq;
  int64_t next; /* bucket chain */
} bhs_ent;
typedef struct {
  bhs_ent *e;
  size_t ne, cap, head; /* live entries: [head, ne) */
  int64_t *bucket;
  size_t nbucket;
  uint32_t limit, seq;
} bhs_t;

typedef struct {
  int mod;
  int kind; /* SmartModuleKind */
  uint8_t *needle;
  size_t needle_len;
  rxprog rx;
  int rx_keep_match;
  uint8_t *acc; /* aggregate accumulator */
  size_t acc_len;
  int32_t prev; /* filter_look_back: static PREV (AtomicI32, starts at 0) */
  bhs_t *set;   /* filter_hashset: static SET */
  uint64_t rs_k0; /* aggregate-json: the instance's next RandomState k0 (std's KEYS thread-local) */
} stage_t;

static uint64_t bhs_hash(const uint8_t *b, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}
static void bhs_free(bhs_t *s) {
  if (!s) return;
  for (size_t i = s->head; i < s->ne; i++) free(s->e[i].b);
  free(s->e);
  free(s->bucket);
  free(s);
}
static void bhs_rebuild(bhs_t *s, size_t nb) {
  free(s->bucket);
  s->nbucket = nb;
  s->bucket = (int64_t *)malloc(nb * sizeof(int64_t));
  for (size_t i = 0; i < nb; i++) s->bucket[i] = -1;
  for (size_t i = s->head; i < s->ne; i++) {
    size_t k = bhs_hash(s->e[i].b, s->e[i].n) & (nb - 1);
    s->e[i].next = s->bucket[k];
    s->bucket[k] = (int64_t)i;
  }
}
/* BoundedHashSet::insert: true when the value was vacant */
static int bhs_insert(bhs_t *s, const uint8_t *b, size_t n) {
  s->seq = s->seq == 0xFFFFFFFFu ? s->seq : s->seq + 1; /* saturating_add */
  if (!s->bucket) bhs_rebuild(s, 1024);
  size_t k = bhs_hash(b, n) & (s->nbucket - 1);
  for (int64_t i = s->bucket[k]; i >= 0; i = s->e[i].next)
    if (s->e[i].n == n && !memcmp(s->e[i].b, b, n)) return 0; /* Occupied */
  if (s->ne == s->cap) {
    /* compact the evicted prefix away before growing */
    size_t live = s->ne - s->head;
    if (s->head > live) {
      memmove(s->e, s->e + s->head, live * sizeof(bhs_ent));
      s->ne = live;
      s->head = 0;
    } else {
      s->cap = s->cap ? 2 * s->cap : 1024;
      s->e = (bhs_ent *)realloc(s->e, s->cap * sizeof(bhs_ent));
    }
    bhs_rebuild(s, s->nbucket);
  }
  bhs_ent ne;
  ne.b = dup_bytes(b, n);
  ne.n = n;
  ne.seq = s->seq;
  s->e[s->ne] = ne;
  s->ne++;
  if ((s->ne - s->head) > 2 * s->nbucket) bhs_rebuild(s, 4 * s->nbucket);
  else {
    s->e[s->ne - 1].next = s->bucket[k];
    s->bucket[k] = (int64_t)(s->ne - 1);
  }
  if ((uint64_t)(s->ne - s->head) > (uint64_t)s->limit) { /* remove_first: the smallest seq */
    bhs_ent *h = &s->e[s->head];
    size_t hk = bhs_hash(h->b, h->n) & (s->nbucket - 1);
    int64_t *pp = &s->bucket[hk];
    while (*pp != (int64_t)s->head) pp = &s->e[*pp].next;
    *pp = h->next;
    free(h->b);
    h->b = NULL;
    s->head++;
  }
  return 1;
}
/* usize::from_str on wasm32 (u32): optional '+', digits; 0 ok, else ParseIntError kind */
static int parse_u32(const char *t, uint32_t *out) {
  size_t n = strlen(t), i = 0;
  if (n == 0) return 1;
  if (t[0] == '+') {
    i = 1;
    if (n == 1) return 2;
  }
  uint64_t acc = 0;
  for (; i < n; i++) {
    if (t[i] < '0' || t[i] > '9') return 2;
    acc = acc * 10 + (uint64_t)(t[i] - '0');
    if (acc > 0xFFFFFFFFull) return 3;
  }
  *out = (uint32_t)acc;
  return 0;
}

struct orc_chain {
  stage_t *st;
  size_t n;
};

orc_chain *orc_chain_new(void) { return (orc_chain *)calloc(1, sizeof(orc_chain)); }
void orc_chain_free(orc_chain *c) {
  if (!c) return;
  for (size_t i = 0; i < c->n; i++) {
    free(c->st[i].needle);
    free(c->st[i].acc);
    bhs_free(c->st[i].set);
    rxprog_free(&c->st[i].rx);
  }
  free(c->st);
  free(c);
}

static const char *param_get(const char **keys, const char **vals, size_t n, const char *k) {
  /* BTreeMap: a later insert of the same key overwrites */
  const char *r = NULL;
  for (size_t i = 0; i < n; i++)
    if (strcmp(keys[i], k) == 0) r = vals[i];
  return r;
}

int orc_chain_add(orc_chain *c, const char *module, const char **keys, const char **vals, size_t n_params,
                  const uint8_t *acc, size_t acc_len, int has_acc, char **msg_out) {
  stage_t s;
  memset(&s, 0, sizeof s);
  if (msg_out) *msg_out = NULL;
  const char *v;
  if (!strcmp(module, "filter")) { /* examples/filter: contains('a') */
    s.mod = M_FILTER_CONTAINS;
    s.kind = K_FILTER;
    s.needle = dup_bytes((const uint8_t *)"a", 1);
    s.needle_len = 1;
  } else if (!strcmp(module, "filter_init")) { /* key required */
    v = param_get(keys, vals, n_params, "key");
    if (!v) {
      if (msg_out) *msg_out = dup_str("Missing param key\n\nSmartModule Init Error: \n");
      return ORC_E_INIT;
    }
    s.mod = M_FILTER_CONTAINS;
    s.kind = K_FILTER;
    s.needle_len = strlen(v);
    s.needle = dup_bytes((const uint8_t *)v, s.needle_len);
  } else if (!strcmp(module, "filter_with_param")) { /* key defaults to "a" */
    v = param_get(keys, vals, n_params, "key");
    if (!v) v = "a";
    s.mod = M_FILTER_CONTAINS;
    s.kind = K_FILTER;
    s.needle_len = strlen(v);
    s.needle = dup_bytes((const uint8_t *)v, s.needle_len);
  } else if (!strcmp(module, "regex-filter") || !strcmp(module, "filter_regex")) {
    const char *pat;
    if (!strcmp(module, "regex-filter")) {
      pat = param_get(keys, vals, n_params, "regex");
      if (!pat) {
        if (msg_out) *msg_out = dup_str("Missing param regex\n\nSmartModule Init Error: \n");
        return ORC_E_INIT;
      }
      s.rx_keep_match = 1;
    } else {
      pat = "\\d{3}-\\d{2}-\\d{4}";
      s.rx_keep_match = 0;
    }
    char *em = NULL;
    int rc = rx_compile(pat, &s.rx, &em);
    if (rc) {
      rxprog_free(&s.rx);
      if (msg_out && rc == ORC_E_INIT) { /* the init error Display (SmartModuleInitError) */
        size_t k = strlen(em);
        char *t = (char *)malloc(k + 32);
        sprintf(t, "%s\n\nSmartModule Init Error: \n", em);
        *msg_out = t;
      } else if (msg_out) {
        *msg_out = dup_str(em);
      }
      free(em);
      return rc;
    }
    free(em);
    s.mod = M_FILTER_REGEX;
    s.kind = K_FILTER;
  } else if (!strcmp(module, "filter_json")) {
    s.mod = M_FILTER_JSON;
    s.kind = K_FILTER;
  } else if (!strcmp(module, "filter_odd")) {
    s.mod = M_FILTER_ODD;
    s.kind = K_FILTER;
  } else if (!strcmp(module, "map")) {
    s.mod = M_MAP_UPPER;
    s.kind = K_MAP;
  } else if (!strcmp(module, "map_double")) {
    s.mod = M_MAP_DOUBLE;
    s.kind = K_MAP;
  } else if (!strcmp(module, "filter_map")) {
    s.mod = M_FILTER_MAP_EVEN_HALF;
    s.kind = K_FILTER_MAP;
  } else if (!strcmp(module, "aggregate-sum")) {
    s.mod = M_AGG_SUM;
    s.kind = K_AGGREGATE;
  } else if (!strcmp(module, "aggregate")) {
    s.mod = M_AGG_CONCAT;
    s.kind = K_AGGREGATE;
  } else if (!strcmp(module, "array_map_json_array")) {
    s.mod = M_ARRAY_MAP;
    s.kind = K_ARRAY_MAP;
  } else if (!strcmp(module, "aggregate-json")) {
    s.mod = M_AGG_JSON;
    s.kind = K_AGGREGATE;
    s.rs_k0 = 1; /* hashmap_random_keys() = (1, 2) on wasm32-unknown-unknown */
  } else if (!strcmp(module, "map_json_project")) { /* param field, default "message" */
    v = param_get(keys, vals, n_params, "field");
    if (!v) v = "message";
    s.mod = M_PROJECT;
    s.kind = K_FILTER_MAP;
    s.needle_len = strlen(v);
    s.needle = dup_bytes((const uint8_t *)v, s.needle_len + 1);
    s.needle[s.needle_len] = 0;
  } else if (!strcmp(module, "filter_look_back")) {
    s.mod = M_FILTER_LOOKBACK;
    s.kind = K_FILTER;
  } else if (!strcmp(module, "filter_hashset")) {
    /* init: count = params.get("count").parse()? else usize::MAX - 1 (lib.rs:28-37) */
    uint32_t limit = 0xFFFFFFFEu;
    v = param_get(keys, vals, n_params, "count");
    if (v) {
      int pk = parse_u32(v, &limit);
      if (pk) {
        if (msg_out) *msg_out = fmt_str("%s\n\nSmartModule Init Error: \n", parse_int_hint(pk));
        return ORC_E_INIT;
      }
    }
    s.mod = M_FILTER_HASHSET;
    s.kind = K_FILTER;
    s.set = (bhs_t *)calloc(1, sizeof(bhs_t));
    s.set->limit = limit;
  } else {
    return ORC_E_UNKNOWN_SM;
  }
  if (s.kind == K_AGGREGATE) {
    s.acc = dup_bytes(acc, has_acc ? acc_len : 0);
    s.acc_len = has_acc ? acc_len : 0;
  }
  c->st = (stage_t *)realloc(c->st, (c->n + 1) * sizeof(stage_t));
  c->st[c->n++] = s;
  return ORC_OK;
}

int orc_chain_accumulator(orc_chain *c, size_t stage, uint8_t **acc, size_t *len) {
  if (stage >= c->n || c->st[stage].kind != K_AGGREGATE) return ORC_E_INVALID_ARG;
  *acc = dup_bytes(c->st[stage].acc, c->st[stage].acc_len);
  *len = c->st[stage].acc_len;
  return 0;
}

static int mem_contains(const uint8_t *h, size_t hn, const uint8_t *n, size_t nn) {
  if (nn == 0) return 1;
  if (nn > hn) return 0;
  for (size_t i = 0; i + nn <= hn; i++)
    if (h[i] == n[0] && !memcmp(h + i, n, nn)) return 1;
  return 0;
}

static void i32_to_str(int32_t v, char *buf, size_t *len) { *len = (size_t)sprintf(buf, "%d", v); }

/* ------------------------------------------------------------------------
 * std::collections::HashMap<String, u32> as the aggregate-json guest builds it
 * (examples/aggregate-json/src/lib.rs:22-36; Rust 1.75, examples/rust-toolchain,
 * for wasm32-unknown-unknown), which fixes the key order of its output:
 *  - RandomState::new() (std/src/hash/random.rs) hands out (k0, k1) from a
 *    thread-local seeded by sys::hashmap_random_keys() = (1, 2) on this target
 *    (std/src/sys/unsupported/common.rs) and bumps k0 per call (stage_t.rs_k0);
 *  - DefaultHasher = SipHash-1-3 (core/src/hash/sip.rs), a String hashes as its
 *    bytes then 0xFF (Hasher::write_str);
 *  - the table is hashbrown 0.14 (std's backend): generic 8-byte control
 *    groups (GroupWord = u64 on wasm32), h1 = the hash as a 32-bit usize, h2 =
 *    its top 7 bits, triangular probing by groups over control bytes whose
 *    trailing group mirrors the first, fix_insert_slot's rescan from bucket 0
 *    for tables smaller than a group, growth by capacity_to_buckets
 *    (0 -> 4 -> 8 -> 2x), resize re-inserting in bucket order, iteration in
 *    bucket order.
 * ---------------------------------------------------------------------- */
uint64_t orc_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1, const uint8_t *m, size_t n) {
#define ORC_ROTL(x, b) (((x) << (b)) | ((x) >> (64 - (b))))
#define ORC_SIPROUND                                                     \
  do {                                                                   \
    v0 += v1; v1 = ORC_ROTL(v1, 13); v1 ^= v0; v0 = ORC_ROTL(v0, 32);    \
    v2 += v3; v3 = ORC_ROTL(v3, 16); v3 ^= v2;                           \
    v0 += v3; v3 = ORC_ROTL(v3, 21); v3 ^= v0;                           \
    v2 += v1; v1 = ORC_ROTL(v1, 17); v1 ^= v2; v2 = ORC_ROTL(v2, 32);    \
  } while (0)
  uint64_t v0 = k0 ^ 0x736f6d6570736575ull, v1 = k1 ^ 0x646f72616e646f6dull;
  uint64_t v2 = k0 ^ 0x6c7967656e657261ull, v3 = k1 ^ 0x7465646279746573ull;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w = 0;
    for (int b = 0; b < 8; b++) w |= (uint64_t)m[i + b] << (8 * b);
    v3 ^= w;
    for (int r = 0; r < c_rounds; r++) ORC_SIPROUND;
    v0 ^= w;
  }
  uint64_t b = (uint64_t)(n & 0xff) << 56;
  for (size_t t = 0; i + t < n; t++) b |= (uint64_t)m[i + t] << (8 * t);
  v3 ^= b;
  for (int r = 0; r < c_rounds; r++) ORC_SIPROUND;
  v0 ^= b;
  v2 ^= 0xff;
  for (int r = 0; r < d_rounds; r++) ORC_SIPROUND;
  return v0 ^ v1 ^ v2 ^ v3;
#undef ORC_SIPROUND
#undef ORC_ROTL
}

static uint64_t hb_str_hash(uint64_t k0, const uint8_t *key, size_t n) {
  uint8_t *t = (uint8_t *)malloc(n + 1);
  if (n) memcpy(t, key, n);
  t[n] = 0xff;
  const uint64_t h = orc_siphash(1, 3, k0, 2, t, n + 1);
  free(t);
  return h;
}

enum { HB_GROUP = 8, HB_EMPTY = 0xff };
typedef struct {
  uint64_t k0;
  size_t buckets; /* 0: the empty singleton */
  size_t items;
  uint8_t *ctrl;  /* buckets + HB_GROUP control bytes */
  uint8_t **key;  /* per bucket (owned) */
  size_t *klen;
  uint32_t *val;
  uint32_t *h1;   /* per bucket: the key's hash as usize */
} hb_t;

static size_t hb_capacity(size_t buckets) {
  if (!buckets) return 0;
  const size_t mask = buckets - 1;
  return mask < 8 ? mask : ((mask + 1) / 8) * 7;
}
static size_t hb_cap_to_buckets(size_t cap) {
  if (cap < 8) return cap < 4 ? 4 : 8;
  size_t adj = cap * 8 / 7, b = 1;
  while (b < adj) b <<= 1;
  return b;
}
static void hb_alloc(hb_t *t, size_t buckets) {
  t->buckets = buckets;
  t->items = 0;
  t->ctrl = (uint8_t *)malloc(buckets + HB_GROUP);
  memset(t->ctrl, HB_EMPTY, buckets + HB_GROUP);
  t->key = (uint8_t **)calloc(buckets, sizeof(uint8_t *));
  t->klen = (size_t *)calloc(buckets, sizeof(size_t));
  t->val = (uint32_t *)calloc(buckets, sizeof(uint32_t));
  t->h1 = (uint32_t *)calloc(buckets, sizeof(uint32_t));
}
static void hb_free(hb_t *t) {
  for (size_t i = 0; i < t->buckets; i++) free(t->key[i]);
  free(t->ctrl);
  free(t->key);
  free(t->klen);
  free(t->val);
  free(t->h1);
  memset(t, 0, sizeof *t);
}
static int hb_full(const hb_t *t, size_t i) { return !(t->ctrl[i] & 0x80); }
/* set_ctrl: the byte and its mirror among the trailing HB_GROUP bytes */
static void hb_set_ctrl(hb_t *t, size_t i, uint8_t c) {
  t->ctrl[i] = c;
  t->ctrl[((i - HB_GROUP) & (t->buckets - 1)) + HB_GROUP] = c;
}
/* find_insert_slot: the first EMPTY/DELETED byte of the group at the probe
 * position, then fix_insert_slot */
static size_t hb_find_insert_slot(const hb_t *t, uint32_t h1) {
  const size_t mask = t->buckets - 1;
  size_t pos = h1 & mask, stride = 0;
  for (;;) {
    for (size_t bit = 0; bit < HB_GROUP; bit++) {
      if (!(t->ctrl[pos + bit] & 0x80)) continue;
      size_t idx = (pos + bit) & mask;
      if (hb_full(t, idx)) { /* a table smaller than a group: rescan the aligned first group */
        idx = 0;
        while (!(t->ctrl[idx] & 0x80)) idx++;
      }
      return idx;
    }
    stride += HB_GROUP;
    pos = (pos + stride) & mask;
  }
}
static void hb_place(hb_t *t, uint8_t *key, size_t klen, uint32_t val, uint64_t hash) {
  const uint32_t h1 = (uint32_t)hash;
  const size_t i = hb_find_insert_slot(t, h1);
  hb_set_ctrl(t, i, (uint8_t)((h1 >> 25) & 0x7f));
  t->key[i] = key;
  t->klen[i] = klen;
  t->val[i] = val;
  t->h1[i] = h1;
  t->items++;
}
/* reserve(1): reserve_rehash -> resize(max(items + 1, capacity + 1)), old
 * buckets re-inserted in bucket order (no tombstones here: no removals) */
static void hb_reserve1(hb_t *t) {
  const size_t cap = hb_capacity(t->buckets);
  if (cap - t->items >= 1) return;
  hb_t n;
  memset(&n, 0, sizeof n);
  n.k0 = t->k0;
  hb_alloc(&n, hb_cap_to_buckets(t->items + 1 > cap + 1 ? t->items + 1 : cap + 1));
  for (size_t i = 0; i < t->buckets; i++) {
    if (!hb_full(t, i)) continue;
    hb_place(&n, t->key[i], t->klen[i], t->val[i], t->h1[i]);
    t->key[i] = NULL;
  }
  hb_free(t);
  *t = n;
}
static long hb_lookup(const hb_t *t, const uint8_t *key, size_t klen) {
  for (size_t i = 0; i < t->buckets; i++)
    if (hb_full(t, i) && t->klen[i] == klen && !memcmp(t->key[i], key, klen)) return (long)i;
  return -1;
}
/* HashMap::insert: find_or_find_insert_slot reserves before the lookup */
static void hb_insert(hb_t *t, const uint8_t *key, size_t klen, uint32_t val) {
  hb_reserve1(t);
  const long at = hb_lookup(t, key, klen);
  if (at >= 0) {
    t->val[at] = val;
    return;
  }
  hb_place(t, dup_bytes(key, klen), klen, val, hb_str_hash(t->k0, key, klen));
}
/* entry(key).and_modify(+= v).or_insert(v): rustc_entry reserves for a vacant key only */
static void hb_entry_add(hb_t *t, const uint8_t *key, size_t klen, uint32_t val) {
  const long at = hb_lookup(t, key, klen);
  if (at >= 0) {
    t->val[at] += val; /* u32 wrapping (release wasm) */
    return;
  }
  hb_reserve1(t);
  hb_place(t, dup_bytes(key, klen), klen, val, hb_str_hash(t->k0, key, klen));
}
static int json_ws_first_is_brace(const uint8_t *s, size_t n) {
  size_t i = 0;
  while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
  return i < n && s[i] == '{';
}

/* per-record user fn outcome */
typedef struct {
  int err; /* 1 -> runtime error */
  char *hint;
  int unsupported;
} fnres;

/* run one stage over decoded records (derive generator loops) */
typedef struct {
  recvec out;
  int has_error;
  rec_t err_rec; /* owned clone of the failing record */
  char *hint;
  size_t hint_len; /* 0: strlen(hint) (a serde_json text may hold a NUL: its length is kept) */
  int64_t err_offset;
  int kind;
  int unsupported;
} stage_out;

static void stage_run(stage_t *s, recvec *in, int64_t base_offset, stage_out *o) {
  memset(o, 0, sizeof *o);
  o->kind = s->kind;
  for (size_t i = 0; i < in->n; i++) {
    rec_t *r = &in->r[i];
    char *hint = NULL;
    size_t hint_len = 0;
    size_t vut;
    int el;
    int keep = 0;
    rec_t outr;
    int emit = 0;
    switch (s->mod) {
      case M_FILTER_CONTAINS:
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        keep = mem_contains(r->val, r->val_len, s->needle, s->needle_len);
        break;
      case M_FILTER_REGEX: {
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        size_t ncp;
        uint32_t *cp = utf8_decode(r->val, r->val_len, &ncp);
        int m = rx_run(&s->rx, cp, ncp);
        free(cp);
        if (m < 0) {
          o->unsupported = 1;
          return;
        }
        keep = s->rx_keep_match ? m : !m;
        break;
      }
      case M_FILTER_JSON: {
        int level = 0;
        size_t ml = 0;
        char *m = NULL;
        int jr = orc_json_structured_log(r->val, r->val_len, &level, &m, &ml);
        if (jr == ORC_E_UNSUPPORTED) {
          o->unsupported = 1;
          return;
        }
        if (jr) {
          hint = m; /* serde_json::Error Display (may hold a NUL: "unknown variant `..`" of the raw string) */
          hint_len = ml;
          break;
        }
        keep = level > 0;
        break;
      }
      case M_FILTER_ODD: {
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        int32_t x;
        int pk = parse_i32(r->val, r->val_len, &x);
        if (pk) {
          hint = fmt_str("Oops something went wrong\n\nCaused by:\n   0: Failed to parse int\n   1: %s",
                         parse_int_hint(pk));
          break;
        }
        keep = (x % 2) == 0;
        break;
      }
      case M_ARRAY_MAP: {
        /* array_map_json_array/src/lib.rs:38-55; derive generator/array_map.rs:17-42:
         * every element -> Record::new_key_value(None, to_string(element)) with the
         * default preamble (data.rs:465-472: attributes 0, deltas 0, no headers) */
        uint8_t **el;
        size_t *ln, cnt, ml;
        char *m = NULL;
        int jr = orc_json_array_map(r->val, r->val_len, &el, &ln, &cnt, &m, &ml);
        if (jr == ORC_E_UNSUPPORTED) {
          o->unsupported = 1;
          return;
        }
        if (jr) {
          hint = m;
          break;
        }
        for (size_t k = 0; k < cnt; k++) {
          rec_t nr;
          memset(&nr, 0, sizeof nr);
          nr.val = el[k];
          nr.val_len = ln[k];
          rv_push(&o->out, nr);
        }
        free(el);
        free(ln);
        break;
      }
      case M_AGG_JSON: {
        /* aggregate-json/src/lib.rs:22-36: accumulated = from_slice(acc).unwrap_or_default();
         * new = from_slice(value)?; accumulated + new (per key `+=`, u32 wrapping in the
         * release wasm); to_vec_pretty of the accumulated map, in its iteration order
         * (the hb_* restatement above).  RandomState draws: serde's map visitor once
         * deserialize_map has seen '{', and HashMap::default() in unwrap_or_default. */
        uint8_t **ak = NULL, **nk = NULL;
        size_t *al = NULL, *nl = NULL, an = 0, nn = 0, ml;
        uint32_t *av = NULL, *nv = NULL;
        char *m = NULL;
        hb_t acc, rec;
        memset(&acc, 0, sizeof acc);
        memset(&rec, 0, sizeof rec);
        if (json_ws_first_is_brace(s->acc, s->acc_len)) acc.k0 = s->rs_k0++;
        if (orc_json_map_u32(s->acc, s->acc_len, &ak, &al, &av, &an, &m, &ml)) { /* unwrap_or_default */
          free(m);
          m = NULL;
          an = 0;
          acc.k0 = s->rs_k0++;
        }
        for (size_t k = 0; k < an; k++) { /* the visitor's HashMap::insert per entry, text order */
          hb_insert(&acc, ak[k], al[k], av[k]);
          free(ak[k]);
        }
        free(ak); free(al); free(av);
        if (json_ws_first_is_brace(r->val, r->val_len)) rec.k0 = s->rs_k0++;
        int jr = orc_json_map_u32(r->val, r->val_len, &nk, &nl, &nv, &nn, &m, &ml);
        if (jr == ORC_E_UNSUPPORTED) {
          hb_free(&acc);
          o->unsupported = 1;
          return;
        }
        if (jr) {
          hb_free(&acc);
          hint = m;
          break;
        }
        for (size_t k = 0; k < nn; k++) {
          hb_insert(&rec, nk[k], nl[k], nv[k]);
          free(nk[k]);
        }
        free(nk); free(nl); free(nv);
        for (size_t i = 0; i < rec.buckets; i++) /* `for (repo, new_stars) in next.0`: bucket order */
          if (hb_full(&rec, i)) hb_entry_add(&acc, rec.key[i], rec.klen[i], rec.val[i]);
        hb_free(&rec);
        uint8_t **ok = (uint8_t **)malloc((acc.items + 1) * sizeof(uint8_t *));
        size_t *ol = (size_t *)malloc((acc.items + 1) * sizeof(size_t));
        uint32_t *ov = (uint32_t *)malloc((acc.items + 1) * sizeof(uint32_t));
        size_t on = 0;
        for (size_t i = 0; i < acc.buckets; i++) {
          if (!hb_full(&acc, i)) continue;
          ok[on] = acc.key[i];
          ol[on] = acc.klen[i];
          ov[on] = acc.val[i];
          on++;
        }
        uint8_t *pb;
        size_t pl;
        orc_json_pretty_map(ok, ol, ov, on, &pb, &pl);
        free(ok); free(ol); free(ov);
        hb_free(&acc);
        free(s->acc);
        s->acc = pb;
        s->acc_len = pl;
        outr = rec_clone(r);
        free(outr.val);
        outr.val = dup_bytes(s->acc, s->acc_len);
        outr.val_len = s->acc_len;
        emit = 1;
        break;
      }
      case M_PROJECT: {
        uint8_t *pv;
        size_t pl, ml;
        int found;
        char *m = NULL;
        int jr = orc_json_project(r->val, r->val_len, (const char *)s->needle, &pv, &pl, &found, &m, &ml);
        if (jr == ORC_E_UNSUPPORTED) {
          o->unsupported = 1;
          return;
        }
        if (jr) {
          hint = m;
          break;
        }
        if (found) { /* filter_map: Some((key, projected)) keeps key and preamble */
          outr = rec_clone(r);
          free(outr.val);
          outr.val = pv;
          outr.val_len = pl;
          emit = 1;
        }
        break;
      }
      case M_FILTER_LOOKBACK: { /* filter_look_back/src/lib.rs:7-18 */
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        int32_t x;
        int pk = parse_i32(r->val, r->val_len, &x);
        if (pk) {
          hint = dup_str(parse_int_hint(pk));
          break;
        }
        keep = x > s->prev;
        if (keep) s->prev = x;
        break;
      }
      case M_FILTER_HASHSET: /* filter_hashset/src/lib.rs:15-19: SET.insert(value.to_owned()) */
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        keep = bhs_insert(s->set, r->val, r->val_len);
        break;
      case M_MAP_UPPER:
        outr = rec_clone(r);
        for (size_t k = 0; k < outr.val_len; k++)
          if (outr.val[k] >= 'a' && outr.val[k] <= 'z') outr.val[k] -= 32;
        emit = 1;
        break;
      case M_MAP_DOUBLE: {
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        int32_t x;
        int pk = parse_i32(r->val, r->val_len, &x);
        if (pk) {
          hint = dup_str(parse_int_hint(pk));
          break;
        }
        char buf[16];
        size_t bl;
        i32_to_str((int32_t)((uint32_t)x * 2u), buf, &bl);
        outr = rec_clone(r);
        free(outr.val);
        outr.val = dup_bytes((const uint8_t *)buf, bl);
        outr.val_len = bl;
        emit = 1;
        break;
      }
      case M_FILTER_MAP_EVEN_HALF: {
        /* String::from_utf8_lossy + parse::<i32>: any non-ASCII byte is a non-digit */
        int32_t x;
        int pk = parse_i32(r->val, r->val_len, &x);
        if (pk) {
          hint = dup_str(parse_int_hint(pk));
          break;
        }
        if (x % 2 == 0) {
          char buf[16];
          size_t bl;
          i32_to_str(x / 2, buf, &bl);
          outr = rec_clone(r);
          free(outr.val);
          outr.val = dup_bytes((const uint8_t *)buf, bl);
          outr.val_len = bl;
          emit = 1;
        }
        break;
      }
      case M_AGG_SUM: {
        if (!utf8_check(s->acc, s->acc_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        size_t b, e;
        utf8_trim(s->acc, s->acc_len, &b, &e);
        int32_t a = 0;
        if (parse_i32(s->acc + b, e - b, &a)) a = 0; /* unwrap_or(0) */
        utf8_trim(r->val, r->val_len, &b, &e);
        int32_t x;
        int pk = parse_i32(r->val + b, e - b, &x);
        if (pk) {
          hint = dup_str(parse_int_hint(pk));
          break;
        }
        char buf[16];
        size_t bl;
        i32_to_str((int32_t)((uint32_t)a + (uint32_t)x), buf, &bl); /* wrapping (release wasm) */
        free(s->acc);
        s->acc = dup_bytes((const uint8_t *)buf, bl);
        s->acc_len = bl;
        outr = rec_clone(r);
        free(outr.val);
        outr.val = dup_bytes(s->acc, s->acc_len);
        outr.val_len = s->acc_len;
        emit = 1;
        break;
      }
      case M_AGG_CONCAT: {
        if (!utf8_check(s->acc, s->acc_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        if (!utf8_check(r->val, r->val_len, &vut, &el)) {
          hint = utf8_hint(vut, el);
          break;
        }
        uint8_t *na = (uint8_t *)malloc(s->acc_len + r->val_len + 1);
        memcpy(na, s->acc, s->acc_len);
        memcpy(na + s->acc_len, r->val, r->val_len);
        free(s->acc);
        s->acc = na;
        s->acc_len += r->val_len;
        outr = rec_clone(r);
        free(outr.val);
        outr.val = dup_bytes(s->acc, s->acc_len);
        outr.val_len = s->acc_len;
        emit = 1;
        break;
      }
    }
    if (hint) {
      /* SmartModuleTransformRuntimeError::new(record, base_offset, kind, err) */
      o->has_error = 1;
      o->hint = hint;
      o->hint_len = hint_len;
      o->err_offset = base_offset + r->off_delta;
      o->err_rec = rec_clone(r);
      return; /* break */
    }
    if (s->kind == K_FILTER) {
      if (keep) rv_push(&o->out, rec_clone(r));
    } else if (emit) {
      rv_push(&o->out, outr);
    }
  }
}

static void res_set_error(orc_result *out, stage_out *so) {
  out->has_error = 1;
  out->hint = so->hint;
  so->hint = NULL;
  out->hint_len = so->hint_len ? so->hint_len : strlen(out->hint);
  out->err_offset = so->err_offset;
  out->err_kind = so->kind;
  out->has_key = so->err_rec.has_key;
  out->key = so->err_rec.key;
  out->key_len = so->err_rec.key_len;
  out->value = so->err_rec.val;
  out->value_len = so->err_rec.val_len;
  so->err_rec.key = so->err_rec.val = NULL;
}

/* SmartModuleChainInstance::process (engine.rs:135-185).  On success out->bytes
 * holds SmartModuleOutput.successes encoded as Vec<Record>. */
int orc_chain_process(orc_chain *c, const uint8_t *raw, size_t raw_len, int64_t base_offset, int64_t base_ts,
                      orc_result *out) {
  (void)base_ts;
  memset(out, 0, sizeof *out);
  out->m_bytes_in = raw_len;
  out->m_invocations = 1;
  if (c->n == 0) {
    recvec rv;
    if (recs_decode(raw, raw_len, &rv)) {
      out->status = ORC_E_IO;
      return out->status;
    }
    obuf b = {0};
    recs_encode(&b, &rv);
    out->bytes = b.p;
    out->bytes_len = b.n;
    out->n_records = (uint32_t)rv.n;
    rv_free(&rv);
    return 0;
  }
  obuf cur = {0};
  ob_put(&cur, raw, raw_len);
  for (size_t si = 0; si < c->n; si++) {
    recvec rv;
    if (recs_decode(cur.p, cur.n, &rv)) {
      ob_free(&cur);
      out->status = ORC_E_DECODING_BASE_INPUT;
      return out->status;
    }
    stage_out so;
    stage_run(&c->st[si], &rv, base_offset, &so);
    rv_free(&rv);
    if (so.unsupported) {
      rv_free(&so.out);
      ob_free(&cur);
      out->status = ORC_E_UNSUPPORTED;
      return out->status;
    }
    obuf nb = {0};
    recs_encode(&nb, &so.out);
    ob_free(&cur);
    cur = nb;
    size_t nout = so.out.n;
    rv_free(&so.out);
    if (so.has_error || si + 1 == c->n) {
      if (si + 1 == c->n) out->m_records_out = nout;
      if (so.has_error) res_set_error(out, &so);
      out->bytes = cur.p;
      out->bytes_len = cur.n;
      out->n_records = (uint32_t)nout;
      return 0;
    }
  }
  return 0; /* unreachable */
}

static uint64_t rd_be(const uint8_t *p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 8) | p[i];
  return v;
}

/* SPU process_batch (fluvio-spu/src/smartengine/batch.rs:41-142) over a file
 * slice framed like FileBatchIterator (fluvio-storage/src/iterators.rs:55-160).
 * out->bytes = encoded output Batch (batch.rs:398-430), CRC32C computed. */
int orc_process_batch(orc_chain *c, const uint8_t *slice, size_t slice_len, uint64_t max_bytes, orc_result *out) {
  memset(out, 0, sizeof *out);
  int64_t sm_base = -1;
  int32_t sm_lod = -1;
  int16_t sm_attr = 0;
  recvec acc = {0};
  uint64_t total = 0;
  size_t pos = 0;
  int stop = 0;
  while (pos < slice_len && !stop) {
    /* FileBatchIterator::next */
    if (slice_len - pos < 57) {
      rv_free(&acc);
      out->status = ORC_E_IO;
      return out->status;
    }
    const uint8_t *h = slice + pos;
    int64_t b_base = (int64_t)rd_be(h, 8);
    int32_t b_len = (int32_t)rd_be(h + 8, 4);
    int16_t b_attr = (int16_t)rd_be(h + 21, 2);
    int32_t b_lod = (int32_t)rd_be(h + 23, 4);
    int64_t b_first_ts = (int64_t)rd_be(h + 27, 8);
    if (b_len < 45) {
      rv_free(&acc);
      out->status = ORC_E_IO;
      return out->status;
    }
    size_t rem = (size_t)b_len - 45;
    if (slice_len - pos - 57 < rem) {
      rv_free(&acc);
      out->status = ORC_E_IO;
      return out->status;
    }
    int comp = b_attr & 7;
    const uint8_t *recs = slice + pos + 57;
    uint8_t *dec = NULL;
    size_t rlen = rem;
    if (comp != 0) { /* iterators.rs:136-156: compression.uncompress(records) (fsg_codec.c) */
      int drc = comp > 4 ? -1 : orc_decompress(comp, recs, rem, &dec, &rlen);
      if (drc) {
        rv_free(&acc);
        out->status = drc == ORC_E_UNSUPPORTED ? ORC_E_UNSUPPORTED : ORC_E_IO;
        return out->status;
      }
      recs = dec;
    }
    pos += 57 + rem;
    /* chain.process(SmartModuleInput::new(records, base_offset, first_timestamp)) */
    orc_result pr;
    int rc = orc_chain_process(c, recs, rlen, b_base, b_first_ts, &pr);
    free(dec);
    out->m_bytes_in += pr.m_bytes_in;
    out->m_invocations += pr.m_invocations;
    out->m_records_out += pr.m_records_out;
    if (rc) {
      orc_result_free(&pr);
      rv_free(&acc);
      out->status = rc;
      return rc;
    }
    recvec rv;
    recs_decode(pr.bytes, pr.bytes_len, &rv);
    int had_err = pr.has_error;
    if (rv.n) {
      if (sm_base == -1) {
        sm_attr = (int16_t)(comp & 7); /* set_compression */
        sm_base = b_base;
      }
      int64_t rel = sm_base - b_base;
      for (size_t i = 0; i < rv.n; i++) rv.r[i].off_delta += rel;
      uint64_t rb = recs_size(&rv);
      if (total + rb > max_bytes) {
        rv_free(&rv);
        if (had_err) {
          /* the error of the cut batch is returned alongside (batch.rs:106-110) */
          out->has_error = 1;
          out->hint = pr.hint;
          pr.hint = NULL;
          out->hint_len = pr.hint_len;
          out->err_offset = pr.err_offset;
          out->err_kind = pr.err_kind;
          out->has_key = pr.has_key;
          out->key = pr.key;
          pr.key = NULL;
          out->key_len = pr.key_len;
          out->value = pr.value;
          pr.value = NULL;
          out->value_len = pr.value_len;
        }
        orc_result_free(&pr);
        break;
      }
      total += rb;
      for (size_t i = 0; i < rv.n; i++) rv_push(&acc, rv.r[i]);
      free(rv.r);
    } else {
      rv_free(&rv);
    }
    if (sm_base != -1) sm_lod += b_lod + 1;
    if (had_err) {
      out->has_error = 1;
      out->hint = pr.hint;
      pr.hint = NULL;
      out->hint_len = pr.hint_len;
      out->err_offset = pr.err_offset;
      out->err_kind = pr.err_kind;
      out->has_key = pr.has_key;
      out->key = pr.key;
      pr.key = NULL;
      out->key_len = pr.key_len;
      out->value = pr.value;
      pr.value = NULL;
      out->value_len = pr.value_len;
      stop = 1;
    }
    orc_result_free(&pr);
  }
  /* Batch::encode (batch.rs:398-430) with Batch::default() header (batch.rs:482-497) */
  obuf body = {0};
  ob_be(&body, (uint16_t)sm_attr, 2);
  ob_be(&body, (uint32_t)sm_lod, 4);
  ob_be(&body, (uint64_t)(int64_t)-1, 8); /* first_timestamp */
  ob_be(&body, (uint64_t)(int64_t)-1, 8); /* max_time_stamp */
  ob_be(&body, (uint64_t)(int64_t)-1, 8); /* producer_id */
  ob_be(&body, (uint16_t)(int16_t)-1, 2); /* producer_epoch */
  ob_be(&body, (uint32_t)(int32_t)-1, 4); /* first_sequence */
  recs_encode(&body, &acc);
  uint32_t crc = orc_crc32c(body.p, body.n);
  obuf b = {0};
  ob_be(&b, (uint64_t)sm_base, 8);
  ob_be(&b, (uint32_t)(45 + recs_size(&acc)), 4);
  ob_be(&b, (uint32_t)(int32_t)-1, 4); /* partition_leader_epoch */
  ob_u8(&b, 2);                        /* magic */
  ob_be(&b, crc, 4);
  ob_put(&b, body.p, body.n);
  ob_free(&body);
  out->bytes = b.p;
  out->bytes_len = b.n;
  out->n_records = (uint32_t)acc.n;
  out->base_offset = sm_base;
  out->last_offset_delta = sm_lod;
  rv_free(&acc);
  return 0;
}

/* SmartModuleChainInstance::look_back (engine.rs:187-218) for one stage: the
 * records read_fn returned (SmartModuleInput::try_from_records: base offset 0)
 * through the module's look_back (derive generator/look_back.rs: the first Err
 * stops with SmartModuleLookbackRuntimeError{hint, offset = base + offset_delta,
 * key, value}).  Stages without a look_back export are skipped (instance.rs:92-95). */
int orc_chain_look_back(orc_chain *c, size_t stage, const uint8_t *raw, size_t raw_len, orc_result *out) {
  memset(out, 0, sizeof *out);
  if (stage >= c->n) return ORC_E_INVALID_ARG;
  stage_t *s = &c->st[stage];
  if (s->mod != M_FILTER_LOOKBACK && s->mod != M_FILTER_HASHSET) return 0;
  out->m_bytes_in = raw_len; /* metrics.add_bytes_in: bytes + one invocation */
  out->m_invocations = 1;
  recvec rv;
  if (recs_decode(raw, raw_len, &rv)) {
    out->status = ORC_E_DECODING_BASE_INPUT;
    return out->status;
  }
  for (size_t i = 0; i < rv.n; i++) {
    rec_t *r = &rv.r[i];
    size_t vut;
    int el;
    char *hint = NULL;
    if (!utf8_check(r->val, r->val_len, &vut, &el)) {
      hint = utf8_hint(vut, el);
    } else if (s->mod == M_FILTER_LOOKBACK) { /* filter_look_back/src/lib.rs:20-26: PREV = parse()? */
      int32_t x;
      int pk = parse_i32(r->val, r->val_len, &x);
      if (pk) hint = dup_str(parse_int_hint(pk));
      else s->prev = x;
    } else {
      (void)bhs_insert(s->set, r->val, r->val_len); /* filter_hashset/src/lib.rs:21-26 */
    }
    if (hint) {
      out->has_error = 1;
      out->hint = hint;
      out->hint_len = strlen(hint);
      out->err_offset = r->off_delta; /* base_offset 0 */
      out->has_key = r->has_key;
      out->key = r->key;
      out->key_len = r->key_len;
      out->value = r->val;
      out->value_len = r->val_len;
      r->key = r->val = NULL;
      break;
    }
  }
  rv_free(&rv);
  return 0;
}

void orc_result_free(orc_result *r) {
  if (!r) return;
  free(r->bytes);
  free(r->hint);
  free(r->key);
  free(r->value);
  free(r->message);
  memset(r, 0, sizeof *r);
}
