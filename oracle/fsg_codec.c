/* fsg_codec.c — CPU restatement of the record-section codecs of
 * crates/fluvio-compression (lib.rs:94-112: Compression::uncompress per
 * `attributes & 7`), used by FileBatchIterator (fluvio-storage iterators.rs:
 * 136-156) and ProduceBatchIterator (fluvio-spu produce_batch.rs:65-84).
 *
 * TEST INFRASTRUCTURE ONLY (the checker and the test-data generator): the
 * product path never links this file.
 *
 * The codecs are third-party crates absent from /root/reference (pinned in the
 * reference's Cargo.lock): flate2 (gzip member, RFC 1952 over RFC 1951 inflate),
 * lz4_flex 0.11 (LZ4 frame format), snap 1.x (Snappy framing format).  Restated
 * from their published formats:
 *   gzip   : zlib's inflate with the gzip wrapper (the canonical RFC 1951/1952
 *            implementation; header fields, CRC-32 and ISIZE are checked as
 *            GzDecoder checks them); one member, trailing bytes ignored
 *   lz4    : frames (magic 0x184D2204, FLG/BD, optional content size, header
 *            checksum = (xxh32(descriptor) >> 8) & 0xFF, blocks with optional
 *            xxh32 block checksums, end mark, optional xxh32 content checksum),
 *            skippable frames, concatenated frames, linked or independent blocks
 *   snappy : stream identifier "sNaPpY", compressed (0x00) / uncompressed (0x01)
 *            chunks with masked CRC-32C of the uncompressed data, padding (0xfe)
 *            and skippable (0x80-0xfd) chunks; raw snappy blocks inside
 *   zstd   : the zstd crate 0.13 (zstd-sys: libzstd) Decoder (zstd.rs:15-20):
 *            concatenated frames and skippable frames, no dictionary; here the
 *            system's libzstd itself (libzstd.so.1, loaded at first use), the
 *            canonical implementation of RFC 8878, as zlib is for gzip
 * Parity of the formats is pinned by round trips with independent encoders:
 * Python's zlib (gzip) and this file's LZ4 / Snappy encoders, plus the xxhash
 * module for xxh32 (tests/test_codecs.py), and by produce_batch.rs:124-153's
 * decoded record bytes.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <dlfcn.h>
#include <zlib.h>

#include "fsg_oracle.h"

typedef struct {
  uint8_t *p;
  size_t n, cap;
} cbuf;
static void cb_put(cbuf *b, const uint8_t *s, size_t n) {
  if (b->n + n > b->cap) {
    size_t c = b->cap ? b->cap : 256;
    while (c < b->n + n) c *= 2;
    b->p = (uint8_t *)realloc(b->p, c);
    b->cap = c;
  }
  if (n) memcpy(b->p + b->n, s, n);
  b->n += n;
}
static void cb_u8(cbuf *b, uint8_t v) { cb_put(b, &v, 1); }
static void cb_le32(cbuf *b, uint32_t v) {
  uint8_t t[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)};
  cb_put(b, t, 4);
}
static uint32_t le32(const uint8_t *p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

/* ---- xxh32 (XXH32 specification) ---- */
static const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
uint32_t orc_xxh32(const uint8_t *p, size_t n, uint32_t seed) {
  const uint8_t *e = p + n;
  uint32_t h;
  if (n >= 16) {
    uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    while (p + 16 <= e) {
      v1 = rotl(v1 + le32(p) * P2, 13) * P1;
      v2 = rotl(v2 + le32(p + 4) * P2, 13) * P1;
      v3 = rotl(v3 + le32(p + 8) * P2, 13) * P1;
      v4 = rotl(v4 + le32(p + 12) * P2, 13) * P1;
      p += 16;
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
  } else {
    h = seed + P5;
  }
  h += (uint32_t)n;
  while (p + 4 <= e) {
    h = rotl(h + le32(p) * P3, 17) * P4;
    p += 4;
  }
  while (p < e) h = rotl(h + (*p++) * P5, 11) * P1;
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

/* ---- gzip (flate2 GzDecoder / GzEncoder) via zlib ---- */
static int gzip_decode(const uint8_t *s, size_t n, cbuf *o) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (inflateInit2(&z, 16 + MAX_WBITS) != Z_OK) return -1;
  z.next_in = (Bytef *)s;
  z.avail_in = (uInt)n;
  uint8_t tmp[16384];
  int rc;
  do {
    z.next_out = tmp;
    z.avail_out = sizeof tmp;
    rc = inflate(&z, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&z);
      return -1;
    }
    cb_put(o, tmp, sizeof tmp - z.avail_out);
    if (rc == Z_OK && z.avail_in == 0 && z.avail_out != 0) { /* truncated member */
      inflateEnd(&z);
      return -1;
    }
  } while (rc != Z_STREAM_END);
  inflateEnd(&z);
  return 0;
}
static int gzip_encode(const uint8_t *s, size_t n, int level, cbuf *o) {
  z_stream z;
  memset(&z, 0, sizeof z);
  if (deflateInit2(&z, level, Z_DEFLATED, 16 + MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
  z.next_in = (Bytef *)s;
  z.avail_in = (uInt)n;
  uint8_t tmp[16384];
  int rc;
  do {
    z.next_out = tmp;
    z.avail_out = sizeof tmp;
    rc = deflate(&z, Z_FINISH);
    cb_put(o, tmp, sizeof tmp - z.avail_out);
  } while (rc == Z_OK);
  deflateEnd(&z);
  return rc == Z_STREAM_END ? 0 : -1;
}

/* ---- LZ4 block + frame ---- */
/* one block into o (o->n grows); the match window starts at `win0` of o */
static int lz4_block(const uint8_t *s, size_t n, cbuf *o, size_t win0) {
  size_t i = 0;
  for (;;) {
    if (i >= n) return -1;
    const uint8_t tok = s[i++];
    size_t lit = tok >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (i >= n) return -1;
        b = s[i++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - i) return -1;
    cb_put(o, s + i, lit);
    i += lit;
    if (i == n) return 0; /* the last sequence has literals only */
    if (n - i < 2) return -1;
    const size_t off = s[i] | (s[i + 1] << 8);
    i += 2;
    size_t ml = (tok & 15) + 4;
    if ((tok & 15) == 15) {
      uint8_t b;
      do {
        if (i >= n) return -1;
        b = s[i++];
        ml += b;
      } while (b == 255);
    }
    if (off == 0 || off > o->n - win0) return -1;
    for (size_t k = 0; k < ml; k++) {
      const uint8_t c = o->p[o->n - off];
      cb_put(o, &c, 1);
    }
  }
}
static int lz4_frames(const uint8_t *s, size_t n, cbuf *o) {
  size_t i = 0;
  while (i < n) {
    if (n - i < 4) return -1;
    const uint32_t magic = le32(s + i);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) { /* skippable frame */
      if (n - i < 8) return -1;
      const uint32_t len = le32(s + i + 4);
      if (len > n - i - 8) return -1;
      i += 8 + (size_t)len;
      continue;
    }
    if (magic != 0x184D2204u) return -1;
    i += 4;
    const size_t d0 = i;
    if (n - i < 3) return -1;
    const uint8_t flg = s[i], bd = s[i + 1];
    if ((flg >> 6) != 1 || (flg & 2) || (bd & 0x8F)) return -1;
    const int indep = (flg >> 5) & 1, bsum = (flg >> 4) & 1, csize = (flg >> 3) & 1, csum = (flg >> 2) & 1,
              dict = flg & 1;
    const int bsz = (bd >> 4) & 7;
    if (bsz < 4) return -1;
    const size_t bmax = (size_t)1 << (2 * bsz + 8); /* 4: 64 KiB .. 7: 4 MiB */
    i += 2;
    uint64_t content = 0;
    if (csize) {
      if (n - i < 8) return -1;
      content = (uint64_t)le32(s + i) | ((uint64_t)le32(s + i + 4) << 32);
      i += 8;
    }
    if (dict) return -1; /* dictionaries: not supported by the decoder */
    if (n - i < 1) return -1;
    if (s[i] != ((orc_xxh32(s + d0, i - d0, 0) >> 8) & 0xFF)) return -1;
    i++;
    const size_t f0 = o->n;
    for (;;) {
      if (n - i < 4) return -1;
      const uint32_t bs = le32(s + i);
      i += 4;
      if (bs == 0) break; /* end mark */
      const size_t len = bs & 0x7FFFFFFFu;
      if (len > bmax || len > n - i) return -1;
      const size_t b0 = o->n;
      if (bs & 0x80000000u)
        cb_put(o, s + i, len);
      else if (lz4_block(s + i, len, o, indep ? b0 : f0))
        return -1;
      if (o->n - b0 > bmax) return -1;
      if (bsum) {
        if (n - i - len < 4 || le32(s + i + len) != orc_xxh32(s + i, len, 0)) return -1;
        i += 4;
      }
      i += len;
    }
    if (csize && o->n - f0 != content) return -1;
    if (csum) {
      if (n - i < 4 || le32(s + i) != orc_xxh32(o->p + f0, o->n - f0, 0)) return -1;
      i += 4;
    }
  }
  return 0;
}
/* greedy LZ4 compressor (hash of 4 bytes, one candidate): test data only */
static void lz4_compress_block(const uint8_t *s, size_t n, cbuf *o) {
  int32_t *ht = (int32_t *)malloc(4096 * sizeof(int32_t));
  for (int k = 0; k < 4096; k++) ht[k] = -1;
  size_t i = 0, anchor = 0;
  while (n >= 13 && i + 12 < n) { /* matches must end >= 5 bytes before the end */
    const uint32_t v = le32(s + i);
    const uint32_t h = (v * 2654435761u) >> 20;
    const int32_t c = ht[h];
    ht[h] = (int32_t)i;
    if (c < 0 || i - (size_t)c > 65535 || le32(s + c) != v) {
      i++;
      continue;
    }
    size_t ml = 4;
    while (i + ml + 5 < n && s[c + ml] == s[i + ml]) ml++;
    const size_t lit = i - anchor;
    uint8_t tok = (uint8_t)(((lit >= 15 ? 15 : lit) << 4) | (ml - 4 >= 15 ? 15 : ml - 4));
    cb_u8(o, tok);
    if (lit >= 15) {
      size_t r = lit - 15;
      for (; r >= 255; r -= 255) cb_u8(o, 255);
      cb_u8(o, (uint8_t)r);
    }
    cb_put(o, s + anchor, lit);
    const size_t off = i - (size_t)c;
    cb_u8(o, (uint8_t)off);
    cb_u8(o, (uint8_t)(off >> 8));
    if (ml - 4 >= 15) {
      size_t r = ml - 4 - 15;
      for (; r >= 255; r -= 255) cb_u8(o, 255);
      cb_u8(o, (uint8_t)r);
    }
    i += ml;
    anchor = i;
  }
  const size_t lit = n - anchor;
  cb_u8(o, (uint8_t)((lit >= 15 ? 15 : lit) << 4));
  if (lit >= 15) {
    size_t r = lit - 15;
    for (; r >= 255; r -= 255) cb_u8(o, 255);
    cb_u8(o, (uint8_t)r);
  }
  cb_put(o, s + anchor, lit);
  free(ht);
}
/* flags: bit0 block checksums, bit1 content checksum, bit2 content size,
 * bit3 linked blocks, bit4 store blocks uncompressed; block size 64 KiB */
static void lz4_encode(const uint8_t *s, size_t n, int flags, cbuf *o) {
  cb_le32(o, 0x184D2204u);
  const size_t d0 = o->n;
  uint8_t flg = 0x40 | ((flags & 8) ? 0 : 0x20) | ((flags & 1) ? 0x10 : 0) | ((flags & 4) ? 0x08 : 0) |
                ((flags & 2) ? 0x04 : 0);
  cb_u8(o, flg);
  cb_u8(o, 0x40); /* 64 KiB blocks */
  if (flags & 4) {
    cb_le32(o, (uint32_t)n);
    cb_le32(o, (uint32_t)((uint64_t)n >> 32));
  }
  cb_u8(o, (uint8_t)((orc_xxh32(o->p + d0, o->n - d0, 0) >> 8) & 0xFF));
  for (size_t b = 0; b < n; b += 65536) {
    const size_t len = n - b < 65536 ? n - b : 65536;
    cbuf blk = {0};
    if (!(flags & 16)) lz4_compress_block(s + b, len, &blk);
    if ((flags & 16) || blk.n >= len) {
      cb_le32(o, 0x80000000u | (uint32_t)len);
      cb_put(o, s + b, len);
      if (flags & 1) cb_le32(o, orc_xxh32(s + b, len, 0));
    } else {
      cb_le32(o, (uint32_t)blk.n);
      cb_put(o, blk.p, blk.n);
      if (flags & 1) cb_le32(o, orc_xxh32(blk.p, blk.n, 0));
    }
    free(blk.p);
  }
  cb_le32(o, 0);
  if (flags & 2) cb_le32(o, orc_xxh32(s, n, 0));
}

/* ---- Snappy raw + framing ---- */
static uint32_t snappy_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
static int snappy_raw(const uint8_t *s, size_t n, cbuf *o) {
  size_t i = 0;
  uint64_t want = 0;
  int sh = 0;
  for (;;) { /* varint32 uncompressed length */
    if (i >= n || sh > 28) return -1;
    const uint8_t b = s[i++];
    want |= (uint64_t)(b & 0x7F) << sh;
    sh += 7;
    if (!(b & 0x80)) break;
  }
  if (want > 0xFFFFFFFFull) return -1;
  const size_t o0 = o->n;
  while (i < n) {
    const uint8_t tag = s[i++];
    size_t len, off = 0;
    switch (tag & 3) {
      case 0: {
        len = tag >> 2;
        if (len >= 60) {
          const size_t nb = len - 59;
          if (n - i < nb) return -1;
          len = 0;
          for (size_t k = 0; k < nb; k++) len |= (size_t)s[i + k] << (8 * k);
          i += nb;
        }
        len += 1;
        if (len > n - i) return -1;
        cb_put(o, s + i, len);
        i += len;
        continue;
      }
      case 1:
        if (i >= n) return -1;
        len = ((tag >> 2) & 7) + 4;
        off = ((size_t)(tag >> 5) << 8) | s[i++];
        break;
      case 2:
        if (n - i < 2) return -1;
        len = (tag >> 2) + 1;
        off = s[i] | (s[i + 1] << 8);
        i += 2;
        break;
      default:
        if (n - i < 4) return -1;
        len = (tag >> 2) + 1;
        off = le32(s + i);
        i += 4;
        break;
    }
    if (off == 0 || off > o->n - o0) return -1;
    for (size_t k = 0; k < len; k++) {
      const uint8_t c = o->p[o->n - off];
      cb_put(o, &c, 1);
    }
    if (o->n - o0 > want) return -1;
  }
  return o->n - o0 == want ? 0 : -1;
}
static int snappy_frames(const uint8_t *s, size_t n, cbuf *o) {
  size_t i = 0;
  int seen_id = 0;
  while (i < n) {
    if (n - i < 4) return -1;
    const uint8_t t = s[i];
    const size_t len = s[i + 1] | (s[i + 2] << 8) | (s[i + 3] << 16);
    i += 4;
    if (len > n - i) return -1;
    const uint8_t *d = s + i;
    i += len;
    if (t == 0xff) {
      if (len != 6 || memcmp(d, "sNaPpY", 6)) return -1;
      seen_id = 1;
      continue;
    }
    if (!seen_id) return -1;
    if (t == 0x00 || t == 0x01) {
      if (len < 4) return -1;
      const uint32_t want = le32(d);
      const size_t o0 = o->n;
      if (t == 0x00) {
        if (snappy_raw(d + 4, len - 4, o)) return -1;
      } else {
        cb_put(o, d + 4, len - 4);
      }
      if (o->n - o0 > 65536) return -1;
      if (snappy_mask(orc_crc32c(o->p + o0, o->n - o0)) != want) return -1;
    } else if (t >= 0x02 && t <= 0x7f) {
      return -1; /* reserved unskippable */
    } /* 0x80-0xfd skippable, 0xfe padding */
  }
  return 0;
}
static void snappy_compress_raw(const uint8_t *s, size_t n, cbuf *o) {
  for (uint64_t v = n;;) { /* varint32 */
    uint8_t b = v & 0x7F;
    v >>= 7;
    if (v) b |= 0x80;
    cb_u8(o, b);
    if (!v) break;
  }
  int32_t *ht = (int32_t *)malloc(4096 * sizeof(int32_t));
  for (int k = 0; k < 4096; k++) ht[k] = -1;
  size_t i = 0, anchor = 0;
  while (n >= 4 && i + 4 <= n) {
    const uint32_t v = le32(s + i);
    const uint32_t h = (v * 0x1e35a7bdu) >> 20;
    const int32_t c = ht[h];
    ht[h] = (int32_t)i;
    if (c < 0 || i - (size_t)c > 65535 || le32(s + c) != v) {
      i++;
      continue;
    }
    size_t ml = 4;
    while (i + ml < n && ml < 64 && s[c + ml] == s[i + ml]) ml++;
    for (size_t p = anchor; p < i;) { /* literals, <= 60 per element */
      size_t l = i - p < 60 ? i - p : 60;
      cb_u8(o, (uint8_t)((l - 1) << 2));
      cb_put(o, s + p, l);
      p += l;
    }
    const size_t off = i - (size_t)c;
    cb_u8(o, (uint8_t)(((ml - 1) << 2) | 2)); /* copy2 */
    cb_u8(o, (uint8_t)off);
    cb_u8(o, (uint8_t)(off >> 8));
    i += ml;
    anchor = i;
  }
  for (size_t p = anchor; p < n;) {
    size_t l = n - p < 60 ? n - p : 60;
    cb_u8(o, (uint8_t)((l - 1) << 2));
    cb_put(o, s + p, l);
    p += l;
  }
  free(ht);
}
/* flags: bit0 store chunks uncompressed, bit1 add a padding and a skippable chunk */
static void snappy_encode(const uint8_t *s, size_t n, int flags, cbuf *o) {
  const uint8_t id[10] = {0xff, 6, 0, 0, 's', 'N', 'a', 'P', 'p', 'Y'};
  cb_put(o, id, 10);
  if (flags & 2) {
    const uint8_t pad[7] = {0xfe, 3, 0, 0, 0, 0, 0}, skip[6] = {0x99, 2, 0, 0, 7, 7};
    cb_put(o, pad, 7);
    cb_put(o, skip, 6);
  }
  for (size_t b = 0; b < n; b += 65536) {
    const size_t len = n - b < 65536 ? n - b : 65536;
    const uint32_t crc = snappy_mask(orc_crc32c(s + b, len));
    cbuf c = {0};
    if (!(flags & 1)) snappy_compress_raw(s + b, len, &c);
    const int raw = (flags & 1) || c.n >= len;
    const size_t clen = 4 + (raw ? len : c.n);
    cb_u8(o, raw ? 0x01 : 0x00);
    cb_u8(o, (uint8_t)clen);
    cb_u8(o, (uint8_t)(clen >> 8));
    cb_u8(o, (uint8_t)(clen >> 16));
    cb_le32(o, crc);
    cb_put(o, raw ? s + b : c.p, raw ? len : c.n);
    free(c.p);
  }
}

/* ---- zstd (zstd crate Decoder / Encoder level 1) through the system libzstd ----
 * (prototypes of the stable API, zstd.h 1.4; no header in this image) */
typedef struct { const void *src; size_t size; size_t pos; } zin_t;
typedef struct { void *dst; size_t size; size_t pos; } zout_t;
static struct {
  int tried, ok;
  void *(*createDStream)(void);
  size_t (*freeDStream)(void *);
  size_t (*initDStream)(void *);
  size_t (*decompressStream)(void *, zout_t *, zin_t *);
  unsigned (*isError)(size_t);
  size_t (*compressBound)(size_t);
  void *(*createCCtx)(void);
  size_t (*freeCCtx)(void *);
  size_t (*setParameter)(void *, int, int);
  size_t (*compress2)(void *, void *, size_t, const void *, size_t);
} Z;
static int zstd_load(void) {
  if (Z.tried) return Z.ok;
  Z.tried = 1;
  void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return 0;
  *(void **)&Z.createDStream = dlsym(h, "ZSTD_createDStream");
  *(void **)&Z.freeDStream = dlsym(h, "ZSTD_freeDStream");
  *(void **)&Z.initDStream = dlsym(h, "ZSTD_initDStream");
  *(void **)&Z.decompressStream = dlsym(h, "ZSTD_decompressStream");
  *(void **)&Z.isError = dlsym(h, "ZSTD_isError");
  *(void **)&Z.compressBound = dlsym(h, "ZSTD_compressBound");
  *(void **)&Z.createCCtx = dlsym(h, "ZSTD_createCCtx");
  *(void **)&Z.freeCCtx = dlsym(h, "ZSTD_freeCCtx");
  *(void **)&Z.setParameter = dlsym(h, "ZSTD_CCtx_setParameter");
  *(void **)&Z.compress2 = dlsym(h, "ZSTD_compress2");
  Z.ok = Z.createDStream && Z.freeDStream && Z.initDStream && Z.decompressStream && Z.isError && Z.compressBound &&
         Z.createCCtx && Z.freeCCtx && Z.setParameter && Z.compress2;
  return Z.ok;
}
/* read_to_end of zstd::stream::read::Decoder: frames until the input ends; the
 * input ending inside a frame, or bytes that are not a frame, is an error */
static int zstd_decode(const uint8_t *s, size_t n, cbuf *o) {
  if (!zstd_load()) return ORC_E_UNSUPPORTED;
  void *d = Z.createDStream();
  if (!d || Z.isError(Z.initDStream(d))) {
    if (d) Z.freeDStream(d);
    return -1;
  }
  zin_t in = {s, n, 0};
  uint8_t tmp[1 << 16];
  size_t hint = 1; /* zio::Reader starts with finished_frame = false: an empty input is an incomplete frame */
  int rc = 0;
  for (;;) {
    zout_t out = {tmp, sizeof tmp, 0};
    hint = Z.decompressStream(d, &out, &in);
    if (Z.isError(hint)) {
      rc = -1;
      break;
    }
    cb_put(o, tmp, out.pos);
    if (in.pos == in.size && out.pos < out.size) break; /* input consumed, output flushed */
  }
  if (!rc && hint) rc = -1; /* the input ended inside a frame ("incomplete frame") */
  Z.freeDStream(d);
  return rc;
}
/* flags: low byte = level (0 -> 1, the crate's Encoder::new(_, 1)); 0x100 content
 * checksum; 0x200 no content size; 0x400 two concatenated frames; 0x800 a
 * skippable frame first */
static int zstd_encode(const uint8_t *s, size_t n, int flags, cbuf *o) {
  if (!zstd_load()) return ORC_E_UNSUPPORTED;
  const int level = (flags & 0xFF) ? (flags & 0xFF) : 1;
  if (flags & 0x800) {
    const uint8_t skip[12] = {0x53, 0x2A, 0x4D, 0x18, 4, 0, 0, 0, 'f', 's', 'g', '!'};
    cb_put(o, skip, sizeof skip);
  }
  const int parts = (flags & 0x400) && n > 1 ? 2 : 1;
  for (int k = 0; k < parts; k++) {
    const size_t a = parts == 1 ? 0 : (k ? n / 2 : 0), b = parts == 1 ? n : (k ? n : n / 2);
    void *c = Z.createCCtx();
    if (!c) return -1;
    Z.setParameter(c, 100, level);                        /* ZSTD_c_compressionLevel */
    Z.setParameter(c, 201, (flags & 0x100) ? 1 : 0);      /* ZSTD_c_checksumFlag */
    Z.setParameter(c, 200, (flags & 0x200) ? 0 : 1);      /* ZSTD_c_contentSizeFlag */
    const size_t cap = Z.compressBound(b - a);
    uint8_t *tmp = (uint8_t *)malloc(cap ? cap : 1);
    const size_t r = Z.compress2(c, tmp, cap, s + a, b - a);
    Z.freeCCtx(c);
    if (Z.isError(r)) {
      free(tmp);
      return -1;
    }
    cb_put(o, tmp, r);
    free(tmp);
  }
  return 0;
}

/* Compression::uncompress: 0 ok (*out malloc'd), -1 a decode error (io::Error) */
int orc_decompress(int codec, const uint8_t *s, size_t n, uint8_t **out, size_t *out_len) {
  cbuf o = {0};
  int rc;
  switch (codec) {
    case 1: rc = gzip_decode(s, n, &o); break;
    case 2: rc = snappy_frames(s, n, &o); break;
    case 3: rc = lz4_frames(s, n, &o); break;
    case 4: rc = zstd_decode(s, n, &o); break;
    default: rc = -1; break;
  }
  if (rc) {
    free(o.p);
    return rc;
  }
  *out = o.p ? o.p : (uint8_t *)malloc(1);
  *out_len = o.n;
  return 0;
}
/* test-data encoders: codec 1 gzip (flags = zlib level, 0 -> 6), 2 snappy, 3 lz4, 4 zstd */
int orc_compress(int codec, const uint8_t *s, size_t n, int flags, uint8_t **out, size_t *out_len) {
  cbuf o = {0};
  int rc = 0;
  switch (codec) {
    case 1: rc = gzip_encode(s, n, flags ? flags : 6, &o); break;
    case 2: snappy_encode(s, n, flags, &o); break;
    case 3: lz4_encode(s, n, flags, &o); break;
    case 4: rc = zstd_encode(s, n, flags, &o); break;
    default: rc = -1;
  }
  if (rc) {
    free(o.p);
    return rc;
  }
  *out = o.p ? o.p : (uint8_t *)malloc(1);
  *out_len = o.n;
  return 0;
}
