// fsg_codec_dev.h — record-section decompression on the GPU.
//
// FileBatchIterator (fluvio-storage iterators.rs:136-156) and
// ProduceBatchIterator (fluvio-spu produce_batch.rs:65-84) hand each batch's
// record section through Compression::uncompress (fluvio-compression
// lib.rs:94-112) chosen by `attributes & 7`: 1 gzip (flate2 GzDecoder), 2
// snappy (snap FrameDecoder), 3 lz4 (lz4_flex FrameDecoder), 4 zstd.  The
// formats (third-party crates, not in the reference tree) are restated here
// from their specifications; zstd is not (FSG_E_UNSUPPORTED at that batch).
//
// One thread decodes one batch's section (a ~16 KiB batch is one serial LZ77 /
// Huffman stream; thousands of batches in flight fill the GPU).  The same code
// runs twice: a sizing pass (write = false: structure checked, output only
// counted) and the writing pass, which also checks every checksum (gzip CRC-32
// + ISIZE, lz4 header / block / content xxh32, snappy masked CRC-32C).
#pragma once
#include <stdint.h>

namespace fsg {

enum DecStatus : int64_t { DEC_BAD = -1, DEC_UNSUP = -2 };

struct DecOut {
  uint8_t* p;     // output (nullptr in the sizing pass)
  uint64_t n;     // bytes produced
  uint64_t cap;   // the writing pass: exact size from the sizing pass
  bool write;
  __device__ bool put(uint8_t c) {
    if (write) {
      if (n >= cap) return false;
      p[n] = c;
    }
    n++;
    return true;
  }
  // LZ77 back-reference of `len` bytes at distance `off` (overlap allowed)
  __device__ bool copy(uint64_t off, uint64_t len, uint64_t win0) {
    if (off == 0 || off > n - win0) return false;
    if (!write) {
      n += len;
      return true;
    }
    if (n + len > cap) return false;
    for (uint64_t k = 0; k < len; k++, n++) p[n] = p[n - off];
    return true;
  }
  __device__ bool put_span(const uint8_t* s, uint64_t len) {
    if (write) {
      if (n + len > cap) return false;
      for (uint64_t k = 0; k < len; k++) p[n + k] = s[k];
    }
    n += len;
    return true;
  }
};

__device__ __forceinline__ uint32_t dec_le32(const uint8_t* p) {
  return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
}

// ---- checksums
__device__ __forceinline__ uint32_t xxh_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ uint32_t dev_xxh32(const uint8_t* p, uint64_t n) {  // seed 0
  const uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
  const uint8_t* e = p + n;
  uint32_t h;
  if (n >= 16) {
    uint32_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0u - P1;
    while (p + 16 <= e) {
      v1 = xxh_rotl(v1 + dec_le32(p) * P2, 13) * P1;
      v2 = xxh_rotl(v2 + dec_le32(p + 4) * P2, 13) * P1;
      v3 = xxh_rotl(v3 + dec_le32(p + 8) * P2, 13) * P1;
      v4 = xxh_rotl(v4 + dec_le32(p + 12) * P2, 13) * P1;
      p += 16;
    }
    h = xxh_rotl(v1, 1) + xxh_rotl(v2, 7) + xxh_rotl(v3, 12) + xxh_rotl(v4, 18);
  } else {
    h = P5;
  }
  h += (uint32_t)n;
  while (p + 4 <= e) {
    h = xxh_rotl(h + dec_le32(p) * P3, 17) * P4;
    p += 4;
  }
  while (p < e) h = xxh_rotl(h + (*p++) * P5, 11) * P1;
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}
// CRC-32 (IEEE, reflected 0xEDB88320) byte table, built at compile time
struct Crc32Tab {
  uint32_t t[256];
  constexpr Crc32Tab() : t() {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
      t[i] = c;
    }
  }
};
__device__ constexpr Crc32Tab g_crc32_ieee{};

// ---- LZ4 (block + frame)
__device__ bool lz4_block_dev(const uint8_t* s, uint64_t n, DecOut& o, uint64_t win0) {
  uint64_t i = 0;
  for (;;) {
    if (i >= n) return false;
    const uint8_t tok = s[i++];
    uint64_t lit = tok >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (i >= n) return false;
        b = s[i++];
        lit += b;
      } while (b == 255);
    }
    if (lit > n - i) return false;
    if (!o.put_span(s + i, lit)) return false;
    i += lit;
    if (i == n) return true;  // the last sequence has literals only
    if (n - i < 2) return false;
    const uint64_t off = s[i] | (s[i + 1] << 8);
    i += 2;
    uint64_t ml = (tok & 15) + 4;
    if ((tok & 15) == 15) {
      uint8_t b;
      do {
        if (i >= n) return false;
        b = s[i++];
        ml += b;
      } while (b == 255);
    }
    if (!o.copy(off, ml, win0)) return false;
  }
}
__device__ bool lz4_frames_dev(const uint8_t* s, uint64_t n, DecOut& o) {
  uint64_t i = 0;
  while (i < n) {
    if (n - i < 4) return false;
    const uint32_t magic = dec_le32(s + i);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (n - i < 8) return false;
      const uint32_t len = dec_le32(s + i + 4);
      if (len > n - i - 8) return false;
      i += 8 + (uint64_t)len;
      continue;
    }
    if (magic != 0x184D2204u) return false;
    i += 4;
    const uint64_t d0 = i;
    if (n - i < 3) return false;
    const uint8_t flg = s[i], bd = s[i + 1];
    if ((flg >> 6) != 1 || (flg & 2) || (bd & 0x8F)) return false;
    const bool indep = (flg >> 5) & 1, bsum = (flg >> 4) & 1, csize = (flg >> 3) & 1, csum = (flg >> 2) & 1,
               dict = flg & 1;
    const int bsz = (bd >> 4) & 7;
    if (bsz < 4 || dict) return false;
    const uint64_t bmax = 1ull << (2 * bsz + 8);
    i += 2;
    uint64_t content = 0;
    if (csize) {
      if (n - i < 8) return false;
      content = (uint64_t)dec_le32(s + i) | ((uint64_t)dec_le32(s + i + 4) << 32);
      i += 8;
    }
    if (n - i < 1) return false;
    if (s[i] != ((dev_xxh32(s + d0, i - d0) >> 8) & 0xFF)) return false;
    i++;
    const uint64_t f0 = o.n;
    for (;;) {
      if (n - i < 4) return false;
      const uint32_t bs = dec_le32(s + i);
      i += 4;
      if (bs == 0) break;  // end mark
      const uint64_t len = bs & 0x7FFFFFFFu;
      if (len > bmax || len > n - i) return false;
      const uint64_t b0 = o.n;
      if (bs & 0x80000000u) {
        if (!o.put_span(s + i, len)) return false;
      } else if (!lz4_block_dev(s + i, len, o, indep ? b0 : f0)) {
        return false;
      }
      if (o.n - b0 > bmax) return false;
      if (bsum) {
        if (n - i - len < 4 || dec_le32(s + i + len) != dev_xxh32(s + i, len)) return false;
        i += 4;
      }
      i += len;
    }
    if (csize && o.n - f0 != content) return false;
    if (csum) {
      if (n - i < 4) return false;
      if (o.write && dec_le32(s + i) != dev_xxh32(o.p + f0, o.n - f0)) return false;
      i += 4;
    }
  }
  return true;
}

// ---- Snappy (raw + framing)
__device__ bool snappy_raw_dev(const uint8_t* s, uint64_t n, DecOut& o) {
  uint64_t i = 0, want = 0;
  int sh = 0;
  for (;;) {
    if (i >= n || sh > 28) return false;
    const uint8_t b = s[i++];
    want |= (uint64_t)(b & 0x7F) << sh;
    sh += 7;
    if (!(b & 0x80)) break;
  }
  if (want > 0xFFFFFFFFull) return false;
  const uint64_t o0 = o.n;
  while (i < n) {
    const uint8_t tag = s[i++];
    uint64_t len, off;
    const uint32_t kind = tag & 3;
    if (kind == 0) {
      len = tag >> 2;
      if (len >= 60) {
        const uint64_t nb = len - 59;
        if (n - i < nb) return false;
        len = 0;
        for (uint64_t k = 0; k < nb; k++) len |= (uint64_t)s[i + k] << (8 * k);
        i += nb;
      }
      len += 1;
      if (len > n - i || !o.put_span(s + i, len)) return false;
      i += len;
      continue;
    }
    if (kind == 1) {
      if (i >= n) return false;
      len = ((tag >> 2) & 7) + 4;
      off = ((uint64_t)(tag >> 5) << 8) | s[i++];
    } else if (kind == 2) {
      if (n - i < 2) return false;
      len = (tag >> 2) + 1;
      off = s[i] | (s[i + 1] << 8);
      i += 2;
    } else {
      if (n - i < 4) return false;
      len = (tag >> 2) + 1;
      off = dec_le32(s + i);
      i += 4;
    }
    if (!o.copy(off, len, o0) || o.n - o0 > want) return false;
  }
  return o.n - o0 == want;
}
__device__ bool snappy_frames_dev(const uint8_t* s, uint64_t n, DecOut& o, const uint32_t* crc32c_tab) {
  uint64_t i = 0;
  bool seen_id = false;
  while (i < n) {
    if (n - i < 4) return false;
    const uint8_t t = s[i];
    const uint64_t len = s[i + 1] | (s[i + 2] << 8) | ((uint32_t)s[i + 3] << 16);
    i += 4;
    if (len > n - i) return false;
    const uint8_t* d = s + i;
    i += len;
    if (t == 0xff) {  // stream identifier
      if (len != 6 || d[0] != 's' || d[1] != 'N' || d[2] != 'a' || d[3] != 'P' || d[4] != 'p' || d[5] != 'Y')
        return false;
      seen_id = true;
      continue;
    }
    if (!seen_id) return false;
    if (t == 0x00 || t == 0x01) {
      if (len < 4) return false;
      const uint32_t want = dec_le32(d);
      const uint64_t o0 = o.n;
      if (t == 0x00) {
        if (!snappy_raw_dev(d + 4, len - 4, o)) return false;
      } else if (!o.put_span(d + 4, len - 4)) {
        return false;
      }
      if (o.n - o0 > 65536) return false;
      if (o.write) {  // masked CRC-32C of the uncompressed data
        uint32_t c = 0xFFFFFFFFu;
        for (uint64_t k = o0; k < o.n; k++) c = crc32c_tab[(c ^ o.p[k]) & 0xff] ^ (c >> 8);
        c ^= 0xFFFFFFFFu;
        if (((c >> 15) | (c << 17)) + 0xa282ead8u != want) return false;
      }
    } else if (t >= 0x02 && t <= 0x7f) {
      return false;  // reserved unskippable
    }  // 0x80-0xfd skippable, 0xfe padding
  }
  return true;
}

// ---- gzip member (RFC 1952) over inflate (RFC 1951)
// The canonical-code construction (count / offs / sym) and the stored / fixed /
// dynamic block walk follow the structure of Mark Adler's public-domain puff.c
// (zlib contrib/puff); decoding is table-driven here (9-bit first-level table,
// canonical walk only for longer codes).
struct Bits {
  const uint8_t* s;
  uint64_t n, i;
  uint32_t buf, cnt;
  bool bad;
  __device__ void fill(uint32_t k) {  // up to k (<= 24) bits buffered, fewer at the end of the stream
    while (cnt < k && i < n) {
      buf |= (uint32_t)s[i++] << cnt;
      cnt += 8;
    }
  }
  // to the next byte boundary: whole bytes fill() read ahead go back to the stream
  __device__ void align() {
    i -= cnt >> 3;
    buf = 0;
    cnt = 0;
  }
  __device__ uint32_t get(uint32_t k) {  // k <= 24
    while (cnt < k) {
      if (i >= n) {
        bad = true;
        return 0;
      }
      buf |= (uint32_t)s[i++] << cnt;
      cnt += 8;
    }
    const uint32_t v = buf & ((1u << k) - 1u);
    buf >>= k;
    cnt -= k;
    return v;
  }
};
constexpr int kHuffFast = 9;  // first-level table bits
struct Huff {
  uint16_t cnt[16];
  uint16_t sym[288];
  uint16_t fast[1 << kHuffFast];  // stream bits (LSB first) -> sym << 4 | len, 0 = longer code
};
// canonical code lengths -> counts / symbols; false if over-subscribed
// (incomplete codes are allowed, as zlib allows a single distance code)
__device__ bool huff_build(Huff& h, const uint8_t* len, int n) {
  for (int k = 0; k < 16; k++) h.cnt[k] = 0;
  for (int s = 0; s < n; s++) h.cnt[len[s]]++;
  for (int k = 0; k < (1 << kHuffFast); k++) h.fast[k] = 0;
  if (h.cnt[0] == n) return true;
  int left = 1;
  for (int k = 1; k < 16; k++) {
    left <<= 1;
    left -= h.cnt[k];
    if (left < 0) return false;
  }
  uint16_t offs[16];
  offs[1] = 0;
  for (int k = 1; k < 15; k++) offs[k + 1] = offs[k] + h.cnt[k];
  for (int s = 0; s < n; s++)
    if (len[s]) h.sym[offs[len[s]]++] = (uint16_t)s;
  // first-level table: canonical codes in symbol order within each length,
  // bit-reversed (deflate sends codes MSB first into an LSB-first stream)
  int code = 0, idx = 0;
  for (int L = 1; L <= kHuffFast; L++) {
    for (int j = 0; j < h.cnt[L]; j++, code++) {
      uint32_t r = 0;
      for (int q = 0; q < L; q++) r |= (uint32_t)((code >> q) & 1) << (L - 1 - q);
      const uint16_t e = (uint16_t)((h.sym[idx + j] << 4) | L);
      for (uint32_t f = r; f < (1u << kHuffFast); f += 1u << L) h.fast[f] = e;
    }
    idx += h.cnt[L];
    code <<= 1;
  }
  return true;
}
__device__ int huff_decode(Bits& b, const Huff& h) {
  b.fill(kHuffFast);
  const uint32_t e = h.fast[b.buf & ((1u << kHuffFast) - 1u)];
  if (e && (e & 15u) <= b.cnt) {
    b.buf >>= e & 15u;
    b.cnt -= e & 15u;
    return (int)(e >> 4);
  }
  int code = 0, first = 0, index = 0;
  for (int k = 1; k < 16; k++) {
    code |= (int)b.get(1);
    if (b.bad) return -1;
    const int count = h.cnt[k];
    if (code - count < first) return h.sym[index + (code - first)];
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -1;
}
__device__ bool inflate_codes(Bits& b, DecOut& o, const Huff& lc, const Huff& dc, uint64_t win0) {
  const uint16_t lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                              35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
  const uint8_t lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
  const uint16_t dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                              193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
  const uint8_t dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
  for (;;) {
    int sym = huff_decode(b, lc);
    if (sym < 0) return false;
    if (sym < 256) {
      if (!o.put((uint8_t)sym)) return false;
      continue;
    }
    if (sym == 256) return true;
    sym -= 257;
    if (sym >= 29) return false;
    const uint64_t len = lbase[sym] + b.get(lext[sym]);
    const int ds = huff_decode(b, dc);
    if (ds < 0 || ds >= 30) return false;
    const uint64_t dist = dbase[ds] + b.get(dext[ds]);
    if (b.bad || !o.copy(dist, len, win0)) return false;
  }
}
__device__ bool inflate_dev(Bits& b, DecOut& o) {
  const uint64_t win0 = o.n;
  Huff lc, dc;
  uint8_t lens[320];
  for (;;) {
    const uint32_t last = b.get(1), type = b.get(2);
    if (b.bad) return false;
    if (type == 0) {  // stored
      b.align();  // to a byte boundary
      if (b.n - b.i < 4) return false;
      const uint32_t len = b.s[b.i] | (b.s[b.i + 1] << 8), nlen = b.s[b.i + 2] | (b.s[b.i + 3] << 8);
      b.i += 4;
      if (len != (~nlen & 0xFFFFu) || len > b.n - b.i || !o.put_span(b.s + b.i, len)) return false;
      b.i += len;
    } else if (type == 1) {  // fixed codes
      for (int s = 0; s < 144; s++) lens[s] = 8;
      for (int s = 144; s < 256; s++) lens[s] = 9;
      for (int s = 256; s < 280; s++) lens[s] = 7;
      for (int s = 280; s < 288; s++) lens[s] = 8;
      huff_build(lc, lens, 288);
      for (int s = 0; s < 30; s++) lens[s] = 5;
      huff_build(dc, lens, 30);
      if (!inflate_codes(b, o, lc, dc, win0)) return false;
    } else if (type == 2) {  // dynamic codes
      const int nlen = (int)b.get(5) + 257, ndist = (int)b.get(5) + 1, ncode = (int)b.get(4) + 4;
      if (b.bad || nlen > 286 || ndist > 30) return false;
      const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
      uint8_t cl[19];
      for (int k = 0; k < 19; k++) cl[k] = 0;
      for (int k = 0; k < ncode; k++) cl[order[k]] = (uint8_t)b.get(3);
      if (b.bad || !huff_build(lc, cl, 19)) return false;
      int idx = 0;
      while (idx < nlen + ndist) {
        const int sym = huff_decode(b, lc);
        if (sym < 0) return false;
        if (sym < 16) {
          lens[idx++] = (uint8_t)sym;
          continue;
        }
        uint8_t v = 0;
        int rep;
        if (sym == 16) {
          if (idx == 0) return false;
          v = lens[idx - 1];
          rep = 3 + (int)b.get(2);
        } else if (sym == 17) {
          rep = 3 + (int)b.get(3);
        } else {
          rep = 11 + (int)b.get(7);
        }
        if (b.bad || idx + rep > nlen + ndist) return false;
        while (rep--) lens[idx++] = v;
      }
      if (lens[256] == 0) return false;  // no end-of-block code
      if (!huff_build(lc, lens, nlen) || !huff_build(dc, lens + nlen, ndist)) return false;
      if (!inflate_codes(b, o, lc, dc, win0)) return false;
    } else {
      return false;
    }
    if (last) return true;
  }
}
__device__ bool gzip_dev(const uint8_t* s, uint64_t n, DecOut& o) {
  if (n < 18 || s[0] != 0x1f || s[1] != 0x8b || s[2] != 8) return false;
  const uint8_t flg = s[3];
  if (flg & 0xE0) return false;  // reserved flag bits
  uint64_t i = 10;
  if (flg & 4) {  // FEXTRA
    if (n - i < 2) return false;
    const uint32_t xl = s[i] | (s[i + 1] << 8);
    if (xl > n - i - 2) return false;
    i += 2 + xl;
  }
  for (int f = 8; f <= 16; f <<= 1)
    if (flg & f) {  // FNAME, FCOMMENT: NUL-terminated
      while (i < n && s[i]) i++;
      if (i >= n) return false;
      i++;
    }
  if (flg & 2) {  // FHCRC: low 16 bits of the header's CRC-32
    if (n - i < 2) return false;
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t k = 0; k < i; k++) c = g_crc32_ieee.t[(c ^ s[k]) & 0xff] ^ (c >> 8);
    if (((c ^ 0xFFFFFFFFu) & 0xFFFFu) != (uint32_t)(s[i] | (s[i + 1] << 8))) return false;
    i += 2;
  }
  Bits b{s, n, i, 0, 0, false};
  const uint64_t o0 = o.n;
  if (!inflate_dev(b, o)) return false;
  b.align();
  if (b.n - b.i < 8) return false;  // trailer after the byte-aligned end (unused bits dropped)
  const uint32_t crc = dec_le32(b.s + b.i), isize = dec_le32(b.s + b.i + 4);
  if ((uint32_t)(o.n - o0) != isize) return false;
  if (o.write) {
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t k = o0; k < o.n; k++) c = g_crc32_ieee.t[(c ^ o.p[k]) & 0xff] ^ (c >> 8);
    if ((c ^ 0xFFFFFFFFu) != crc) return false;
  }
  return true;  // bytes after the member are ignored
}

}  // namespace fsg
#include "fsg_zstd_dev.h"
namespace fsg {

// Compression::uncompress of one record section: the output length or DEC_BAD
// (io::Error "uncompress error")
__device__ int64_t dev_decompress(uint32_t codec, const uint8_t* s, uint64_t n, DecOut& o,
                                  const uint32_t* crc32c_tab) {
  bool ok;
  switch (codec) {
    case 1: ok = gzip_dev(s, n, o); break;
    case 2: ok = snappy_frames_dev(s, n, o, crc32c_tab); break;
    case 3: ok = lz4_frames_dev(s, n, o); break;
    case 4: ok = zstd::zstd_frames_dev(s, n, o); break;
    default: return DEC_BAD;
  }
  return ok ? (int64_t)o.n : DEC_BAD;
}

}  // namespace fsg
