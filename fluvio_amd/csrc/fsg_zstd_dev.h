// fsg_zstd_dev.h — zstd frames (RFC 8878) decoded on the GPU, one thread per
// stored batch, inside the sizing / writing passes of fsg_codec_dev.h.
//
// Fluvio's Compression::Zstd (crates/fluvio-compression/src/zstd.rs:15-20)
// reads the record section with the zstd crate's streaming Decoder
// (zstd 0.13 / libzstd, third-party, absent from the reference tree): any
// number of zstd frames and skippable frames until the input ends, no
// dictionary; the input ending inside a frame is an error.  Restated from
// the format specification:
//   frame header (descriptor, window, dictionary id, content size), raw /
//   RLE / compressed blocks, literals (raw, RLE, Huffman with 1 or 4 streams,
//   treeless), sequences (predefined / RLE / FSE / repeat tables for literal
//   length, offset and match length codes, repeat offsets), optional XXH64
//   content checksum.
// Decoded literals of a Huffman block are staged at the end of the batch's
// output region (the writing pass knows its exact size from the sizing pass):
// every literal is read before the output reaches its slot.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fsg {
namespace zstd {

__device__ __forceinline__ int hbit32(uint32_t x) { return 31 - __builtin_clz(x); }  // x > 0

// forward bit reader (FSE table descriptions): LSB first within each byte
struct FBits {
  const uint8_t* s;
  uint64_t n;    // bytes available
  uint64_t pos;  // bit position
  bool bad;
  __device__ uint32_t read(int k) {
    if (k == 0) return 0;
    if (pos + (uint64_t)k > 8 * n) {
      bad = true;
      return 0;
    }
    uint32_t v = 0;
    for (int i = 0; i < k; i++, pos++) v |= (uint32_t)((s[pos >> 3] >> (pos & 7)) & 1u) << i;
    return v;
  }
};

// backward bit reader (Huffman / FSE streams): the stream ends with a 1 bit
// marking its last byte's padding; bits are read from the marker down, bits
// below the start read as zeros (off < 0)
struct RBits {
  const uint8_t* s;
  uint64_t n;
  int64_t off;  // data bits left above position 0
  __device__ bool init(const uint8_t* p, uint64_t len) {
    s = p;
    n = len;
    if (!len || !p[len - 1]) return false;
    off = 8 * (int64_t)(len - 1) + hbit32(p[len - 1]);
    return true;
  }
  __device__ uint64_t read(int k) {  // k <= 56
    if (k == 0) return 0;
    off -= k;
    const int64_t start = off;
    if (start + k <= 0) return 0;
    const int64_t lo = start < 0 ? 0 : start;
    const int drop = (int)(lo - start);
    const uint64_t byte = (uint64_t)lo >> 3;
    uint64_t w = 0;
    for (int i = 0; i < 8 && byte + i < n; i++) w |= (uint64_t)s[byte + i] << (8 * i);
    const int need = k - drop;
    const uint64_t v = (w >> (lo & 7)) & ((need >= 64) ? ~0ull : ((1ull << need) - 1ull));
    return v << drop;
  }
};

// ---- FSE
constexpr int kFseMax = 512;
struct Fse {
  uint8_t sym[kFseMax];
  uint8_t nb[kFseMax];
  uint16_t base[kFseMax];
  int al;  // accuracy log
};
// decoding table from normalized counts (-1 = "less than one")
__device__ bool fse_build(Fse& t, const int16_t* cnt, int nsym, int al) {
  const int size = 1 << al;
  uint16_t next[256];
  int high = size;
  for (int s = 0; s < nsym; s++)
    if (cnt[s] == -1) {
      t.sym[--high] = (uint8_t)s;
      next[s] = 1;
    }
  const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  int pos = 0;
  for (int s = 0; s < nsym; s++) {
    if (cnt[s] <= 0) continue;
    next[s] = (uint16_t)cnt[s];
    for (int i = 0; i < cnt[s]; i++) {
      t.sym[pos] = (uint8_t)s;
      do {
        pos = (pos + step) & mask;
      } while (pos >= high);
    }
  }
  if (pos != 0) return false;
  for (int i = 0; i < size; i++) {
    const uint16_t d = next[t.sym[i]]++;
    t.nb[i] = (uint8_t)(al - hbit32(d));
    t.base[i] = (uint16_t)(((uint32_t)d << t.nb[i]) - (uint32_t)size);
  }
  t.al = al;
  return true;
}
__device__ void fse_rle(Fse& t, uint8_t sym) {
  t.sym[0] = sym;
  t.nb[0] = 0;
  t.base[0] = 0;
  t.al = 0;
}
// a table description (forward bits); *used = its bytes
__device__ bool fse_read(Fse& t, const uint8_t* s, uint64_t n, int max_al, int max_sym, uint64_t* used) {
  FBits b{s, n, 0, false};
  const int al = 5 + (int)b.read(4);
  if (b.bad || al > max_al) return false;
  int16_t cnt[256];
  int remaining = 1 << al, sym = 0;
  while (remaining > 0 && sym <= max_sym) {
    const int bits = hbit32((uint32_t)remaining + 1) + 1;
    uint32_t v = b.read(bits);
    const uint32_t lower = (1u << (bits - 1)) - 1u;
    const uint32_t thr = (1u << bits) - 1u - ((uint32_t)remaining + 1u);
    if ((v & lower) < thr) {
      b.pos -= 1;  // the small range takes one bit less
      v &= lower;
    } else if (v > lower) {
      v -= thr;
    }
    const int p = (int)v - 1;
    remaining -= p < 0 ? -p : p;
    cnt[sym++] = (int16_t)p;
    if (p == 0) {
      for (;;) {
        const int rep = (int)b.read(2);
        for (int i = 0; i < rep && sym <= max_sym; i++) cnt[sym++] = 0;
        if (rep != 3) break;
      }
    }
    if (b.bad) return false;
  }
  if (remaining != 0 || sym > max_sym + 1 || b.bad) return false;
  *used = (b.pos + 7) >> 3;
  return fse_build(t, cnt, sym, al);
}

// ---- Huffman (literals)
constexpr int kHufMaxBits = 11;
struct Huf {
  uint8_t sym[1 << kHufMaxBits];
  uint8_t nb[1 << kHufMaxBits];
  int maxbits;
  bool valid;
};
// tree description -> table; *used = its bytes
__device__ bool huf_read(Huf& h, Fse& ft, const uint8_t* s, uint64_t n, uint64_t* used) {
  if (n < 1) return false;
  uint8_t w[256];
  int nw = 0;
  const uint32_t hb = s[0];
  if (hb < 128) {  // FSE-compressed weights: hb bytes
    if (hb == 0 || 1 + (uint64_t)hb > n) return false;
    uint64_t tu = 0;
    if (!fse_read(ft, s + 1, hb, 6, 255, &tu) || tu >= hb) return false;
    RBits b;
    if (!b.init(s + 1 + tu, hb - tu)) return false;
    uint32_t s1 = (uint32_t)b.read(ft.al), s2 = (uint32_t)b.read(ft.al);
    for (;;) {
      if (nw >= 255) return false;
      w[nw++] = ft.sym[s1];
      s1 = ft.base[s1] + (uint32_t)b.read(ft.nb[s1]);
      if (b.off < 0) {
        if (nw >= 255) return false;
        w[nw++] = ft.sym[s2];
        break;
      }
      if (nw >= 255) return false;
      w[nw++] = ft.sym[s2];
      s2 = ft.base[s2] + (uint32_t)b.read(ft.nb[s2]);
      if (b.off < 0) {
        if (nw >= 255) return false;
        w[nw++] = ft.sym[s1];
        break;
      }
    }
    *used = 1 + hb;
  } else {  // direct: hb - 127 weights of 4 bits
    nw = (int)hb - 127;
    const uint64_t nb = ((uint64_t)nw + 1) / 2;
    if (1 + nb > n) return false;
    for (int i = 0; i < nw; i++) w[i] = (uint8_t)((i & 1) ? (s[1 + i / 2] & 15) : (s[1 + i / 2] >> 4));
    *used = 1 + nb;
  }
  // the last symbol's weight completes a power of two
  uint32_t tot = 0;
  for (int i = 0; i < nw; i++) {
    if (w[i] > kHufMaxBits) return false;
    if (w[i]) tot += 1u << (w[i] - 1);
  }
  if (tot == 0) return false;
  const int maxbits = hbit32(tot) + 1;
  if (maxbits > kHufMaxBits) return false;
  const uint32_t rest = (1u << maxbits) - tot;
  if (rest & (rest - 1)) return false;
  if (nw >= 256) return false;
  w[nw++] = (uint8_t)(hbit32(rest) + 1);
  // table: longest codes first (rank by bits), symbols in order within a rank
  uint8_t bits[256];
  int rank[kHufMaxBits + 2] = {0};
  for (int i = 0; i < nw; i++) {
    bits[i] = w[i] ? (uint8_t)(maxbits + 1 - w[i]) : 0;
    rank[bits[i]]++;
  }
  int start[kHufMaxBits + 2];
  start[maxbits] = 0;
  for (int b2 = maxbits; b2 >= 1; b2--) start[b2 - 1] = start[b2] + rank[b2] * (1 << (maxbits - b2));
  if (start[0] != (1 << maxbits)) return false;
  for (int i = 0; i < nw; i++) {
    if (!bits[i]) continue;
    const int len = 1 << (maxbits - bits[i]);
    for (int k = 0; k < len; k++) {
      h.sym[start[bits[i]] + k] = (uint8_t)i;
      h.nb[start[bits[i]] + k] = bits[i];
    }
    start[bits[i]] += len;
  }
  h.maxbits = maxbits;
  h.valid = true;
  return true;
}
// one stream of `cnt` symbols; out == nullptr: validate only
__device__ bool huf_stream(const Huf& h, const uint8_t* s, uint64_t n, uint8_t* out, uint64_t cnt) {
  RBits b;
  if (!b.init(s, n)) return false;
  const uint32_t mask = (1u << h.maxbits) - 1u;
  uint32_t st = (uint32_t)b.read(h.maxbits);
  for (uint64_t i = 0; i < cnt; i++) {
    const uint8_t nbits = h.nb[st];
    if (out) out[i] = h.sym[st];
    st = ((st << nbits) + (uint32_t)b.read(nbits)) & mask;
  }
  return b.off == -(int64_t)h.maxbits;  // every bit of the stream consumed
}

// ---- sequences
__device__ __forceinline__ void ll_code(uint32_t c, uint32_t& base, int& nb) {
  const uint32_t lb[20] = {16, 18, 20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
  const uint8_t lx[20] = {1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  if (c < 16) {
    base = c;
    nb = 0;
  } else {
    base = lb[c - 16];
    nb = lx[c - 16];
  }
}
__device__ __forceinline__ void ml_code(uint32_t c, uint32_t& base, int& nb) {
  const uint32_t mb[21] = {35, 37, 39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
  const uint8_t mx[21] = {1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
  if (c < 32) {
    base = c + 3;
    nb = 0;
  } else {
    base = mb[c - 32];
    nb = mx[c - 32];
  }
}
// predefined distributions (RFC 8878 3.1.1.3.2.2)
__device__ void fse_predef(Fse& t, int which) {
  const int16_t ll[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
                          -1, -1, -1, -1};
  const int16_t ml[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                          1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
  const int16_t of[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
  if (which == 0)
    fse_build(t, ll, 36, 6);
  else if (which == 1)
    fse_build(t, of, 29, 5);
  else
    fse_build(t, ml, 53, 6);
}

struct FrameState {
  Huf huf;             // the previous Huffman table (treeless literals)
  Fse tab[3];          // LL, OF, ML (repeat mode)
  bool tab_ok[3];
  Fse scratch;         // Huffman weight decoding
  uint32_t rep[3];
};

// one compressed block of `bs` bytes; frame output starts at f0
__device__ bool zstd_block(FrameState& F, const uint8_t* s, uint64_t bs, DecOut& o, uint64_t f0) {
  if (bs < 1) return false;
  // ---- literals section
  const uint32_t b0 = s[0];
  const uint32_t ltype = b0 & 3, sf = (b0 >> 2) & 3;
  uint64_t lsize = 0, csize = 0, hdr = 0;
  int nstreams = 1;
  if (ltype < 2) {
    if ((sf & 1) == 0) {
      lsize = b0 >> 3;
      hdr = 1;
    } else if (sf == 1) {
      if (bs < 2) return false;
      lsize = (b0 >> 4) | ((uint32_t)s[1] << 4);
      hdr = 2;
    } else {
      if (bs < 3) return false;
      lsize = (b0 >> 4) | ((uint32_t)s[1] << 4) | ((uint32_t)s[2] << 12);
      hdr = 3;
    }
  } else {
    const uint64_t hl = sf < 2 ? 3 : sf == 2 ? 4 : 5;
    if (bs < hl) return false;
    uint64_t h = 0;
    for (uint64_t i = 0; i < hl; i++) h |= (uint64_t)s[i] << (8 * i);
    const int w = sf < 2 ? 10 : sf == 2 ? 14 : 18;
    lsize = (h >> 4) & ((1ull << w) - 1);
    csize = (h >> (4 + w)) & ((1ull << w) - 1);
    nstreams = sf == 0 ? 1 : 4;
    hdr = hl;
  }
  if (lsize > 131072) return false;
  const uint8_t* lit = nullptr;  // raw literals: in the source
  uint8_t rle = 0;
  uint64_t p = hdr;
  if (ltype == 0) {
    if (p + lsize > bs) return false;
    lit = s + p;
    p += lsize;
  } else if (ltype == 1) {
    if (p + 1 > bs) return false;
    rle = s[p];
    p += 1;
  } else {
    if (p + csize > bs) return false;
    const uint8_t* c = s + p;
    uint64_t cn = csize, tu = 0;
    if (ltype == 2) {
      if (!huf_read(F.huf, F.scratch, c, cn, &tu)) return false;
      c += tu;
      cn -= tu;
    } else if (!F.huf.valid) {
      return false;  // treeless without a previous table
    }
    if (nstreams == 4 && lsize < 6) return false;
    // stage the literals at the end of the batch's output (writing pass)
    uint8_t* dst = o.write ? o.p + o.cap - lsize : nullptr;
    if (o.write && o.cap < lsize) return false;
    if (nstreams == 1) {
      if (!huf_stream(F.huf, c, cn, dst, lsize)) return false;
    } else {
      if (cn < 6) return false;
      const uint64_t z1 = c[0] | (c[1] << 8), z2 = c[2] | (c[3] << 8), z3 = c[4] | (c[5] << 8);
      if (6 + z1 + z2 + z3 > cn) return false;
      const uint64_t z4 = cn - 6 - z1 - z2 - z3;
      const uint64_t q = (lsize + 3) / 4;
      if (3 * q > lsize) return false;
      const uint8_t* sp = c + 6;
      const uint64_t zs[4] = {z1, z2, z3, z4};
      for (int k = 0; k < 4; k++) {
        const uint64_t cnt = k < 3 ? q : lsize - 3 * q;
        if (!huf_stream(F.huf, sp, zs[k], dst ? dst + k * q : nullptr, cnt)) return false;
        sp += zs[k];
      }
    }
    lit = dst;
    p += csize;
  }
  // ---- sequences section
  if (p >= bs) return false;
  uint64_t nseq = s[p];
  if (nseq == 0) {
    p += 1;
  } else if (nseq < 128) {
    p += 1;
  } else if (nseq < 255) {
    if (p + 2 > bs) return false;
    nseq = ((nseq - 128) << 8) + s[p + 1];
    p += 2;
  } else {
    if (p + 3 > bs) return false;
    nseq = s[p + 1] + ((uint64_t)s[p + 2] << 8) + 0x7F00;
    p += 3;
  }
  uint64_t lused = 0;  // literals consumed
  auto put_lits = [&](uint64_t k) -> bool {
    if (lused + k > lsize) return false;
    if (o.write) {
      if (o.n + k > o.cap) return false;
      for (uint64_t i = 0; i < k; i++) o.p[o.n + i] = ltype == 1 ? rle : lit[lused + i];
    }
    o.n += k;
    lused += k;
    return true;
  };
  if (nseq == 0) {
    if (p != bs) return false;
    return put_lits(lsize);
  }
  if (p >= bs) return false;
  const uint32_t modes = s[p++];
  if (modes & 3) return false;  // reserved bits
  const int maxal[3] = {9, 8, 9}, maxsym[3] = {35, 31, 52};
  for (int k = 0; k < 3; k++) {
    const uint32_t m = (modes >> (6 - 2 * k)) & 3;
    if (m == 0) {
      fse_predef(F.tab[k], k);
    } else if (m == 1) {
      if (p >= bs || s[p] > (uint32_t)maxsym[k]) return false;
      fse_rle(F.tab[k], s[p]);
      p += 1;
    } else if (m == 2) {
      uint64_t u = 0;
      if (!fse_read(F.tab[k], s + p, bs - p, maxal[k], maxsym[k], &u)) return false;
      p += u;
    } else if (!F.tab_ok[k]) {
      return false;  // repeat without a previous table
    }
    F.tab_ok[k] = true;
  }
  if (p >= bs) return false;
  RBits b;
  if (!b.init(s + p, bs - p)) return false;
  const Fse &TL = F.tab[0], &TO = F.tab[1], &TM = F.tab[2];
  uint32_t sl = (uint32_t)b.read(TL.al), so = (uint32_t)b.read(TO.al), sm = (uint32_t)b.read(TM.al);
  for (uint64_t i = 0; i < nseq; i++) {
    const uint32_t oc = TO.sym[so], mc = TM.sym[sm], lc = TL.sym[sl];
    if (oc > 31) return false;
    uint32_t mb, lb;
    int mnb, lnb;
    ml_code(mc, mb, mnb);
    ll_code(lc, lb, lnb);
    const uint64_t ofv = (1ull << oc) + b.read((int)oc);
    const uint64_t ml = mb + b.read(mnb);
    const uint64_t ll = lb + b.read(lnb);
    uint64_t off;
    if (ofv > 3) {
      off = ofv - 3;
      F.rep[2] = F.rep[1];
      F.rep[1] = F.rep[0];
      F.rep[0] = (uint32_t)off;
    } else {
      const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0 ? 1u : 0u);
      if (idx == 0) {
        off = F.rep[0];
      } else {
        off = idx < 3 ? F.rep[idx] : (uint64_t)F.rep[0] - 1;
        if (idx > 1) F.rep[2] = F.rep[1];
        F.rep[1] = F.rep[0];
        F.rep[0] = (uint32_t)off;
      }
    }
    if (i + 1 < nseq) {  // state updates: literal length, match length, offset
      sl = TL.base[sl] + (uint32_t)b.read(TL.nb[sl]);
      sm = TM.base[sm] + (uint32_t)b.read(TM.nb[sm]);
      so = TO.base[so] + (uint32_t)b.read(TO.nb[so]);
    }
    if (!put_lits(ll)) return false;
    if (off == 0 || off > o.n - f0) return false;
    if (!o.copy(off, ml, f0)) return false;
  }
  if (b.off != 0) return false;  // the sequence bitstream fully consumed
  return put_lits(lsize - lused);
}

__device__ uint64_t xxh64(const uint8_t* p, uint64_t n) {  // seed 0
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                 P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto rd64 = [](const uint8_t* q) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)q[i] << (8 * i);
    return v;
  };
  auto round = [&](uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; };
  auto merge = [&](uint64_t acc, uint64_t v) { return (acc ^ round(0, v)) * P1 + P4; };
  uint64_t h, i = 0;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; i + 32 <= n; i += 32) {
      v1 = round(v1, rd64(p + i));
      v2 = round(v2, rd64(p + i + 8));
      v3 = round(v3, rd64(p + i + 16));
      v4 = round(v4, rd64(p + i + 24));
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h = merge(h, v1);
    h = merge(h, v2);
    h = merge(h, v3);
    h = merge(h, v4);
  } else {
    h = P5;
  }
  h += n;
  for (; i + 8 <= n; i += 8) h = rotl(h ^ round(0, rd64(p + i)), 27) * P1 + P4;
  if (i + 4 <= n) {
    const uint64_t w = (uint64_t)p[i] | ((uint64_t)p[i + 1] << 8) | ((uint64_t)p[i + 2] << 16) | ((uint64_t)p[i + 3] << 24);
    h = rotl(h ^ (w * P1), 23) * P2 + P3;
    i += 4;
  }
  for (; i < n; i++) h = rotl(h ^ (p[i] * P5), 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// frames until the input ends (zstd::stream::read::Decoder::read_to_end)
__device__ bool zstd_frames_dev(const uint8_t* s, uint64_t n, DecOut& o) {
  if (n == 0) return false;  // zio::Reader: an empty input is an incomplete frame
  FrameState F;
  uint64_t i = 0;
  while (i < n) {
    if (n - i < 4) return false;
    const uint32_t magic = (uint32_t)s[i] | ((uint32_t)s[i + 1] << 8) | ((uint32_t)s[i + 2] << 16) |
                           ((uint32_t)s[i + 3] << 24);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (n - i < 8) return false;
      const uint64_t len = (uint64_t)s[i + 4] | ((uint64_t)s[i + 5] << 8) | ((uint64_t)s[i + 6] << 16) |
                           ((uint64_t)s[i + 7] << 24);
      if (n - i - 8 < len) return false;
      i += 8 + len;
      continue;
    }
    if (magic != 0xFD2FB528u) return false;
    i += 4;
    if (i >= n) return false;
    const uint32_t fd = s[i++];
    const uint32_t fcs_flag = fd >> 6, single = (fd >> 5) & 1, csum = (fd >> 2) & 1, did_flag = fd & 3;
    if (fd & 8) return false;  // reserved bit
    uint64_t window = 0;
    if (!single) {
      if (i >= n) return false;
      const uint32_t wd = s[i++];
      const uint32_t e = wd >> 3, m = wd & 7;
      const uint64_t base = 1ull << (10 + e);
      window = base + (base / 8) * m;
    }
    const int did_len = did_flag == 0 ? 0 : did_flag == 1 ? 1 : did_flag == 2 ? 2 : 4;
    if (n - i < (uint64_t)did_len) return false;
    uint64_t did = 0;
    for (int k = 0; k < did_len; k++) did |= (uint64_t)s[i + k] << (8 * k);
    i += did_len;
    if (did != 0) return false;  // a dictionary the decoder does not have
    const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (n - i < (uint64_t)fcs_len) return false;
    uint64_t fcs = 0;
    for (int k = 0; k < fcs_len; k++) fcs |= (uint64_t)s[i + k] << (8 * k);
    if (fcs_len == 2) fcs += 256;
    i += fcs_len;
    if (single) window = fcs;
    const uint64_t f0 = o.n;
    F.huf.valid = false;
    F.tab_ok[0] = F.tab_ok[1] = F.tab_ok[2] = false;
    F.rep[0] = 1;
    F.rep[1] = 4;
    F.rep[2] = 8;
    const uint64_t bmax = window < 131072 ? window : 131072;
    for (;;) {
      if (n - i < 3) return false;
      const uint32_t bh = (uint32_t)s[i] | ((uint32_t)s[i + 1] << 8) | ((uint32_t)s[i + 2] << 16);
      i += 3;
      const bool last = bh & 1;
      const uint32_t bt = (bh >> 1) & 3;
      const uint64_t bs = bh >> 3;
      if (bt == 3) return false;
      if (bt == 1) {  // RLE: one byte, bs times
        if (i >= n || bs > bmax) return false;
        const uint8_t v = s[i++];
        if (o.write && o.n + bs > o.cap) return false;
        if (o.write)
          for (uint64_t k = 0; k < bs; k++) o.p[o.n + k] = v;
        o.n += bs;
      } else {
        if (n - i < bs || bs > bmax) return false;
        if (bt == 0) {
          if (!o.put_span(s + i, bs)) return false;
        } else if (!zstd_block(F, s + i, bs, o, f0)) {
          return false;
        }
        i += bs;
      }
      if (last) break;
    }
    if (fcs_flag || single) {
      if (o.n - f0 != fcs) return false;
    }
    if (csum) {
      if (n - i < 4) return false;
      if (o.write) {
        const uint32_t want = (uint32_t)s[i] | ((uint32_t)s[i + 1] << 8) | ((uint32_t)s[i + 2] << 16) |
                              ((uint32_t)s[i + 3] << 24);
        if ((uint32_t)xxh64(o.p + f0, o.n - f0) != want) return false;
      }
      i += 4;
    }
  }
  return true;
}

}  // namespace zstd
}  // namespace fsg
