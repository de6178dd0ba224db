// fsg_lean.hip — the lean evaluation kernel of the substring / bounded-regex /
// filter_json / projection filters (the C1-C3 hot path) and the record framing
// kernels that feed it (k_chase, k_chase_w).  Batches it cannot decide exactly
// go to k_eval (fsg_kernels.hip) through the deferred list.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <type_traits>

#include "fsg_device.h"
#include "fsg_dev_util.h"
#include "fsg_json_dfa.h"
#include "fsg_launch.h"

namespace fsg {
// ---------------------------------------------------------------------------
// k_eval_lean — persistent workgroups of two waves for chains of substring /
// bounded-regex / filter_json filters and ASCII-uppercase maps (filter /
// filter_init / filter_with_param / regex-filter / filter_json / map), the
// C1/C2 hot path.  Each workgroup walks the batches b = blockIdx.x + i * grid;
// while batch i is evaluated, batch i + 1 is already streaming into a second
// LDS window (LDS-DMA), so HBM latency hides behind the evaluation.  A batch
// takes this path only when its records can neither error nor decode
// unusually: record section inside the 16 KiB window, 1..64 records that frame
// exactly, every value ASCII (then from_utf8 cannot fail, filter.rs / derive
// filter.rs:14-40).  Any other batch is appended to a.list and evaluated
// exactly by k_eval (list mode).
//   1. LDS-DMA the batch (header + record section) into the prefetch window,
//      copied to the evaluation window when its turn comes
//   2. lane 0 chases the record length varints; lane r parses record r exactly
//      (Record::decode, data.rs:534-562) and checks it ends where its length says
//   3. per contains stage, a data-parallel 4-gram scan over the value bytes
//      (16 B + 4 B look-ahead per lane, ballot-filtered); 4-gram hits are parked
//      in registers and resolved after the scan (record lookup + full needle);
//      before the first scan the bytes between values are cleared, so the OR
//      of every scanned word has a high bit iff some value is non-ASCII
//   4. survivors -> compaction descriptors (ballot prefix), BatchStat
// ---------------------------------------------------------------------------
constexpr int kLeanWin = 16464;  // 57-B header + 16 KiB section + 15 B alignment, 16-B multiple
constexpr int kLeanMaxR = 64;    // one record per lane of wave 0
constexpr int kLeanThreads = 128;  // two waves per batch: DMA issue and the scan are split over both
constexpr int kLeanNeedle = 128; // longest needle of the lean path (longer: exact kernel)
constexpr int kLeanBlk = (kLeanWin + 80) / 64 + 1;  // 64-byte blocks of the window
constexpr int kLeanNeedles = 256;  // resident needle bytes of all contains stages
// a stage as the lean kernel needs it, copied to LDS once per workgroup (no
// global reads while a prefetch is in flight)
struct LeanStage {
  uint8_t op;
  uint8_t upper;       // in_type == VT_SRC_UPPER
  uint8_t keep_match;
  uint8_t pad;
  uint32_t m;          // needle_len
  uint32_t max_len, s_bot, s_mid, acc1, acc2;
  uint32_t tt;         // blob offset of the regex rows (tt or tt_up by the input case)
  uint32_t nd;         // blob offset of the needle
  uint32_t nd_off;     // its offset in LeanLds::needles (when resident)
};
struct __attribute__((aligned(16))) LeanLds {
  uint8_t win[kLeanWin + 48];  // + look-ahead of the last scan chunk
  uint32_t r_vs[kLeanMaxR];
  uint32_t r_ve[kLeanMaxR];
  uint32_t match[2];
  uint32_t nst;
  uint32_t red[4];                  // workgroup OR (two alternating pairs)
  uint32_t out_upper;
  uint32_t tt_stage;                // stage whose rows sit in tt for the whole launch (0xFF: reloaded)
  uint32_t nd_res;                  // 1: every needle sits in needles (LeanStage::nd_off)
  uint32_t ghigh;                   // bytes >= 0x80 between values (record headers / trailers), from framing
  uint32_t hcw[2];                  // per wave: bytes >= 0x80 the first scan saw over [first value, last value end)
  LeanStage stg[kMaxStages];
  uint64_t tt[256];                 // the scanned regex stage's byte rows (DfaDesc::tt)
  uint8_t needle[kLeanNeedle + 8];  // the scanned stage's needle
  uint8_t needles[kLeanNeedles];    // the contains stages' needles, back to back (when they fit)
  alignas(4) uint8_t blk[kLeanBlk + 4];  // blk[j] = last record whose value starts <= 64 j (0xFF none)
};
// workgroup OR of p over the two waves; `par` alternates the LDS pair so one
// barrier suffices (a pair is rewritten two calls later, after a barrier that
// every reader of it has passed)
__device__ __forceinline__ bool lean_or(uint32_t* red, uint32_t& par, bool p) {
  const uint64_t bl = __ballot(p);
  uint32_t* r = red + 2 * par;
  if ((threadIdx.x & 63u) == 0) r[threadIdx.x >> 6] = bl != 0 ? 1u : 0u;
  lean_sync();
  par ^= 1u;
  return (r[0] | r[1]) != 0u;
}
// the filter_json variant: per-chunk quote / in-string masks, the token list,
// the token DFA (fsg_json_dfa.h)
// LDS of the JSON variant is sized for 5 workgroups per CU (<= 32 KiB): the
// per-chunk words cover 16 KiB of values (a batch whose values span more takes
// the exact kernel), the token list 1024 entries (a 16 KiB batch of ~1 KB log
// records has ~600), and jn lives in the regex rows' space (LeanLds::tt; a
// chain with regex and JSON stages reloads its rows per batch)
constexpr int kJsonChunks = 1024;
constexpr int kJsonEnt = 1024;  // token entries per batch (more: exact kernel)
constexpr int kJsonSeg = kJsonChunks;  // object members per batch (LeanLdsJ::jn; more: exact kernel)
__device__ constexpr JsonDfaTables g_json_tables{};
static_assert(sizeof(LeanLds::tt) >= 2 * kJsonChunks, "jn overlays the regex rows");
struct __attribute__((aligned(16))) LeanLdsJ : LeanLds {
  uint32_t jm[kJsonChunks];      // pass 1: quote16 | special16 << 16; pass 2: in-string16 | hot16 << 16
  // jn: non-space16 per chunk; then the object members: first token | record start << 15
  __device__ __forceinline__ uint16_t* jn() { return reinterpret_cast<uint16_t*>(tt); }
  uint32_t ent[kJsonEnt];        // pos | in-string bit << 15 | byte << 16 | token class << 24
  uint32_t racc[kLeanMaxR];      // per record: level fields | message fields << 8 | bad << 16
  uint32_t rlvl[kLeanMaxR];      // per record: bit (LogLevel index) of its level value
  unsigned long long rbest[kLeanMaxR];  // projection: (member + 1) << 32 | value span of the last matching member
  uint32_t nseg;
  uint32_t wsum[4];              // cross-wave scan carries
  uint8_t dfa[kJsonStates * kJsonCls2];
  uint8_t bcls[256];
};

__device__ __forceinline__ uint32_t win5(const uint32_t (&w)[5], int j) {
  const int k = j >> 2, al = j & 3;
  return al ? __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)al) : w[k];
}
// 4 window bytes starting at any offset q (two aligned LDS dwords)
__device__ __forceinline__ uint32_t lds_u32_at(const uint8_t* win, uint32_t q) {
  const uint32_t* w = (const uint32_t*)(win + (q & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], q & 3u);
}
// record whose value region holds window offset p: the last r with r_vs[r] <= p
// (-1: none), by the 64-byte block table (lean_blk / clear_gaps built it)
__device__ __forceinline__ int lean_rec_of(const LeanLds& L, int nr, uint32_t p) {
  int r = (int)(int8_t)L.blk[p >> 6];
  while (r + 1 < nr && L.r_vs[r + 1] <= p) r++;
  return r;
}
// ... by binary search over the value starts (no table: for rare lookups)
__device__ __forceinline__ int lean_rec_bs(const LeanLds& L, int nr, uint32_t p) {
  int lo = 0, hi = nr;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (L.r_vs[m] <= p) lo = m + 1; else hi = m;
  }
  return lo - 1;
}
// m needle bytes at window offset p (4 bytes per compare)
__device__ __forceinline__ bool lean_verify(const LeanLds& L, uint32_t p, uint32_t m, bool upper) {
  for (uint32_t t = 0; t < m; t += 4) {
    uint32_t x = lds_u32_at(L.win, p + t);
    if (upper) x = swar_upper(x);
    const uint32_t k = m - t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (m - t))) - 1u);
    if ((x ^ lds_u32_at(L.needle, t)) & k) return false;
  }
  return true;
}
// a 4-gram hit at window offset p: the whole needle inside one value -> record bit
__device__ __forceinline__ void lean_resolve(const LeanLds& L, int nr, uint32_t p, uint32_t m, bool upper,
                                             uint64_t& mask) {
  const int r = lean_rec_bs(L, nr, p);
  if (r < 0 || p < L.r_vs[r] || p + m > L.r_ve[r]) return;
  if (lean_verify(L, p, m, upper)) mask |= 1ull << r;
}
__device__ __forceinline__ void lean_push(const LeanLds& L, int nr, uint32_t p, uint32_t m, bool upper,
                                          uint32_t& s0, uint32_t& s1, uint32_t& nh, uint64_t& mask) {
  if (nh == 0) s0 = p;
  else if (nh == 1) s0 |= p << 16;
  else if (nh == 2) s1 = p;
  else if (nh == 3) s1 |= p << 16;
  else lean_resolve(L, nr, p, m, upper, mask);  // more than 4 hits in one lane: resolve now
  nh++;
}
// One contains stage over the value bytes [lo, hi) of a window whose non-value
// bytes in [lo & ~15, hi + 16) are blanks (clear_gaps).  Returns the OR of the scanned words
// (bit 7 of a byte set <=> some value byte >= 0x80, i.e. a non-ASCII value).
//   kMode 0 (m >= 7): every occurrence covers an aligned word, so each aligned
//           word is compared with the needle's 4-grams at offsets 0..3 (one
//           compare per byte, no byte shifting)
//   kMode 1 (4 <= m <= 6): the 4-gram at each of the 16 positions (alignbyte)
//   kMode 2 (1 <= m <= 3): masked compare of the first m bytes at each position
//   kMode 3 (m == 0): OR only
// kCount (gaps not cleared): instead of the OR, the count of bytes >= 0x80 in
// the scanned words, the first and last chunk masked to [lo, hi); the caller
// compares it with the framing's count of such bytes between values
__device__ __forceinline__ uint32_t bytes_in(uint32_t base, uint32_t lo, uint32_t hi) {  // mask: lo <= base + k < hi
  const uint32_t s = lo > base ? (lo - base < 4u ? lo - base : 4u) : 0u;
  const uint32_t e = hi > base ? (hi - base < 4u ? hi - base : 4u) : 0u;
  if (e <= s) return 0u;
  return (e == 4u ? 0xFFFFFFFFu : ((1u << (8 * e)) - 1u)) & ~((1u << (8 * s)) - 1u);
}
template <int kMode, bool kCount = false>
__device__ __forceinline__ uint32_t lean_scan(LeanLds& L, int nr, uint32_t lo, uint32_t hi, const uint8_t* nd,
                                              uint32_t m, bool upper) {
  const uint32_t l = threadIdx.x;
  uint32_t rot[4] = {0, 0, 0, 0};
  uint32_t k4 = 0xFFFFFFFFu;
  if (kMode == 0) {
    for (int d = 0; d < 4; d++)
      for (int t = 0; t < 4; t++) rot[d] |= (uint32_t)L.needle[d + t] << (8 * t);
  } else if (kMode != 3) {
    const uint32_t m4 = m < 4 ? m : 4;
    for (uint32_t t = 0; t < m4; t++) rot[0] |= (uint32_t)L.needle[t] << (8 * t);
    if (kMode == 2) k4 = (1u << (8 * m4)) - 1u;
  }
  uint32_t acc = 0, s0 = 0, s1 = 0, nh = 0;
  uint64_t mask = 0;  // records of this lane's verified hits
  uint32_t c = (lo & ~15u) + l * 16;
  uint4 nx = c < hi ? *(const uint4*)(&L.win[c]) : make_uint4(0, 0, 0, 0);
  uint32_t nx4 = (kMode == 1 || kMode == 2) && c < hi ? *(const uint32_t*)(&L.win[c + 16]) : 0u;
  constexpr uint32_t kStride = kLeanThreads * 16;
  for (; c < hi; c += kStride) {
    uint32_t wd[5] = {nx.x, nx.y, nx.z, nx.w, nx4};
    if (c + kStride < hi) {  // next chunk's LDS read in flight during this one
      nx = *(const uint4*)(&L.win[c + kStride]);
      if (kMode == 1 || kMode == 2) nx4 = *(const uint32_t*)(&L.win[c + kStride + 16]);
    }
    if (kCount) {
      if (c >= lo && c + 16 <= hi) {
#pragma unroll
        for (int k = 0; k < 4; k++) acc += (uint32_t)__builtin_popcount(wd[k] & 0x80808080u);
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
          acc += (uint32_t)__builtin_popcount(wd[k] & 0x80808080u & bytes_in(c + 4 * k, lo, hi));
      }
    } else {
      acc |= wd[0] | wd[1] | wd[2] | wd[3];
    }
    if (kMode == 3) continue;
    if (upper) {
#pragma unroll
      for (int k = 0; k < 5; k++) wd[k] = swar_upper(wd[k]);
    }
    // min over the compare differences: zero iff some 4-gram hits (vector ops
    // only; a ballot per compare would cost a scalar OR each)
    uint32_t z = 0xFFFFFFFFu;
    if (kMode == 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) z = min(z, min(min(wd[k] ^ rot[0], wd[k] ^ rot[1]), min(wd[k] ^ rot[2], wd[k] ^ rot[3])));
    } else {
#pragma unroll
      for (int j = 0; j < 16; j += 2) z = min(z, min((win5(wd, j) ^ rot[0]) & k4, (win5(wd, j + 1) ^ rot[0]) & k4));
    }
    const bool hl = z == 0u;
    if (!__ballot(hl)) continue;  // wave-uniform: no 4-gram hit in any lane
    if (!hl) continue;            // none in this lane
    if (kMode == 0) {
      // rare hits: parked, resolved after the scan for all lanes at once
#pragma unroll
      for (int k = 0; k < 4; k++)
#pragma unroll
        for (int d = 0; d < 4; d++)
          if (wd[k] == rot[d]) lean_push(L, nr, c + 4 * k - d, m, upper, s0, s1, nh, mask);
    } else {
      uint32_t cand = 0;
#pragma unroll
      for (int j = 0; j < 16; j++) cand |= (uint32_t)(((win5(wd, j) ^ rot[0]) & k4) == 0) << j;
      if (kMode == 1) {
        while (cand) {
          lean_push(L, nr, c + (uint32_t)__builtin_ctz(cand), m, upper, s0, s1, nh, mask);
          cand &= cand - 1;
        }
      } else {
        // m <= 3: the masked compare is the whole needle and hits are dense;
        // one record lookup per chunk, then register compares per hit
        uint32_t p = c + (uint32_t)__builtin_ctz(cand);
        int r = lean_rec_of(L, nr, p);
        uint32_t rvs = r >= 0 ? L.r_vs[r] : 0u, rve = r >= 0 ? L.r_ve[r] : 0u;
        uint32_t nvs = r + 1 < nr ? L.r_vs[r + 1] : 0xFFFFFFFFu;
        while (cand) {
          p = c + (uint32_t)__builtin_ctz(cand);
          cand &= cand - 1;
          while (p >= nvs) {
            r++;
            rvs = nvs;
            rve = L.r_ve[r];
            nvs = r + 1 < nr ? L.r_vs[r + 1] : 0xFFFFFFFFu;
          }
          if (r >= 0 && p >= rvs && p + m <= rve) mask |= 1ull << r;
        }
      }
    }
  }
  if (nh > 0) lean_resolve(L, nr, s0 & 0xFFFFu, m, upper, mask);
  if (nh > 1) lean_resolve(L, nr, s0 >> 16, m, upper, mask);
  if (nh > 2) lean_resolve(L, nr, s1 & 0xFFFFu, m, upper, mask);
  if (nh > 3) lean_resolve(L, nr, s1 >> 16, m, upper, mask);
  if (mask) {
    atomicOr(&L.match[0], (uint32_t)mask);
    atomicOr(&L.match[1], (uint32_t)(mask >> 32));
  }
  return acc;
}

// One bounded-length regex stage over the value bytes [lo, hi) (regex-filter /
// filter_regex with a <= 16-state ASCII DFA, smartmodule/regex-filter/src/lib.rs:
// 24-28): the range is cut into one piece per thread; a thread runs the DFA
// over its piece plus max_len - 1 bytes of overlap, so every match starting
// in the piece ends inside the scan.  Table-driven: the state is 4 bits, one
// LDS read of tt[byte] gives the byte's whole row; FSG_RX_STEP bytes a step, their
// row reads issued before the state chain consumes them (a byte at a time,
// each read waited for at once: C1 eval 2.30 -> 1.36 ms at 8 bytes, 1.53 at 16
// (128-VGPR cap of the lean kernel), 2.55 with two interleaved chains (spills)).
// A value piece starts in s_bot at the value start and in s_mid elsewhere
// (unanchored restart); accept bit0 is sticky (the DFA stays in an accepting
// state), bit1 is checked where a value ends (`$`).  Returns the OR of every
// scanned byte (bit 7 set <=> a non-ASCII value byte).
#ifndef FSG_RX_STEP
#define FSG_RX_STEP 8
#endif
__device__ __forceinline__ uint32_t lean_regex(LeanLds& L, int nr, uint32_t lo, uint32_t hi, uint32_t mlen,
                                               uint32_t s_bot, uint32_t s_mid, uint32_t acc1, uint32_t acc2) {
  constexpr uint32_t kStep = FSG_RX_STEP;
  const uint32_t l = threadIdx.x;
  // piece length: a multiple of 4 whose dword count is odd, so the lanes' window
  // reads (ds_read_b32: bank (a/4) mod 32 per 32-lane group) fall on distinct banks
  uint32_t q_len = ((hi - lo + kLeanThreads - 1) / kLeanThreads + 3u) & ~3u;
  if (!((q_len >> 2) & 1u)) q_len += 4u;
  const uint32_t p0 = lo + l * q_len;
  uint32_t orw = 0;
  uint64_t mask = 0;
  if (p0 < hi) {
    const uint32_t p1 = p0 + q_len < hi ? p0 + q_len : hi;
    const uint32_t pe = p1 + mlen - (mlen ? 1u : 0u);
    const uint32_t pend = pe < hi ? pe : hi;
    int r = lean_rec_bs(L, nr, p0);
    if (r < 0) r = 0;
    for (; r < nr; r++) {
      const uint32_t vs = L.r_vs[r], ve = L.r_ve[r];
      if (vs >= p1) break;
      uint32_t q = vs > p0 ? vs : p0;
      if (q >= ve) continue;
      uint32_t st = q == vs ? s_bot : s_mid;
      const uint32_t end = ve < pend ? ve : pend;
      while (q + kStep <= end) {
        uint32_t w[kStep / 4];
#pragma unroll
        for (uint32_t j = 0; j < kStep / 4; j++) {
          w[j] = lds_u32_at(L.win, q + 4u * j);
          orw |= w[j];
        }
        uint64_t t[kStep];
#pragma unroll
        for (uint32_t k = 0; k < kStep; k++) t[k] = L.tt[(w[k >> 2] >> (8 * (k & 3))) & 0xFFu];
#pragma unroll
        for (uint32_t k = 0; k < kStep; k++) st = (uint32_t)(t[k] >> (4 * st)) & 15u;
        q += kStep;
      }
      while (q < end) {
        const uint32_t w = lds_u32_at(L.win, q);
        const uint32_t n = end - q < 4u ? end - q : 4u;
        orw |= n == 4 ? w : (w & ((1u << (8 * n)) - 1u));
        for (uint32_t k = 0; k < n; k++) st = (uint32_t)(L.tt[(w >> (8 * k)) & 0xFFu] >> (4 * st)) & 15u;
        q += n;
      }
      if (((acc1 >> st) & 1u) || (end == ve && ((acc2 >> st) & 1u))) mask |= 1ull << r;
    }
  }
  // empty values: decided by the start state alone
  if ((int)l < nr && L.r_vs[l] == L.r_ve[l] && (((acc1 | acc2) >> s_bot) & 1u)) mask |= 1ull << l;
  if (mask) {
    atomicOr(&L.match[0], (uint32_t)mask);
    atomicOr(&L.match[1], (uint32_t)(mask >> 32));
  }
  return orw;
}

// 4 bits: which of the 4 bytes of a SWAR mask word carry 0x80
__device__ __forceinline__ uint32_t nib4(uint32_t m80) { return ((((m80 >> 7) & 0x01010101u) * 0x01020408u) >> 24) & 15u; }
// ---------------------------------------------------------------------------
// filter_json in the lean kernel (smartmodule/examples/filter_json/src/lib.rs:
// 54-70, serde_json::from_slice::<StructuredLog>), data-parallel:
//   1. byte classes of every 16-byte chunk of the batch's values (quotes,
//      spaces, "special" bytes: < 0x20, '\\', >= 0x80), one chunk per lane;
//      the in-string mask from a prefix XOR of the quotes carried across the
//      whole batch (a workgroup XOR scan)
//   2. the token list: every quote, special byte and non-space byte outside
//      strings, in order (workgroup prefix sum); opening quotes carry the class
//      of their string ("level", "message", a LogLevel variant, other)
//   3. one thread per record runs the table-driven token DFA of fsg_json_dfa.h
//      over its tokens.  The DFA accepts exactly the flat objects whose
//      outcome is certain: ASCII, no escapes / control bytes, level a variant
//      string, message a string, other values strings / JSON numbers /
//      literals, each field once.  Any other record (and any record starting
//      inside an unbalanced string) sends the batch to the exact kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pxor16(uint32_t q) {  // inclusive prefix XOR of 16 bits
  uint32_t px = q ^ (q << 1);
  px ^= px << 2;
  px ^= px << 4;
  px ^= px << 8;
  return px & 0xFFFFu;
}
// workgroup (128 threads) exclusive prefix of v; returns the exclusive value, *total
__device__ __forceinline__ uint32_t wg_excl_sum(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const uint32_t l = threadIdx.x, lane = l & 63u, w = l >> 6;
  const uint32_t incl = wave_incl_scan(v);
  if (lane == 63) wsum[w] = incl;
  lean_sync();
  const uint32_t w0 = wsum[0];
  *total = w0 + wsum[1];
  lean_sync();
  return incl - v + (w ? w0 : 0u);
}
// the class of the string of n bytes at window offset a: its (up to 8) bytes
// as one little-endian word against immediate constants (string literals would
// be global loads)
template <typename LdsT>
__device__ __forceinline__ uint32_t json_str_class(const LdsT& L, uint32_t a, uint32_t n) {
  if (n < 4 || n > 7) return JC_Q_OTHER;
  const uint64_t lo = lds_u32_at(L.win, a);
  const uint64_t hi = lds_u32_at(L.win, a + 4);
  const uint64_t w = (lo | (hi << 32)) & ((1ull << (8 * n)) - 1ull);
  constexpr auto k = [](const char* t) {
    uint64_t v = 0;
    for (int i = 0; t[i]; i++) v |= (uint64_t)(uint8_t)t[i] << (8 * i);
    return v;
  };
  if (n == 5) return w == k("level") ? JC_Q_LEVEL : w == k("debug") ? JC_Q_DEBUG : w == k("error") ? JC_Q_ERROR : JC_Q_OTHER;
  if (n == 7) return w == k("message") ? JC_Q_MSG : JC_Q_OTHER;
  if (n == 4) return w == k("info") ? JC_Q_INFO : w == k("warn") ? JC_Q_WARN : JC_Q_OTHER;
  return JC_Q_OTHER;
}
// stages 1-3 for the records [0, nr); returns true if the batch must go to the
// exact kernel; match bits of records whose level > Debug in L.match
// lean_json_stage step 3b for the members [0, nseg) of L.jn
template <bool kProj>
__device__ __forceinline__ void json_members(LeanLdsJ& L, int nr, uint32_t ntok, uint32_t nseg) {
  for (uint32_t k = threadIdx.x; k < nseg; k += kLeanThreads) {
    const uint32_t sg = L.jn()[k];
    const bool first = (sg & 0x8000u) != 0u;
    const uint32_t t0 = sg & 0x7FFFu;
    uint32_t t = t0;
    // the member's record: that of its first token (a record start) or of the comma before it
    const uint32_t anchor = L.ent[first ? t : t - 1] & 0x7FFFu;
    const uint32_t rr = (uint32_t)lean_rec_of(L, nr, anchor);
    const uint32_t ve = L.r_ve[rr];
    uint32_t st = first ? (uint32_t)JS_OBJ : (uint32_t)JS_KEY;
    uint32_t prev = first ? 0xFFFFu : anchor;
    uint32_t nlv = 0, nmsg = 0, lv = 0;
    bool ended = false, nbad = false;
    bool khit = false, inval = false, found = false, vneg = false;
    uint32_t vstart = 0, ntv = 0, fs = 0, fe = 0;
    for (; t < ntok; t++) {
      const uint32_t en = L.ent[t];
      const uint32_t pos = en & 0x7FFFu;
      if (pos >= ve) break;
      uint32_t cls = en >> 24;
      const uint32_t adj = pos == prev + 1 ? 1u : 0u;
      const uint32_t st0 = st;
      if constexpr (kProj) {
        const bool q = cls == JC_Q_FIELD;
        if (q) cls = JC_Q_OTHER;  // every string takes the "other" paths of the table
        else if (cls >= JC_Q_LEVEL && cls <= JC_Q_ERROR) cls = JC_Q_OTHER;
        st = L.dfa[st * kJsonCls2 + cls * 2 + adj];
        if (st == JS_INKEY_OTHER) khit = q;
        if (st0 == JS_VAL_OTHER) {
          inval = true;
          vstart = pos;
          ntv = 0;
          vneg = cls == JC_MINUS;
        }
        if (inval) {
          if (st == JS_KEY || st == JS_END) {  // ',' / '}' after the value
            inval = false;
            if (st0 == JS_N_ZERO && vneg && ntv == 2) nbad = true;  // -0
            if (khit) {
              found = true;
              fs = vstart;
              fe = prev + 1;
            }
          } else {
            ntv++;
            if (st == JS_N_DOT || st == JS_N_E || ntv > 18) nbad = true;
          }
        }
      } else {
        if (st >= JS_INV_D && st <= JS_INV_E) lv = 1u << (st - JS_INV_D);
        st = L.dfa[st * kJsonCls2 + cls * 2 + adj];
        nlv += st == JS_INKEY_LV ? 1u : 0u;
        nmsg += st == JS_INKEY_MSG ? 1u : 0u;
      }
      prev = pos;
      if (cls == JC_COMMA || st == JS_FAIL) {
        ended = true;
        break;
      }
    }
    const bool ok = !nbad && (ended ? st == JS_KEY : st == JS_END);
    atomicAdd(&L.racc[rr], nlv | (nmsg << 8) | (ok ? 0u : 1u << 16));
    if (lv) atomicOr(&L.rlvl[rr], lv);
    if (found) atomicMax(&L.rbest[rr], ((unsigned long long)(t0 + 1) << 32) | (fs << 16) | fe);
  }
}

#ifdef FSG_LEAN_TIMING
#define JT_PARAMS , uint64_t *lt_acc, uint64_t &lt_last
#define JT_ARGS , lt_acc, lt_last
#define JMARK(k)                                             \
  {                                                          \
    const uint64_t lt_now = __builtin_amdgcn_s_memtime();    \
    lt_acc[k] += lt_now - lt_last;                           \
    lt_last = lt_now;                                        \
  }
#else
#define JT_PARAMS
#define JT_ARGS
#define JMARK(k)
#endif
__device__ bool lean_json_stage(LeanLdsJ& L, int nr, uint32_t& orpar, bool proj, uint32_t fl JT_PARAMS) {
  const uint32_t l = threadIdx.x;
  const uint32_t c0 = L.r_vs[0] & ~15u, c1 = L.r_ve[nr - 1];
  const uint32_t nch = (c1 - c0 + 15) >> 4;
  if (nch > (uint32_t)kJsonChunks) return true;
  // 1. masks; thread t owns the contiguous chunks [t*per, (t+1)*per), per odd:
  //    the lanes' jm[] dwords and 16-byte window reads then fall on distinct
  //    banks (an even per put 4-8 lanes of a group on one bank)
  const uint32_t per = ((nch + kLeanThreads - 1) / kLeanThreads) | 1u;
  const uint32_t k0 = l * per, k1 = k0 + per < nch ? k0 + per : nch;
  uint32_t par = 0;
  for (uint32_t k = k0; k < k1; k++) {  // byte classes, once: quote, special (< 0x20 incl. 0, '\\', >= 0x80), non-space
    const uint4 v = *(const uint4*)(&L.win[c0 + 16 * k]);
    uint32_t q = 0, sp = 0, ns = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t w = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
      q |= nib4(zbytes(w ^ 0x22222222u)) << (4 * d);
      sp |= nib4(zbytes(w & 0xE0E0E0E0u) | zbytes(w ^ 0x5C5C5C5Cu) | (w & 0x80808080u)) << (4 * d);
      ns |= nib4(zbytes(w ^ 0x20202020u)) << (4 * d);
    }
    L.jm[k] = q | (sp << 16);
    L.jn()[k] = (uint16_t)(~ns & 0xFFFFu);
    par ^= __builtin_popcount(q) & 1u;
  }
  JMARK(6);
  uint32_t tot;
  uint32_t carry = wg_excl_sum(par, L.wsum, &tot) & 1u;  // parity of all quotes before my chunks
  uint32_t cnt = 0;
  for (uint32_t k = k0; k < k1; k++) {
    const uint32_t m = L.jm[k], q = m & 0xFFFFu, sp = m >> 16;
    const uint32_t instr = (pxor16(q) ^ q ^ (carry ? 0xFFFFu : 0u)) & 0xFFFFu;
    carry ^= __builtin_popcount(q) & 1u;
    const uint32_t hot = q | sp | ((uint32_t)L.jn()[k] & ~instr);
    L.jm[k] = instr | (hot << 16);
    cnt += __builtin_popcount(hot);
  }
  JMARK(7);
  // 2. token list
  uint32_t ntok;
  uint32_t e = wg_excl_sum(cnt, L.wsum, &ntok);
  if (ntok > (uint32_t)kJsonEnt) return true;  // uniform: every thread saw the same total
  // positions in order (ALU only: the token count per thread is uneven, the
  // records' heads are dense), then classes strided over the tokens
  for (uint32_t k = k0; k < k1; k++) {
    const uint32_t instr = L.jm[k] & 0xFFFFu;
    uint32_t hot = L.jm[k] >> 16;
    while (hot) {
      const uint32_t j = (uint32_t)__builtin_ctz(hot);
      hot &= hot - 1;
      L.ent[e++] = (c0 + 16 * k + j) | (((instr >> j) & 1u) << 15);
    }
  }
  if (l == 0) L.nseg = 0;
  lean_sync();
  JMARK(8);
  // classes; an opening quote takes the class of its string (the next token
  // closes it).  Bits 0..15 never change here, so a neighbour's position and
  // in-string bit can be read while it is being rewritten.
  for (uint32_t t = l; t < ntok; t += kLeanThreads) {
    const uint32_t en = L.ent[t];
    const uint32_t pos = en & 0x7FFFu;
    const uint32_t b = L.win[pos];
    uint32_t cls = L.bcls[b];
    if (b == '"') {
      cls = (en & 0x8000u) ? (uint32_t)JC_Q_CLOSE : (uint32_t)JC_Q_OTHER;
      if (cls == JC_Q_OTHER && t + 1 < ntok) {
        const uint32_t nx = L.ent[t + 1];
        const uint32_t np = nx & 0x7FFFu;
        if ((nx & 0x8000u) && L.win[np] == '"') {
          const uint32_t a = pos + 1, n = np - a;
          if (proj) {  // the projected field's name (L.needle) or another string
            bool eq = n == fl;
            for (uint32_t k = 0; eq && k < fl; k += 4) {
              const uint32_t mk = fl - k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (fl - k))) - 1u);
              eq = ((lds_u32_at(L.win, a + k) ^ lds_u32_at(L.needle, k)) & mk) == 0u;
            }
            cls = eq ? (uint32_t)JC_Q_FIELD : (uint32_t)JC_Q_OTHER;
          } else {
            cls = json_str_class(L, a, n);
          }
        }
      }
    }
    L.ent[t] = (en & 0xFFFFu) | (b << 16) | (cls << 24);
    // members: the token after a comma starts one (of the comma's record)
    if (cls == JC_COMMA) {
      const uint32_t k = atomicAdd(&L.nseg, 1u);
      if (k < (uint32_t)kJsonSeg) L.jn()[k] = (uint16_t)(t + 1);
    }
  }
  lean_sync();
  JMARK(9);
  // 3a. per record: balanced quotes at its ends, its first token (binary
  //     search on positions) = the start of its first member
  const uint32_t r = 2 * (l & 63u) + (l >> 6);
  auto instr_at = [&](uint32_t p) {
    const uint32_t k = (p - c0) >> 4, j = (p - c0) & 15u;
    if (k >= nch) return 0u;
    return (L.jm[k] >> j) & 1u;
  };
  uint32_t t_first = 0;
  bool bad = false;
  if ((int)r < nr) {
    const uint32_t vs = L.r_vs[r], ve = L.r_ve[r];
    if (instr_at(vs) || instr_at(ve)) bad = true;
    uint32_t lo = 0, hi = ntok;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if ((L.ent[m] & 0x7FFFu) < vs) lo = m + 1; else hi = m;
    }
    t_first = lo;
    // no token inside the value: not an object (and no member may claim it)
    if (lo >= ntok || (L.ent[lo] & 0x7FFFu) >= ve) bad = true;
    L.racc[r] = bad ? 1u << 16 : 0u;
    L.rlvl[r] = 0;
    L.rbest[r] = 0;
    if (!bad) {
      const uint32_t k = atomicAdd(&L.nseg, 1u);
      if (k < (uint32_t)kJsonSeg) L.jn()[k] = (uint16_t)(lo | 0x8000u);
    }
  }
  (void)t_first;
  lean_sync();
  const uint32_t nseg = L.nseg;
  if (nseg > (uint32_t)kJsonSeg) return lean_or(L.red, orpar, true);  // uniform
  // 3b. the token DFA, one thread per object member: a member after a comma
  //     starts in JS_KEY (the only state a comma leads to) and ends with the
  //     next comma, which must lead to JS_KEY again, or at the record's end,
  //     which must be JS_END.  filter_json, per record: each field exactly
  //     once, the level value's variant.  Projection (map_json_project,
  //     Map<String, Value>, last member wins): the value span of the last
  //     member whose key is the field; numbers whose serde_json text differs
  //     from the source (fractions, exponents, -0, more than 18 digits) are
  //     unsupported by the device restatement -> exact kernel
  JMARK(10);
  if (proj)
    json_members<true>(L, nr, ntok, nseg);
  else
    json_members<false>(L, nr, ntok, nseg);
  lean_sync();
  JMARK(11);
  if ((int)r < nr) {
    const uint32_t ac = L.racc[r];
    if (proj) {
      bad = (ac >> 16) != 0u;
      const unsigned long long bst = L.rbest[r];
      if (!bad && bst) {
        atomicOr(&L.match[r >> 5], 1u << (r & 31));
        L.r_vs[r] = (uint32_t)(bst >> 16) & 0xFFFFu;  // the value narrows to the field's text
        L.r_ve[r] = (uint32_t)bst & 0xFFFFu;
      }
    } else {
      // exactly one level and one message field (a duplicate is a serde error)
      bad = (ac >> 16) != 0u || (ac & 0xFFu) != 1u || ((ac >> 8) & 0xFFu) != 1u;
      if (!bad && (L.rlvl[r] & ~1u)) atomicOr(&L.match[r >> 5], 1u << (r & 31));
    }
  }
  return lean_or(L.red, orpar, bad);
}

// blank every byte between values (record headers, keys, lengths) with
// spaces and build the 64-byte block -> record table; thread l < nr owns
// record l (value [vs, vs+vl)).  A space has no high bit (the scans' OR stays
// an ASCII test), is no JSON token (the token list holds value bytes only) and
// a needle hit that reaches into a gap fails its record range check.
__device__ __forceinline__ void clear_gaps(LeanLds& L, int nr, uint32_t vs, uint32_t vl) {
  const uint32_t l = threadIdx.x;
  const uint32_t lo = L.r_vs[0], hi = L.r_ve[nr - 1];
  // [s, e) <- ' ': whole aligned dwords inside the range, bytes at its edges (a
  // dword at an edge may hold another record's value bytes)
  auto zero = [&](uint32_t s, uint32_t e) {
    const uint32_t s4 = (s + 3) & ~3u, e4 = e & ~3u;
    if (s4 >= e4) {
      for (uint32_t p = s; p < e; p++) L.win[p] = 0x20;
      return;
    }
    for (uint32_t p = s; p < s4; p++) L.win[p] = 0x20;
    for (uint32_t p = s4; p < e4; p += 4) *(uint32_t*)(L.win + p) = 0x20202020u;
    for (uint32_t p = e4; p < e; p++) L.win[p] = 0x20;
  };
  if ((int)l < nr) zero(vs + vl, (int)l + 1 < nr ? L.r_vs[l + 1] : ((vs + vl + 15) & ~15u) + 16);
  if (l == 0) zero(lo & ~15u, lo);
  // blk[j] = l for the 64-byte blocks j starting in [vs, next value start)
  if ((int)l < nr) {
    const uint32_t e = (int)l + 1 < nr ? L.r_vs[l + 1] : hi + 80;
    const uint32_t j0 = (vs + 63) >> 6, j1 = (e + 63) >> 6;
    const uint32_t rep = l * 0x01010101u;
    uint32_t j = j0;
    for (; j < j1 && (j & 3u); j++) L.blk[j] = (uint8_t)l;
    for (; j + 4 <= j1; j += 4) *(uint32_t*)(L.blk + j) = rep;
    for (; j < j1; j++) L.blk[j] = (uint8_t)l;
  }
  if (l == 0)
    for (uint32_t j = 0; (j << 6) < lo; j++) L.blk[j] = 0xFF;
}

// the 64-byte block -> record table alone (the part of clear_gaps a short
// needle's dense hits need; thread l < nr owns record l)
__device__ __forceinline__ void lean_blk(LeanLds& L, int nr, uint32_t vs) {
  const uint32_t l = threadIdx.x;
  const uint32_t lo = L.r_vs[0], hi = L.r_ve[nr - 1];
  if ((int)l < nr) {
    const uint32_t e = (int)l + 1 < nr ? L.r_vs[l + 1] : hi + 80;
    const uint32_t j0 = (vs + 63) >> 6, j1 = (e + 63) >> 6;
    const uint32_t rep = l * 0x01010101u;
    uint32_t j = j0;
    for (; j < j1 && (j & 3u); j++) L.blk[j] = (uint8_t)l;
    for (; j + 4 <= j1; j += 4) *(uint32_t*)(L.blk + j) = rep;
    for (; j < j1; j++) L.blk[j] = (uint8_t)l;
  }
  if (l == 0)
    for (uint32_t j = 0; (j << 6) < lo; j++) L.blk[j] = 0xFF;
}

__device__ __forceinline__ uint32_t high_count(const uint8_t* win, uint32_t p, uint32_t e) {  // bytes >= 0x80 in [p, e)
  uint32_t n = 0;
  for (uint32_t q = p & ~3u; q < e; q += 4)
    n += (uint32_t)__builtin_popcount(*(const uint32_t*)(win + q) & 0x80808080u & bytes_in(q, p, e));
  return n;
}
// the 16-byte aligned window [al, al + wlen) of batch b
struct LeanWin {
  uint64_t pos, al;
  uint32_t wlen;
};
__device__ __forceinline__ LeanWin lean_window(const EvalArgs& a, uint32_t b) {
  LeanWin w;
  w.pos = a.bpos[b];
  const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
  w.al = w.pos & ~15ull;
  uint64_t wl = nxt > w.al ? nxt - w.al : 0;
  if (wl > (uint64_t)kLeanWin) wl = kLeanWin;
  w.wlen = (uint32_t)((wl + 15) & ~15ull);
  return w;
}
// 1 KiB LDS-DMA pieces (one 16-byte piece per lane), the last one partial;
// the waves split the pieces
__device__ __forceinline__ void lean_issue(const EvalArgs& a, const LeanWin& w, uint8_t* dst) {
  const uint32_t l = threadIdx.x, lane = l & 63u;
  const uint8_t* src = a.slice + w.al + lane * 16;
  for (uint32_t k = __builtin_amdgcn_readfirstlane(l >> 6); k * 1024 < w.wlen; k += kLeanThreads / 64)
    if (k * 1024 + lane * 16 < w.wlen)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + k * 1024),
                                       (__attribute__((address_space(3))) void*)(dst + k * 1024), 16, 0, 0);
}

// k_chase — record framing of the lean path, one thread per batch: the chain
// of record length varints (Record::decode's first field, data.rs:534-562)
// walked with dependent global loads; thousands of batches in flight hide the
// latency, and k_eval_lean gets every record's start with its window instead
// of a serial walk through LDS.  Conservative: anything unusual (more than
// kLeanMaxR records, a length varint over 4 bytes, a record past the window)
// leaves rend[b] = 0xFFFF and the batch takes the exact path.
// The starts are staged in LDS and written back as one contiguous span per
// workgroup (batches b0 .. b0 + 255 own consecutive record slots), so the
// stores are coalesced instead of one partial line per record.
constexpr int kChaseT = 256;
__global__ __launch_bounds__(kChaseT) void k_chase(EvalArgs a) {
  __shared__ uint16_t st[kChaseT * kLeanMaxR];
  const uint32_t t = threadIdx.x;
  const uint32_t b0 = blockIdx.x * kChaseT;
  const uint32_t b = b0 + t;
  const uint32_t bl = b0 + kChaseT < a.nbatches ? b0 + kChaseT : a.nbatches;  // first batch past the block
  const uint64_t R0 = a.rbase[b0];
  const uint64_t R1 = bl < a.nbatches ? a.rbase[bl] : a.nrec;
  const bool stage = R1 - R0 <= (uint64_t)(kChaseT * kLeanMaxR);
  if (b < a.nbatches) {
    const uint64_t pos = a.bpos[b];
    const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
    const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
    const uint64_t al = pos & ~15ull;
    uint64_t wl = nxt > al ? nxt - al : 0;
    if (wl > (uint64_t)kLeanWin) wl = kLeanWin;
    const uint64_t wlen = (wl + 15) & ~15ull;
    const uint8_t* base = a.slice + al;
    const uint32_t batch_len = __builtin_bswap32(ld_u32_at(a.slice + pos + 8));
    const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
    const uint64_t sec_len = sec_end - sec0;
    const int32_t count = sec_len >= 4 ? (int32_t)__builtin_bswap32(ld_u32_at(a.slice + sec0)) : -1;
    uint32_t end = 0xFFFFu;
    if (sec_len >= 4 && sec_end - al <= wlen && count >= 0 && count <= kLeanMaxR && (uint64_t)count == rn) {
      const uint32_t have = (uint32_t)(sec_end - al);
      uint32_t q = (uint32_t)(sec0 + 4 - al);
      int n = 0;
      for (; n < count; n++) {
        const uint32_t x = ld_u32_at(base + q);
        const uint32_t term = ~x & 0x80808080u;
        if (!term) break;
        const uint32_t nb = (((uint32_t)__builtin_ctz(term)) >> 3) + 1;
        if (q + nb > have) break;
        const uint32_t y = nb == 4 ? x : (x & ((1u << (8 * nb)) - 1u));
        const uint32_t v = (y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u) | ((y >> 3) & 0xFE00000u);
        if (v & 1u) break;  // negative length (zigzag)
        const uint32_t len = v >> 1;
        if (have - (q + nb) < len) break;
        if (stage)
          st[rb - R0 + n] = (uint16_t)q;
        else
          a.rstart[rb + n] = (uint16_t)q;
        q += nb + len;
      }
      if (n == count) end = q;
    }
    a.rend[b] = (uint16_t)end;
  }
  if (!stage) return;  // uniform
  __syncthreads();
  // slots of failed chases hold garbage: the lean kernel never reads them (rend = 0xFFFF)
  const uint64_t n = R1 - R0;
  uint16_t* dst = a.rstart + R0;
  const uint32_t head = (uint32_t)((8u - ((uintptr_t)dst & 15u) / 2u) & 7u);  // u16 slots to 16-B alignment
  for (uint64_t i = t; i < n && i < head; i += kChaseT) dst[i] = st[i];
  for (uint64_t i = head + 8ull * t; i + 8 <= n; i += 8ull * kChaseT) {
    uint4 v;
    v.x = st[i] | ((uint32_t)st[i + 1] << 16);
    v.y = st[i + 2] | ((uint32_t)st[i + 3] << 16);
    v.z = st[i + 4] | ((uint32_t)st[i + 5] << 16);
    v.w = st[i + 6] | ((uint32_t)st[i + 7] << 16);
    *(uint4*)(dst + i) = v;
  }
  const uint64_t tail0 = n > head ? head + ((n - head) & ~7ull) : n;
  for (uint64_t i = tail0 + t; i < n; i += kChaseT) dst[i] = st[i];
}

// k_chase_w — the same record framing for the exact kernel and the lean array
// kernel: any record count, a batch up to 64 KiB from its aligned start.  One
// wave per batch: the window streams through registers 16 KiB at a time (row
// k = 1 KiB, lane = 16 bytes), and the wave-uniform walk reads each length
// varint with two readlanes (no dependent memory loads on the chain); the
// starts are gathered one per lane and stored 64 at a time.
__device__ __forceinline__ uint32_t sel4(const uint4& v, uint32_t c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}
constexpr int kChaseRows = 16;
__global__ __launch_bounds__(256) void k_chase_w(EvalArgs a) {
  const uint32_t lane = lane_id();
  const uint32_t nw = gridDim.x * 4;
  // the batch index is wave-uniform: readfirstlane keeps the whole walk scalar
  for (uint32_t b = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); b < a.nbatches; b += nw) {
    const uint64_t pos = a.bpos[b];
    const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
    const uint64_t al = pos & ~15ull;
    const uint32_t batch_len = __builtin_bswap32(ld_u32_at(a.slice + pos + 8));
    const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
    const uint64_t sec_len = sec_end - sec0;
    const int32_t count = sec_len >= 4 ? (int32_t)__builtin_bswap32(ld_u32_at(a.slice + sec0)) : -1;
    uint32_t end = 0xFFFFu;
    if (sec_len >= 4 && sec_end - al < 0xFFFFu && count >= 0 && (uint64_t)count == rn) {
      const uint32_t have = (uint32_t)(sec_end - al);
      const uint64_t lim = a.slice_len + kSlicePad;  // readable bytes of the slice buffer
      uint32_t q = (uint32_t)(sec0 + 4 - al);
      uint32_t n = 0, acc = 0;
      bool ok = true;
      for (uint32_t blk = 0; ok && n < (uint32_t)count && blk * 1024u * kChaseRows < have; blk++) {
        uint4 R[kChaseRows + 1];
#pragma unroll
        for (int k = 0; k <= kChaseRows; k++) {
          const uint64_t o = al + (uint64_t)(blk * kChaseRows + k) * 1024 + lane * 16;
          R[k] = o + 16 <= lim ? *(const uint4*)(a.slice + o) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < kChaseRows; k++) {
          const uint32_t row_end = (blk * kChaseRows + k + 1) * 1024u;
          while (ok && n < (uint32_t)count && q < row_end) {
            q = __builtin_amdgcn_readfirstlane(q);  // uniform (the compiler cannot see it through the loop)
            n = __builtin_amdgcn_readfirstlane(n);
            const uint32_t d = (q & 1023u) >> 2;  // dword of the row
            const uint32_t w0 = __builtin_amdgcn_readlane(sel4(R[k], d & 3u), d >> 2);
            const uint32_t w1 = d == 255 ? __builtin_amdgcn_readlane(R[k + 1].x, 0)
                                         : __builtin_amdgcn_readlane(sel4(R[k], (d + 1) & 3u), (d + 1) >> 2);
            const uint32_t x = __builtin_amdgcn_alignbyte(w1, w0, q & 3u);
            const uint32_t term = ~x & 0x80808080u;
            const uint32_t nb = (((uint32_t)__builtin_ctz(term | 0x80000000u)) >> 3) + 1;
            const uint32_t y = nb == 4 ? x : (x & ((1u << (8 * nb)) - 1u));
            const uint32_t v = (y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u) | ((y >> 3) & 0xFE00000u);
            const uint32_t len = v >> 1;
            // no terminator in 4 bytes, past the section, a negative length, past the section
            if (!term || q + nb > have || (v & 1u) || have - (q + nb) < len) {
              ok = false;
              break;
            }
            if (lane == (n & 63u)) acc = q;
            if ((n & 63u) == 63u) a.rstart[rb + n - 63 + lane] = (uint16_t)acc;
            n++;
            q += nb + len;
          }
        }
      }
      if (n & 63u)
        if (lane < (n & 63u)) a.rstart[rb + (n & ~63u) + lane] = (uint16_t)acc;
      if (ok && n == (uint32_t)count) end = q;
    }
    if (lane == 0) a.rend[b] = (uint16_t)end;
  }
}
void launch_chase_w(const EvalArgs& a, hipStream_t s) {
  if (a.nbatches) hipLaunchKernelGGL(k_chase_w, dim3(std::min<uint32_t>((a.nbatches + 3) / 4, 8192)), dim3(256), 0, s, a);
}

// four waves per SIMD (eight workgroups per CU, as many as the LDS holds)
// kernel variants by the chain's stage ops (a smaller kernel holds fewer
// registers and less code): substring filters only, regex filters only, both,
// and the filter_json / projection variant (every lean stage)
enum LeanKind { kLeanContains = 0, kLeanRegex = 1, kLeanMixed = 2, kLeanJson = 3 };
template <int kKind>
#ifndef FSG_JSON_WPE
#define FSG_JSON_WPE 3  // waves per SIMD of the JSON lean kernel: <= 168 VGPRs, with <= 32 KiB LDS 5 workgroups per CU
#endif
#ifndef FSG_LEAN_WPE
#define FSG_LEAN_WPE 4
#endif
__global__ __launch_bounds__(kLeanThreads) __attribute__((amdgpu_waves_per_eu(kKind == kLeanJson ? FSG_JSON_WPE : FSG_LEAN_WPE))) void k_eval_lean(EvalArgs a) {
  constexpr bool kJson = kKind == kLeanJson;
  constexpr bool kHasRx = kKind != kLeanContains;  // regex stages compiled in
  constexpr bool kHasCt = kKind != kLeanRegex;     // substring stages compiled in
  __shared__ typename std::conditional<kJson, LeanLdsJ, LeanLds>::type L;
  const uint32_t l = threadIdx.x;
  const uint32_t G = gridDim.x;
  uint32_t b = blockIdx.x;
  if (b >= a.nbatches) return;
  // the chain's stages, needles, regex rows and JSON tables: LDS, once
  {
    const ChainDesc& ch = *a.chain;
    const uint32_t nst = ch.nstages;
    uint32_t nrx = 0, rx = 0xFFu, ndo = 0;
    for (uint32_t s = 0; s < nst; s++)
      if (ch.st[s].op == OP_CONTAINS || ch.st[s].op == OP_PROJECT) ndo += ch.st[s].needle_len;
    const bool nd_res = ndo <= (uint32_t)kLeanNeedles;
    ndo = 0;
    for (uint32_t s = 0; s < nst; s++) {
      const StageDesc& sd = ch.st[s];
      if (sd.op == OP_REGEX) {
        nrx++;
        rx = s;
      }
      if (l == 0) {
        LeanStage g;
        g.op = sd.op;
        g.upper = sd.in_type == VT_SRC_UPPER ? 1 : 0;
        g.keep_match = sd.keep_match;
        g.pad = 0;
        g.m = sd.needle_len;
        g.max_len = (uint32_t)sd.dfa.max_len;
        g.s_bot = sd.dfa.s_bot;
        g.s_mid = sd.dfa.s_mid;
        g.acc1 = sd.dfa.acc1;
        g.acc2 = sd.dfa.acc2;
        g.tt = sd.in_type == VT_SRC_UPPER ? sd.dfa.tt_up : sd.dfa.tt;
        g.nd = sd.needle;
        g.nd_off = ndo;
        L.stg[s] = g;
      }
      if ((sd.op == OP_CONTAINS || sd.op == OP_PROJECT) && nd_res) {
        for (uint32_t t = l; t < sd.needle_len; t += kLeanThreads) L.needles[ndo + t] = a.blob[sd.needle + t];
        ndo += sd.needle_len;
      }
    }
    if (nrx == 1 && !kJson) {  // one regex stage: its rows stay resident (the JSON variant reuses them as jn)
      const StageDesc& sd = ch.st[rx];
      const uint64_t* tt = (const uint64_t*)(a.blob + (sd.in_type == VT_SRC_UPPER ? sd.dfa.tt_up : sd.dfa.tt));
      for (uint32_t t = l; t < 256; t += kLeanThreads) L.tt[t] = tt[t];
    }
    if (l == 0) {
      L.nst = nst;
      L.out_upper = ch.out_type == VT_SRC_UPPER ? 1u : 0u;
      L.tt_stage = nrx == 1 && !kJson ? rx : 0xFFu;
      L.nd_res = nd_res ? 1u : 0u;
    }
    if constexpr (kJson) {
      for (uint32_t t = l; t < (uint32_t)(kJsonStates * kJsonCls2); t += kLeanThreads) L.dfa[t] = g_json_tables.t[t];
      for (uint32_t t = l; t < 256; t += kLeanThreads) L.bcls[t] = g_json_tables.bcls[t];
    }
  }
  uint32_t par = 0;  // lean_or pair
#ifdef FSG_LEAN_TIMING  // experiment builds: per-phase clock sums, printed by workgroup 0
  uint64_t lt_acc[12] = {}, lt_last = __builtin_amdgcn_s_memtime(), lt_nb = 0;
#define LEAN_MARK(k)                                         \
  {                                                          \
    const uint64_t lt_now = __builtin_amdgcn_s_memtime();    \
    lt_acc[k] += lt_now - lt_last;                           \
    lt_last = lt_now;                                        \
  }
#else
#define LEAN_MARK(k)
#endif
  // the previous batch's results, stored once the next window is in flight
  // (a store issued right before the wait for the next window would be waited for too)
  uint32_t p_b = 0xFFFFFFFFu;
  // the regex variant also writes each batch's scan row (BF_ROWDONE); the
  // others would spill for it (measured: 20 / 8 more bytes of scratch)
  const bool kRows = kKind == 1 && a.rows != nullptr;
  const int64_t base0 = kRows ? (int64_t)rd_be(a.slice + a.bpos[0], 8) : 0;  // batch 0's base offset
  bool p_defer = false, p_kept = false;
  uint64_t p_idx = 0;
  KeptRec p_d = {};
  int64_t p_base = 0, p_ts0 = 0;
  int32_t p_lod = 0;
  uint32_t p_comp = 0;
  uint32_t p_nkeep = 0, p_sec = 0;
  auto flush = [&]() {
    if (p_b == 0xFFFFFFFFu) return;
    if (p_defer) {
      if (l == 0) {
        const uint32_t i = atomicAdd(&a.list[0], 1u);
        a.list[1 + i] = p_b;
      }
    } else {
      if (p_kept) a.desc[p_idx] = p_d;
      // the batch's scan row for a first surviving batch 0 (k_size skips BF_ROWDONE batches then)
      const uint64_t rbytes = kRows ? wave_sum((uint64_t)(p_kept ? copy_out_size(p_d, base0 - p_base) : 0u)) : 0ull;
      if (l == 0) {
        BatchStat st = {};
        st.base_offset = p_base;
        st.lod_in = p_lod;
        st.first_ts = p_ts0;
        st.comp = p_comp;
        st.flags = BF_LAST_STAGE;
        if (kRows) {
          ScanRow row = {};
          row.rec_bytes = rbytes;
          row.nonempty = p_nkeep ? 1 : 0;
          row.lod = (uint64_t)(int64_t)(p_lod + 1);
          row.nrec = p_nkeep;
          row.bytes_in = p_sec;
          row.recs_out = p_nkeep;
          a.rows[p_b] = row;
          st.flags |= BF_ROWDONE;
        }
        st.nkeep = p_nkeep;
        st.nout = p_nkeep;
        st.sec_len = p_sec;
        st.err_stage = 0xFFFFFFFFu;
        a.bstat[p_b] = st;
      }
    }
    p_b = 0xFFFFFFFFu;
  };
  for (;;) {
    lean_sync();  // every lane is done with the previous batch's window
    const LeanWin W = lean_window(a, b);
    const uint64_t pos = W.pos, al = W.al;
    const uint32_t wlen = W.wlen;
    const uint64_t rb = a.rbase[b];
    const uint32_t bn = b + G;
    lean_issue(a, W, L.win);
    // the record starts (k_chase) ride along with the window
    const uint32_t rs = l < 64 ? a.rstart[rb + l] : 0u;
    const uint32_t re = a.rend[b];
    __builtin_amdgcn_s_waitcnt(0);  // this wave's pieces have landed
    lean_sync();                    // ... and the other wave's
    LEAN_MARK(0);
    // batch header (file format, batch.rs:163-180), read before the gaps are cleared
    const uint8_t* h = L.win + (pos - al);
    const int64_t base_offset = (int64_t)rd_be(h, 8);
    const uint32_t batch_len = (uint32_t)rd_be(h + 8, 4);
    const int32_t lod_in = (int32_t)rd_be(h + 23, 4);
    const int64_t first_ts = (int64_t)rd_be(h + 27, 8);
    const uint32_t comp = (uint32_t)h[22] & 7u;
    const uint64_t sec0 = pos + 57;
    const uint64_t sec_end = pos + 12 + (uint64_t)batch_len;  // framing validated at ingest
    const uint32_t sec_len = (uint32_t)(sec_end - sec0);
    const int32_t count = sec_len >= 4 ? (int32_t)rd_be(L.win + (sec0 - al), 4) : -1;
    bool defer = sec_len < 4 || sec_end - al > (uint64_t)wlen || count < 0 || count > kLeanMaxR;
    // 2. framing: the record starts k_chase found (rs, loaded with the window);
    //    lane r parses record r.  No lean framing (rend 0xFFFF): exact path.
    if (!defer) defer = re == 0xFFFFu;
    const int nr = defer ? 0 : count;
    bool g = true;
    int64_t ts = 0, od = 0, hdr = 0;
    uint32_t vs = 0, vl = 0, kpos = 0, klen = 0;
    uint8_t attr = 0, tag = 0;
    const uint32_t rs_next = __shfl_down(rs, 1, 64);
    uint32_t gh = 0;  // bytes >= 0x80 of this record between values (non-JSON kernel)
    if ((int)l < nr) {
      uint32_t q = rs;
      const uint32_t lim = (int)l + 1 == nr ? re : rs_next;
      int64_t len, kl, vlen;
      g = !wvarint((const uint8_t*)L.win, q, lim, &len);
      uint32_t vb = q - rs;  // varint bytes of the header (each but its last has bit 7 set)
      uint32_t nv = 1;
      if (g && q < lim) attr = L.win[q++]; else g = false;
      const uint32_t q1 = q;
      g = g && !wvarint((const uint8_t*)L.win, q, lim, &ts) && !wvarint((const uint8_t*)L.win, q, lim, &od);
      vb += q - q1;
      nv += 2;
      if (g && q < lim) tag = L.win[q++]; else g = false;
      g = g && tag <= 1;
      uint32_t kh = 0;
      if (g && tag == 1) {
        const uint32_t q2 = q;
        g = !wvarint((const uint8_t*)L.win, q, lim, &kl) && kl >= 0 && (uint64_t)q + (uint64_t)kl <= lim;
        vb += q - q2;
        nv += 1;
        if (g) {
          kpos = q;
          klen = (uint32_t)kl;
          q += klen;
          if (!kJson) kh = high_count(L.win, kpos, kpos + klen);
        }
      }
      const uint32_t q3 = q;
      g = g && !wvarint((const uint8_t*)L.win, q, lim, &vlen) && vlen >= 0 && (uint64_t)q + (uint64_t)vlen <= lim;
      vb += q - q3;
      nv += 1;
      vs = q;
      if (g) {
        vl = (uint32_t)vlen;
        q += vl;
      }
      const uint32_t q4 = q;
      g = g && !wvarint((const uint8_t*)L.win, q, lim, &hdr) && q == lim;
      L.r_vs[l] = vs;
      L.r_ve[l] = vs + vl;
      // the scans cover [first value start, last value end): the header of
      // every record but the first, the trailer of every record but the last
      if (!kJson && g)
        gh = (l > 0 ? vb - nv + (attr >> 7) + kh : 0u) + ((int)l + 1 < nr ? q - q4 - 1 : 0u);
    }
    if (!kJson && l < 64) {  // wave 0 frames: its sum is the batch's
      const uint32_t t = wave_sum(gh);
      if (l == 0) L.ghigh = t;
    }
    defer = lean_or(L.red, par, defer || !g);  // a record that does not frame exactly
    LEAN_MARK(1);
    uint64_t alive = __ballot((int)l < nr);
    // 3. stages.  Before the first scan every non-value byte of the scanned
    //    range is cleared (record headers, keys, lengths): then the OR of the
    //    scanned words has a high bit iff some value is non-ASCII.
    bool checked = false;  // every value known ASCII (from_utf8 cannot fail)
    bool cleared = false;  // gap bytes zeroed, record block table built
    const uint32_t nst = __builtin_amdgcn_readfirstlane(L.nst);
    for (uint32_t s = 0; !defer && s < nst; s++) {
      const LeanStage sd = L.stg[s];
      const uint32_t op = __builtin_amdgcn_readfirstlane((uint32_t)sd.op);
      if (op == OP_MAP_UPPER) continue;  // representation only
      if constexpr (kJson) if (op == OP_FILTER_JSON || op == OP_PROJECT) {
        const bool proj = op == OP_PROJECT;
        const uint32_t fl = proj ? __builtin_amdgcn_readfirstlane(sd.m) : 0u;
        if (l == 0) {
          L.match[0] = 0;
          L.match[1] = 0;
        }
        if (proj) {  // the field name (<= kLeanNeedle bytes: the runtime checks)
          if (__builtin_amdgcn_readfirstlane(L.nd_res)) {
            const uint32_t o = __builtin_amdgcn_readfirstlane(sd.nd_off);
            for (uint32_t t = l; t < fl; t += kLeanThreads) L.needle[t] = L.needles[o + t];
          } else {
            const uint8_t* nd = a.blob + __builtin_amdgcn_readfirstlane(sd.nd);
            for (uint32_t t = l; t < fl; t += kLeanThreads) L.needle[t] = nd[t];
          }
        }
        if (!cleared && nr > 0) {
          clear_gaps(L, nr, vs, vl);
          cleared = true;
        }
        lean_sync();
        LEAN_MARK(2);
        if (nr > 0 && lean_json_stage(L, nr, par, proj, fl JT_ARGS)) {
          defer = true;
          break;
        }
        LEAN_MARK(3);
        alive &= __ballot(l < 64 && ((L.match[(l >> 5) & 1] >> (l & 31)) & 1u));
        if (proj && (int)l < nr) {  // lane l keeps record l's (narrowed) value span
          vs = L.r_vs[l];
          vl = L.r_ve[l] - vs;
        }
        lean_sync();
        continue;
      }
      const bool rx = op == OP_REGEX;
      const uint32_t m = __builtin_amdgcn_readfirstlane(sd.m);
      if (!rx && m == 0 && checked) continue;  // an empty needle keeps every (UTF-8) value
      if (nr == 0) break;
      const uint32_t lo = L.r_vs[0], hi = L.r_ve[nr - 1];
      if constexpr (kJson) {  // the JSON kernel's scans see cleared gaps (OR of the words)
        if (!cleared) {
          clear_gaps(L, nr, vs, vl);
          cleared = true;
        }
      } else if (!rx && m > 0 && m < 4 && !cleared) {  // a short needle's dense hits use the block table
        lean_blk(L, nr, vs);
        cleared = true;
      }
      if (l == 0) {
        L.match[0] = 0;
        L.match[1] = 0;
      }
      const bool upper = sd.upper != 0;
      if (rx != kHasRx && (rx || !kHasCt)) {  // a stage this variant does not hold (the launcher never picks it)
        defer = true;
        break;
      }
      if constexpr (kHasRx) if (rx) {
        if (__builtin_amdgcn_readfirstlane(L.tt_stage) != s) {  // several regex stages: rows per stage
          const uint64_t* tt = (const uint64_t*)(a.blob + __builtin_amdgcn_readfirstlane(sd.tt));
          lean_sync();  // every lane is done with the previous rows
          for (uint32_t t = l; t < 256; t += kLeanThreads) L.tt[t] = tt[t];
        }
        lean_sync();
        LEAN_MARK(2);
        // (the regex scan reads value bytes only: its OR needs no gap clearing)
        const uint32_t orw = lean_regex(L, nr, lo, hi, sd.max_len, sd.s_bot, sd.s_mid, sd.acc1, sd.acc2);
        const bool high = lean_or(L.red, par, (orw & 0x80808080u) != 0u);  // also orders the match bits
        LEAN_MARK(3);
        if (!checked && high) defer = true;  // a non-ASCII value: exact UTF-8 / Unicode DFA path
        checked = true;
        const bool hit = l < 64 && ((L.match[(l >> 5) & 1] >> (l & 31)) & 1u);
        alive &= __ballot(sd.keep_match ? hit : !hit);
        lean_sync();  // match is rewritten by the next stage
        continue;
      }
      if constexpr (!kHasCt) {
        defer = true;
        break;
      } else {
      if (m > (uint32_t)kLeanNeedle) {
        defer = true;  // long needle: exact kernel
        break;
      }
      if (__builtin_amdgcn_readfirstlane(L.nd_res)) {
        const uint32_t o = __builtin_amdgcn_readfirstlane(sd.nd_off);
        for (uint32_t t = l; t < m; t += kLeanThreads) L.needle[t] = L.needles[o + t];
      } else {
        const uint8_t* nd = a.blob + __builtin_amdgcn_readfirstlane(sd.nd);
        for (uint32_t t = l; t < m; t += kLeanThreads) L.needle[t] = nd[t];
      }
      lean_sync();
      LEAN_MARK(2);
      bool high;
      if constexpr (kJson) {
        uint32_t orw;
        if (m >= 7) orw = lean_scan<0>(L, nr, lo, hi, nullptr, m, upper);
        else if (m >= 4) orw = lean_scan<1>(L, nr, lo, hi, nullptr, m, upper);
        else if (m > 0) orw = lean_scan<2>(L, nr, lo, hi, nullptr, m, upper);
        else orw = lean_scan<3>(L, nr, lo, hi, nullptr, m, upper);
        high = lean_or(L.red, par, (orw & 0x80808080u) != 0u);  // also orders the match bits
      } else {
        // gaps are not cleared: the count of high bytes over [lo, hi) against
        // the framing's count of those between values (equal <=> ASCII values)
        uint32_t cnt;
        if (m >= 7) cnt = lean_scan<0, true>(L, nr, lo, hi, nullptr, m, upper);
        else if (m >= 4) cnt = lean_scan<1, true>(L, nr, lo, hi, nullptr, m, upper);
        else if (m > 0) cnt = lean_scan<2, true>(L, nr, lo, hi, nullptr, m, upper);
        else cnt = lean_scan<3, true>(L, nr, lo, hi, nullptr, m, upper);
        if (!checked) {
          const uint32_t t = wave_sum(cnt);
          if ((l & 63u) == 0) L.hcw[l >> 6] = t;
        }
        (void)lean_or(L.red, par, false);  // orders the match bits and the counts
        high = !checked && L.hcw[0] + L.hcw[1] != L.ghigh;
      }
      if (!checked && high) defer = true;  // a non-ASCII value: exact UTF-8 path
      checked = true;
      if (m > 0) alive &= __ballot(l < 64 && ((L.match[(l >> 5) & 1] >> (l & 31)) & 1u));
      LEAN_MARK(3);
      lean_sync();  // match / needle are rewritten by the next stage
      }
    }
    // 4. survivors -> descriptors (stored by the next iteration's flush)
    p_b = b;
    p_defer = defer;
    p_kept = !defer && l < 64 && ((alive >> (l & 63)) & 1ull);
    if (p_kept) {
      p_idx = rb + __popcll(alive & ((1ull << l) - 1ull));
      p_d.src = al + rs;
      p_d.vpos = al + vs;
      p_d.kpos = tag ? al + kpos : 0;
      p_d.od = od;
      p_d.ts = ts;
      p_d.hdr = hdr;
      p_d.vlen = vl;
      p_d.klen = klen;
      p_d.ival = 0;
      p_d.mode = L.out_upper ? KM_UPPER : KM_COPY;
      p_d.has_key = tag;
      p_d.attr = attr;
      p_d.pad = 0;
    }
    p_base = base_offset;
    p_ts0 = first_ts;
    p_comp = comp;
    p_lod = lod_in;
    p_nkeep = (uint32_t)__popcll(alive);
    p_sec = sec_len;
    flush();
    LEAN_MARK(4);
#ifdef FSG_LEAN_TIMING
    lt_nb++;
#endif
    if (bn >= a.nbatches) break;
    b = bn;
  }
#ifdef FSG_LEAN_TIMING
  if (blockIdx.x < 2 && (threadIdx.x & 63u) == 0)
    printf("lean wg %u wave %u batches %lu wait %lu frame %lu gaps %lu scan %lu tail %lu | j1 %lu j1b %lu j2 %lu j2c %lu j3a %lu j3b %lu\n",
           blockIdx.x, threadIdx.x >> 6, (unsigned long)lt_nb, (unsigned long)lt_acc[0], (unsigned long)lt_acc[1],
           (unsigned long)lt_acc[2], (unsigned long)lt_acc[3], (unsigned long)lt_acc[4], (unsigned long)lt_acc[6],
           (unsigned long)lt_acc[7], (unsigned long)lt_acc[8], (unsigned long)lt_acc[9], (unsigned long)lt_acc[10],
           (unsigned long)lt_acc[11]);
#endif
}

// ---------------------------------------------------------------------------
// Flat substring path: a chain whose one scanning stage is a substring filter
// (filter / filter_init / filter_with_param: value.contains(needle), needle of
// 4..128 bytes) decouples streaming from the batch structure:
//   k_flat_scan   every byte of the slice once, as a flat array (headers and
//                 gaps included): one 16-byte chunk a lane, 8 rounds of 1 KiB
//                 per wave in flight; per chunk two bits: "a needle occurrence
//                 is anchored here" and "a byte >= 0x80 here", stored as one
//                 64-bit ballot per bitmap per round.  Needles of >= 7 bytes:
//                 every occurrence covers an aligned dword; each aligned dword
//                 is compared with the needle's 4-grams at offsets 0..3 and an
//                 occurrence is anchored at the chunk of its first covered
//                 aligned dword (starts in [16 C - 3, 16 C + 12]).  Needles of
//                 4..6 bytes: the 4-gram at each of the 16 positions, anchored
//                 at the chunk of its start.  Candidates are verified in full.
//   k_flat_decide one thread per batch (the k_chase walk): each record framed
//                 from its header bytes (one 24-byte read, varints decoded in
//                 registers, the trailing headers varint checked where the
//                 length says the record ends), then decided from the bits
//                 over its value: anchors whose every start lies in [vs, ve - m]
//                 match, edge chunks are re-checked on their bytes (the
//                 record's own lines); a high bit in a chunk of the value
//                 (exact at the edges: gap bytes hold varint continuation
//                 bytes) defers the batch.  Anything unusual (more than 64
//                 records, a varint over 4 bytes, framing that does not close)
//                 defers the batch to k_eval.
// The batch results (BatchStat, KeptRec) are those k_eval_lean writes.
// ---------------------------------------------------------------------------
#ifndef FSG_FLAT_ROUNDS
#define FSG_FLAT_ROUNDS 8
#endif
// a workgroup per 4 x kFlatRounds KiB (no cap: measured on MI355X, c2 eval
// 1.142 -> 1.067 ms with the nontemporal loads below, against 4096 workgroups)
#ifndef FSG_FLAT_GRID
#define FSG_FLAT_GRID 1000000
#endif
constexpr int kFlatRounds = FSG_FLAT_ROUNDS;  // 1 KiB rounds per wave in flight
__device__ __forceinline__ bool flat_verify(const uint8_t* s, uint64_t p, const uint8_t* nd, uint32_t m, bool upper) {
  for (uint32_t t = 0; t < m; t += 4) {
    uint32_t x = ld_u32_at(s + p + t);
    if (upper) x = swar_upper(x);
    const uint32_t k = m - t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (m - t))) - 1u);
    if ((x ^ ld_u32_at(nd + t)) & k) return false;
  }
  return true;
}
// JSON-interesting bytes of a dword (0x80 per byte): '"', '\\', < 0x20, >= 0x80;
// special: the same without the quote
__device__ __forceinline__ uint32_t fj_special(uint32_t w) {
  return zbytes(w ^ 0x5C5C5C5Cu) | zbytes(w & 0xE0E0E0E0u) | (w & 0x80808080u);
}
__device__ __forceinline__ uint32_t fj_bytes(uint32_t w) { return zbytes(w ^ 0x22222222u) | fj_special(w); }
// kLong: m >= 7, aligned dwords against the 4 offsets.  kJson: the second word
// of a round holds the chunks with a JSON-interesting byte (fj_bytes) instead
// of the high bytes (the flat JSON path); kNone: no substring stage (occurrence word 0)
template <bool kLong, bool kJson = false, bool kNone = false>
__global__ __launch_bounds__(256) void k_flat_scan(EvalArgs a, uint32_t stage) {
  // a wave's round staged in LDS when it holds candidates: the needle is
  // verified from there (a global re-read per candidate stalled the stream)
  __shared__ uint32_t rbuf[4][256 + 4];  // (+4: the alignbyte of the last dword reads one past)
  __shared__ uint32_t ndw[kLeanNeedle / 4 + 1];
  const StageDesc& sd = a.chain->st[kNone ? 0 : stage];
  const uint32_t m = kNone ? 4u : sd.needle_len;
  const bool upper = !kNone && sd.in_type == VT_SRC_UPPER;
  const uint8_t* nd = a.blob + sd.needle;
  uint32_t rot[4] = {0, 0, 0, 0};
  if (!kNone) {
    for (uint32_t t = threadIdx.x; t < (m + 3) / 4; t += 256) ndw[t] = ld_u32_at(nd + 4 * t);
    __syncthreads();
#pragma unroll
    for (int d = 0; d < 4; d++) rot[d] = ld_u32_at(nd + (kLong ? d : 0));
  }
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t* rb = rbuf[wv];
  const uint64_t nrounds = a.fbm_words;  // 1 KiB rounds of the slice
  const uint64_t w0 = (uint64_t)blockIdx.x * 4 + wv;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  // the two bitmaps interleaved per 1 KiB round: occurrence word r at fbm[2r],
  // high-byte word at fbm[2r + 1] (k_flat_decide reads both from one line)
  ulonglong2* bm2 = (ulonglong2*)a.fbm;
  for (uint64_t r0 = w0 * kFlatRounds; r0 < nrounds; r0 += nw * kFlatRounds) {
    uint4 v[kFlatRounds];
    uint32_t nx[kFlatRounds];
#pragma unroll
    for (int i = 0; i < kFlatRounds; i++) {  // every round's loads in flight before the first use
      const uint64_t c = (r0 + i) * 1024 + lane * 16;
#ifndef FSG_FLAT_NO_NT  // streamed once: nontemporal, the later kernels' lines stay cached
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      v[i] = make_uint4(0, 0, 0, 0);
      if (r0 + i < nrounds) {
        const v4u t = __builtin_nontemporal_load((const v4u*)(a.slice + c));
        v[i] = make_uint4(t.x, t.y, t.z, t.w);
      }
#else
      v[i] = r0 + i < nrounds ? *(const uint4*)(a.slice + c) : make_uint4(0, 0, 0, 0);
#endif
      if (!kLong) nx[i] = r0 + i < nrounds ? *(const uint32_t*)(a.slice + c + 16) : 0u;
    }
#pragma unroll
    for (int i = 0; i < kFlatRounds; i++) {
      if (r0 + i >= nrounds) break;  // uniform
      const uint64_t R = (r0 + i) * 1024;
      uint32_t w[5] = {v[i].x, v[i].y, v[i].z, v[i].w, kLong ? 0u : nx[i]};
      const bool high = kJson ? ((fj_bytes(w[0]) | fj_bytes(w[1]) | fj_bytes(w[2]) | fj_bytes(w[3])) != 0u)
                              : ((w[0] | w[1] | w[2] | w[3]) & 0x80808080u) != 0u;
      if (kNone) {
        const uint64_t hh = __ballot(high);
        if (lane == 0) bm2[r0 + i] = make_ulonglong2(0ull, hh);
        continue;
      }
      if (upper) {
#pragma unroll
        for (int k = 0; k < 5; k++) w[k] = swar_upper(w[k]);
      }
      // min over the compare differences: zero iff some 4-gram hits (the
      // candidate masks are built only when a lane of the wave has one)
      uint32_t z = 0xFFFFFFFFu;
      if (kLong) {
#pragma unroll
        for (int k = 0; k < 4; k++) z = min(z, min(min(w[k] ^ rot[0], w[k] ^ rot[1]), min(w[k] ^ rot[2], w[k] ^ rot[3])));
      } else {
#pragma unroll
        for (int j = 0; j < 16; j++)
          z = min(z, ((j & 3) ? __builtin_amdgcn_alignbyte(w[(j >> 2) + 1], w[j >> 2], (uint32_t)(j & 3)) : w[j >> 2]) ^ rot[0]);
      }
      bool hit = false;
      if (__ballot(z == 0u)) {  // rare: stage the round, verify every candidate from LDS
        // candidates: bit (4k + d) = aligned dword k against the needle at
        // offset d (kLong), bit j = the 4-gram at position j (else)
        uint32_t cm = 0;
        if (kLong) {
#pragma unroll
          for (int k = 0; k < 4; k++)
#pragma unroll
            for (int d = 0; d < 4; d++) cm |= (uint32_t)(w[k] == rot[d]) << (4 * k + d);
        } else {
#pragma unroll
          for (int j = 0; j < 16; j++)
            cm |= (uint32_t)(((j & 3) ? __builtin_amdgcn_alignbyte(w[(j >> 2) + 1], w[j >> 2], (uint32_t)(j & 3)) : w[j >> 2]) ==
                             rot[0]) << j;
        }
        rb[4 * lane] = v[i].x;
        rb[4 * lane + 1] = v[i].y;
        rb[4 * lane + 2] = v[i].z;
        rb[4 * lane + 3] = v[i].w;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        while (cm && !hit) {
          const uint32_t j = (uint32_t)__builtin_ctz(cm);
          cm &= cm - 1;
          const int64_t rel = kLong ? (int64_t)(16 * lane + 4 * (j >> 2)) - (int64_t)(j & 3) : (int64_t)(16 * lane + j);
          if (rel < 0 || rel + m > 1024) {  // beyond the staged round: from memory
            if ((int64_t)R + rel < 0) continue;  // a start before the slice (round 0): no occurrence
            hit = flat_verify(a.slice, R + rel, nd, m, upper);
            continue;
          }
          bool eq = true;
          for (uint32_t t = 0; t < m && eq; t += 4) {
            const uint32_t q = (uint32_t)rel + t;
            uint32_t x = __builtin_amdgcn_alignbyte(rb[(q >> 2) + 1], rb[q >> 2], q & 3u);
            if (upper) x = swar_upper(x);
            const uint32_t k = m - t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (m - t))) - 1u);
            eq = ((x ^ ndw[t >> 2]) & k) == 0u;
          }
          hit = eq;
        }
      }
      const uint64_t hb = __ballot(hit), hh = __ballot(high);
      if (lane == 0) bm2[r0 + i] = make_ulonglong2(hb, hh);
    }
  }
}
// bm: the interleaved bitmaps offset by the one wanted (0 occurrences, 1 high bytes): word w at bm[kS w]
// (kS = 2; the flat JSON path interleaves four words per round)
template <int kS = 2>
__device__ __forceinline__ bool bm_bit(const unsigned long long* bm, uint64_t c) { return (bm[kS * (c >> 6)] >> (c & 63)) & 1ull; }
// bits [c0, c1) of a bitmap: any set
template <int kS = 2>
__device__ __forceinline__ bool flat_any(const unsigned long long* bm, uint64_t c0, uint64_t c1) {
  for (uint64_t c = c0; c < c1;) {
    const uint64_t w = c >> 6, lo = c & 63;
    const uint64_t hi = (c1 - (w << 6)) < 64 ? (c1 - (w << 6)) : 64;
    const uint64_t mask = (hi == 64 ? ~0ull : ((1ull << hi) - 1ull)) & ~((1ull << lo) - 1ull);
    if (bm[kS * w] & mask) return true;
    c = (w + 1) << 6;
  }
  return false;
}
// a varint of at most 4 bytes at the start of w: its length (0: longer) and zigzag value (varint.rs:43-66)
__device__ __forceinline__ uint32_t var4(uint32_t w, int64_t& val) {
  const uint32_t term = ~w & 0x80808080u;
  const uint32_t nb = term ? (((uint32_t)__builtin_ctz(term)) >> 3) + 1 : 0u;
  const uint32_t y = nb == 4 ? w : (w & ((1u << (8 * nb)) - 1u));
  const uint32_t u = (y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u) | ((y >> 3) & 0xFE00000u);
  val = (int64_t)(u >> 1) ^ -(int64_t)(u & 1u);
  return nb;
}
// the 24 header bytes of a record at absolute q, as aligned dwords from q & ~3
struct FlatHdr {
  uint32_t x[6];
};
__device__ __forceinline__ FlatHdr flat_hdr(const uint8_t* S, uint64_t q) {
  FlatHdr h;
  const uint64_t a0 = q & ~3ull;
#pragma unroll
  for (int k = 0; k < 6; k++) h.x[k] = *(const uint32_t*)(S + a0 + 4 * k);
  return h;
}
__device__ __forceinline__ uint32_t flat_at(const FlatHdr& h, uint32_t o) {  // bytes [o, o + 4), o < 20
  const uint32_t d = o >> 2;
  uint32_t lo = h.x[0], hi = h.x[1];
#pragma unroll
  for (uint32_t k = 1; k < 5; k++)
    if (d == k) {
      lo = h.x[k];
      hi = h.x[k + 1];
    }
  return __builtin_amdgcn_alignbyte(hi, lo, o & 3u);
}
// Software-pipelined walk: record n + 1's header load is issued as soon as
// record n's length varint says where it starts, together with record n's
// trailer, bitmap words and edge chunks, so one memory round trip per record
// sits on the thread's critical path (the plain walk had five).
template <bool kLong>
__global__ __launch_bounds__(256) void k_flat_decide(EvalArgs a, uint32_t stage) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= a.nbatches) return;
  const StageDesc& sd = a.chain->st[stage];
  const uint32_t m = sd.needle_len;
  const bool upper = sd.in_type == VT_SRC_UPPER;
  const bool out_upper = a.chain->out_type == VT_SRC_UPPER;
  const uint8_t* nd = a.blob + sd.needle;
  const unsigned long long* hit_bm = a.fbm;  // interleaved (k_flat_scan): hit word w at [2 w], high at [2 w + 1]
  const unsigned long long* hi_bm = a.fbm + 1;
  const uint8_t* S = a.slice;
  const uint64_t pos = a.bpos[b];
  // output sizes for a first surviving batch 0 (k_size skips BF_ROWDONE batches then)
  const int64_t rel0 = (int64_t)rd_be(S + a.bpos[0], 8) - (int64_t)rd_be(S + pos, 8);
  uint64_t rbytes = 0;
  const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
  const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
  const uint64_t al = pos & ~15ull;
  uint64_t wl = nxt > al ? nxt - al : 0;
  if (wl > (uint64_t)kLeanWin) wl = kLeanWin;
  const uint64_t wlen = (wl + 15) & ~15ull;
  const uint32_t batch_len = __builtin_bswap32(ld_u32_at(S + pos + 8));
  const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
  const uint64_t sec_len = sec_end - sec0;
  const int32_t count = sec_len >= 4 ? (int32_t)__builtin_bswap32(ld_u32_at(S + sec0)) : -1;
  bool ok = sec_len >= 4 && sec_end - al <= wlen && count >= 0 && count <= kLeanMaxR && (uint64_t)count == rn;
  uint32_t nkeep = 0;
  uint64_t q = sec0 + 4;  // absolute start of record n
  FlatHdr H = flat_hdr(S, ok && count > 0 ? q : sec0);
  for (int32_t n = 0; ok && n < count; n++) {
    uint32_t o = (uint32_t)(q & 3), nb;
    int64_t len, ts, od, kl = 0, vlen, hdr;
    nb = var4(flat_at(H, o), len);
    ok = nb != 0 && len >= 0;
    const uint64_t end = q + nb + (uint64_t)len;  // where the record ends (Record::decode's length)
    ok = ok && end <= sec_end;
    if (!ok) break;
    const FlatHdr Hn = flat_hdr(S, n + 1 < count ? end : q);  // the next record's header, in flight now
    o += nb;
    const uint8_t attr = (uint8_t)flat_at(H, o);
    o += 1;
    nb = var4(flat_at(H, o), ts);
    ok = nb != 0;
    o += nb;
    nb = var4(flat_at(H, o), od);
    ok = ok && nb != 0;
    o += nb;
    const uint8_t tag = (uint8_t)flat_at(H, o);
    o += 1;
    ok = ok && tag <= 1;
    if (!ok) break;
    uint64_t p = (q & ~3ull) + o, kpos = 0;
    uint32_t klen = 0;
    if (tag == 1) {
      nb = var4(flat_at(H, o), kl);
      ok = nb != 0 && kl >= 0;
      p += nb;
      kpos = p;
      klen = (uint32_t)kl;
      p += klen;
    }
    nb = var4(tag == 1 ? ld_u32_at(S + p) : flat_at(H, o), vlen);
    ok = ok && nb != 0 && vlen >= 0;
    const uint64_t va = p + nb, ve = va + (uint64_t)vlen;
    ok = ok && ve <= end;
    if (!ok) break;
    // every load of this record at once: trailer, bitmap words, edge chunks
    const uint32_t tw = ld_u32_at(S + ve);
    const uint64_t c0 = va >> 4, c1 = (ve + 15) >> 4, i0 = (va + 15) >> 4, i1 = ve >> 4;
    const uint64_t wb = c0 >> 6;  // first bitmap word touching the value
    const ulonglong2 bw0 = *(const ulonglong2*)(a.fbm + 2 * wb), bw1 = *(const ulonglong2*)(a.fbm + 2 * wb + 2);
    const unsigned long long mb0 = bw0.x, hb0 = bw0.y, mb1 = bw1.x, hb1 = bw1.y;
    const uint4 ea = *(const uint4*)(S + (c0 << 4));
    const uint4 eb = *(const uint4*)(S + (((ve ? ve - 1 : 0) >> 4) << 4));
    nb = var4(tw, hdr);
    ok = nb != 0 && ve + nb == end;
    if (!ok) break;
    // bits [x0, x1) of a bitmap from the two loaded words (a longer range reads more)
    auto bits_any = [&](const unsigned long long* bm, unsigned long long w0v, unsigned long long w1v, uint64_t x0,
                        uint64_t x1) {
      if (x1 <= x0) return false;
      if (x1 > (wb + 2) << 6) return flat_any(bm, x0, x1);
      const uint64_t lo = x0 - (wb << 6), hi = x1 - (wb << 6);  // in [0, 128]
      const unsigned long long m0 = (lo < 64 ? (~0ull << lo) : 0ull) & (hi >= 64 ? ~0ull : ((1ull << hi) - 1ull));
      const unsigned long long m1 = (hi > 64 ? (hi >= 128 ? ~0ull : ((1ull << (hi - 64)) - 1ull)) : 0ull) &
                                    (lo > 64 ? (~0ull << (lo - 64)) : ~0ull);
      return ((w0v & m0) | (w1v & m1)) != 0ull;
    };
    auto bit = [&](unsigned long long w0v, unsigned long long w1v, uint64_t c) {
      const uint64_t r = c - (wb << 6);
      return r < 64 ? ((w0v >> r) & 1ull) != 0ull : r < 128 ? ((w1v >> (r - 64)) & 1ull) != 0ull : false;
    };
    // bytes >= 0x80 in the value: chunks inside it by their bits, the edge
    // chunks (which hold gap bytes) by their bytes
    if (ve > va) {
      bool hi = bits_any(hi_bm, hb0, hb1, i0, i1);
      auto hi_edge = [&](const uint4& u, uint64_t c) {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
        uint32_t f = 0;
#pragma unroll
        for (int k = 0; k < 4; k++)
          f |= w[k] & bytes_in((uint32_t)(((c << 4) + 4 * k) - al), (uint32_t)(va - al), (uint32_t)(ve - al));
        return (f & 0x80808080u) != 0u;
      };
      if (!hi && c0 < i0) hi = hi_edge(ea, c0);
      if (!hi && i1 < c1 && (i1 >= i0 || c0 != i1)) hi = hi_edge(eb, i1);
      ok = !hi;
      if (!ok) break;
    }
    // an occurrence starting in [va, ve - m]
    bool match = false;
    if ((uint64_t)vlen >= m) {
      const uint64_t sl = ve - m;  // last valid start
      // anchors of chunk C: starts [16C - 3, 16C + 12] (kLong), [16C, 16C + 15]
      const uint64_t blo = kLong ? 3 : 0, bhi = kLong ? 12 : 15;
      const uint64_t j0 = (va + blo + 15) >> 4;                   // first chunk whose every start is >= va
      const uint64_t j1 = sl >= bhi ? ((sl - bhi) >> 4) + 1 : 0;  // chunks < j1: every start <= sl
      match = j0 < j1 && bits_any(hit_bm, mb0, mb1, j0, j1);
      if (!match) {  // chunks holding some valid start but not all: the bytes decide
        const uint64_t e0 = va >= bhi ? (va - bhi + 15) >> 4 : 0, e1 = (sl + blo) >> 4;
        for (uint64_t c = e0; c <= e1 && !match; c++) {
          if (c >= j0 && c < j1) {
            c = j1 - 1;
            continue;
          }
          if (c >= (wb << 6) && c < ((wb + 2) << 6) ? !bit(mb0, mb1, c) : !bm_bit(hit_bm, c)) continue;  // the loaded words
          const uint64_t lo = (c << 4) >= va + blo ? (c << 4) - blo : va;
          const uint64_t hi = (c << 4) + bhi <= sl ? (c << 4) + bhi : sl;
          for (uint64_t s0 = lo; s0 <= hi && !match; s0++) match = flat_verify(S, s0, nd, m, upper);
        }
      }
    }
    if (match) {
      KeptRec d;
      d.src = q;
      d.vpos = va;
      d.kpos = tag ? kpos : 0;
      d.od = od;
      d.ts = ts;
      d.hdr = hdr;
      d.vlen = (uint32_t)vlen;
      d.klen = klen;
      d.ival = 0;
      d.mode = out_upper ? KM_UPPER : KM_COPY;
      d.has_key = tag;
      d.attr = attr;
      d.pad = 0;
      rbytes += copy_out_size(d, rel0);
      a.desc[rb + nkeep++] = d;
    }
    q = end;
    H = Hn;
  }
  ok = ok && q == sec_end;
  if (!ok) {  // the exact kernel frames and evaluates this batch (no record starts from here)
    a.rend[b] = 0xFFFFu;
    const uint32_t i = atomicAdd(&a.list[0], 1u);
    a.list[1 + i] = b;
    return;
  }
  const uint8_t* h = S + pos;  // batch header (file format, batch.rs:163-180)
  BatchStat st = {};
  st.base_offset = (int64_t)rd_be(h, 8);
  st.lod_in = (int32_t)rd_be(h + 23, 4);
  st.first_ts = (int64_t)rd_be(h + 27, 8);
  st.comp = (uint32_t)h[22] & 7u;
  st.flags = BF_LAST_STAGE;
  if (a.rows) {
    ScanRow row = {};
    row.rec_bytes = rbytes;
    row.nonempty = nkeep ? 1 : 0;
    row.lod = (uint64_t)(int64_t)(st.lod_in + 1);
    row.nrec = nkeep;
    row.bytes_in = sec_len;
    row.recs_out = nkeep;
    a.rows[b] = row;
    st.flags |= BF_ROWDONE;
  }
  st.nkeep = st.nout = nkeep;
  st.sec_len = (uint32_t)sec_len;
  st.err_stage = 0xFFFFFFFFu;
  a.bstat[b] = st;
}

// ---------------------------------------------------------------------------
// Flat JSON path: filter_json (serde_json::from_slice::<StructuredLog>,
// smartmodule/examples/filter_json/src/lib.rs:54-70) and the field projection
// (map_json_project), with at most one substring stage and uppercase maps
// beside them.  k_flat_scan<., kJson> streams the slice once and marks every
// 16-byte chunk holding a JSON-interesting byte ('"', '\\', < 0x20, >= 0x80),
// beside the needle's occurrence anchors when there is a substring stage;
// k_fj_decide walks each batch's records with one thread (k_flat_decide's
// pipelined framing) and parses every value as a flat object: bytes outside
// strings one by one, strings by their first interesting byte, the clean
// chunks between skipped with the bitmap (a clean chunk holds no quote, so the
// string goes on through it).  Accepted is what the lean kernel's token DFA
// accepts (fsg_json_dfa.h): { "key": value (, "key": value)* } with ' ' as the
// only whitespace, keys and strings without escapes / control / high bytes,
// level a LogLevel variant string, message a string, other values a string, a
// JSON number or true / false / null, each field once; with a projection
// (Map<String, Value>: every number is parsed) numbers are integers of at most
// 18 characters other than -0, and the last member named by the field is the
// output span.  Every byte of an accepted value was either examined or lies in
// a clean chunk, so the value is ASCII (from_utf8 cannot fail).  Any other
// record, and framing k_flat_decide would not take, defers the batch to k_eval.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t u4_dw(uint4 v, uint32_t k) {  // (values, not lvalues: no memory select)
  const uint32_t x = v.x, y = v.y, z = v.z, w = v.w;
  return (k & 2u) ? ((k & 1u) ? w : z) : ((k & 1u) ? y : x);
}
// 16 bits: the JSON-interesting bytes of a chunk
__device__ __forceinline__ uint32_t fj_mask(const uint4& v) {
  return nib4(fj_bytes(v.x)) | (nib4(fj_bytes(v.y)) << 4) | (nib4(fj_bytes(v.z)) << 8) | (nib4(fj_bytes(v.w)) << 12);
}
__device__ __forceinline__ uint4 sel4(uint4 a0, uint4 a1, uint4 a2, uint4 a3, uint32_t k) {
  uint4 r;
  r.x = u4_dw(make_uint4(a0.x, a1.x, a2.x, a3.x), k);
  r.y = u4_dw(make_uint4(a0.y, a1.y, a2.y, a3.y), k);
  r.z = u4_dw(make_uint4(a0.z, a1.z, a2.z, a3.z), k);
  r.w = u4_dw(make_uint4(a0.w, a1.w, a2.w, a3.w), k);
  return r;
}
// A record's value as the walk sees it: the 64 bytes from its first chunk (the
// head window) and the 80 bytes up to its last chunk (the tail window), staged
// in this thread's LDS slot, every other byte from memory (rare: members in the
// middle of a long value), and the interesting-chunk bitmap for strings that
// run between the windows.  Positions are 32-bit offsets from B (the batch's
// 16-aligned start); the windows start at chunk boundaries.
constexpr uint32_t kFjHead = 64, kFjTail = 80, kFjSlot = kFjHead + kFjTail;  // bytes per thread in LDS
struct FjCur {
  const uint8_t* B;
  uint8_t* W;                     // this thread's LDS slot: head window, then tail window
  const unsigned long long* fbm;  // two words per round r: occurrences, interesting at fbm[2 r], fbm[2 r + 1]
  uint64_t cb;                    // B's chunk index in the slice
  uint32_t hb, tb;                // offsets of the head / tail windows
  uint32_t c;                     // chunk of v (the current chunk) and m its interesting bytes
  uint4 v;
  uint32_t m;
  bool mv;                        // m computed
  uint64_t wb;                    // the slice rounds wb, wb + 1 preloaded: interesting words j0, j1
  unsigned long long j0, j1;
  // the slot offset of position p, or >= kFjSlot outside both windows
  __device__ __forceinline__ uint32_t loff(uint32_t p) const {
    const uint32_t dh = p - hb, dt = p - tb;
    return dh < kFjHead ? dh : dt < kFjTail ? kFjHead + dt : kFjSlot;
  }
  __device__ __forceinline__ uint4 chunk(uint32_t ci) {
    if (ci != c) {
      const uint32_t o = loff(16u * ci);
      if (o < kFjSlot) v = *(const uint4*)(W + o);
      else v = *(const uint4*)(B + 16u * ci);
      c = ci;
      mv = false;
    }
    return v;
  }
  __device__ __forceinline__ uint32_t mask(uint32_t ci) {  // interesting bytes of chunk ci
    chunk(ci);
    if (!mv) {
      m = fj_mask(v);
      mv = true;
    }
    return m;
  }
  __device__ __forceinline__ uint32_t at(uint32_t p) {
    const uint32_t o = loff(p);
    if (o < kFjSlot) return W[o];
    return B[p];
  }
  // the n <= 8 bytes at p as a little-endian word
  __device__ __forceinline__ uint64_t word(uint32_t p, uint32_t n) {
    const uint32_t o = loff(p);
    uint64_t w = 0;
    if (o < kFjHead ? o + n <= kFjHead : o + n <= kFjSlot) {  // inside one window: three aligned dwords
      const uint32_t* d = (const uint32_t*)(W + (o & ~3u));
      const uint32_t e0 = d[0], e1 = d[1], e2 = d[2], sh = o & 3u;
      w = (uint64_t)__builtin_amdgcn_alignbyte(e1, e0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(e2, e1, sh) << 32);
    } else {
      for (uint32_t i = 0; i < n; i++) w |= (uint64_t)at(p + i) << (8 * i);
    }
    return n >= 8 ? w : (w & ((1ull << (8 * n)) - 1ull));
  }
  // the first position >= p (< ve) holding a byte that is not an ASCII digit, or ve
  __device__ __forceinline__ uint32_t digits_end(uint32_t p, uint32_t ve) {
    for (;;) {
      const uint4 u = chunk(p >> 4);
      uint32_t nd = 0;
#pragma unroll
      for (int d = 0; d < 4; d++) {
        const uint32_t w = u4_dw(u, (uint32_t)d), x = w & 0x7F7F7F7Fu;
        const uint32_t dig = (x + 0x50505050u) & ~(x + 0x46464646u) & ~w & 0x80808080u;  // 0x30 <= b <= 0x39
        nd |= nib4(~dig & 0x80808080u) << (4 * d);
      }
      nd &= 0xFFFFu << (p & 15u);
      if (nd) {
        const uint32_t x = (p & ~15u) + (uint32_t)__builtin_ctz(nd);
        return x < ve ? x : ve;
      }
      p = (p | 15u) + 1;
      if (p >= ve) return ve;
    }
  }
  // the first chunk in [ci, lim) with an interesting byte, or lim
  __device__ __forceinline__ uint32_t next(uint32_t ci, uint32_t lim) {
    while (ci < lim) {
      const uint64_t ac = cb + ci, r = ac >> 6;
      unsigned long long w = r == wb ? j0 : r == wb + 1 ? j1 : fbm[2 * r + 1];
      w &= ~0ull << (ac & 63u);
      if (w) {
        const uint32_t x = ci + (uint32_t)__builtin_ctzll(w) - (uint32_t)(ac & 63u);
        return x < lim ? x : lim;
      }
      ci += 64u - (uint32_t)(ac & 63u);
    }
    return lim;
  }
};
// the closing quote of the string whose bytes start at s (before ve), or ~0u:
// an escape, a control or high byte, or no quote before ve
__device__ __forceinline__ uint32_t fj_str_end(FjCur& C, uint32_t s, uint32_t ve) {
  uint32_t ci = s >> 4;
  uint32_t m = C.mask(ci) & (0xFFFFu << (s & 15u));
  const uint32_t lim = (ve + 15) >> 4;
  while (!m) {
    ci = C.next(ci + 1, lim);
    if (ci >= lim) return ~0u;
    m = C.mask(ci);
  }
  const uint32_t x = (ci << 4) + (uint32_t)__builtin_ctz(m);
  if (x >= ve || ((u4_dw(C.v, (x >> 2) & 3u) >> (8u * (x & 3u))) & 0xFFu) != 0x22u) return ~0u;
  return x;
}
constexpr uint64_t fj_k(const char* t) {
  uint64_t v = 0;
  for (int i = 0; t[i]; i++) v |= (uint64_t)(uint8_t)t[i] << (8 * i);
  return v;
}
__device__ __forceinline__ bool fj_digit(uint32_t c) { return c - 0x30u < 10u; }
// one record's value [va, ve) (offsets from C.B); false: the batch goes to
// k_eval.  fj: the StructuredLog filter (lvl = 1 << LogLevel index); proj: the
// field fld[0, fl) (fw: as a word when fl <= 8), its last member's value span
// [fs, fe) when found
__device__ __forceinline__ bool fj_walk(FjCur& C, uint32_t va, uint32_t ve, bool fj, bool proj, const uint8_t* fld,
                                        uint32_t fl, uint64_t fw, uint32_t& lvl, bool& found, uint32_t& fs,
                                        uint32_t& fe) {
  uint32_t p = va;
  uint32_t nlv = 0, nmsg = 0;
  lvl = 0;
  found = false;
  auto sp = [&]() {
    while (p < ve && C.at(p) == 0x20u) p++;
  };
  sp();
  if (p >= ve || C.at(p) != '{') return false;
  p++;
  for (;;) {
    sp();
    if (p >= ve || C.at(p) != '"') return false;  // (an empty object goes to k_eval too)
    const uint32_t k0 = p + 1, k1 = fj_str_end(C, k0, ve);
    if (k1 == ~0u) return false;
    const uint32_t kn = k1 - k0;
    p = k1 + 1;
    if (p + 2 <= ve && (uint32_t)C.word(p, 2) == 0x223Au) {  // `:"` (the common layout): one word
      p++;
    } else {
      sp();
      if (p >= ve || C.at(p) != ':') return false;
      p++;
      sp();
      if (p >= ve) return false;
    }
    uint32_t key = 0;  // 1 level, 2 message
    if (fj && (kn == 5 || kn == 7)) {
      const uint64_t w = C.word(k0, kn);
      key = kn == 5 && w == fj_k("level") ? 1u : kn == 7 && w == fj_k("message") ? 2u : 0u;
    }
    bool fhit = false;
    if (proj && kn == fl && fl <= 8) {
      fhit = C.word(k0, fl) == fw;
    } else if (proj && kn == fl) {
      fhit = true;
      for (uint32_t t = 0; fhit && t < fl; t += 4) {
        const uint32_t mk = fl - t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (fl - t))) - 1u);
        fhit = ((ld_u32_at(C.B + k0 + t) ^ ld_u32_at(fld + t)) & mk) == 0u;
      }
    }
    const uint32_t v0 = p;
    const uint32_t c = C.at(p);
    if (c == '"') {
      const uint32_t s1 = fj_str_end(C, p + 1, ve);
      if (s1 == ~0u) return false;
      if (key == 1) {
        const uint32_t n = s1 - p - 1;
        const uint64_t w = n == 4 || n == 5 ? C.word(p + 1, n) : 0ull;
        const uint32_t v = n == 5 && w == fj_k("debug") ? 1u : n == 4 && w == fj_k("info") ? 2u
                         : n == 4 && w == fj_k("warn") ? 4u : n == 5 && w == fj_k("error") ? 8u : 0u;
        if (!v || nlv++) return false;  // unknown variant / duplicate field: serde errors
        lvl = v;
      } else if (key == 2) {
        if (nmsg++) return false;
      }
      p = s1 + 1;
    } else {
      if (key) return false;  // level / message not a string: invalid type
      if (c == '-' || fj_digit(c)) {
        const bool neg = c == '-';
        if (neg) p++;
        if (p >= ve) return false;
        const uint32_t d = C.at(p);
        if (d == '0') {
          p++;
          if (p < ve && fj_digit(C.at(p))) return false;  // a leading zero
        } else if (fj_digit(d)) {
          p = C.digits_end(p + 1, ve);
        } else {
          return false;
        }
        bool real = false;
        if (p < ve && C.at(p) == '.') {
          real = true;
          if (++p >= ve || !fj_digit(C.at(p))) return false;
          p = C.digits_end(p + 1, ve);
        }
        if (p < ve && (C.at(p) | 0x20u) == 'e') {
          real = true;
          if (++p < ve && (C.at(p) == '+' || C.at(p) == '-')) p++;
          if (p >= ve || !fj_digit(C.at(p))) return false;
          p = C.digits_end(p + 1, ve);
        }
        // a projection parses every number into a Value: integers of <= 18
        // characters only (no f64 reading, no -0)
        if (proj && (real || p - v0 > 18 || (neg && p - v0 == 2 && d == '0'))) return false;
      } else {
        const uint32_t n = c == 'f' ? 5u : 4u;
        if (p + n > ve) return false;
        const uint64_t w = C.word(p, n);
        if (!(c == 't' ? w == fj_k("true") : c == 'f' ? w == fj_k("false") : c == 'n' && w == fj_k("null")))
          return false;
        p += n;
      }
    }
    if (fhit) {
      found = true;
      fs = v0;
      fe = p;
    }
    if (p + 2 <= ve && (uint32_t)C.word(p, 2) == 0x222Cu) {  // `,"` (the common layout): the next key
      p++;
      continue;
    }
    sp();
    if (p >= ve) return false;
    const uint32_t e = C.at(p++);
    if (e == '}') break;
    if (e != ',') return false;
  }
  sp();
  if (p != ve) return false;                       // trailing characters
  return !fj || (nlv == 1 && nmsg == 1);           // a missing field: serde error
}
// one record's framing (Record::decode, data.rs:534-562) from its header bytes
struct FjRec {
  uint64_t q, end, va, ve, kpos;
  int64_t ts, od;
  uint32_t klen;
  uint8_t attr, tag;
  bool ok;
};
__device__ __forceinline__ FjRec fj_frame(const uint8_t* S, const FlatHdr& H, uint64_t q, uint64_t sec_end,
                                          bool allow_empty = false) {
  FjRec r;
  r.q = q;
  r.kpos = 0;
  r.klen = 0;
  r.ts = r.od = 0;
  r.attr = r.tag = 0;
  r.va = r.ve = r.end = q;
  uint32_t o = (uint32_t)(q & 3), nb;
  int64_t len, kl = 0, vlen;
  nb = var4(flat_at(H, o), len);
  r.ok = nb != 0 && len >= 0;
  r.end = q + nb + (uint64_t)len;  // where the record ends (Record::decode's length)
  r.ok = r.ok && r.end <= sec_end;
  if (!r.ok) return r;
  o += nb;
  r.attr = (uint8_t)flat_at(H, o);
  o += 1;
  nb = var4(flat_at(H, o), r.ts);
  r.ok = nb != 0;
  o += nb;
  nb = var4(flat_at(H, o), r.od);
  r.ok = r.ok && nb != 0;
  o += nb;
  r.tag = (uint8_t)flat_at(H, o);
  o += 1;
  r.ok = r.ok && r.tag <= 1;
  if (!r.ok) return r;
  uint64_t p = (q & ~3ull) + o;
  if (r.tag == 1) {
    nb = var4(flat_at(H, o), kl);
    r.ok = nb != 0 && kl >= 0;
    p += nb;
    r.kpos = p;
    r.klen = (uint32_t)kl;
    p += r.klen;
  }
  nb = var4(r.tag == 1 ? ld_u32_at(S + p) : flat_at(H, o), vlen);
  r.ok = r.ok && nb != 0 && vlen >= 0;
  r.va = p + nb;
  r.ve = r.va + (uint64_t)vlen;
  r.ok = r.ok && r.ve <= r.end && (allow_empty || r.ve > r.va);  // (JSON: an empty value is a serde error, k_eval)
  return r;
}
// ---------------------------------------------------------------------------
// Flat regex path: a chain whose one scanning stage is a bounded regex filter
// (regex-filter / filter_regex, smartmodule/regex-filter/src/lib.rs:24-28:
// Regex::is_match on the value) whose ASCII DFA has <= 16 states and a longest
// match of <= 17 bytes (no word boundaries, no multi-line anchors: the compiler
// then gives a restart state s_mid that needs no previous byte).
//   k_rx_scan    every 16-byte chunk C of the slice once, as a flat array: the
//                DFA from s_mid over the chunk's window [16 C - ctx, 16 C + 16)
//                (ctx = 4 ceil((max_len - 1) / 4) bytes of the previous chunk);
//                bit "the sticky accept was reached in the window" and bit "a
//                byte >= 0x80 in the chunk", one 64-bit ballot each per 1 KiB
//                round (k_flat_scan's interleaved layout)
//   k_rx_decide  one thread per batch (k_flat_decide's framing): a record
//                matches when an interior chunk (window inside the value) has
//                the bit; the chunks whose windows leave the value (its first
//                chunks, its last) are decided by an exact scan of their bytes
//                (from s_bot at the value start, acceptance at its end), which
//                an anchor-free pattern (s_bot = s_mid, no end-only accept)
//                skips when their bits are clear.  Every match of at most
//                max_len bytes lies in the window of the chunk holding its last
//                byte, so the bits plus the edge scans see every match.
// ---------------------------------------------------------------------------
// The rows sit in LDS as 32 interleaved copies (row b of copy k at u64 index
// 32 b + k, lane l reads copy l mod 32): a 32-lane group's ds_read_b64 then
// touches banks 2 k, 2 k + 1 whatever the bytes, no conflicts (one copy had
// ~3.2 conflict cycles per lookup on C1 text).  64 KiB per 512-thread workgroup.
constexpr int kRxThreads = 512;
template <int kCtx>  // context dwords before each chunk: ceil((max_len - 1) / 4)
__global__ __launch_bounds__(kRxThreads) void k_rx_scan(EvalArgs a, uint32_t stage) {
  __shared__ unsigned long long T32[256 * 32];
  const StageDesc& sd = a.chain->st[stage];
  const bool upper = sd.in_type == VT_SRC_UPPER;
  {
    const unsigned long long* tt = (const unsigned long long*)(a.blob + (upper ? sd.dfa.tt_up : sd.dfa.tt));
    for (uint32_t i = threadIdx.x; i < 256 * 32; i += kRxThreads) T32[i] = tt[i >> 5];
  }
  __syncthreads();
  const unsigned long long* T = T32 + (threadIdx.x & 31u);  // this lane's copy: row b at T[32 b]
  const uint32_t s0 = sd.dfa.s_mid, acc1 = sd.dfa.acc1;
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  const uint64_t nrounds = a.fbm_words;
  constexpr uint32_t kW = kRxThreads / 64;  // waves per workgroup
  const uint64_t w0 = (uint64_t)blockIdx.x * kW + wv;
  const uint64_t nw = (uint64_t)gridDim.x * kW;
  ulonglong2* bm2 = (ulonglong2*)a.fbm;
  for (uint64_t r0 = w0 * kFlatRounds; r0 < nrounds; r0 += nw * kFlatRounds) {
    uint4 v[kFlatRounds], pv[kFlatRounds];
#pragma unroll
    for (int i = 0; i < kFlatRounds; i++) {  // every round's loads in flight before the first use
      const uint64_t c = (r0 + i) * 1024 + lane * 16;
      v[i] = r0 + i < nrounds ? *(const uint4*)(a.slice + c) : make_uint4(0, 0, 0, 0);
      if (kCtx) pv[i] = r0 + i < nrounds && c >= 16 ? *(const uint4*)(a.slice + c - 16) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kFlatRounds; i++) {
      if (r0 + i >= nrounds) break;  // uniform
      uint32_t w[4 + kCtx];
#pragma unroll
      for (int d = 0; d < kCtx; d++) w[d] = u4_dw(pv[i], (uint32_t)(4 - kCtx + d));
      w[kCtx] = v[i].x;
      w[kCtx + 1] = v[i].y;
      w[kCtx + 2] = v[i].z;
      w[kCtx + 3] = v[i].w;
      unsigned long long row[4 * (4 + kCtx)];
#pragma unroll
      for (int k = 0; k < 4 * (4 + kCtx); k++) row[k] = T[32u * ((w[k >> 2] >> (8 * (k & 3))) & 0xFFu)];  // rows ahead of the chain
      uint32_t st = s0;
#pragma unroll
      for (int k = 0; k < 4 * (4 + kCtx); k++) st = (uint32_t)(row[k] >> (4 * st)) & 15u;
      const bool hit = (acc1 >> st) & 1u;
      const bool high = ((v[i].x | v[i].y | v[i].z | v[i].w) & 0x80808080u) != 0u;
      const uint64_t hb = __ballot(hit), hh = __ballot(high);
      if (lane == 0) bm2[r0 + i] = make_ulonglong2(hb, hh);
    }
  }
}
// the DFA over the bytes [p0, p1) of the three chunks from chunk cb (every
// position stepped in order, inactive ones predicated off: no divergent loop)
__device__ __noinline__ uint32_t rx_win(const unsigned long long* T, const uint8_t* S, uint64_t cb, uint64_t p0,
                                           uint64_t p1, uint32_t st) {
  const uint4* src = (const uint4*)(S + (cb << 4));
  const uint4 u[3] = {src[0], src[1], src[2]};
  const uint64_t base = cb << 4;
  const uint32_t lo = p0 > base ? (uint32_t)(p0 - base) : 0u, hi = p1 > base ? (uint32_t)(p1 - base) : 0u;
#pragma unroll
  for (uint32_t k = 0; k < 48; k++) {
    const uint32_t w = k < 16 ? u4_dw(u[0], (k >> 2) & 3u) : k < 32 ? u4_dw(u[1], (k >> 2) & 3u) : u4_dw(u[2], (k >> 2) & 3u);
    const uint32_t nx = (uint32_t)(T[(w >> (8 * (k & 3u))) & 0xFFu] >> (4 * st)) & 15u;
    st = k >= lo && k < hi ? nx : st;
  }
  return st;
}
// the DFA over bytes [p0, p1) of S from state st (the rows in T); the
// sticky accept, or acceptance at the end.  The bytes arrive 64 at a time
// (four 16-byte loads in flight together), the steps run from registers.
__device__ __noinline__ uint32_t rx_run(const unsigned long long* T, const uint8_t* S, uint64_t p0, uint64_t p1, uint32_t st) {
  for (uint64_t a0 = p0 & ~15ull; a0 < p1; a0 += 64) {
    const uint4* src = (const uint4*)(S + a0);
    const uint4 u0 = src[0], u1 = src[1], u2 = src[2], u3 = src[3];
    const uint64_t lo = p0 > a0 ? p0 - a0 : 0, hi = p1 - a0 < 64 ? p1 - a0 : 64;
    for (uint32_t k = (uint32_t)lo; k < (uint32_t)hi; k++) {
      const uint32_t w = u4_dw(sel4(u0, u1, u2, u3, k >> 4), (k >> 2) & 3u);
      st = (uint32_t)(T[(w >> (8 * (k & 3u))) & 0xFFu] >> (4 * st)) & 15u;
    }
  }
  return st;
}
__global__ __launch_bounds__(256) void k_rx_decide(EvalArgs a, uint32_t stage) {
  __shared__ unsigned long long T[256];
  const StageDesc& sd = a.chain->st[stage];
  const bool upper = sd.in_type == VT_SRC_UPPER;
  T[threadIdx.x] = ((const unsigned long long*)(a.blob + (upper ? sd.dfa.tt_up : sd.dfa.tt)))[threadIdx.x];
  __syncthreads();
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= a.nbatches) return;
  const uint32_t s_bot = sd.dfa.s_bot, s_mid = sd.dfa.s_mid, acc1 = sd.dfa.acc1, acc2 = sd.dfa.acc2;
  const uint32_t ml = (uint32_t)sd.dfa.max_len;
  const uint64_t ctx = 4 * ((ml + 2) / 4);  // context bytes of a chunk's window (k_rx_scan's kCtx dwords)
  const bool free_ = s_bot == s_mid && (acc2 & ~acc1) == 0u;  // no begin / end anchors: clear bits decide edges
  const bool keep_match = sd.keep_match != 0;
  const bool out_upper = a.chain->out_type == VT_SRC_UPPER;
  const unsigned long long* hit_bm = a.fbm;  // interleaved: window bits of round w at [2 w], high bytes at [2 w + 1]
  const unsigned long long* hi_bm = a.fbm + 1;
  const uint8_t* S = a.slice;
  const uint64_t pos = a.bpos[b];
  // output sizes for a first surviving batch 0 (k_size skips BF_ROWDONE batches then)
  const int64_t rel0 = (int64_t)rd_be(S + a.bpos[0], 8) - (int64_t)rd_be(S + pos, 8);
  uint64_t rbytes = 0;
  const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
  const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
  const uint64_t al = pos & ~15ull;
  uint64_t wl = nxt > al ? nxt - al : 0;
  if (wl > (uint64_t)kLeanWin) wl = kLeanWin;
  const uint64_t wlen = (wl + 15) & ~15ull;
  const uint32_t batch_len = __builtin_bswap32(ld_u32_at(S + pos + 8));
  const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
  const uint64_t sec_len = sec_end - sec0;
  const int32_t count = sec_len >= 4 ? (int32_t)__builtin_bswap32(ld_u32_at(S + sec0)) : -1;
  bool ok = sec_len >= 4 && sec_end - al <= wlen && count >= 0 && count <= kLeanMaxR && (uint64_t)count == rn;
  uint32_t nkeep = 0;
  uint64_t q = sec0 + 4;  // absolute start of record n
  FlatHdr H = flat_hdr(S, ok && count > 0 ? q : sec0);
  // software pipeline: record n + 1 is framed and its loads are issued before
  // record n is decided; record n + 2's header is in flight meanwhile
  struct RxLoads {
    uint32_t tw;
    ulonglong2 bw0, bw1;
    uint4 ea, eb;
  };
  auto issue = [&](const FjRec& r) {
    RxLoads L;
    L.tw = ld_u32_at(S + r.ve);
    const uint64_t wb0 = (r.va >> 4) >> 6;
    L.bw0 = *(const ulonglong2*)(a.fbm + 2 * wb0);
    L.bw1 = *(const ulonglong2*)(a.fbm + 2 * wb0 + 2);
    L.ea = *(const uint4*)(S + ((r.va >> 4) << 4));
    L.eb = *(const uint4*)(S + (((r.ve ? r.ve - 1 : 0) >> 4) << 4));
    return L;
  };
  FjRec R = {};
  RxLoads LD = {};
  if (ok && count > 0) {
    R = fj_frame(S, H, q, sec_end, true);
    ok = R.ok;
    if (ok) {
      LD = issue(R);
      q = R.end;
      if (count > 1) H = flat_hdr(S, q);
    }
  }
  for (int32_t n = 0; ok && n < count; n++) {
    const FjRec cur = R;
    const RxLoads CL = LD;
    if (n + 1 < count) {
      R = fj_frame(S, H, q, sec_end, true);
      ok = R.ok;
      if (!ok) break;
      LD = issue(R);
      q = R.end;
      if (n + 2 < count) H = flat_hdr(S, q);
    }
    const uint64_t va = cur.va, ve = cur.ve, end = cur.end;
    const uint64_t c0 = va >> 4, c1 = (ve + 15) >> 4, i0 = (va + 15) >> 4, i1 = ve >> 4;
    const uint64_t wb = c0 >> 6;  // first bitmap word touching the value
    const unsigned long long mb0 = CL.bw0.x, hb0 = CL.bw0.y, mb1 = CL.bw1.x, hb1 = CL.bw1.y;
    const uint4 ea = CL.ea, eb = CL.eb;
    int64_t hdr;
    uint32_t nb = var4(CL.tw, hdr);
    ok = nb != 0 && ve + nb == end;
    if (!ok) break;
    auto bits_any = [&](const unsigned long long* bm, unsigned long long w0v, unsigned long long w1v, uint64_t x0,
                        uint64_t x1) {
      if (x1 <= x0) return false;
      if (x1 > (wb + 2) << 6) return flat_any(bm, x0, x1);
      const uint64_t lo = x0 - (wb << 6), hi = x1 - (wb << 6);  // in [0, 128]
      const unsigned long long m0 = (lo < 64 ? (~0ull << lo) : 0ull) & (hi >= 64 ? ~0ull : ((1ull << hi) - 1ull));
      const unsigned long long m1 = (hi > 64 ? (hi >= 128 ? ~0ull : ((1ull << (hi - 64)) - 1ull)) : 0ull) &
                                    (lo > 64 ? (~0ull << (lo - 64)) : ~0ull);
      return ((w0v & m0) | (w1v & m1)) != 0ull;
    };
    // bytes >= 0x80 in the value: chunks inside it by their bits, the edge
    // chunks (which hold gap bytes) by their bytes
    if (ve > va) {
      bool hi = bits_any(hi_bm, hb0, hb1, i0, i1);
      auto hi_edge = [&](const uint4& u, uint64_t c) {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
        uint32_t f = 0;
#pragma unroll
        for (int k = 0; k < 4; k++)
          f |= w[k] & bytes_in((uint32_t)(((c << 4) + 4 * k) - al), (uint32_t)(va - al), (uint32_t)(ve - al));
        return (f & 0x80808080u) != 0u;
      };
      if (!hi && c0 < i0) hi = hi_edge(ea, c0);
      if (!hi && i1 < c1 && (i1 >= i0 || c0 != i1)) hi = hi_edge(eb, i1);
      ok = !hi;
      if (!ok) break;
    }
    bool match;
    if (ve == va) {
      match = (((acc1 | acc2) >> s_bot) & 1u) != 0u;
    } else {
      const uint64_t l1 = (ve - 1) >> 4;                      // the value's last chunk
      const uint64_t j0 = (va + ctx + 15) >> 4, j1 = ve >> 4;  // interior chunks [j0, j1): window inside the value
      match = j0 < j1 && bits_any(hit_bm, mb0, mb1, j0, j1);
      if (!match) {
        // head chunks [c0, h1) hold the matches ending near the value start,
        // tail chunks [t0, l1] those ending near its end; an anchored pattern
        // scans both always (a ^ match can end in an interior chunk, a $ match
        // at an aligned end has no tail chunk)
        const uint64_t h1 = j0 < l1 + 1 ? j0 : l1 + 1, t0 = j1 > j0 ? j1 : j0;
        const bool head = !free_ || bits_any(hit_bm, mb0, mb1, c0, h1);
        const bool tail = free_ ? t0 <= l1 && bits_any(hit_bm, mb0, mb1, t0, l1 + 1) : true;
        uint64_t he = (h1 << 4) < ve ? (h1 << 4) : ve;  // the head scan's end
        if (!free_ && he < va + ml) he = va + ml < ve ? va + ml : ve;
        if (head) {  // from the value start
          const uint32_t st = he - (c0 << 4) <= 48 ? rx_win(T, S, c0, va, he, s_bot) : rx_run(T, S, va, he, s_bot);
          match = ((acc1 >> st) & 1u) || (he == ve && ((acc2 >> st) & 1u));
        }
        if (!match && tail && !(head && he == ve)) {
          const uint64_t e = t0 <= l1 ? (t0 << 4) : ve - 1;  // the earliest end of a match left to see
          const uint64_t back = ml ? ml - 1 : 0;
          const uint64_t st0 = e > va + back ? e - back : va;
          const uint64_t cs = st0 >> 4;
          const uint32_t s1 = st0 == va ? s_bot : s_mid;
          const uint32_t st = ve - (cs << 4) <= 48 ? rx_win(T, S, cs, st0, ve, s1) : rx_run(T, S, st0, ve, s1);
          match = ((acc1 >> st) & 1u) || ((acc2 >> st) & 1u);
        }
      }
    }
    if (match == keep_match) {
      KeptRec d;
      d.src = cur.q;
      d.vpos = va;
      d.kpos = cur.tag ? cur.kpos : 0;
      d.od = cur.od;
      d.ts = cur.ts;
      d.hdr = hdr;
      d.vlen = (uint32_t)(ve - va);
      d.klen = cur.klen;
      d.ival = 0;
      d.mode = out_upper ? KM_UPPER : KM_COPY;
      d.has_key = cur.tag;
      d.attr = cur.attr;
      d.pad = 0;
      rbytes += copy_out_size(d, rel0);
      a.desc[rb + nkeep++] = d;
    }
  }
  ok = ok && q == sec_end;  // (q: the end of the last record framed)
  if (!ok) {  // the exact kernel frames and evaluates this batch
    a.rend[b] = 0xFFFFu;
    const uint32_t i = atomicAdd(&a.list[0], 1u);
    a.list[1 + i] = b;
    return;
  }
  const uint8_t* h = S + pos;  // batch header (file format, batch.rs:163-180)
  BatchStat st = {};
  st.base_offset = (int64_t)rd_be(h, 8);
  st.lod_in = (int32_t)rd_be(h + 23, 4);
  st.first_ts = (int64_t)rd_be(h + 27, 8);
  st.comp = (uint32_t)h[22] & 7u;
  st.flags = BF_LAST_STAGE;
  if (a.rows) {
    ScanRow row = {};
    row.rec_bytes = rbytes;
    row.nonempty = nkeep ? 1 : 0;
    row.lod = (uint64_t)(int64_t)(st.lod_in + 1);
    row.nrec = nkeep;
    row.bytes_in = sec_len;
    row.recs_out = nkeep;
    a.rows[b] = row;
    st.flags |= BF_ROWDONE;
  }
  st.nkeep = st.nout = nkeep;
  st.sec_len = (uint32_t)sec_len;
  st.err_stage = 0xFFFFFFFFu;
  a.bstat[b] = st;
}

// a record's loads, issued together: its value's head and tail windows, the
// bitmap rounds over its first chunk, its trailer (the headers varint)
struct FjLoads {
  uint4 h0, h1, h2, h3, t0, t1, t2, t3, t4;
  ulonglong2 bw0, bw1;  // rounds wb, wb + 1: (occurrences, interesting)
  uint32_t tw;
  uint64_t tc;
};
__device__ __forceinline__ FjLoads fj_issue(const uint8_t* S, const unsigned long long* fbm, const FjRec& r) {
  FjLoads L;
  const uint64_t c0 = r.va >> 4, wb = c0 >> 6;
  const uint4* hp = (const uint4*)(S + (c0 << 4));
  L.tc = ((r.ve - 1) >> 4) >= c0 + 4 ? ((r.ve - 1) >> 4) - 4 : c0;
  const uint4* tp = (const uint4*)(S + (L.tc << 4));
  L.h0 = hp[0];
  L.h1 = hp[1];
  L.h2 = hp[2];
  L.h3 = hp[3];
  L.t0 = tp[0];
  L.t1 = tp[1];
  L.t2 = tp[2];
  L.t3 = tp[3];
  L.t4 = tp[4];
  L.bw0 = *(const ulonglong2*)(fbm + 2 * wb);
  L.bw1 = *(const ulonglong2*)(fbm + 2 * wb + 2);
  L.tw = ld_u32_at(S + r.ve);
  return L;
}
#ifndef FSG_FJ_WPE
#define FSG_FJ_WPE 3  // waves per SIMD of k_fj_decide (<= 168 VGPRs, no scratch)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FSG_FJ_WPE))) void k_fj_decide(EvalArgs a) {
  __shared__ uint4 slots[256 * (kFjSlot / 16) + 1];  // (+1: a word read past the last slot's end)
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= a.nbatches) return;
  // a.flat_st: substring stage (0xFF none) | needle length << 8 | filter_json << 16 | projection << 17 | its stage << 24
  const uint32_t fst = a.flat_st;
  const uint32_t sub = fst & 0xFFu, m = (fst >> 8) & 0xFFu;
  const bool has_sub = sub != 0xFFu, fj = (fst >> 16) & 1u, proj = (fst >> 17) & 1u;
  const bool kLong = m >= 7;
  const StageDesc& sd = a.chain->st[has_sub ? sub : 0];
  const bool upper = has_sub && sd.in_type == VT_SRC_UPPER;
  const bool out_upper = a.chain->out_type == VT_SRC_UPPER;
  const uint8_t* nd = a.blob + sd.needle;
  const StageDesc& pd = a.chain->st[fst >> 24];
  const uint8_t* fld = a.blob + pd.needle;
  const uint32_t fl = proj ? pd.needle_len : 0u;
  uint64_t fw = 0;  // a field name of <= 8 bytes as a word
  for (uint32_t t = 0; t < fl && fl <= 8; t++) fw |= (uint64_t)fld[t] << (8 * t);
  const unsigned long long* hit_bm = a.fbm;  // k_flat_scan<., kJson>: occurrence word w at [2 w]
  const uint8_t* S = a.slice;
  const uint64_t pos = a.bpos[b];
  // output sizes for a first surviving batch 0 (k_size skips BF_ROWDONE batches then)
  const int64_t rel0 = (int64_t)rd_be(S + a.bpos[0], 8) - (int64_t)rd_be(S + pos, 8);
  uint64_t rbytes = 0;
  const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
  const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
  const uint64_t al = pos & ~15ull;
  uint64_t wl = nxt > al ? nxt - al : 0;
  if (wl > (uint64_t)kLeanWin) wl = kLeanWin;
  const uint64_t wlen = (wl + 15) & ~15ull;
  const uint32_t batch_len = __builtin_bswap32(ld_u32_at(S + pos + 8));
  const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
  const uint64_t sec_len = sec_end - sec0;
  const int32_t count = sec_len >= 4 ? (int32_t)__builtin_bswap32(ld_u32_at(S + sec0)) : -1;
  bool ok = sec_len >= 4 && sec_end - al <= wlen && count >= 0 && count <= kLeanMaxR && (uint64_t)count == rn;
  uint32_t nkeep = 0;
  FjCur C;
  C.B = S + al;
  C.W = (uint8_t*)&slots[threadIdx.x * (kFjSlot / 16)];
  C.cb = al >> 4;
  C.fbm = a.fbm;
  // software pipeline: record n + 1's header is framed and its loads issued
  // before record n is walked; record n + 2's header is in flight meanwhile
  FjRec R = {};
  FjLoads L = {};
  FlatHdr H = flat_hdr(S, sec0);
  uint64_t q = sec0 + 4;  // absolute start of the next record to frame
  if (ok && count > 0) {
    H = flat_hdr(S, q);
    R = fj_frame(S, H, q, sec_end);
    ok = R.ok;
    if (ok) {
      L = fj_issue(S, a.fbm, R);
      q = R.end;
      if (count > 1) H = flat_hdr(S, q);
    }
  }
  for (int32_t n = 0; ok && n < count; n++) {
    // record n's loads have landed: its windows into the slot
    {
      uint4* w = (uint4*)C.W;
      w[0] = L.h0;
      w[1] = L.h1;
      w[2] = L.h2;
      w[3] = L.h3;
      w[4] = L.t0;
      w[5] = L.t1;
      w[6] = L.t2;
      w[7] = L.t3;
      w[8] = L.t4;
    }
    const FjRec cur = R;
    const uint64_t va = cur.va, ve = cur.ve;
    const uint64_t c0 = va >> 4, wb = c0 >> 6;
    const ulonglong2 bw0 = L.bw0, bw1 = L.bw1;
    int64_t hdr;
    uint32_t nb = var4(L.tw, hdr);
    ok = nb != 0 && ve + nb == cur.end;
    if (!ok) break;
    C.hb = (uint32_t)(va - al) & ~15u;
    C.tb = (uint32_t)((L.tc << 4) - al);
    C.c = ~0u;
    C.wb = wb;
    C.j0 = bw0.y;
    C.j1 = bw1.y;
    // the next record: framed now, its loads in flight during this walk
    if (n + 1 < count) {
      R = fj_frame(S, H, q, sec_end);
      ok = R.ok;
      if (!ok) break;
      L = fj_issue(S, a.fbm, R);
      q = R.end;
      if (n + 2 < count) H = flat_hdr(S, q);
    }
    bool keep = true;
    if (has_sub) {  // an occurrence starting in [va, ve - m] (k_flat_decide's anchors)
      const unsigned long long mb0 = bw0.x, mb1 = bw1.x;
      auto bits_any = [&](uint64_t x0, uint64_t x1) {
        if (x1 <= x0) return false;
        if (x1 > (wb + 2) << 6) return flat_any(hit_bm, x0, x1);
        const uint64_t lo = x0 - (wb << 6), hi = x1 - (wb << 6);  // in [0, 128]
        const unsigned long long m0 = (lo < 64 ? (~0ull << lo) : 0ull) & (hi >= 64 ? ~0ull : ((1ull << hi) - 1ull));
        const unsigned long long m1 = (hi > 64 ? (hi >= 128 ? ~0ull : ((1ull << (hi - 64)) - 1ull)) : 0ull) &
                                      (lo > 64 ? (~0ull << (lo - 64)) : ~0ull);
        return ((mb0 & m0) | (mb1 & m1)) != 0ull;
      };
      bool match = false;
      const uint64_t vlen = ve - va;
      if (vlen >= m) {
        const uint64_t sl = ve - m;
        const uint64_t blo = kLong ? 3 : 0, bhi = kLong ? 12 : 15;
        const uint64_t j0 = (va + blo + 15) >> 4;
        const uint64_t j1 = sl >= bhi ? ((sl - bhi) >> 4) + 1 : 0;
        match = j0 < j1 && bits_any(j0, j1);
        if (!match) {
          const uint64_t e0 = va >= bhi ? (va - bhi + 15) >> 4 : 0, e1 = (sl + blo) >> 4;
          for (uint64_t c = e0; c <= e1 && !match; c++) {
            if (c >= j0 && c < j1) {
              c = j1 - 1;
              continue;
            }
            const uint64_t r = c - (wb << 6);
            const bool bt = c >= (wb << 6) && r < 128 ? (((r < 64 ? mb0 : mb1) >> (r & 63)) & 1ull) != 0ull
                                                      : bm_bit(hit_bm, c);
            if (!bt) continue;
            const uint64_t lo = (c << 4) >= va + blo ? (c << 4) - blo : va;
            const uint64_t hi = (c << 4) + bhi <= sl ? (c << 4) + bhi : sl;
            for (uint64_t s0 = lo; s0 <= hi && !match; s0++) match = flat_verify(S, s0, nd, m, upper);
          }
        }
      }
      keep = match;
    }
    uint32_t lvl = 0, fs = (uint32_t)(va - al), fe = (uint32_t)(ve - al);
    bool found = false;
#ifdef FSG_FJ_NOWALK  // experiment builds: the decide without the JSON walk (framing, loads and staging only)
    lvl = 2u;
    found = true;
    (void)fw;
#else
    ok = fj_walk(C, fs, fe, fj, proj, fld, fl, fw, lvl, found, fs, fe);
#endif
    if (!ok) break;
    keep = keep && (!fj || lvl > 1u) && (!proj || found);  // level > Debug
    if (keep) {
      KeptRec d;
      d.src = cur.q;
      d.vpos = al + fs;
      d.kpos = cur.tag ? cur.kpos : 0;
      d.od = cur.od;
      d.ts = cur.ts;
      d.hdr = hdr;
      d.vlen = fe - fs;
      d.klen = cur.klen;
      d.ival = 0;
      d.mode = out_upper ? KM_UPPER : KM_COPY;
      d.has_key = cur.tag;
      d.attr = cur.attr;
      d.pad = 0;
      rbytes += copy_out_size(d, rel0);
      a.desc[rb + nkeep++] = d;
    }
  }
  ok = ok && q == sec_end;  // (q: the end of the last record framed)
  if (!ok) {  // the exact kernel frames and evaluates this batch
    a.rend[b] = 0xFFFFu;
    const uint32_t i = atomicAdd(&a.list[0], 1u);
    a.list[1 + i] = b;
    return;
  }
  const uint8_t* h = S + pos;  // batch header (file format, batch.rs:163-180)
  BatchStat st = {};
  st.base_offset = (int64_t)rd_be(h, 8);
  st.lod_in = (int32_t)rd_be(h + 23, 4);
  st.first_ts = (int64_t)rd_be(h + 27, 8);
  st.comp = (uint32_t)h[22] & 7u;
  st.flags = BF_LAST_STAGE;
  if (a.rows) {
    ScanRow row = {};
    row.rec_bytes = rbytes;
    row.nonempty = nkeep ? 1 : 0;
    row.lod = (uint64_t)(int64_t)(st.lod_in + 1);
    row.nrec = nkeep;
    row.bytes_in = sec_len;
    row.recs_out = nkeep;
    a.rows[b] = row;
    st.flags |= BF_ROWDONE;
  }
  st.nkeep = st.nout = nkeep;
  st.sec_len = (uint32_t)sec_len;
  st.err_stage = 0xFFFFFFFFu;
  a.bstat[b] = st;
}

// resident workgroups of k_eval_lean<kind> on the current device (CUs x occupancy)
template <int kKind>
static uint32_t lean_grid() {
  static std::mutex mu;
  static uint32_t cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  std::lock_guard<std::mutex> lock(mu);
  uint32_t& c = cache[dev];
  if (!c) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_eval_lean<kKind>, kLeanThreads, 0);
    c = (uint32_t)std::max(1, cus) * (uint32_t)std::max(1, per);
  }
  return c;
}
template <int kKind>
static void launch_lean_kind(const EvalArgs& a, hipStream_t s) {
  // persistent: as many workgroups as fit on the device at once
  const uint32_t g = std::min<uint32_t>(a.nbatches, lean_grid<kKind>());
  hipLaunchKernelGGL(k_eval_lean<kKind>, dim3(g), dim3(kLeanThreads), 0, s, a);
}

// ---------------------------------------------------------------------------
// k_eval_int — chains of integer stages over decimal values (filter_odd,
// map_double, filter_map, aggregate-sum: from_utf8 + parse::<i32>, the
// aggregate after str::trim) on batches of many small records.  One
// 256-thread workgroup per batch: the window in LDS by LDS-DMA, the record
// starts from k_chase_w (kept with the slice), thread t takes the contiguous
// records [t R, t R + R) (R <= kIntR, unrolled: no indexed registers).
//   pass 1  every field of each record parsed from LDS (Record::decode, the
//           same checks walk_fast makes), the value parsed and the stages
//           run in registers: a keep bit and the output integer per record
//   scans   kept records and the aggregate's wrapping i32 sum, in record order
//           (thread runs are contiguous): wave scans + the four wave totals
//   pass 2  the kept records' fields again, their descriptors at the prefix
// A batch with a byte >= 0x80 in a value, a value that does not parse, a
// record that does not tile its span, more than 256 kIntR records or starts
// k_chase_w could not find is deferred whole to k_eval (list mode), which
// reports its error exactly.
// ---------------------------------------------------------------------------
constexpr int kIntR = 8;
struct __attribute__((aligned(16))) IntLds {
  uint8_t win[kLeanWin + 64];
  uint32_t wk[4], wa[4];
  uint32_t defer;
};
struct IntRec {  // one record's fields (window offsets)
  uint32_t vs, vl, kpos, klen;
  int64_t ts, od, hdr;
  uint8_t attr, tag;
};
// Record::decode of the record spanning window offsets [s, e): false unless it tiles the span
__device__ __forceinline__ bool int_rec(const uint8_t* w, uint32_t s, uint32_t e, IntRec& r) {
  uint32_t q = s;
  int64_t len, kl, vl;
  bool g = !wvarint(w, q, e, &len) && len >= 0 && (uint64_t)q + (uint64_t)len == e;
  if (g && q < e) r.attr = w[q++]; else g = false;
  g = g && !wvarint(w, q, e, &r.ts) && !wvarint(w, q, e, &r.od);
  if (g && q < e) r.tag = w[q++]; else g = false;
  g = g && r.tag <= 1;
  r.kpos = 0;
  r.klen = 0;
  if (g && r.tag == 1) {
    g = !wvarint(w, q, e, &kl) && kl >= 0 && (uint64_t)q + (uint64_t)kl <= e;
    if (g) {
      r.kpos = q;
      r.klen = (uint32_t)kl;
      q += r.klen;
    }
  }
  g = g && !wvarint(w, q, e, &vl) && vl >= 0 && (uint64_t)q + (uint64_t)vl <= e;
  r.vs = q;
  r.vl = g ? (uint32_t)vl : 0u;
  if (g) q += r.vl;
  g = g && !wvarint(w, q, e, &r.hdr) && q == e;
  return g;
}
__device__ __forceinline__ bool int_ws(uint32_t c) { return c == 0x20 || (c >= 0x09 && c <= 0x0D); }
template <int kAgg>  // kAgg: the chain ends in aggregate-sum
__device__ __forceinline__ void eval_int_body(const EvalArgs& a, uint32_t bid) {
  __shared__ IntLds L;
  const uint32_t b = bid;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const ChainDesc& ch = *a.chain;
  const uint8_t* S = a.slice;
  const uint64_t pos = a.bpos[b];
  const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
  const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
  const uint32_t rend = a.rend[b];
  const uint64_t al = pos & ~15ull;
  uint64_t wl = nxt > al ? nxt - al : 0;
  if (wl > (uint64_t)kLeanWin) wl = kLeanWin;
  const uint32_t wlen = (uint32_t)((wl + 15) & ~15ull);
  // the window (every byte of the batch when it fits) by LDS-DMA
  for (uint32_t k = wv; k * 1024u < wlen; k += 4)
    if (k * 1024u + lane * 16u < wlen)  // (an inactive lane writes nothing)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S + al + k * 1024u + lane * 16u),
                                       (__attribute__((address_space(3))) void*)(L.win + k * 1024u), 16, 0, 0);
  if (t == 0) L.defer = 0;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const uint32_t batch_len = (uint32_t)rd_be(L.win + (pos - al) + 8, 4);
  const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
  const uint32_t count = (uint32_t)rn;
  bool ok = rend != 0xFFFFu && sec_end - al <= wlen && sec_end - al == rend && count > 0 &&
            count <= 256u * (uint32_t)kIntR && sec_end >= sec0 + 4 &&
            (uint32_t)rd_be(L.win + (sec0 - al), 4) == count;
  const uint16_t* rs = a.rstart + rb;
  const uint32_t R = (count + 255u) >> 8;
  const uint32_t r0 = t * R;
  uint32_t keep = 0, kc = 0, asum = 0;
  bool simple = true;  // every kept record fits a KeptC (no key, no headers, 32-bit deltas)
  int32_t xv[kIntR];
  const bool src_out = ch.out_type != VT_I32;
  // pass 1: fields, value, stages
#pragma unroll
  for (int i = 0; i < kIntR; i++) {
    xv[i] = 0;
    const uint32_t k = r0 + (uint32_t)i;
    if (!ok || i >= (int)R || k >= count) continue;
    const uint32_t s = rs[k], e = k + 1 < count ? rs[k + 1] : rend;
    IntRec r;
    ok = s < e && e <= rend && int_rec(L.win, s, e, r);
    if (!ok) continue;
    // from_utf8: ASCII only here; the aggregate trims (str::trim) before parsing
    uint32_t vb = r.vs, ve = r.vs + r.vl;
    for (uint32_t j = vb; j < ve; j++) ok = ok && L.win[j] < 0x80u;
    if (!ok) continue;
    if (ch.st[0].op == OP_AGG_SUM) {
      while (vb < ve && int_ws(L.win[vb])) vb++;
      while (ve > vb && int_ws(L.win[ve - 1])) ve--;
    }
    int32_t x = 0;
    ok = parse_i32(L.win + vb, ve - vb, &x) == 0;
    if (!ok) continue;
    bool alive = true;
    for (uint32_t st = 0; st < ch.nstages && alive; st++) {
      const uint8_t op = ch.st[st].op;
      if (op == OP_FILTER_ODD) {
        alive = x % 2 == 0;
      } else if (op == OP_MAP_DOUBLE) {
        x = (int32_t)((uint32_t)x * 2u);
      } else if (op == OP_FILTER_MAP) {
        if (x % 2 == 0) x /= 2; else alive = false;
      }
    }
    xv[i] = x;
    if (alive) {
      keep |= 1u << i;
      kc++;
      if (kAgg) asum += (uint32_t)x;
      simple = simple && r.tag == 0 && r.hdr == 0 && r.od == (int64_t)(int32_t)r.od && r.ts == (int64_t)(int32_t)r.ts;
    }
  }
  if (__syncthreads_or(!ok)) {  // the exact kernel takes the whole batch
    if (t == 0) {
      const uint32_t j = atomicAdd(&a.list[0], 1u);
      a.list[1 + j] = b;
    }
    return;
  }
  const bool compact = kAgg && __syncthreads_and(simple);
  // record-order prefixes: kept records, aggregate sum (wrapping)
  const uint32_t ik = wave_incl_scan(kc), ia = wave_incl_scan(asum);
  if (lane == 63) {
    L.wk[wv] = ik;
    L.wa[wv] = ia;
  }
  __syncthreads();
  uint32_t kbase = ik - kc, abase = ia - asum;
  for (uint32_t w2 = 0; w2 < wv; w2++) {
    kbase += L.wk[w2];
    abase += L.wa[w2];
  }
  // pass 2: the kept records' descriptors
  const uint8_t mode = kAgg ? (uint8_t)KM_AGG : src_out ? (ch.out_type == VT_SRC_UPPER ? (uint8_t)KM_UPPER : (uint8_t)KM_COPY)
                                                        : (uint8_t)KM_I32;
  uint32_t kn = 0, run = abase;
#pragma unroll
  for (int i = 0; i < kIntR; i++) {
    if (!((keep >> i) & 1u)) continue;
    const uint32_t k = r0 + (uint32_t)i;
    const uint32_t s = rs[k], e = k + 1 < count ? rs[k + 1] : rend;
    IntRec r;
    (void)int_rec(L.win, s, e, r);
    run += (uint32_t)xv[i];
    if (compact) {
      KeptC c;
      c.od = (int32_t)r.od;
      c.ts = (int32_t)r.ts;
      c.ival = (int32_t)run;
      c.mode = mode;
      c.attr = r.attr;
      c.pad = 0;
      ((KeptC*)(a.desc + rb))[kbase + kn++] = c;
      continue;
    }
    KeptRec d;
    d.src = al + s;
    d.vpos = al + r.vs;
    d.kpos = r.tag ? al + r.kpos : 0;
    d.od = r.od;
    d.ts = r.ts;
    d.hdr = r.hdr;
    d.vlen = r.vl;
    d.klen = r.klen;
    d.ival = kAgg ? (int32_t)run : xv[i];
    d.mode = mode;
    d.has_key = r.tag;
    d.attr = r.attr;
    d.pad = 0;
    a.desc[rb + kbase + kn++] = d;
  }
  if (t == 0) {
    const uint8_t* h = L.win + (pos - al);  // batch header (file format, batch.rs:163-180)
    BatchStat st = {};
    st.base_offset = (int64_t)rd_be(h, 8);
    st.lod_in = (int32_t)rd_be(h + 23, 4);
    st.first_ts = (int64_t)rd_be(h + 27, 8);
    st.comp = (uint32_t)h[22] & 7u;
    st.flags = BF_LAST_STAGE | (compact ? BF_COMPACT : 0u);
    st.nkeep = st.nout = L.wk[0] + L.wk[1] + L.wk[2] + L.wk[3];
    st.sec_len = (uint32_t)(sec_end - sec0);
    st.err_stage = 0xFFFFFFFFu;
    st.agg_sum = kAgg ? (int64_t)(int32_t)(L.wa[0] + L.wa[1] + L.wa[2] + L.wa[3]) : 0;
    a.bstat[b] = st;
  }
}
template <int kAgg>
__global__ __launch_bounds__(256) void k_eval_int(EvalArgs a) { eval_int_body<kAgg>(a, blockIdx.x); }
// the aggregate-sum group path: every chain's batches in one grid (fsg_launch.h GaJob)
__device__ __forceinline__ uint32_t ga_find(const uint32_t* off, uint32_t n, uint32_t bid) {
  uint32_t lo = 0, hi = n - 1;  // the last job with off[j] <= bid
  while (lo < hi) {
    const uint32_t m = (lo + hi + 1) >> 1;
    if (off[m] <= bid) lo = m; else hi = m - 1;
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_ga_eval_int(const GaJob* J, const uint32_t* off, uint32_t n) {
  const uint32_t j = ga_find(off, n, blockIdx.x);
  eval_int_body<1>(J[j].ea, blockIdx.x - off[j]);
}
void launch_ga_eval_int(const GaJob* jobs, uint32_t n, const uint32_t* off, uint32_t total, hipStream_t s) {
  if (total) hipLaunchKernelGGL(k_ga_eval_int, dim3(total), dim3(256), 0, s, jobs, off, n);
}

bool int_lean_eligible(const ChainDesc& ch, uint32_t ops) {
  if (!ch.nstages) return false;
  if (ops & ~((1u << OP_FILTER_ODD) | (1u << OP_MAP_DOUBLE) | (1u << OP_FILTER_MAP) | (1u << OP_AGG_SUM))) return false;
  if (ch.st[0].in_type != VT_SRC) return false;
  for (uint32_t k = 0; k < ch.nstages; k++) {
    const StageDesc& sd = ch.st[k];
    if (sd.op == OP_AGG_SUM && (k + 1 != ch.nstages || sd.acc_bad || !(ch.flags & CF_AGG_SUM))) return false;
  }
  return true;
}
void launch_eval_int(const EvalArgs& a, bool agg, hipStream_t s) {
  if (!a.nbatches) return;
  if (agg)
    hipLaunchKernelGGL(k_eval_int<1>, dim3(a.nbatches), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_eval_int<0>, dim3(a.nbatches), dim3(256), 0, s, a);
}

int flat_stage(const ChainDesc& ch, uint32_t ops) {
  if (ops & ~((1u << OP_CONTAINS) | (1u << OP_MAP_UPPER))) return -1;
  int st = -1;
  for (uint32_t k = 0; k < ch.nstages; k++)
    if (ch.st[k].op == OP_CONTAINS) {
      if (st >= 0) return -1;  // more than one substring stage: k_eval_lean
      st = (int)k;
    }
  if (st < 0) return -1;
  const uint32_t m = ch.st[st].needle_len;
  return m >= 4 && m <= (uint32_t)kLeanNeedle ? st : -1;
}

void launch_eval_flat(const EvalArgs& a, uint32_t flat_st, hipStream_t s) {
  if (!a.nbatches) return;
  const uint32_t stage = flat_st & 0xFFu, m = flat_st >> 8;
  const uint64_t waves = (a.fbm_words + kFlatRounds - 1) / kFlatRounds;
  const uint32_t g1 = (uint32_t)std::max<uint64_t>(std::min<uint64_t>((waves + 3) / 4, FSG_FLAT_GRID), 1);
  const uint32_t g2 = (a.nbatches + 255) / 256;
  if (m >= 7) {
    hipLaunchKernelGGL(k_flat_scan<true>, dim3(g1), dim3(256), 0, s, a, stage);
    hipLaunchKernelGGL(k_flat_decide<true>, dim3(g2), dim3(256), 0, s, a, stage);
  } else {
    hipLaunchKernelGGL(k_flat_scan<false>, dim3(g1), dim3(256), 0, s, a, stage);
    hipLaunchKernelGGL(k_flat_decide<false>, dim3(g2), dim3(256), 0, s, a, stage);
  }
}

int fjson_flags(const ChainDesc& ch, uint32_t ops) {
  const uint32_t jops = (1u << OP_FILTER_JSON) | (1u << OP_PROJECT);
  if (!(ops & jops) || (ops & ~((1u << OP_CONTAINS) | (1u << OP_MAP_UPPER) | jops))) return -1;
  int sub = -1, fjs = -1, pjs = -1;
  for (uint32_t k = 0; k < ch.nstages; k++) {
    const StageDesc& sd = ch.st[k];
    if (pjs >= 0 && sd.op != OP_MAP_UPPER) return -1;  // after a projection: uppercase maps only
    if (sd.op == OP_CONTAINS) {
      if (sub >= 0) return -1;
      sub = (int)k;
    } else if (sd.op == OP_FILTER_JSON || sd.op == OP_PROJECT) {
      if (sd.in_type != VT_SRC) return -1;
      if (sd.op == OP_FILTER_JSON) {
        if (fjs >= 0) return -1;
        fjs = (int)k;
      } else {
        if (sd.needle_len > (uint32_t)kLeanNeedle) return -1;
        pjs = (int)k;
      }
    }
  }
  uint32_t m = 0;
  if (sub >= 0) {
    m = ch.st[sub].needle_len;
    if (m < 4 || m > (uint32_t)kLeanNeedle) return -1;
  }
  return (int)((sub >= 0 ? (uint32_t)sub : 0xFFu) | (m << 8) | ((fjs >= 0 ? 1u : 0u) << 16) |
               ((pjs >= 0 ? 1u : 0u) << 17) | ((uint32_t)(pjs >= 0 ? pjs : 0) << 24));
}

void launch_eval_fjson(const EvalArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  const uint32_t sub = a.flat_st & 0xFFu, m = (a.flat_st >> 8) & 0xFFu;
  const uint64_t waves = (a.fbm_words + kFlatRounds - 1) / kFlatRounds;
  const uint32_t g1 = (uint32_t)std::max<uint64_t>(std::min<uint64_t>((waves + 3) / 4, 4096), 1);
  const uint32_t g2 = (a.nbatches + 255) / 256;
  if (sub == 0xFFu)
    hipLaunchKernelGGL((k_flat_scan<true, true, true>), dim3(g1), dim3(256), 0, s, a, 0u);
  else if (m >= 7)
    hipLaunchKernelGGL((k_flat_scan<true, true, false>), dim3(g1), dim3(256), 0, s, a, sub);
  else
    hipLaunchKernelGGL((k_flat_scan<false, true, false>), dim3(g1), dim3(256), 0, s, a, sub);
  hipLaunchKernelGGL(k_fj_decide, dim3(g2), dim3(256), 0, s, a);
}

int rx_flat_stage(const ChainDesc& ch, uint32_t ops) {
  if (ops & ~((1u << OP_REGEX) | (1u << OP_MAP_UPPER))) return -1;
  int st = -1;
  for (uint32_t k = 0; k < ch.nstages; k++)
    if (ch.st[k].op == OP_REGEX) {
      if (st >= 0) return -1;  // several regex stages: k_eval_lean
      st = (int)k;
    }
  if (st < 0) return -1;
  const DfaDesc& d = ch.st[st].dfa;
  return d.lean && d.max_len >= 0 && d.max_len <= 17 ? st : -1;
}
void launch_eval_rx(const EvalArgs& a, uint32_t stage, hipStream_t s) {
  if (!a.nbatches) return;
  const uint32_t ml = (uint32_t)a.chain_host_max_len;
  const uint64_t waves = (a.fbm_words + kFlatRounds - 1) / kFlatRounds;
  constexpr uint32_t kW = kRxThreads / 64;
  const uint32_t g1 = (uint32_t)std::max<uint64_t>(std::min<uint64_t>((waves + kW - 1) / kW, 2048), 1);
  const uint32_t g2 = (a.nbatches + 255) / 256;
  switch ((ml + 2) / 4) {  // context dwords of a chunk's window
    case 0: hipLaunchKernelGGL(k_rx_scan<0>, dim3(g1), dim3(kRxThreads), 0, s, a, stage); break;
    case 1: hipLaunchKernelGGL(k_rx_scan<1>, dim3(g1), dim3(kRxThreads), 0, s, a, stage); break;
    case 2: hipLaunchKernelGGL(k_rx_scan<2>, dim3(g1), dim3(kRxThreads), 0, s, a, stage); break;
    case 3: hipLaunchKernelGGL(k_rx_scan<3>, dim3(g1), dim3(kRxThreads), 0, s, a, stage); break;
    default: hipLaunchKernelGGL(k_rx_scan<4>, dim3(g1), dim3(kRxThreads), 0, s, a, stage); break;
  }
  hipLaunchKernelGGL(k_rx_decide, dim3(g2), dim3(256), 0, s, a, stage);
}

void launch_eval_lean(const EvalArgs& a, uint32_t ops, hipStream_t s) {
  if (!a.nbatches) return;
  hipLaunchKernelGGL(k_chase, dim3((a.nbatches + kChaseT - 1) / kChaseT), dim3(kChaseT), 0, s, a);
  const bool json = (ops & ((1u << OP_FILTER_JSON) | (1u << OP_PROJECT))) != 0;
  const bool rx = (ops & (1u << OP_REGEX)) != 0, ct = (ops & (1u << OP_CONTAINS)) != 0;
  if (json)
    launch_lean_kind<kLeanJson>(a, s);
  else if (rx && ct)
    launch_lean_kind<kLeanMixed>(a, s);
  else if (rx)
    launch_lean_kind<kLeanRegex>(a, s);
  else
    launch_lean_kind<kLeanContains>(a, s);
}

}  // namespace fsg
