// fsg_kernels.hip — CDNA4 (gfx950) kernels of the SmartModule record-transform path.
//
// Pipeline of one process_batch call over an HBM-resident slice:
//   k_eval     one wave per stored batch: header decode, LDS-staged record
//              windows, record framing (Record::decode, data.rs:534-562), the
//              fused SmartModule chain per record, first-error semantics
//              (engine.rs:135-185 + derive generator loops), compaction
//              descriptors of the surviving records
//   k_size     one wave per batch: output record sizes after the offset fix-up
//              (spu batch.rs:95-105)
//   k_scan_*   cross-batch exclusive scan (bytes, offsets, metrics, aggregate)
//              + max_bytes cut detection (batch.rs:101-111)
//   k_plan     one thread: the process_batch stop rules (batch.rs:41-142)
//   k_header   output Batch header (batch.rs:398-430, Batch::default 482-497)
//   k_write    one wave per included batch: canonical record re-encode
//              (data.rs:504-532, varint.rs:43-66) into the output batch
//   k_crc_*    CRC32C over attributes..records, chunked + GF(2) combine
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "fsg_device.h"
#include "fsg_dev_util.h"
#include "fsg_codec_dev.h"
#include "fsg_json_dev.h"
#include "fsg_json_dfa.h"

namespace fsg {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dec_len_i32(int32_t v) {
  uint32_t u = v < 0 ? (uint32_t)(-(int64_t)v) : (uint32_t)v;
  uint32_t n = 1;
  while (u >= 10) {
    u /= 10;
    n++;
  }
  return n + (v < 0 ? 1 : 0);
}
__device__ __forceinline__ uint32_t fmt_i32(int32_t v, uint8_t* out) {
  uint8_t t[12];
  uint32_t n = 0;
  uint32_t u = v < 0 ? (uint32_t)(-(int64_t)v) : (uint32_t)v;
  do {
    t[n++] = (uint8_t)('0' + u % 10);
    u /= 10;
  } while (u);
  uint32_t k = 0;
  if (v < 0) out[k++] = '-';
  while (n) out[k++] = t[--n];
  return k;
}

// ---------------------------------------------------------------------------
// Rust core::str::from_utf8 (run_utf8_validation) — serial, one lane per value
// returns 1 valid; else 0 with valid_up_to and error_len (0 = None)
// ---------------------------------------------------------------------------
template <typename P>
__device__ int utf8_check(P s, uint32_t n, uint32_t* vut, uint32_t* elen) {
  uint32_t i = 0;
  while (i < n) {
    uint32_t f = s[i];
    if (f < 0x80) {
      i++;
      continue;
    }
    int w = (f >= 0xC2 && f <= 0xDF) ? 2 : (f >= 0xE0 && f <= 0xEF) ? 3 : (f >= 0xF0 && f <= 0xF4) ? 4 : 0;
    if (w == 0) { *vut = i; *elen = 1; return 0; }
    if (i + 1 >= n) { *vut = i; *elen = 0; return 0; }
    uint32_t b1 = s[i + 1];
    if (w == 2) {
      if ((b1 & 0xC0) != 0x80) { *vut = i; *elen = 1; return 0; }
      i += 2;
      continue;
    }
    bool ok1;
    if (w == 3)
      ok1 = (f == 0xE0 && b1 >= 0xA0 && b1 <= 0xBF) || (f >= 0xE1 && f <= 0xEC && b1 >= 0x80 && b1 <= 0xBF) ||
            (f == 0xED && b1 >= 0x80 && b1 <= 0x9F) || (f >= 0xEE && f <= 0xEF && b1 >= 0x80 && b1 <= 0xBF);
    else
      ok1 = (f == 0xF0 && b1 >= 0x90 && b1 <= 0xBF) || (f >= 0xF1 && f <= 0xF3 && b1 >= 0x80 && b1 <= 0xBF) ||
            (f == 0xF4 && b1 >= 0x80 && b1 <= 0x8F);
    if (!ok1) { *vut = i; *elen = 1; return 0; }
    if (i + 2 >= n) { *vut = i; *elen = 0; return 0; }
    if ((s[i + 2] & 0xC0) != 0x80) { *vut = i; *elen = 2; return 0; }
    if (w == 3) {
      i += 3;
      continue;
    }
    if (i + 3 >= n) { *vut = i; *elen = 0; return 0; }
    if ((s[i + 3] & 0xC0) != 0x80) { *vut = i; *elen = 3; return 0; }
    i += 4;
  }
  return 1;
}

// char::is_whitespace on a code point
__device__ __forceinline__ bool cp_ws(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F ||
         c == 0x3000;
}
template <typename P>
__device__ __forceinline__ uint32_t cp_at(P s, uint32_t i, uint32_t* w) {
  uint32_t f = s[i];
  if (f < 0x80) { *w = 1; return f; }
  if (f < 0xE0) { *w = 2; return ((f & 0x1F) << 6) | (s[i + 1] & 0x3F); }
  if (f < 0xF0) { *w = 3; return ((f & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); }
  *w = 4;
  return ((f & 0x07) << 18) | ((uint32_t)(s[i + 1] & 0x3F) << 12) | ((uint32_t)(s[i + 2] & 0x3F) << 6) |
         (s[i + 3] & 0x3F);
}
// str::trim on valid UTF-8 -> [b, e)
template <typename P>
__device__ void utf8_trim(P s, uint32_t n, uint32_t* b, uint32_t* e) {
  uint32_t i = 0, w;
  while (i < n) {
    uint32_t c = cp_at(s, i, &w);
    if (!cp_ws(c)) break;
    i += w;
  }
  uint32_t j = n;
  while (j > i) {
    uint32_t k = j - 1;
    while (k > i && (s[k] & 0xC0) == 0x80) k--;
    uint32_t c = cp_at(s, k, &w);
    if (!cp_ws(c)) break;
    j = k;
  }
  *b = i;
  *e = j;
}


// ---------------------------------------------------------------------------
// k_eval: per-wave LDS state
// ---------------------------------------------------------------------------
enum RecFlags : uint32_t {
  RF_ALIVE = 1u,
  RF_MATCH = 2u,
  RF_NONASCII = 4u,
  RF_UTF8_DONE = 8u,
  RF_UTF8_BAD = 16u,
};

constexpr int kDfaLds = 4096;
constexpr int kEvalThreads = 256;  // one 4-wave workgroup per stored batch
// compile-time op sets of the k_eval variants
constexpr uint32_t opbit(int op) { return 1u << op; }
constexpr uint32_t kOpsContains = opbit(OP_CONTAINS) | opbit(OP_MAP_UPPER);
constexpr uint32_t kOpsRegex = opbit(OP_REGEX) | opbit(OP_CONTAINS) | opbit(OP_MAP_UPPER);
constexpr uint32_t kOpsJson = opbit(OP_FILTER_JSON) | opbit(OP_CONTAINS) | opbit(OP_MAP_UPPER) | opbit(OP_PROJECT) |
                              opbit(OP_REGEX);
constexpr uint32_t kOpsArray = opbit(OP_ARRAY_MAP) | opbit(OP_CONTAINS) | opbit(OP_MAP_UPPER);
constexpr uint32_t kOpsInt = opbit(OP_FILTER_ODD) | opbit(OP_MAP_DOUBLE) | opbit(OP_FILTER_MAP) | opbit(OP_AGG_SUM) |
                             opbit(OP_AGG_CONCAT) | opbit(OP_CONTAINS) | opbit(OP_MAP_UPPER) | opbit(OP_LB_MAX) |
                             opbit(OP_DEDUP);
constexpr uint32_t kOpsAll = 0xFFFFu;
constexpr int kDfaDyn = 768 + kDfaLds;  // dynamic LDS of a chain with a regex stage
extern __shared__ __attribute__((aligned(16))) uint8_t g_dyn_lds[];

struct __attribute__((aligned(16))) WaveLds {
  uint8_t win[kWin + 64];
  uint32_t r_vs[kMaxR];     // value start (window offset)
  uint32_t r_vl[kMaxR];     // value length
  uint32_t r_start[kMaxR];  // record start (window offset)
  uint32_t r_kpos[kMaxR];   // key bytes (window offset)
  uint32_t r_klen[kMaxR];
  uint32_t r_flags[kMaxR];
  uint32_t r_aux[kMaxR];    // utf8 valid_up_to / parse kind
  uint32_t r_aux2[kMaxR];   // utf8 error_len
  uint32_t r_aux3[kMaxR];   // serde_json error span end
  int32_t r_ival[kMaxR];    // VT_I32 value
  int32_t r_ival_in[kMaxR]; // value entering the erroring stage
  uint32_t r_ec[kMaxR];     // error code word (ErrCode | detail)
  uint8_t r_es[kMaxR];      // first error stage (0xFF none)
  uint8_t r_attr[kMaxR];
  uint8_t r_haskey[kMaxR];
  int64_t r_od[kMaxR];
  int64_t r_ts[kMaxR];
  int64_t r_hdr[kMaxR];
  uint32_t r_end[kMaxR];    // fast walk: record end (window offset)
  // wave-uniform scalars
  int32_t nr;
  int32_t walk_status;      // 0 ok, 1 decode error, 2 window incomplete (need next window)
  uint32_t err_stage_b, err_idx_b;  // broadcast of the batch's first error (wave 0 -> all)
  uint32_t next_cursor_lo, next_cursor_hi;
  BatchStat bs;             // the batch's result, assembled by lane 0 (keeps long-lived state out of VGPRs)
};

// Serial exact walk of records (lane 0).  Window bytes w[0..wlen) map to
// absolute offsets wbase..; the record section ends at absolute sec_end.
// Record::decode semantics (data.rs:534-562): fields parsed in order, the next
// record starts where the headers varint ends.
template <typename P>
__device__ void walk_records(WaveLds& L, P w, uint64_t wbase, uint32_t wlen, uint64_t sec_end, uint64_t cursor,
                             uint32_t rec_remaining, int max_recs) {
  // window limit in window offsets; section limit in window offsets (may exceed wlen)
  const uint64_t sec_lim64 = sec_end - wbase;
  const uint32_t wlim = wlen;
  uint32_t q = (uint32_t)(cursor - wbase);
  int nr = 0;
  int status = 0;
  const int lim = max_recs < kMaxR ? max_recs : kMaxR;
  while (nr < lim && (uint32_t)nr < rec_remaining) {
    const uint32_t start = q;
    const uint32_t have = wlim < sec_lim64 ? wlim : (uint32_t)sec_lim64;  // readable bytes in window
    const bool win_short = (uint64_t)wlim < sec_lim64;                        // more section bytes exist
#define WALK_FAIL()            \
  do {                         \
    status = win_short ? 2 : 1; \
    goto done;                 \
  } while (0)
    int64_t len;
    if (wvarint(w, q, have, &len)) WALK_FAIL();
    if ((int64_t)(sec_lim64 - q) < len) {  // "not enough for record" (remaining is section-relative)
      status = 1;
      goto done;
    }
    if (q >= have) WALK_FAIL();
    uint8_t attr = w[q++];
    int64_t ts, od;
    if (wvarint(w, q, have, &ts)) WALK_FAIL();
    if (wvarint(w, q, have, &od)) WALK_FAIL();
    if (q >= have) WALK_FAIL();
    uint8_t tag = w[q++];
    if (tag > 1) {
      status = 1;
      goto done;
    }
    uint32_t kpos = 0, klen = 0;
    if (tag == 1) {
      int64_t kl;
      if (wvarint(w, q, have, &kl)) WALK_FAIL();
      uint64_t want = (uint64_t)kl, rem = sec_lim64 - q;
      uint64_t take = want < rem ? want : rem;
      if ((uint64_t)q + take > have) {
        status = 2;  // bytes exist in the section but not in the window
        goto done;
      }
      kpos = q;
      klen = (uint32_t)take;
      q += (uint32_t)take;
    }
    int64_t vl;
    if (wvarint(w, q, have, &vl)) WALK_FAIL();
    {
      uint64_t want = (uint64_t)vl, rem = sec_lim64 - q;
      uint64_t take = want < rem ? want : rem;
      if ((uint64_t)q + take > have) {
        status = 2;
        goto done;
      }
      L.r_vs[nr] = q;
      L.r_vl[nr] = (uint32_t)take;
      q += (uint32_t)take;
    }
    int64_t hdr;
    if (wvarint(w, q, have, &hdr)) WALK_FAIL();
#undef WALK_FAIL
    L.r_start[nr] = start;
    L.r_kpos[nr] = kpos;
    L.r_klen[nr] = klen;
    L.r_haskey[nr] = tag;
    L.r_attr[nr] = attr;
    L.r_od[nr] = od;
    L.r_ts[nr] = ts;
    L.r_hdr[nr] = hdr;
    L.r_flags[nr] = RF_ALIVE;
    L.r_es[nr] = 0xFF;
    L.r_ec[nr] = 0;
    L.r_ival[nr] = 0;
    nr++;
  }
done:
  if (status == 2 && nr > 0) status = 0;  // stop the window before the incomplete record
  L.nr = nr;
  L.walk_status = status;
  const uint64_t nc = wbase + (nr > 0 ? (uint64_t)(L.r_vs[nr - 1] + L.r_vl[nr - 1]) : (cursor - wbase));
  // next record starts after the headers varint of the last record: recompute
  uint64_t nxt = cursor;
  if (nr > 0) {
    uint32_t qq = L.r_vs[nr - 1] + L.r_vl[nr - 1];
    int64_t h;
    wvarint(w, qq, wlen, &h);
    nxt = wbase + qq;
  }
  (void)nc;
  L.next_cursor_lo = (uint32_t)nxt;
  L.next_cursor_hi = (uint32_t)(nxt >> 32);
}

// Fast walk: lane 0 chases only the length varints (record i+1 starts at
// start_i + varint_size + len when the record is well formed); then every lane
// parses its own records exactly (Record::decode) and checks that the fields end
// where the length said.  Any inconsistency -> caller runs the exact serial walk.
// Returns true when the window was walked.
__device__ __forceinline__ bool walk_fast(WaveLds& L, const uint8_t* w, uint64_t wbase, uint32_t wlen, uint64_t sec_end,
                          uint64_t cursor, uint32_t rec_remaining, const uint16_t* rsb = nullptr, uint64_t al0 = 0,
                          uint32_t done = 0, uint32_t rend = 0) {
  const uint32_t tid = threadIdx.x;
  const uint64_t sec_lim64 = sec_end - wbase;
  const uint32_t have = wlen < sec_lim64 ? wlen : (uint32_t)sec_lim64;
  if (rsb) {
    // record starts precomputed by k_chase_w (offsets from al0): every lane
    // takes its records' bounds; the records that end inside the window are a prefix
    const uint32_t lim = rec_remaining < (uint32_t)kMaxR ? rec_remaining : (uint32_t)kMaxR;
    bool in = false;
    if (tid < lim) {
      const uint64_t st = al0 + rsb[done + tid];
      const uint64_t en = al0 + (tid + 1 < rec_remaining ? rsb[done + tid + 1] : rend);
      in = st >= wbase && en - wbase <= have;
      if (in) {
        L.r_start[tid] = (uint32_t)(st - wbase);
        L.r_end[tid] = (uint32_t)(en - wbase);
      }
    }
    const int n = __syncthreads_count(in);
    if (tid == 0) L.nr = n;
  } else if (tid == 0) {
    uint32_t q = (uint32_t)(cursor - wbase);
    int n = 0;
    const int lim = (int)(rec_remaining < (uint32_t)kMaxR ? rec_remaining : (uint32_t)kMaxR);
    while (n < lim) {
      uint32_t q0 = q;
      int64_t len;
      if (wvarint(w, q, have, &len)) break;
      if (len < 0 || (int64_t)(sec_lim64 - q) < len) break;
      const uint64_t end = (uint64_t)q + (uint64_t)len;
      if (end > have) break;
      L.r_start[n] = q0;
      L.r_end[n] = (uint32_t)end;
      q = (uint32_t)end;
      n++;
    }
    L.nr = n;
  }
  __syncthreads();
  const int nr = L.nr;
  if (nr == 0) return false;
  bool ok = true;
  for (int r = (int)tid; r < nr; r += kEvalThreads) {
    uint32_t q = L.r_start[r];
    const uint32_t lim = L.r_end[r];
    int64_t len, ts, od, kl, vl, hdr;
    bool g = !wvarint(w, q, lim, &len);
    uint8_t attr = 0, tag = 0;
    if (g && q < lim) attr = w[q++]; else g = false;
    g = g && !wvarint(w, q, lim, &ts) && !wvarint(w, q, lim, &od);
    if (g && q < lim) tag = w[q++]; else g = false;
    g = g && tag <= 1;
    uint32_t kpos = 0, klen = 0;
    if (g && tag == 1) {
      g = !wvarint(w, q, lim, &kl) && kl >= 0 && (uint64_t)q + (uint64_t)kl <= lim;
      if (g) {
        kpos = q;
        klen = (uint32_t)kl;
        q += klen;
      }
    }
    g = g && !wvarint(w, q, lim, &vl) && vl >= 0 && (uint64_t)q + (uint64_t)vl <= lim;
    uint32_t vs = q;
    if (g) q += (uint32_t)vl;
    g = g && !wvarint(w, q, lim, &hdr) && q == lim;
    if (g) {
      L.r_vs[r] = vs;
      L.r_vl[r] = (uint32_t)vl;
      L.r_kpos[r] = kpos;
      L.r_klen[r] = klen;
      L.r_haskey[r] = tag;
      L.r_attr[r] = attr;
      L.r_od[r] = od;
      L.r_ts[r] = ts;
      L.r_hdr[r] = hdr;
      L.r_flags[r] = RF_ALIVE;
      L.r_es[r] = 0xFF;
      L.r_ec[r] = 0;
      L.r_ival[r] = 0;
    }
    ok &= g;
  }
  ok = __syncthreads_and(ok);
  if (ok && tid == 0) {
    L.walk_status = 0;
    const uint64_t nxt = wbase + L.r_end[nr - 1];
    L.next_cursor_lo = (uint32_t)nxt;
    L.next_cursor_hi = (uint32_t)(nxt >> 32);
  }
  __syncthreads();
  return ok;
}

// ---------------------------------------------------------------------------
// Parallel framing of a batch of many small records (k_eval<kOpsInt / kOpsAll>,
// a batch whose section is resident in the window and holds more than kMaxR
// records: aggregate-sum, filter_hashset, integer maps over decimal values).
// The lane-0 chase costs one dependent LDS round trip per record and a window
// reload per kMaxR records; here every byte position p of the section gets
// nx(p) = where a record starting at p would end (its length varint decoded as
// walk_fast decodes it), J = nx^32 by five in-place squarings, lane 0 follows
// J from the first record (one hop per 32 records), and one lane per hop fills
// in its 32 record starts with nx.  Any position whose length does not decode,
// a chain that does not end exactly at the section end, or a record count
// other than the header's leaves the batch to the exact walk (nothing is
// decided from here: walk_fast re-parses every record it is given).
// ---------------------------------------------------------------------------
constexpr int kParMaxR = 4096;  // record starts held (a 16 KiB section of 7-byte records: ~2,340)
constexpr int kParHop = 32;     // J = nx^kParHop
constexpr uint32_t kParBad = 0xFFFFu;
struct __attribute__((aligned(16))) ParLds {
  uint16_t J[kWin + 16];               // section-relative successor^32 (n = exact end, kParBad = undecodable)
  uint16_t rs[kParMaxR];               // record starts (window offsets)
  uint16_t lead[kParMaxR / kParHop];   // every kParHop-th record start (section-relative)
  uint32_t nlead, total, ok;
};
// where a record starting at window offset q would end (section-relative to c0), or kParBad
__device__ __forceinline__ uint32_t par_next(const uint8_t* w, uint32_t q, uint32_t c0, uint32_t lim) {
  int64_t len;
  if (wvarint(w, q, lim, &len)) return kParBad;
  if (len < 0 || (int64_t)(lim - q) < len) return kParBad;
  return q + (uint32_t)len - c0;
}
// record starts of the section [c0, lim) (window offsets) into P.rs; true when
// exactly `count` records tile it
__device__ __forceinline__ bool par_frame(const uint8_t* w, ParLds& P, uint32_t c0, uint32_t lim, uint32_t count) {
  const uint32_t tid = threadIdx.x;
  const uint32_t n = lim - c0;
  for (uint32_t i = tid; i < n; i += kEvalThreads) P.J[i] = (uint16_t)par_next(w, c0 + i, c0, lim);
  __syncthreads();
  // five squarings in place: a chunk's successors-of-successors are read before any is written
  constexpr int kC = 16;
  for (int r = 0; r < 5; r++) {
    for (uint32_t base = 0; base < n; base += kEvalThreads * kC) {
      uint16_t v[kC];
#pragma unroll
      for (int k = 0; k < kC; k++) {
        const uint32_t i = base + (uint32_t)k * kEvalThreads + tid;
        const uint32_t j = i < n ? P.J[i] : kParBad;
        v[k] = (uint16_t)(j >= n ? j : P.J[j]);
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < kC; k++) {
        const uint32_t i = base + (uint32_t)k * kEvalThreads + tid;
        if (i < n) P.J[i] = v[k];
      }
      __syncthreads();
    }
  }
  if (tid == 0) {
    uint32_t p = 0, k = 0;
    bool ok = true;
    while (p < n) {
      if (k >= (uint32_t)(kParMaxR / kParHop)) {
        ok = false;
        break;
      }
      P.lead[k++] = (uint16_t)p;
      p = P.J[p];
    }
    P.nlead = k;
    P.ok = ok && p == n;
  }
  __syncthreads();
  if (!P.ok) return false;
  const uint32_t nl = P.nlead;
  if (tid < nl) {  // hop t: records [32 t, 32 t + 32)
    uint32_t p = P.lead[tid], s = 0;
    for (; s < (uint32_t)kParHop && p < n; s++) {
      P.rs[tid * kParHop + s] = (uint16_t)(c0 + p);
      p = par_next(w, c0 + p, c0, lim);
    }
    if (tid + 1 == nl) P.total = tid * kParHop + s;
  }
  __syncthreads();
  return P.total == count;
}

// find the record whose [start, ...) region contains window offset p (largest r with r_vs[r] <= p)
__device__ __forceinline__ int find_rec(const WaveLds& L, int nr, uint32_t p) {
  int lo = 0, hi = nr - 1, r = -1;
  while (lo <= hi) {
    int m = (lo + hi) >> 1;
    if (L.r_vs[m] <= p) {
      r = m;
      lo = m + 1;
    } else
      hi = m - 1;
  }
  return r;
}

// Data-parallel substring scan + non-ASCII marking over the values of the window.
// Marks RF_MATCH on records whose (optionally uppercased) value contains needle.
// Each lane takes 16-byte chunks (32 bytes from two ds_read_b128 of the LDS
// window).  Filter: the 4-byte window at each of the 16 positions is compared
// with the needle's first min(m, 4) bytes (one v_alignbyte + one compare per
// position); the compares are OR-ed as wave ballots on the scalar unit, so a
// wave with no 4-gram hit anywhere pays ~2 VALU per position and moves on.
// Lanes with a hit rebuild their position mask and verify the rest of the
// needle byte by byte.
__device__ __forceinline__ uint32_t win_at(const uint32_t (&w)[8], int j) {
  const int k = j >> 2, a = j & 3;
  return a ? __builtin_amdgcn_alignbyte(w[k + 1], w[k], (uint32_t)a) : w[k];
}
template <bool kLds, typename P>
__device__ __forceinline__ void scan_contains(WaveLds& L, P w, uint32_t wlen, int nr, const uint8_t* needle,
                                              uint32_t m, bool upper, bool mark_nonascii) {
  (void)wlen;
  if (nr == 0) return;
  const uint32_t lo = L.r_vs[0];
  const uint32_t hi = L.r_vs[nr - 1] + L.r_vl[nr - 1];
  const uint32_t l = threadIdx.x;
  const uint32_t m4 = m < 4 ? m : 4;
  uint32_t n4 = 0;
  for (uint32_t t = 0; t < m4; t++) n4 |= (uint32_t)needle[t] << (8 * t);
  const uint32_t k4 = m4 == 4 ? 0xFFFFFFFFu : ((1u << (8 * m4)) - 1u);
  for (uint32_t c = (lo & ~15u) + l * 16; c < hi; c += kEvalThreads * 16) {
    uint32_t wd[8];
    if constexpr (kLds) {
      const uint4 v0 = *(const uint4*)(&L.win[c]);
      const uint4 v1 = *(const uint4*)(&L.win[c + 16]);
      wd[0] = v0.x; wd[1] = v0.y; wd[2] = v0.z; wd[3] = v0.w;
      wd[4] = v1.x; wd[5] = v1.y; wd[6] = v1.z; wd[7] = v1.w;
    } else {
      for (int k = 0; k < 8; k++)
        wd[k] = (uint32_t)w[c + 4 * k] | ((uint32_t)w[c + 4 * k + 1] << 8) | ((uint32_t)w[c + 4 * k + 2] << 16) |
                ((uint32_t)w[c + 4 * k + 3] << 24);
    }
    if (mark_nonascii && ((wd[0] | wd[1] | wd[2] | wd[3]) & 0x80808080u)) {
      for (int k = 0; k < 4; k++)
        for (int j = 0; j < 4; j++) {
          uint32_t p = c + 4 * k + j;
          if (((wd[k] >> (8 * j)) & 0x80) && p >= lo && p < hi) {
            int r = find_rec(L, nr, p);
            if (r >= 0 && p < L.r_vs[r] + L.r_vl[r]) atomicOr(&L.r_flags[r], RF_NONASCII);
          }
        }
    }
    if (m == 0) continue;
    if (upper)
      for (int k = 0; k < 8; k++) wd[k] = swar_upper(wd[k]);
    uint64_t any = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) any |= __ballot(((win_at(wd, j) ^ n4) & k4) == 0);
    if (!any) continue;                    // wave-uniform: no 4-gram hit in any lane
    if (!((any >> (l & 63)) & 1)) continue;  // this lane has no hit
    uint32_t cand = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) cand |= (uint32_t)(((win_at(wd, j) ^ n4) & k4) == 0) << j;
    while (cand) {
      const uint32_t p = c + (uint32_t)__builtin_ctz(cand);
      cand &= cand - 1;
      if (p < lo || p >= hi) continue;
      const int r = find_rec(L, nr, p);
      if (r < 0) continue;
      if (p + m > L.r_vs[r] + L.r_vl[r]) continue;
      bool ok = true;
      for (uint32_t t = 4; t < m; t++) {
        uint8_t y = kLds ? L.win[p + t] : w[p + t];
        if (upper) y = up(y);
        if (y != needle[t]) {
          ok = false;
          break;
        }
      }
      if (ok) atomicOr(&L.r_flags[r], RF_MATCH);
    }
  }
}

// records with an empty value never get a scan hit; an empty needle matches all
// Data-parallel non-ASCII marking only
template <bool kLds, typename P>
__device__ __forceinline__ void scan_nonascii(WaveLds& L, P w, uint32_t wlen, int nr) {
  scan_contains<kLds>(L, w, wlen, nr, nullptr, 0, false, true);
}

// DFA helpers
struct DfaView {
  const uint8_t* cls;
  const uint8_t* trans;
  const uint8_t* acc;
  uint32_t ncls;
};

// Bounded-length regex: each lane scans its 16-byte chunks plus max_len bytes of
// overlap, restarting at value starts; any match inside a value marks RF_MATCH.
template <typename P>
__device__ void scan_regex_bounded(WaveLds& L, P w, int nr, const DfaView& d, uint32_t s_bot, uint32_t s_mid,
                                   uint32_t max_len) {
  if (nr == 0) return;
  const uint32_t lo = L.r_vs[0];
  const uint32_t hi = L.r_vs[nr - 1] + L.r_vl[nr - 1];
  const uint32_t l = threadIdx.x;
  for (uint32_t c0 = (lo & ~15u) + l * 16; c0 < hi; c0 += kEvalThreads * 16) {
    uint32_t c = c0 < lo ? lo : c0;
    int r = find_rec(L, nr, c);
    if (r < 0) r = 0;
    uint32_t send = c0 + 16 + max_len;
    if (send > hi) send = hi;
    uint32_t q = c;
    bool have_state = false;
    uint32_t st = 0;
    while (q < send && r < nr) {
      const uint32_t vs = L.r_vs[r], ve = vs + L.r_vl[r];
      if (q >= ve) {
        if (have_state && (d.acc[st] & 2)) atomicOr(&L.r_flags[r], RF_MATCH);
        have_state = false;
        r++;
        continue;
      }
      if (q < vs) {
        q = vs;
        have_state = false;
        continue;
      }
      if (!have_state) {
        st = (q == vs) ? s_bot : s_mid;
        have_state = true;
        if (d.acc[st] & 1) {
          atomicOr(&L.r_flags[r], RF_MATCH);
          q = ve;
          continue;
        }
      }
      st = d.trans[st * d.ncls + d.cls[w[q]]];
      q++;
      if (d.acc[st] & 1) {
        atomicOr(&L.r_flags[r], RF_MATCH);
        q = ve;  // value decided; skip its remainder
        have_state = false;
        r++;
        continue;
      }
    }
    // a value that ends exactly at send: check end-of-text acceptance
    if (have_state && r < nr && q == L.r_vs[r] + L.r_vl[r] && (d.acc[st] & 2)) atomicOr(&L.r_flags[r], RF_MATCH);
  }
}

// serial DFA over one byte sequence (unbounded patterns / short values)
template <typename P>
__device__ bool dfa_run(P s, uint32_t n, const DfaView& d, uint32_t s_bot) {
  uint32_t st = s_bot;
  if (d.acc[st] & 1) return true;
  for (uint32_t i = 0; i < n; i++) {
    st = d.trans[st * d.ncls + d.cls[s[i]]];
    if (d.acc[st] & 1) return true;
  }
  return (d.acc[st] & 2) != 0;
}

// serial full (Unicode) DFA: u16 transitions read through L1/L2
template <typename P>
__device__ bool dfa_run_full(P s, uint32_t n, const uint8_t* blob, const DfaDesc& f, bool upper) {
  const uint8_t* cls = blob + (upper ? f.f_classmap_up : f.f_classmap);
  const uint16_t* tr = (const uint16_t*)(blob + f.f_trans);
  const uint8_t* acc = blob + f.f_accept;
  uint32_t st = f.f_s_bot;
  if (acc[st] & 1) return true;
  for (uint32_t i = 0; i < n; i++) {
    st = tr[st * f.f_nclasses + cls[s[i]]];
    if (acc[st] & 1) return true;
  }
  return (acc[st] & 2) != 0;
}

// a code point of the valid UTF-8 value in the DFA's version-uncertain ranges
// (fsg_u_newer: assigned, or recategorized, after this build's Unicode 13
// tables; binary search over the blob's (lo, hi) pairs)
template <typename P>
__device__ bool utf8_has_newer(P s, uint32_t n, const uint8_t* blob, const DfaDesc& f) {
  const uint32_t* vt = (const uint32_t*)(blob + f.vtab);
  for (uint32_t i = 0; i < n;) {
    const uint32_t c0 = s[i];
    if (c0 < 0x80) {
      i++;
      continue;
    }
    const uint32_t w = c0 < 0xE0 ? 2u : c0 < 0xF0 ? 3u : 4u;
    uint32_t cp = w == 2 ? (c0 & 0x1Fu) : w == 3 ? (c0 & 0x0Fu) : (c0 & 0x07u);
    for (uint32_t k = 1; k < w && i + k < n; k++) cp = (cp << 6) | (s[i + k] & 0x3Fu);
    uint32_t lo = 0, hi = f.vtab_n;
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (vt[2 * m + 1] < cp) lo = m + 1; else hi = m;
    }
    if (lo < f.vtab_n && vt[2 * lo] <= cp) return true;
    i += w;
  }
  return false;
}

// the marked walk (Unicode \b / \B, fsg_regex.h): before each code point the
// marker of its class (0xFC a \w code point, 0xFE \n, 0xFD any other), then
// its bytes; \w membership by binary search over the blob's ranges.  The
// value is valid UTF-8 here (checked before the stage).
template <typename P>
__device__ bool dfa_run_marked(P s, uint32_t n, const uint8_t* blob, const DfaDesc& f, bool upper) {
  const uint8_t* cls = blob + (upper ? f.f_classmap_up : f.f_classmap);
  const uint8_t* mcls = blob + f.f_classmap;  // the markers' classes (uppercasing leaves them)
  const uint16_t* tr = (const uint16_t*)(blob + f.f_trans);
  const uint8_t* acc = blob + f.f_accept;
  const uint32_t* wt = (const uint32_t*)(blob + f.wtab);
  uint32_t st = f.f_s_bot;
  if (acc[st] & 1) return true;
  for (uint32_t i = 0; i < n;) {
    const uint32_t c0 = s[i];
    const uint32_t w = c0 < 0x80 ? 1u : c0 < 0xE0 ? 2u : c0 < 0xF0 ? 3u : 4u;
    uint32_t cp = w == 1 ? c0 : w == 2 ? (c0 & 0x1Fu) : w == 3 ? (c0 & 0x0Fu) : (c0 & 0x07u);
    for (uint32_t k = 1; k < w && i + k < n; k++) cp = (cp << 6) | (s[i + k] & 0x3Fu);
    bool word;
    if (cp < 0x80) {
      word = (cp >= '0' && cp <= '9') || (cp >= 'A' && cp <= 'Z') || (cp >= 'a' && cp <= 'z') || cp == '_';
    } else {
      uint32_t lo = 0, hi = f.wtab_n;
      while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (wt[2 * m + 1] < cp) lo = m + 1; else hi = m;
      }
      word = lo < f.wtab_n && wt[2 * lo] <= cp;
    }
    const uint32_t mk = cp == '\n' ? 0xFEu : word ? 0xFCu : 0xFDu;
    st = tr[st * f.f_nclasses + mcls[mk]];
    if (acc[st] & 1) return true;
    for (uint32_t k = 0; k < w && i + k < n; k++) {
      st = tr[st * f.f_nclasses + cls[s[i + k]]];
      if (acc[st] & 1) return true;
    }
    i += w;
  }
  return (acc[st] & 2) != 0;
}

// ---------------------------------------------------------------------------
// evaluate the chain (stages [0, nst)) over the records of one window
// ---------------------------------------------------------------------------
template <uint32_t kOps, bool kLds, typename P>
__device__ __forceinline__ void eval_window(WaveLds& L, P w, uint32_t wlen, int nr, const ChainDesc& ch, const uint8_t* blob,
                            int nst, int lds_stage, bool& unsupported, uint64_t wbase, ElemRec* elem) {
  const uint32_t l = threadIdx.x;
  bool nonascii_done = false;
  for (int s = 0; s < nst; s++) {
    const StageDesc sd = ch.st[s];  // by value: one scalar load, no re-reads inside the loops
    const uint8_t op = sd.op;
    const bool src = sd.in_type != VT_I32;
    const bool upper = sd.in_type == VT_SRC_UPPER;
    if (op == OP_MAP_UPPER) continue;  // value representation changes statically
    const bool need_utf8 = src && (op == OP_CONTAINS || op == OP_REGEX || op == OP_FILTER_ODD ||
                                   op == OP_MAP_DOUBLE || op == OP_AGG_SUM || op == OP_AGG_CONCAT ||
                                   op == OP_LB_MAX || op == OP_DEDUP);
    // ---- data-parallel phase over window bytes
    for (int r = l; r < nr; r += kEvalThreads) L.r_flags[r] &= ~RF_MATCH;
    __syncthreads();
    if ((kOps & opbit(OP_CONTAINS)) && src && op == OP_CONTAINS) {
      scan_contains<kLds>(L, w, wlen, nr, blob + sd.needle, sd.needle_len, upper, !nonascii_done);
      nonascii_done = true;
    } else if (need_utf8 && !nonascii_done) {
      scan_nonascii<kLds>(L, w, wlen, nr);
      nonascii_done = true;
    }
    DfaView dv;
    if ((kOps & opbit(OP_REGEX)) && op == OP_REGEX) {
      const bool in_lds = s == lds_stage;
      dv.cls = in_lds ? (upper ? g_dyn_lds + 256 : g_dyn_lds) : blob + (upper ? sd.dfa.classmap_up : sd.dfa.classmap);
      dv.trans = in_lds ? g_dyn_lds + 768 : blob + sd.dfa.trans;
      dv.acc = in_lds ? g_dyn_lds + 512 : blob + sd.dfa.accept;
      dv.ncls = sd.dfa.nclasses;
      if (src && sd.dfa.max_len >= 0)
        scan_regex_bounded(L, w, nr, dv, sd.dfa.s_bot, sd.dfa.s_mid, (uint32_t)sd.dfa.max_len);
    }
    __syncthreads();
    // ---- per-record phase (thread per record; record r = 4 * lane + wave so
    // that the records of a window are spread over the four waves)
    static_assert(kMaxR <= kEvalThreads, "one pass covers every record");
    for (int r = (int)(((l & 63u) << 2) | (l >> 6)); r < nr; r += kEvalThreads) {
      uint32_t f = L.r_flags[r];
      if (!(f & RF_ALIVE)) continue;
      const uint32_t vs = L.r_vs[r], vl = L.r_vl[r];
      if (need_utf8 && (f & RF_NONASCII) && !(f & RF_UTF8_DONE)) {
        uint32_t vut = 0, el = 0;
        if (!utf8_check(w + vs, vl, &vut, &el)) {
          f |= RF_UTF8_BAD;
          L.r_aux[r] = vut;
          L.r_aux2[r] = el;
        }
        f |= RF_UTF8_DONE;
      }
      bool err = false;
      uint32_t ec = 0;
      const int32_t ival_in = L.r_ival[r];
      if ((kOps & (opbit(OP_AGG_SUM) | opbit(OP_AGG_CONCAT))) && (op == OP_AGG_SUM || op == OP_AGG_CONCAT) &&
          sd.acc_bad) {
        err = true;
        ec = EC_ACC_UTF8;
        L.r_aux[r] = sd.acc_vut;
        L.r_aux2[r] = sd.acc_elen;
      } else if (need_utf8 && (f & RF_UTF8_BAD)) {
        err = true;
        ec = EC_UTF8;
      } else {
        switch (op) {
          case OP_CONTAINS: {
            if constexpr (!(kOps & opbit(OP_CONTAINS))) break;
            bool keep;
            if (src) {
              keep = (f & RF_MATCH) || sd.needle_len == 0;
            } else {
              uint8_t t[12];
              uint32_t n = fmt_i32(ival_in, t);
              keep = sd.needle_len == 0;
              const uint8_t* nd = blob + sd.needle;
              for (uint32_t i = 0; !keep && i + sd.needle_len <= n; i++) {
                uint32_t k = 0;
                while (k < sd.needle_len && t[i + k] == nd[k]) k++;
                keep = k == sd.needle_len;
              }
            }
            if (!keep) f &= ~RF_ALIVE;
            break;
          }
          case OP_REGEX: {
            if constexpr (!(kOps & opbit(OP_REGEX))) break;
            bool m;
            if (src) {
              if (f & RF_NONASCII) {
                if ((sd.dfa.unicode_word && !sd.dfa.f_marked) ||
                    (sd.dfa.vtab_n && utf8_has_newer(w + vs, vl, blob, sd.dfa))) {
                  // (?-u) \b on a non-ASCII value, or a code point whose class
                  // membership differs between Unicode versions: surfaces only if
                  // this record is reached
                  err = true;
                  ec = EC_UNSUP;
                  break;
                }
                m = sd.dfa.f_marked ? dfa_run_marked(w + vs, vl, blob, sd.dfa, upper)
                                    : dfa_run_full(w + vs, vl, blob, sd.dfa, upper);
              } else if (sd.dfa.max_len >= 0) {
                m = (f & RF_MATCH) != 0;
                // an empty value is never visited by the chunk scan
                if (vl == 0) m = dfa_run(w + vs, 0u, dv, sd.dfa.s_bot);
              } else {
                m = dfa_run(w + vs, vl, dv, sd.dfa.s_bot);
              }
            } else {
              uint8_t t[12];
              uint32_t n = fmt_i32(ival_in, t);
              m = dfa_run((const uint8_t*)t, n, dv, sd.dfa.s_bot);
            }
            bool keep = sd.keep_match ? m : !m;
            if (!keep) f &= ~RF_ALIVE;
            break;
          }
          case OP_FILTER_JSON: {
            if constexpr (!(kOps & opbit(OP_FILTER_JSON))) break;
            uint8_t t[12];
            const uint8_t* js = (const uint8_t*)&w[vs];
            uint32_t jn = vl;
            if (!src) {
              jn = fmt_i32(ival_in, t);
              js = t;
            }
            const JRes jr = json_structured_log(js, jn, src && upper);
            if (!jr.ok) {
              err = true;
              ec = EC_JSON | ((uint32_t)jr.code << 8) | ((uint32_t)jr.sub << 16);
              L.r_aux[r] = jr.pos;
              L.r_aux2[r] = jr.a;
              L.r_aux3[r] = jr.b;
            } else if (jr.level == 0) {
              f &= ~RF_ALIVE;  // level > Debug keeps the record
            }
            break;
          }
          case OP_ARRAY_MAP: {
            // array_map_json_array: serde_json::from_slice::<Vec<Value>> (no from_utf8 first)
            if constexpr (!(kOps & opbit(OP_ARRAY_MAP))) break;
            uint8_t t[12];
            const uint8_t* js = (const uint8_t*)&w[vs];
            uint32_t jn = vl;
            if (!src) {
              jn = fmt_i32(ival_in, t);
              js = t;
            }
            const uint64_t av = wbase + vs;
            uint32_t ne = 0;
            const JRes jr = json_array_explode(js, jn, src && upper, elem + (av >> 1), av, &ne);
            if (!jr.ok) {
              err = true;
              if (jr.code == JE_UNSUP) {
                ec = EC_UNSUP;
              } else {
                ec = EC_JSON | ((uint32_t)jr.code << 8) | ((uint32_t)jr.sub << 16);
                L.r_aux[r] = jr.pos;
                L.r_aux2[r] = jr.a;
                L.r_aux3[r] = jr.b;
              }
            } else {
              L.r_ival[r] = (int32_t)ne;  // element count
              if (jr.sub) L.bs.pad = 1u;  // non-verbatim elements (same value from every lane)
            }
            break;
          }
          case OP_AGG_JSON: {
            // aggregate-json: serde_json::from_slice::<HashMap<String, u32>> of the
            // value (the accumulator side never fails: unwrap_or_default); the
            // entries go to elem[], k_aggj folds them in stream order
            if constexpr (!(kOps & opbit(OP_AGG_JSON))) break;
            uint8_t t[12];
            const uint8_t* js = (const uint8_t*)&w[vs];
            uint32_t jn = vl;
            if (!src) {
              jn = fmt_i32(ival_in, t);
              js = t;
            }
            const uint64_t av = wbase + vs;
            uint32_t ne = 0;
            const JRes jr = json_map_u32(js, jn, src && upper, elem + (av >> 1), av, &ne);
            if (!jr.ok) {
              err = true;
              if (jr.code == JE_UNSUP) {
                ec = EC_UNSUP;
              } else {
                ec = EC_JSON | ((uint32_t)jr.code << 8) | ((uint32_t)jr.sub << 16);
                L.r_aux[r] = jr.pos;
                L.r_aux2[r] = jr.a;
                L.r_aux3[r] = jr.b;
              }
            } else {
              L.r_ival[r] = (int32_t)ne;  // entry count
            }
            break;
          }
          case OP_PROJECT: {
            // map_json_project: the value becomes its field's JSON text (a view
            // into the source value), a missing field drops the record
            if constexpr (!(kOps & opbit(OP_PROJECT))) break;
            uint8_t t[12];
            const uint8_t* js = (const uint8_t*)&w[vs];
            uint32_t jn = vl;
            if (!src) {
              jn = fmt_i32(ival_in, t);
              js = t;
            }
            uint32_t ps = 0, pl = 0;
            bool found = false;
            const JRes jr = json_project(js, jn, src && upper, blob + sd.needle, sd.needle_len, &ps, &pl, &found);
            if (!jr.ok) {
              err = true;
              if (jr.code == JE_UNSUP) {
                ec = EC_UNSUP;
              } else {
                ec = EC_JSON | ((uint32_t)jr.code << 8) | ((uint32_t)jr.sub << 16);
                L.r_aux[r] = jr.pos;
                L.r_aux2[r] = jr.a;
                L.r_aux3[r] = jr.b;
              }
            } else if (!found) {
              f &= ~RF_ALIVE;
            } else {
              L.r_vs[r] = vs + ps;  // valid JSON text: valid UTF-8 from here on
              L.r_vl[r] = pl;
              f = (f | RF_UTF8_DONE) & ~RF_UTF8_BAD;
            }
            break;
          }
          case OP_AGG_CONCAT: {
            // aggregate: acc.push_str(from_utf8(value)?) — the bytes this record appends
            if constexpr (!(kOps & opbit(OP_AGG_CONCAT))) break;
            L.r_ival[r] = src ? (int32_t)vl : (int32_t)dec_len_i32(ival_in);
            if (!src) L.r_ival_in[r] = ival_in;
            break;
          }
          case OP_FILTER_ODD:
          case OP_MAP_DOUBLE:
          case OP_FILTER_MAP:
          case OP_AGG_SUM:
          case OP_LB_MAX: {
            if constexpr (!(kOps & (opbit(OP_FILTER_ODD) | opbit(OP_MAP_DOUBLE) | opbit(OP_FILTER_MAP) |
                                    opbit(OP_AGG_SUM) | opbit(OP_LB_MAX))))
              break;
            int32_t x = 0;
            int pk = 0;
            if (src) {
              uint32_t b = 0, e = vl;
              if (op == OP_AGG_SUM) utf8_trim(w + vs, vl, &b, &e);
              pk = parse_i32(w + vs + b, e - b, &x);
            } else {
              x = ival_in;
            }
            if (pk) {
              err = true;
              ec = EC_PARSE;
              L.r_aux[r] = (uint32_t)pk;
              break;
            }
            if (op == OP_FILTER_ODD) {
              if (x % 2 != 0) f &= ~RF_ALIVE;
            } else if (op == OP_MAP_DOUBLE) {
              L.r_ival[r] = (int32_t)((uint32_t)x * 2u);
            } else if (op == OP_FILTER_MAP) {
              if (x % 2 == 0)
                L.r_ival[r] = x / 2;
              else
                f &= ~RF_ALIVE;
            } else {
              // aggregate input (running sum formed by the cross-batch scan) /
              // filter_look_back value (kept or not by k_sf_compact)
              L.r_ival[r] = x;
            }
            break;
          }
          default: break;
        }
      }
      if (err) {
        f &= ~RF_ALIVE;
        L.r_es[r] = (uint8_t)s;
        L.r_ec[r] = ec;
        L.r_ival_in[r] = ival_in;
      }
      L.r_flags[r] = f;
    }
    __syncthreads();
  }
}

// stage window bytes [al, al+wlen) into LDS: 1 KiB LDS-DMA pieces
// (global_load_lds_dwordx4, one per wave instruction), all issued before one wait
__device__ __forceinline__ void load_window(WaveLds& L, const uint8_t* slice, uint64_t al, uint32_t wlen) {
  const uint32_t l = lane_id();
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t npieces = (wlen + 1023) / 1024;
  const uint8_t* src = slice + al + l * 16;
  for (uint32_t k = wv; k < npieces; k += kEvalThreads / 64)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + k * 1024),
                                     (__attribute__((address_space(3))) void*)(L.win + k * 1024), 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);  // all counters: the LDS-DMA pieces have landed
  __syncthreads();
}

// ---------------------------------------------------------------------------
// k_eval — one 256-thread (4-wave) workgroup per stored batch: the window is
// shared, the scans and per-record work spread over the 4 waves, the serial
// walk and the ordered emission run on wave 0
// ---------------------------------------------------------------------------
#ifdef FSG_EVAL_TIMING  // experiment builds: per-phase clock sums of workgroup 0, printed at its end
__shared__ unsigned long long et_acc[6];
#define ET_MARK(v) const unsigned long long v = (threadIdx.x == 0) ? (unsigned long long)clock64() : 0ull
#define ET_ADD(i, a0, a1) \
  if (threadIdx.x == 0) et_acc[i] += (a1) - (a0)
#else
#define ET_MARK(v)
#define ET_ADD(i, a0, a1)
#endif
template <uint32_t kOps>
__device__ __forceinline__ void eval_batch(const EvalArgs& a, WaveLds& L, const uint32_t b, ParLds* PL = nullptr) {
  const uint32_t l = lane_id();
  const uint32_t tid = threadIdx.x;
  const bool wave0 = tid < 64;
  const ChainDesc& ch = *a.chain;
  const uint8_t* S = a.slice;
  const uint64_t pos = a.bpos[b];
  // ---- batch header (file format, batch.rs:163-180)
  // the first window starts at the batch header: one LDS-DMA burst brings the
  // header, the record count and (for batches up to ~17 KB) every record
  const uint64_t al0 = pos & ~15ull;
  load_window(L, S, al0, kWin);
  const uint8_t* h = L.win + (pos - al0);
  const int32_t batch_len = (int32_t)rd_be(h + 8, 4);
  if (tid == 0) {
    L.bs.base_offset = (int64_t)rd_be(h, 8);
    L.bs.lod_in = (int32_t)rd_be(h + 23, 4);
    L.bs.first_ts = (int64_t)rd_be(h + 27, 8);
    L.bs.comp = (uint32_t)rd_be(h + 22, 1) & 7u;
    L.bs.err_code = 0;
    L.bs.err_pos = 0;
    L.bs.err_od = 0;
    L.bs.err_ival = 0;
    L.bs.err_aux = 0;
    L.bs.err_aux2 = 0;
    L.bs.err_aux3 = 0;
    L.bs.pad = 0;  // set: array elements for k_canon_len / k_write_canon
  }
  const uint64_t sec0 = pos + 57;
  const uint64_t sec_end = pos + 12 + (uint64_t)(uint32_t)batch_len;  // framing validated at ingest
  const uint32_t sec_len = (uint32_t)(sec_end - sec0);
  // ---- stage the DFA of a regex stage into LDS (first one that fits)
  int lds_stage = -1;
  for (int s = 0; s < (int)ch.nstages; s++) {
    const StageDesc& sd = ch.st[s];
    if (sd.op == OP_REGEX && sd.dfa.nstates * sd.dfa.nclasses <= (uint32_t)kDfaLds) {
      lds_stage = s;
      for (uint32_t i = tid; i < 256; i += kEvalThreads) {
        g_dyn_lds[i] = a.blob[sd.dfa.classmap + i];
        g_dyn_lds[256 + i] = a.blob[sd.dfa.classmap_up + i];
        g_dyn_lds[512 + i] = i < sd.dfa.nstates ? a.blob[sd.dfa.accept + i] : 0;
      }
      for (uint32_t i = tid; i < sd.dfa.nstates * sd.dfa.nclasses; i += kEvalThreads)
        g_dyn_lds[768 + i] = a.blob[sd.dfa.trans + i];
      break;
    }
  }
  // ---- Vec<Record> count (decoder.rs:43-55)
  uint32_t flags = 0;
  int32_t count = 0;
  if (sec_len < 4) {
    flags |= BF_DECODE;
  } else {
    count = (int32_t)rd_be(L.win + (sec0 - al0), 4);
  }
  bool first_window = true;  // the window at al0 is already resident
  const uint32_t nrec_total = count > 0 ? (uint32_t)count : 0u;
  // record starts from k_chase_w / k_chase when they framed this batch
  uint32_t rend_b = a.rend ? a.rend[b] : 0xFFFFu;
  const uint16_t* rsb = (a.rstart && rend_b != 0xFFFFu) ? a.rstart + a.rbase[b] : nullptr;
  const uint64_t rb = a.rbase[b];
  // many small records in a resident section: framed in parallel (par_frame),
  // the window kept for every group of kMaxR records
  bool resident = false;
  ET_MARK(tp0);
  if (PL && !rsb && nrec_total > (uint32_t)kMaxR && nrec_total <= (uint32_t)kParMaxR &&
      sec_end + 16 <= al0 + (uint64_t)kWin) {
    if (par_frame((const uint8_t*)L.win, *PL, (uint32_t)(sec0 + 4 - al0), (uint32_t)(sec_end - al0), nrec_total)) {
      rsb = PL->rs;
      rend_b = (uint32_t)(sec_end - al0);
      resident = true;
    }
  }
  ET_MARK(tp1);
  ET_ADD(0, tp0, tp1);
#ifdef FSG_EVAL_TIMING
  if (threadIdx.x == 0) et_acc[5] += resident ? 1000000ull : 1ull;
#endif
  // phase A: full chain; phase B (only if a record error occurred): truncated
  // chain.  A pass-through batch runs no stage: its records are kept as they are.
  const bool passthru = a.pass && a.pass[b];
  int nst = passthru ? 0 : (int)ch.nstages;
  uint32_t err_stage = 0xFFFFFFFFu, err_idx = 0xFFFFFFFFu;
  bool unsupported = false;
  uint32_t kcount = 0, nout = 0;
  int64_t aggsum = 0;
  uint64_t catsum = 0;
  for (int phase = 0; phase < 2 && !(flags & BF_DECODE); phase++) {
    if (phase == 1) {
      if (err_stage == 0xFFFFFFFFu) break;
      nst = (int)err_stage + 1;
    }
    kcount = 0;
    nout = 0;
    aggsum = 0;
    catsum = 0;
    uint64_t cursor = sec0 + 4;
    uint32_t done_recs = 0;
    const uint32_t rec_cap = phase == 1 ? err_idx : nrec_total;
    const bool full = nst == (int)ch.nstages;  // this phase's output is the last stage's
    const bool agg_on = (kOps & opbit(OP_AGG_SUM)) && (ch.flags & CF_AGG_SUM) && full;
    const bool cat_on = (kOps & opbit(OP_AGG_CONCAT)) && (ch.flags & CF_AGG_CAT) && full;
    const bool arr_on = (kOps & opbit(OP_ARRAY_MAP)) && (ch.flags & CF_ARRAY) && full;
    const bool aggj_on = (kOps & opbit(OP_AGG_JSON)) && (ch.flags & CF_AGG_JSON) && full;
    const uint8_t last_in = ch.st[ch.nstages - 1].in_type;
    const int last = nst - 1;
    const uint8_t out_type = (nst == (int)ch.nstages) ? (uint8_t)ch.out_type : ch.st[nst].in_type;
    while (done_recs < nrec_total && done_recs < (phase == 1 ? rec_cap + 1 : nrec_total)) {
      // window [al, al + wlen)
      const uint64_t al = (first_window || resident) ? al0 : (cursor & ~15ull);
      uint64_t wend = al + kWin;
      const uint64_t sec_end16 = (sec_end + 15) & ~15ull;
      if (wend > sec_end16) wend = sec_end16;
      const uint32_t wlen = (uint32_t)(wend - al);
      __syncthreads();
      if (!first_window && !resident) load_window(L, S, al, wlen);
      first_window = false;
      ET_MARK(tw0);
      if (!walk_fast(L, (const uint8_t*)L.win, al, wlen, sec_end, cursor, nrec_total - done_recs, rsb, al0, done_recs,
                     rend_b)) {
        if (tid == 0)
          walk_records(L, (const uint8_t*)L.win, al, wlen, sec_end, cursor, nrec_total - done_recs, kMaxR);
        __syncthreads();
      }
      int nr = L.nr;
      const int ws = L.walk_status;
      bool global_mode = false;
      uint64_t gbase = 0;
      if (nr == 0) {
        if (ws == 1) {
          flags |= BF_DECODE;
          break;
        }
        // a record larger than the window: evaluate it from global memory
        global_mode = true;
        gbase = cursor;
        __syncthreads();
        if (tid == 0) walk_records(L, S + gbase, gbase, (uint32_t)(sec_end - gbase), sec_end, cursor, 1, 1);
        __syncthreads();
        nr = L.nr;
        if (nr == 0) {
          flags |= BF_DECODE;
          break;
        }
      }
      // phase B: only records before the error record
      int nr_eval = nr;
      if (phase == 1 && done_recs + (uint32_t)nr > err_idx + 1) nr_eval = (int)(err_idx + 1 - done_recs);
      if (global_mode)
        eval_window<kOps, false>(L, S + gbase, (uint32_t)(sec_end - gbase), nr_eval, ch, a.blob, nst, lds_stage,
                           unsupported, gbase, a.elem);
      else
        eval_window<kOps, true>(L, (const uint8_t*)L.win, wlen, nr_eval, ch, a.blob, nst, lds_stage,
                          unsupported, al, a.elem);
      ET_MARK(tw2);
      ET_ADD(1, tw0, tw2);
      const uint64_t wbase = global_mode ? gbase : al;
      // ---- error tracking (phase A) and descriptor emission: wave 0, in record order
      for (int r0 = 0; wave0 && r0 < nr_eval; r0 += 64) {
        const int r = r0 + (int)l;
        const bool valid = r < nr_eval;
        const uint32_t gidx = done_recs + (uint32_t)r;
        bool is_err = false;
        uint32_t es = 0xFFu;
        if (valid) {
          es = L.r_es[r];
          is_err = es != 0xFFu;
        }
        if (phase == 0) {
          // lexicographic min (stage, index) over the wave
          uint64_t key = is_err ? (((uint64_t)es << 32) | gidx) : ~0ull;
          for (int o = 32; o > 0; o >>= 1) {
            uint64_t t = __shfl_xor(key, o, 64);
            key = t < key ? t : key;
          }
          if (key != ~0ull) {
            const uint32_t ks = (uint32_t)(key >> 32), ki = (uint32_t)key;
            if (ks < err_stage || (ks == err_stage && ki < err_idx)) {
              err_stage = ks;
              err_idx = ki;
              const int rr = (int)(ki - done_recs);
              if (l == 0) {
                L.bs.err_code = L.r_ec[rr];
                L.bs.err_aux = L.r_aux[rr];
                L.bs.err_aux2 = L.r_aux2[rr];
                L.bs.err_aux3 = L.r_aux3[rr];
                L.bs.err_ival = L.r_ival_in[rr];
                L.bs.err_pos = wbase + L.r_start[rr];
                L.bs.err_od = L.r_od[rr];
                L.bs.err_vpos = wbase + L.r_vs[rr];
                L.bs.err_vlen = L.r_vl[rr];
              }
            }
          }
        }
        bool kept = valid && !is_err && (L.r_flags[r] & RF_ALIVE);
        if (phase == 1 && gidx >= err_idx) kept = false;
        const uint64_t bal = ballot(kept);
        const uint32_t pre = (uint32_t)__popcll(bal & ((1ull << l) - 1ull));
        int32_t local = 0;
        uint32_t cat_local = 0;
        uint32_t outs = kept ? 1u : 0u;
        if (arr_on) outs = kept ? (uint32_t)L.r_ival[r] : 0u;
        if (cat_on) {
          // u32 inclusive scan of the appended byte counts
          uint32_t uv = kept ? (uint32_t)L.r_ival[r] : 0u;
          for (int o = 1; o < 64; o <<= 1) {
            uint32_t t = __shfl_up(uv, o, 64);
            if ((int)l >= o) uv += t;
          }
          cat_local = (uint32_t)catsum + uv;
          catsum += __shfl(uv, 63, 64);
        }
        nout += (uint32_t)wave_sum(outs);
        if (agg_on) {
          int32_t v = kept ? L.r_ival[r] : 0;
          // wrapping i32 inclusive scan
          uint32_t uv = (uint32_t)v;
          for (int o = 1; o < 64; o <<= 1) {
            uint32_t t = __shfl_up(uv, o, 64);
            if ((int)l >= o) uv += t;
          }
          local = (int32_t)((uint32_t)aggsum + uv);
          aggsum = (int64_t)(int32_t)((uint32_t)aggsum + (uint32_t)__shfl(uv, 63, 64));
        }
        if (kept) {
          KeptRec d;
          d.src = wbase + L.r_start[r];
          d.od = L.r_od[r];
          const uint32_t klen = L.r_klen[r];
          d.kpos = L.r_haskey[r] ? (wbase + L.r_kpos[r]) : 0;
          d.klen = klen;
          d.has_key = L.r_haskey[r];
          d.attr = L.r_attr[r];
          d.ts = L.r_ts[r];
          d.hdr = L.r_hdr[r];
          d.vpos = wbase + L.r_vs[r];
          d.vlen = L.r_vl[r];
          d.pad = 0;
          if (agg_on) {
            d.mode = KM_AGG;
            d.ival = local;
          } else if (arr_on) {
            d.mode = KM_ARRAY;
            d.ival = L.r_ival[r];
            d.pad = last_in == VT_SRC_UPPER ? KF_UPPER : 0;
          } else if (aggj_on) {
            d.mode = KM_AGGJ;  // vpos locates the entries; k_aggj sets src / vlen to the map text in cat
            d.ival = L.r_ival[r];
            d.pad = last_in == VT_SRC_UPPER ? KF_UPPER : 0;
          } else if (cat_on) {
            d.mode = KM_CONCAT;
            d.ival = (int32_t)cat_local;
            if (last_in == VT_I32) {
              d.pad = KF_I32;
              d.vlen = (uint32_t)L.r_ival_in[r];
            } else {
              d.pad = last_in == VT_SRC_UPPER ? KF_UPPER : 0;
            }
          } else if (out_type == VT_I32) {
            d.mode = KM_I32;
            d.ival = L.r_ival[r];
          } else {
            d.mode = out_type == VT_SRC_UPPER ? KM_UPPER : KM_COPY;
            d.ival = L.r_ival[r];  // filter_look_back: the parsed value for k_sf_*
          }
          a.desc[rb + kcount + pre] = d;
        }
        kcount += (uint32_t)__popcll(bal);
      }
      if (tid == 0) {
        L.err_stage_b = err_stage;
        L.err_idx_b = err_idx;
      }
      __syncthreads();
      err_stage = L.err_stage_b;  // every wave learns the first error (uniform control flow)
      err_idx = L.err_idx_b;
      done_recs += (uint32_t)nr;
      cursor = ((uint64_t)L.next_cursor_hi << 32) | L.next_cursor_lo;
      ET_MARK(tw3);
      ET_ADD(2, tw2, tw3);
#ifdef FSG_EVAL_TIMING
      if (threadIdx.x == 0) et_acc[3] += 1;
#endif
      (void)last;
    }
    if (phase == 0 && err_stage == 0xFFFFFFFFu) break;
  }
  unsupported = __syncthreads_or(unsupported);  // also orders lane 0's L.bs writes
  if (tid == 0) {
    if (!(flags & BF_DECODE) && err_stage != 0xFFFFFFFFu)
      flags |= (L.bs.err_code == EC_UNSUP) ? BF_UNSUPPORTED : BF_ERR;
    if (!passthru && (err_stage == 0xFFFFFFFFu || err_stage + 1 == ch.nstages)) flags |= BF_LAST_STAGE;
    if (unsupported) flags |= BF_UNSUPPORTED;
    BatchStat st = L.bs;
    st.flags = flags;
    st.nkeep = kcount;
    st.sec_len = sec_len;
    st.err_stage = err_stage;
    const bool agg_ran = !passthru && (err_stage == 0xFFFFFFFFu || err_stage + 1 == ch.nstages);
    st.agg_sum = (ch.has_agg && agg_ran) ? aggsum : 0;
    st.nout = nout;
    st.cat_sum = (ch.has_agg && agg_ran) ? catsum : 0;
    a.bstat[b] = st;  // the cross-batch minima are reduced by k_mins
  }
}

// k_eval: batches blockIdx.x (direct mode) or the deferred list written by
// k_eval_lean (list mode: a.list[0] = count, a.list[1..] = batch indices)
template <uint32_t kOps>
__global__ __launch_bounds__(kEvalThreads, (kOps == kOpsContains) ? 4 : 2) void k_eval(EvalArgs a) {
  __shared__ WaveLds L;
  const uint32_t n = a.list ? a.list[0] : a.nbatches;
  if constexpr (kOps == kOpsInt || kOps == kOpsAll) {  // batches of many small records: parallel framing
    __shared__ ParLds P;
#ifdef FSG_EVAL_TIMING
    if (threadIdx.x < 6) et_acc[threadIdx.x] = 0;
    __syncthreads();
    const unsigned long long tk0 = clock64();
#endif
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
      eval_batch<kOps>(a, L, a.list ? a.list[1 + i] : i, &P);
      __syncthreads();
    }
#ifdef FSG_EVAL_TIMING
    if (threadIdx.x == 0 && blockIdx.x == 0)
      printf("k_eval timing wg0: total %llu par %llu walk+eval %llu emit %llu windows %llu resident %llu\n",
             (unsigned long long)(clock64() - tk0), et_acc[0], et_acc[1], et_acc[2], et_acc[3], et_acc[5]);
#endif
  } else {
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
      eval_batch<kOps>(a, L, a.list ? a.list[1 + i] : i);
      __syncthreads();  // the window is reused by the next batch
    }
  }
}

// ---------------------------------------------------------------------------
// k_mins: first surviving / erroring / undecodable / unsupported batch
// ---------------------------------------------------------------------------
__device__ __forceinline__ void mins_body(const BatchStat* bstat, uint32_t n, Mins* mins, uint32_t bid, uint32_t gdim) {
  __shared__ uint32_t sh[4][4];
  uint32_t fk = 0xFFFFFFFFu, fe = 0xFFFFFFFFu, fd = 0xFFFFFFFFu, fu = 0xFFFFFFFFu;
  for (uint32_t b = bid * 256 + threadIdx.x; b < n; b += gdim * 256) {
    const uint32_t f = bstat[b].flags;
    const uint32_t nk = bstat[b].nout;  // batches whose stage output is non-empty
    if (f & BF_DECODE) fd = fd < b ? fd : b;
    if (f & BF_UNSUPPORTED) fu = fu < b ? fu : b;
    if (!(f & BF_DECODE)) {
      if (nk) fk = fk < b ? fk : b;
      if (f & BF_ERR) fe = fe < b ? fe : b;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t t;
    t = __shfl_xor(fk, o, 64); fk = t < fk ? t : fk;
    t = __shfl_xor(fe, o, 64); fe = t < fe ? t : fe;
    t = __shfl_xor(fd, o, 64); fd = t < fd ? t : fd;
    t = __shfl_xor(fu, o, 64); fu = t < fu ? t : fu;
  }
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w][0] = fk; sh[w][1] = fe; sh[w][2] = fd; sh[w][3] = fu;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    uint32_t m = sh[0][threadIdx.x];
    for (int k = 1; k < 4; k++) m = sh[k][threadIdx.x] < m ? sh[k][threadIdx.x] : m;
    if (m != 0xFFFFFFFFu) atomicMin(&((uint32_t*)mins)[threadIdx.x], m);  // first_keep, first_err, first_dec, first_unsup
  }
}
__global__ __launch_bounds__(256) void k_mins(const BatchStat* bstat, uint32_t n, Mins* mins) {
  mins_body(bstat, n, mins, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------
// output record size of a descriptor after the offset fix-up
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t out_vlen(const KeptRec& d, int32_t agg_base, uint64_t cat_base) {
  if (d.mode == KM_I32) return dec_len_i32(d.ival);
  if (d.mode == KM_AGG) return dec_len_i32((int32_t)((uint32_t)agg_base + (uint32_t)d.ival));
  if (d.mode == KM_CONCAT) return (uint32_t)(cat_base + (uint32_t)d.ival);  // whole accumulator after this record
  return d.vlen;
}
__device__ __forceinline__ uint32_t rec_out_size(const KeptRec& d, int64_t rel, int32_t agg_base, uint64_t cat_base) {
  const uint32_t vl = out_vlen(d, agg_base, cat_base);
  uint32_t inner = 1 + vsize(d.ts) + vsize(d.od + rel) + 1 + (d.has_key ? vsize((int64_t)d.klen) + d.klen : 0) +
                   vsize((int64_t)vl) + vl + vsize(d.hdr);
  return vsize((int64_t)inner) + inner;
}
// one array_map output record: Record::new_key_value(None, element) — default
// preamble (attributes 0, timestamp_delta 0, offset_delta 0 + rel, no headers)
__device__ __forceinline__ uint32_t elem_inner(uint32_t len, int64_t rel) {
  return 1 + 1 + vsize(rel) + 1 + vsize((int64_t)len) + len + 1;
}
__device__ __forceinline__ uint32_t elem_out_size(uint32_t len, int64_t rel) {
  const uint32_t inner = elem_inner(len, rel);
  return vsize((int64_t)inner) + inner;
}
// Σ output record sizes of the elements of one KM_ARRAY record
__device__ __forceinline__ uint64_t array_rec_bytes(const KeptRec& d, const ElemRec* elem, int64_t rel) {
  // k_arr_lean's sums: every element shorter than 40 bytes has an inner length
  // below 64 (one varint byte), so its record is 5 + vsize(rel) + vsize(len) + len
  if ((d.pad & KF_ESUM) && d.hdr == 0) return (uint64_t)d.ival * (5 + vsize(rel)) + (uint64_t)d.ts;
  const ElemRec* e = elem + (d.vpos >> 1);
  uint64_t s = 0;
  for (int32_t j = 0; j < d.ival; j++) s += elem_out_size(e[j].out_len & 0x7FFFFFFFu, rel);
  return s;
}

// k_size: one wave per batch (4 batches per 256-thread block)
__device__ __forceinline__ void size_batch(const SizeArgs& a, uint32_t b) {
  const uint32_t l = lane_id();
  const BatchStat st = a.bstat[b];
  const uint32_t f = a.mins->first_keep;
  // a flat decide already wrote this row for f = 0 (the offset fix-up against batch 0)
  if ((st.flags & BF_ROWDONE) && f == 0 && a.mins->carry == 0xFFFFFFFFu && !a.seg && !a.agg_only) return;
  ScanRow row = {};
  if (a.agg_only) {
    row.agg = st.agg_sum;
    row.cat = st.cat_sum;
    if (l == 0) a.rows[b] = row;
    return;
  }
  row.bytes_in = st.sec_len;
  row.recs_out = (st.flags & BF_LAST_STAGE) ? st.nout : 0;
  row.agg = st.agg_sum;
  row.cat = st.cat_sum;
  if (f != 0xFFFFFFFFu && b >= f && !(st.flags & BF_DECODE)) {
    const int64_t first_base = a.mins->carry != 0xFFFFFFFFu ? a.mins->carry_base : a.bstat[f].base_offset;
    const int64_t rel = a.seg ? 0 : first_base - st.base_offset;
    const int32_t agg_base = a.agg_pre ? (int32_t)((uint64_t)a.acc0 + (uint64_t)a.agg_pre[b].agg) : 0;
    const uint64_t cat_base = a.agg_pre ? a.acc_len + a.agg_pre[b].cat : 0;
    uint64_t sum = 0;
    if (st.flags & BF_ARR_LEAN) {  // k_arr_lean's counts (fsg_array.hip): elements with L >= 60 - vsize(rel)
      const ArrBatch& ab = a.arr_b[b];  // take one more inner-length varint byte
      const uint32_t vr = vsize(rel);
      sum = (uint64_t)ab.ne * (5 + vr) + ab.esum + ab.c59;
      for (uint32_t L = 60 - vr < 50 ? 50 : 60 - vr; L <= 58; L++) sum += ab.cnt[L - 50];
    } else {
      const KeptRec* d = a.desc + a.rbase[b];
      const bool compact = (st.flags & BF_COMPACT) != 0;
      for (uint32_t k = l; k < st.nkeep; k += 64) {
        const KeptRec r = kept_at(d, k, compact);
        sum += r.mode == KM_ARRAY ? array_rec_bytes(r, a.elem, rel) : rec_out_size(r, rel, agg_base, cat_base);
      }
      sum = wave_sum(sum);
    }
    row.rec_bytes = sum;
    row.nonempty = st.nout ? 1 : 0;
    row.lod = (uint64_t)(int64_t)(st.lod_in + 1);
    row.nrec = st.nout;
  }
  if (l == 0) a.rows[b] = row;
}
__global__ __launch_bounds__(256) void k_size(SizeArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b < a.nbatches) size_batch(a, b);
}

// ---------------------------------------------------------------------------
// cross-batch exclusive scan of ScanRow (3 kernels)
// ---------------------------------------------------------------------------
constexpr int kScanBlock = 256;
constexpr int kScanPer = 8;  // rows per thread
constexpr int kScanTile = kScanBlock * kScanPer;

__device__ __forceinline__ void row_add(ScanRow& a, const ScanRow& b) {
  a.rec_bytes += b.rec_bytes;
  a.nonempty += b.nonempty;
  a.lod += b.lod;
  a.nrec += b.nrec;
  a.bytes_in += b.bytes_in;
  a.recs_out += b.recs_out;
  a.agg = (int64_t)(int32_t)((uint32_t)a.agg + (uint32_t)b.agg);
  a.cat += b.cat;
}

__device__ void block_excl_scan(ScanRow& v, ScanRow* sh, ScanRow& total) {
  // Hillis-Steele over 256 threads through LDS (rows are 64 B)
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int o = 1; o < kScanBlock; o <<= 1) {
    ScanRow x = sh[t];
    if (t >= o) row_add(x, sh[t - o]);
    __syncthreads();
    sh[t] = x;
    __syncthreads();
  }
  total = sh[kScanBlock - 1];
  ScanRow ex = {};
  if (t > 0) ex = sh[t - 1];
  v = ex;
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_scan_reduce(const ScanRow* rows, uint32_t n, ScanRow* tile_sums) {
  __shared__ ScanRow sh[kScanBlock];
  const uint32_t base = blockIdx.x * kScanTile;
  ScanRow acc = {};
  for (int k = 0; k < kScanPer; k++) {
    uint32_t i = base + threadIdx.x * kScanPer + k;
    if (i < n) row_add(acc, rows[i]);
  }
  ScanRow total;
  block_excl_scan(acc, sh, total);
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(256) void k_scan_top(ScanRow* tile_sums, uint32_t ntiles, ScanRow* grand) {
  __shared__ ScanRow sh[kScanBlock];
  ScanRow carry = {};
  for (uint32_t base = 0; base < ntiles; base += kScanBlock) {
    uint32_t i = base + threadIdx.x;
    ScanRow v = {};
    if (i < ntiles) v = tile_sums[i];
    ScanRow total;
    block_excl_scan(v, sh, total);
    row_add(v, carry);
    if (i < ntiles) tile_sums[i] = v;
    row_add(carry, total);
    __syncthreads();
  }
  if (threadIdx.x == 0) *grand = carry;
}

struct ScanDownArgs {
  const ScanRow* rows;
  ScanRow* pre;
  const ScanRow* tile_sums;
  uint32_t n;
  uint32_t detect_cut;
  uint64_t max_bytes;
  Mins* mins;
  const BatchStat* bstat;
};

__device__ __forceinline__ void scan_down_body(const ScanDownArgs& a, uint32_t bid) {
  __shared__ ScanRow sh[kScanBlock];
  const uint32_t base = bid * kScanTile;
  ScanRow acc = {};
  for (int k = 0; k < kScanPer; k++) {
    uint32_t i = base + threadIdx.x * kScanPer + k;
    if (i < a.n) row_add(acc, a.rows[i]);
  }
  ScanRow total;
  block_excl_scan(acc, sh, total);
  ScanRow run = a.tile_sums ? a.tile_sums[bid] : ScanRow{};  // null: the slice is one tile
  row_add(run, acc);
  const uint32_t f = a.mins->first_keep;
  for (int k = 0; k < kScanPer; k++) {
    uint32_t i = base + threadIdx.x * kScanPer + k;
    if (i >= a.n) break;
    const ScanRow v = a.rows[i];
    a.pre[i] = run;
    row_add(run, v);
    // max_bytes cut (batch.rs:101-111): total + records.write_size(0) > max_bytes
    if (a.detect_cut && f != 0xFFFFFFFFu && i >= f && v.nonempty) {
      const uint64_t incl = run.rec_bytes + 4ull * run.nonempty;
      if (incl > a.max_bytes) atomicMin(&a.mins->cut, i);
    }
  }
}
__global__ __launch_bounds__(256) void k_scan_down(ScanDownArgs a) { scan_down_body(a, blockIdx.x); }

// ---------------------------------------------------------------------------
// k_plan: the process_batch stop rules (batch.rs:41-142), one thread
// ---------------------------------------------------------------------------


__device__ __forceinline__ ScanRow incl_at(const PlanArgs& a, uint32_t i) {
  ScanRow r = a.pre[i];
  row_add(r, a.rows[i]);
  return r;
}

__device__ __forceinline__ void plan_run(const PlanArgs& a) {
  const uint32_t NONE = 0xFFFFFFFFu;
  const uint32_t n = a.nbatches;
  const uint32_t f = a.mins->first_keep, e = a.mins->first_err, d = a.mins->first_dec, u = a.mins->first_unsup;
  const uint32_t c = a.mins->cut;
  Plan p = {};
  p.err_batch = -1;
  p.first = -1;
  p.last = -1;
  p.stop = -1;
  p.done = -1;
  p.lod = -1;
  p.base_offset = -1;
  // stop batch: min(error batch, cut batch); the cut batch was processed too
  uint32_t stop = n ? n - 1 : NONE;
  bool cut = false, err = false;
  if (c != NONE && (e == NONE || c <= e)) {
    stop = c;
    cut = true;
    err = (c == e);
  } else if (e != NONE) {
    stop = e;
    err = true;
  }
  int status = 0;
  uint32_t fail_at = NONE;
  if (d != NONE && (stop == NONE || d <= stop)) {
    status = a.empty_chain ? -104 : -11;  // FSG_E_IO / FSG_E_DECODING_BASE_INPUT
    fail_at = d;
  }
  if (u != NONE && (stop == NONE || u <= stop) && (fail_at == NONE || u < fail_at)) {
    status = -103;  // FSG_E_UNSUPPORTED
    fail_at = u;
  }
  if (status == 0 && a.tail_status != 0 && !cut && !err) {
    status = a.tail_status;  // the iterator hit a bad batch after the last framed one
  }
  if (status != 0) {
    p.status = status;
    // process() completed for the batches before the failing one (all of them
    // when the iterator failed after the last framed batch)
    p.done = fail_at != NONE ? (int32_t)fail_at - 1 : (int32_t)n - 1;
    // FSG_E_UNSUPPORTED: the input is valid for the reference and the caller
    // falls back (e.g. to wasm) and replays it, so no state moves; a segment
    // keeps `done` (its output slice ends there, the final stop decides)
    if (status == -103 && !a.seg) p.done = -1;
    const uint32_t m = fail_at != NONE ? fail_at : (n ? n - 1 : NONE);
    if (m != NONE) {
      ScanRow r = incl_at(a, m);
      p.bytes_in = r.bytes_in;
      p.invocations = m + 1;
    }
    if (a.has_agg && p.done >= 0) {
      // the aggregate's accumulator after the completed calls: the chain
      // instance keeps it although process_batch returns the error
      // (smartengine batch loop: `process(input)?` per batch)
      const ScanRow rd = incl_at(a, (uint32_t)p.done);
      p.acc_final = (int64_t)(int32_t)((uint64_t)a.acc0 + (uint64_t)rd.agg);
      p.cat_final = rd.cat;
      p.acc_touched = rd.recs_out > 0;
      p.stop = p.done;  // k_cat appends through it
    }
    *a.plan = p;
    return;
  }
  if (stop == NONE) {  // no batches at all
    *a.plan = p;
    return;
  }
  p.stop = (int32_t)stop;
  p.done = (int32_t)stop;
  const ScanRow rs = incl_at(a, stop);
  p.bytes_in = rs.bytes_in;
  p.invocations = stop + 1;
  p.records_out = rs.recs_out;
  if (a.has_agg) {
    p.acc_final = (int64_t)(int32_t)((uint64_t)a.acc0 + (uint64_t)rs.agg);
    p.cat_final = rs.cat;
    p.acc_touched = rs.recs_out > 0;  // aggregate emits one record per aggregated input
  }
  const int64_t last = cut ? (int64_t)c - 1 : (int64_t)stop;
  if (err) p.err_batch = (int32_t)e;
  if (f != NONE && f <= stop) {
    p.first = (int32_t)f;
    // set before the max_bytes check (batch.rs:85-91); set_compression of the
    // first surviving batch — a continuation carries both from an earlier chunk
    const bool carry = a.mins->carry != 0xFFFFFFFFu;
    p.base_offset = carry ? a.mins->carry_base : a.bstat[f].base_offset;
    p.comp = carry ? (int32_t)(a.mins->carry & 7u) : (int32_t)a.bstat[f].comp;
    if ((int64_t)f <= last) {
      p.last = (int32_t)last;
      const ScanRow rl = incl_at(a, (uint32_t)last);
      const ScanRow rf = a.pre[f];
      p.lod = (int32_t)(-1 + (int64_t)(rl.lod - rf.lod));
      p.n_records = rl.nrec - rf.nrec;
      p.rec_bytes = rl.rec_bytes - rf.rec_bytes;
      p.nonempty = (int32_t)(rl.nonempty - rf.nonempty);
    }
  }
  *a.plan = p;
}
__global__ void k_plan(PlanArgs a) {
  if (threadIdx.x == 0) plan_run(a);
}

// k_state: the aggregate-sum accumulator after this call, kept in HBM
// (SmartModuleAggregate.accumulator, transforms/aggregate.rs:95): unchanged
// unless the aggregate emitted records
__global__ void k_state(const Plan* plan, int32_t* state) {
  if (threadIdx.x != 0) return;
  const Plan p = *plan;
  if (p.acc_touched) *state = (int32_t)p.acc_final;  // also through `done` when the call fails
}

// ---------------------------------------------------------------------------
// k_seg_headers: a segment's output as the next segment's input slice: per
// batch the source header with batch_len / count of the segment's records for
// it (the records themselves were written by k_write / k_write_lean with
// WriteArgs::seg), positions, record-count prefix and pass-through flags.  The
// next segment decodes these records exactly as the reference's next stage
// decodes SmartModuleInput::try_from_records (engine.rs:160-165).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_seg_headers(SegArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nb) return;
  const uint64_t o = 61ull * b + a.pre[b].rec_bytes;
  const uint8_t* h = a.src + a.bpos[b];
  uint8_t* d = a.dst + o;
  const uint64_t rb = a.rows[b].rec_bytes;
  const uint32_t cnt = (uint32_t)a.rows[b].nrec;
  const uint32_t blen = (uint32_t)(49 + rb);
  if (l < 57) {
    uint8_t x = h[l];
    if (l >= 8 && l < 12) x = (uint8_t)(blen >> (8 * (11 - l)));
    d[l] = x;
  } else if (l < 61) {
    d[l] = (uint8_t)(cnt >> (8 * (60 - l)));
  }
  if (l == 0) {
    a.dbpos[b] = o;
    a.drbase[b] = a.pre[b].nrec;
    a.dpass[b] = ((int32_t)b == a.pass_batch || (a.pass_in && a.pass_in[b])) ? 1 : 0;
  }
}
void launch_seg_headers(const SegArgs& a, hipStream_t s) {
  if (a.nb) hipLaunchKernelGGL(k_seg_headers, dim3((a.nb + 3) / 4), dim3(256), 0, s, a);
}

// ---------------------------------------------------------------------------
// k_header: output batch header (Batch::default() + base offset, lod, count)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void header_run(const Plan* plan, uint8_t* out) {
  const Plan p = *plan;
  uint8_t h[61];
  auto be = [&](int off, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) h[off + i] = (uint8_t)(v >> (8 * (nb - 1 - i)));
  };
  be(0, (uint64_t)p.base_offset, 8);
  be(8, (uint32_t)(45 + 4 + p.rec_bytes), 4);
  be(12, (uint32_t)-1, 4);  // partition_leader_epoch
  h[16] = 2;                // magic
  be(17, 0, 4);             // crc placeholder
  be(21, (uint32_t)p.comp & 7u, 2);  // attributes: the first surviving batch's compression
  be(23, (uint32_t)p.lod, 4);
  be(27, (uint64_t)-1, 8);  // first_timestamp
  be(35, (uint64_t)-1, 8);  // max_time_stamp
  be(43, (uint64_t)-1, 8);  // producer_id
  be(51, (uint16_t)-1, 2);  // producer_epoch
  be(53, (uint32_t)-1, 4);  // first_sequence
  be(57, (uint32_t)p.n_records, 4);
  for (int i = 0; i < 61; i++) out[i] = h[i];
}
__global__ void k_header(const Plan* plan, uint8_t* out) {
  if (threadIdx.x == 0) header_run(plan, out);
}

// ---------------------------------------------------------------------------
// k_write: canonical re-encode of the kept records, one wave per included batch
// ---------------------------------------------------------------------------


// copy n source bytes at slice offset s0 to out offset d0 (ASCII-uppercased when
// `upper`), all lanes of the wave: 16-byte aligned destination units, lane u
// takes units u, u + 64, ...  Every unit of a segment has the same source
// misalignment, so each unit is two aligned dwordx4 loads and four alignbytes
// selected by a wave-uniform switch; interior units are one dwordx4 store,
// the two edge units byte stores.
__device__ __forceinline__ void copy_seg(uint8_t* __restrict__ out, const uint8_t* __restrict__ slice, uint64_t d0,
                                         uint64_t s0, uint32_t n, bool upper) {
  if (!n) return;
  const uint32_t lane = lane_id();
  const uint64_t u0 = d0 >> 4;
  const uint32_t nunits = (uint32_t)(((d0 + n + 15) >> 4) - u0);
  const uint32_t sh = (uint32_t)((s0 - d0) & 15);  // source offset of a destination unit start, mod 16
  const uint64_t e = d0 + n;
  for (uint32_t u = lane; u < nunits; u += 64) {
    const uint64_t D = (u0 + u) << 4;
    const uint64_t A = s0 + D - d0;  // >= s0 - 15: the value sits >= 61 B into the slice
    const uint4* src = (const uint4*)(slice + (A & ~15ull));
    const uint4 x0 = src[0], x1 = src[1];
    const uint32_t w[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    const uint32_t bs = sh & 3u;
    uint32_t v[4];
    switch (sh >> 2) {  // wave-uniform
      case 0:
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], bs);
        break;
      case 1:
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = __builtin_amdgcn_alignbyte(w[k + 2], w[k + 1], bs);
        break;
      case 2:
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = __builtin_amdgcn_alignbyte(w[k + 3], w[k + 2], bs);
        break;
      default:
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = __builtin_amdgcn_alignbyte(w[k + 4], w[k + 3], bs);
        break;
    }
    if (upper) {
#pragma unroll
      for (int k = 0; k < 4; k++) v[k] = swar_upper(v[k]);
    }
    const uint64_t lo = D > d0 ? D : d0;
    const uint64_t hi = D + 16 < e ? D + 16 : e;
    if (lo == D && hi == D + 16) {
      *(uint4*)(out + D) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
      const uint32_t jl = (uint32_t)(lo - D), jh = (uint32_t)(hi - D);
#pragma unroll
      for (int jj = 0; jj < 16; jj++)
        if ((uint32_t)jj >= jl && (uint32_t)jj < jh) out[D + jj] = (uint8_t)(v[jj >> 2] >> (8 * (jj & 3)));
    }
  }
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, uint32_t lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// Every lane's segment out[d0, d0 + n) <- src[s0, s0 + n) at once: the
// segments' 16-byte destination units are numbered across the wave (a scan)
// and dealt out 64 at a time, so the loads of many records are in flight
// together instead of one record's per wave round trip.  Units a segment
// shares with its neighbours are written bytewise inside the segment only.
__device__ __forceinline__ void copy_segs(uint8_t* __restrict__ out, const uint8_t* __restrict__ src, uint64_t d0,
                                          uint64_t s0, uint32_t n, bool upper) {
  const uint64_t act = __ballot(n != 0u);
  if (__builtin_popcountll(act) <= 1) {  // one segment (a one-record batch): no scan
    if (act) {
      const uint32_t i = (uint32_t)__builtin_ctzll(act);
      copy_seg(out, src, readlane_u64(d0, i), readlane_u64(s0, i), __builtin_amdgcn_readlane(n, i),
               __builtin_amdgcn_readlane((uint32_t)upper, i) != 0u);
    }
    return;
  }
  const uint32_t lane = lane_id();
  const uint32_t units = n ? (uint32_t)(((d0 + n + 15) >> 4) - (d0 >> 4)) : 0u;
  const uint32_t incl = wave_incl_scan(units), ex = incl - units;
  const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
  for (uint32_t u0 = 0; u0 < tot; u0 += 64) {
    const uint32_t u = u0 + lane;
    // the segment of unit u: the last lane whose exclusive prefix <= u (empty
    // segments share their successor's prefix and are passed over)
    uint32_t rr = 0;
#pragma unroll
    for (uint32_t st = 32; st > 0; st >>= 1) {
      const uint32_t c = rr + st;
      const uint32_t pc = __shfl(ex, (int)(c & 63), 64);
      if (c < 64 && pc <= u) rr = c;
    }
    const uint32_t rex = __shfl(ex, (int)rr, 64);
    const uint64_t rd = ((uint64_t)__shfl((uint32_t)(d0 >> 32), (int)rr, 64) << 32) | __shfl((uint32_t)d0, (int)rr, 64);
    const uint64_t rs = ((uint64_t)__shfl((uint32_t)(s0 >> 32), (int)rr, 64) << 32) | __shfl((uint32_t)s0, (int)rr, 64);
    const uint32_t rn = __shfl(n, (int)rr, 64);
    const bool rup = __shfl((uint32_t)upper, (int)rr, 64) != 0u;
    if (u >= tot) continue;
    const uint64_t D = ((rd >> 4) + (u - rex)) << 4;
    const uint64_t A = rs + D - rd;  // the source of D (may start before rs: the unit's head is masked)
    const uint4* sp = (const uint4*)(src + (A & ~15ull));
    const uint4 x0 = sp[0], x1 = sp[1];
    const uint32_t w[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    const uint32_t sh = (uint32_t)(A & 15), q = sh >> 2, bs = sh & 3u;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t lo = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
      const uint32_t hi = q == 0 ? w[k + 1] : q == 1 ? w[k + 2] : q == 2 ? w[k + 3] : w[k + 4];
      v[k] = __builtin_amdgcn_alignbyte(hi, lo, bs);
      if (rup) v[k] = swar_upper(v[k]);
    }
    const uint64_t e = rd + rn;
    const uint64_t lo = D > rd ? D : rd;
    const uint64_t hi = D + 16 < e ? D + 16 : e;
    if (lo == D && hi == D + 16) {
      *(uint4*)(out + D) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
      const uint32_t jl = (uint32_t)(lo - D), jh = (uint32_t)(hi - D);
#pragma unroll
      for (int jj = 0; jj < 16; jj++)
        if ((uint32_t)jj >= jl && (uint32_t)jj < jh) out[D + jj] = (uint8_t)(v[jj >> 2] >> (8 * (jj & 3)));
    }
  }
}

constexpr uint32_t kElemLaneCopy = 48;  // array elements up to this size are copied by their own lane

// array_map batch (derive generator/array_map.rs:17-42): the elements of the
// batch's kept records, flattened 64 at a time over the wave.  Lane = element:
// size, wave scan, record header (default preamble + offset fix-up), payload
// (short verbatim elements by the lane, long ones by the whole wave, the rest
// through the canonicalizer).
template <bool kCanon>  // kCanon: only the payloads of non-verbatim elements (k_write_canon)
__device__ void write_array_batch(const WriteArgs& a, const KeptRec* d, uint32_t nkeep, int64_t rel, uint64_t obase) {
  const uint32_t lane = lane_id();
  uint8_t* out = a.out;
  uint64_t run = 0;
  for (uint32_t k0 = 0; k0 < nkeep; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool v = k < nkeep;
    uint32_t ne = 0, flg = 0;
    uint64_t sb = 0;
    if (v) {
      const KeptRec r = d[k];
      ne = (uint32_t)r.ival;
      sb = r.vpos >> 1;
      flg = r.pad;
    }
    const uint32_t eincl = wave_incl_scan(ne);
    const uint32_t eex = eincl - ne;
    const uint32_t tot = __builtin_amdgcn_readlane(eincl, 63);
    for (uint32_t e0 = 0; e0 < tot; e0 += 64) {
      const uint32_t e = e0 + lane;
      const bool ev = e < tot;
      // record of element e: the last lane whose exclusive prefix <= e
      uint32_t rr = 0;
#pragma unroll
      for (uint32_t st = 32; st > 0; st >>= 1) {
        const uint32_t c = rr + st;
        const uint32_t pc = __shfl(eex, (int)(c & 63), 64);
        if (c < 64 && pc <= e) rr = c;
      }
      const uint32_t rex = __shfl(eex, (int)rr, 64);
      const uint64_t rsb = ((uint64_t)__shfl((uint32_t)(sb >> 32), (int)rr, 64) << 32) | __shfl((uint32_t)sb, (int)rr, 64);
      const bool upper = (__shfl(flg, (int)rr, 64) & KF_UPPER) != 0;
      ElemRec er = {0, 0, 0};
      if (ev) er = a.elem[rsb + (e - rex)];
      const uint32_t len = er.out_len & 0x7FFFFFFFu;
      const bool verb = (er.out_len >> 31) != 0;
      const uint32_t sz = ev ? elem_out_size(len, rel) : 0u;
      const uint64_t incl = wave_incl_scan((uint64_t)sz);
      const uint64_t my = obase + run + incl - sz;
      bool wave_copy = false;
      if (kCanon) {
        if (ev && !verb) {  // the payload after the header k_write wrote
          uint8_t t[16];
          const uint32_t hw = venc((int64_t)elem_inner(len, rel), t) + 2 + venc(rel, t) + 1 + venc((int64_t)len, t);
          json_canon<const uint8_t*>(a.slice + er.pos, er.src_len, upper, out + my + hw);
        }
      } else if (ev) {
        uint8_t* q = out + my;
        uint8_t t[16];
        uint32_t w = 0;
        uint32_t nn = venc((int64_t)elem_inner(len, rel), t);
        for (uint32_t i = 0; i < nn; i++) q[w++] = t[i];
        q[w++] = 0;  // attributes
        q[w++] = 0;  // timestamp_delta
        nn = venc(rel, t);
        for (uint32_t i = 0; i < nn; i++) q[w++] = t[i];
        q[w++] = 0;  // key: None
        nn = venc((int64_t)len, t);
        for (uint32_t i = 0; i < nn; i++) q[w++] = t[i];
        if (!verb) {
          // floats, key order, whitespace, escapes: the payload by k_write_canon
        } else if (len <= kElemLaneCopy) {
          const uint8_t* src = a.slice + er.pos;
          for (uint32_t i = 0; i < len; i++) q[w + i] = upper ? up(src[i]) : src[i];
        } else {
          wave_copy = true;
        }
        q[w + len] = 0;  // headers
      }
      // long verbatim elements: whole-wave copies
      uint64_t pend = __ballot(wave_copy);
      while (pend) {
        const uint32_t i = (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1;
        const uint32_t il = __builtin_amdgcn_readlane(len, i);
        const uint64_t dst = readlane_u64(my, i) + elem_out_size(il, rel) - il - 1;
        copy_seg(out, a.slice, dst, readlane_u64(er.pos, i), il, __builtin_amdgcn_readlane((uint32_t)upper, i) != 0);
      }
      run += readlane_u64(incl, 63);
    }
  }
}

// k_write — one wave per included batch (four per 256-thread block).  Per chunk
// of up to 64 survivors: lane = record: size, wave scan, varint header fields
// and i32 values; then the wave walks the chunk's records in order and copies
// each key/value payload with all 64 lanes (copy_seg).  aggregate (concat)
// values are prefixes of the accumulator stream built by k_cat.
constexpr int kWriteThreads = 256;
__device__ __forceinline__ void write_batch(const WriteArgs& a, const Plan& p, int32_t b) {
  const uint32_t lane = lane_id();
  const BatchStat st = a.bstat[b];
  const int64_t rel = a.seg ? 0 : a.base - st.base_offset;
  const int32_t agg_base = a.agg_pre ? (int32_t)((uint64_t)a.acc0 + (uint64_t)a.agg_pre[b].agg) : 0;
  const uint64_t cat_base = a.agg_pre ? a.acc_len + a.agg_pre[b].cat : 0;
  const KeptRec* d = a.desc + a.rbase[b];
  const uint64_t obase = a.seg ? 61ull * (uint64_t)(b + 1) + a.pre[b].rec_bytes
                               : 61 + (a.pre[b].rec_bytes - a.pre[p.first].rec_bytes);
  uint8_t* out = a.out;
  if (st.flags & BF_ARR_LEAN) return;  // k_arr_write (fsg_array.hip)
  const bool compact = (st.flags & BF_COMPACT) != 0;
  const uint8_t mode0 = st.nkeep ? (compact ? (uint8_t)KM_AGG : d[0].mode) : (uint8_t)0;
  if (mode0 == KM_ARRAY) {  // a batch's descriptors share one mode
    write_array_batch<false>(a, d, st.nkeep, rel, obase);
    return;
  }
  uint64_t run = 0;
  for (uint32_t k0 = 0; k0 < st.nkeep; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool v = k < st.nkeep;
    KeptRec r = {};
    uint32_t sz = 0;
    if (v) {
      r = kept_at(d, k, compact);
      sz = rec_out_size(r, rel, agg_base, cat_base);
    }
    const uint64_t incl = wave_incl_scan((uint64_t)sz);
    const uint64_t my = obase + run + incl - sz;
    uint64_t kd = 0, vd = 0, vsrc = 0;
    uint32_t kl = 0, vc = 0;
    if (v) {
      uint8_t* q = out + my;
      const uint32_t vl = out_vlen(r, agg_base, cat_base);
      const uint32_t inner = 1 + vsize(r.ts) + vsize(r.od + rel) + 1 +
                             (r.has_key ? vsize((int64_t)r.klen) + r.klen : 0) + vsize((int64_t)vl) + vl + vsize(r.hdr);
      uint8_t t[16];
      uint32_t n = venc((int64_t)inner, t), w = 0;
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      q[w++] = r.attr;
      n = venc(r.ts, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      n = venc(r.od + rel, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      q[w++] = r.has_key ? 1 : 0;
      if (r.has_key) {
        n = venc((int64_t)r.klen, t);
        for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
        kd = my + w;
        kl = r.klen;
        w += r.klen;
      }
      n = venc((int64_t)vl, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      vd = my + w;
      if (r.mode == KM_I32 || r.mode == KM_AGG) {
        const int32_t x = r.mode == KM_I32 ? r.ival : (int32_t)((uint32_t)agg_base + (uint32_t)r.ival);
        w += fmt_i32(x, q + w);
      } else {
        vc = vl;
        vsrc = r.mode == KM_CONCAT ? kCatOff : r.mode == KM_AGGJ ? r.src : r.vpos;  // KM_AGGJ: the map text in cat
        w += vl;
      }
      n = venc(r.hdr, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
    }
    // payloads: the chunk's keys, then its values, each spread over the wave
    const bool cat = mode0 == KM_CONCAT || mode0 == KM_AGGJ;
    if (__ballot(kl != 0u)) copy_segs(out, a.slice, kd, r.kpos, kl, false);
    copy_segs(out, cat ? a.cat : a.slice, vd, vsrc, vc, r.mode == KM_UPPER);
    run += readlane_u64(incl, 63);
  }
}
__global__ __launch_bounds__(kWriteThreads) void k_write(WriteArgs a) {
  const Plan p = *a.plan;
  const int32_t b = p.first + (int32_t)(blockIdx.x * (kWriteThreads / 64) + (threadIdx.x >> 6));
  if (p.first < 0 || b > p.last) return;
  write_batch(a, p, b);
}

// k_write_gen — batches of records whose values are generated integers
// (KM_I32: map_double / filter_map outputs; KM_AGG: aggregate-sum's running
// sum): one 256-thread workgroup per included batch, thread t the contiguous
// kept records [t R, t R + R) (R <= 8, unrolled); output sizes, a block scan,
// every record's bytes assembled in LDS (varint fields, key, decimal value,
// trailer), then 16-byte stores.  Batches of another mode, more than 2048
// records or more output than the stage holds take write_batch on wave 0.
constexpr int kWgObuf = 32768;
constexpr int kWgR = 8;
struct __attribute__((aligned(16))) WgLds {
  uint8_t ob[kWgObuf + 16];
  uint32_t wt[4];
};
__device__ __forceinline__ void write_gen_body(const WriteArgs& a, uint32_t bid) {
  __shared__ WgLds L;
  const int32_t b = a.first + (int32_t)bid;
  if (a.first < 0 || b > a.last) return;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const BatchStat st = a.bstat[b];
  const uint32_t nk = st.nkeep;
  if (!nk) return;
  const int64_t rel = a.seg ? 0 : a.base - st.base_offset;
  const int32_t agg_base = a.agg_pre ? (int32_t)((uint64_t)a.acc0 + (uint64_t)a.agg_pre[b].agg) : 0;
  const KeptRec* d = a.desc + a.rbase[b];
  const uint64_t obase = a.seg ? 61ull * (uint64_t)(b + 1) + a.pre[b].rec_bytes
                               : 61 + (a.pre[b].rec_bytes - a.pre[a.first].rec_bytes);
  const bool compact = (st.flags & BF_COMPACT) != 0;
  const uint8_t mode0 = compact ? (uint8_t)KM_AGG : d[0].mode;  // a batch's descriptors share one mode
  const uint32_t R = (nk + 255u) >> 8;
  const bool gen = (mode0 == KM_I32 || mode0 == KM_AGG) && R <= (uint32_t)kWgR && !(st.flags & BF_ARR_LEAN);
  Plan p = {};
  p.first = a.first;
  if (!gen) {
    if (t < 64) write_batch(a, p, b);
    return;
  }
  const uint32_t k0 = t * R;
  uint32_t sz[kWgR], mine = 0;
#pragma unroll
  for (int i = 0; i < kWgR; i++) {
    sz[i] = 0;
    if (i < (int)R && k0 + i < nk) {
      sz[i] = rec_out_size(kept_at(d, k0 + i, compact), rel, agg_base, 0);
      mine += sz[i];
    }
  }
  const uint32_t incl = wave_incl_scan(mine);
  if (lane == 63) L.wt[wv] = incl;
  __syncthreads();
  uint32_t off = incl - mine;
  for (uint32_t w2 = 0; w2 < wv; w2++) off += L.wt[w2];
  const uint32_t total = L.wt[0] + L.wt[1] + L.wt[2] + L.wt[3];
  const uint32_t d0 = (uint32_t)(obase & 15);
  if (d0 + total > (uint32_t)kWgObuf) {  // uniform
    if (t < 64) write_batch(a, p, b);
    return;
  }
  uint32_t q = d0 + off;
#pragma unroll
  for (int i = 0; i < kWgR; i++) {
    if (!sz[i]) continue;
    const KeptRec r = kept_at(d, k0 + i, compact);
    const int32_t x = r.mode == KM_I32 ? r.ival : (int32_t)((uint32_t)agg_base + (uint32_t)r.ival);
    const uint32_t vl = dec_len_i32(x);
    const uint32_t inner = 1 + vsize(r.ts) + vsize(r.od + rel) + 1 +
                           (r.has_key ? vsize((int64_t)r.klen) + r.klen : 0) + vsize((int64_t)vl) + vl + vsize(r.hdr);
    uint8_t* o = L.ob + q;
    uint32_t w = venc((int64_t)inner, o);
    o[w++] = r.attr;
    w += venc(r.ts, o + w);
    w += venc(r.od + rel, o + w);
    o[w++] = r.has_key ? 1 : 0;
    if (r.has_key) {
      w += venc((int64_t)r.klen, o + w);
      const uint8_t* ks = a.slice + r.kpos;
      for (uint32_t j = 0; j < r.klen; j++) o[w + j] = ks[j];
      w += r.klen;
    }
    w += venc((int64_t)vl, o + w);
    w += fmt_i32(x, o + w);
    w += venc(r.hdr, o + w);
    q += w;
  }
  __syncthreads();
  const uint32_t E = d0 + total;
  uint8_t* og = a.out + obase - d0;
  for (uint32_t u = t; u < (E + 15) >> 4; u += 256) {
    const uint32_t D = u << 4;
    if (D >= d0 && D + 16 <= E) {
      *(uint4*)(og + D) = *(const uint4*)(L.ob + D);
    } else {
      const uint32_t lo = D > d0 ? D : d0, hi = D + 16 < E ? D + 16 : E;
      for (uint32_t j = lo; j < hi; j++) og[j] = L.ob[j];
    }
  }
}
__global__ __launch_bounds__(256) void k_write_gen(WriteArgs a) { write_gen_body(a, blockIdx.x); }
void launch_write_gen(const WriteArgs& a, uint32_t nblocks, hipStream_t s) {
  if (nblocks) hipLaunchKernelGGL(k_write_gen, dim3(nblocks), dim3(256), 0, s, a);
}

// Array elements whose canonical text differs from their source text (floats,
// keys out of BTreeMap order, whitespace, escapes): json_canon measures them
// after k_eval (k_canon_len, before k_size) and writes them after k_write
// (k_write_canon, the same position walk as k_write), only in the batches
// k_eval flagged (BatchStat::pad).  One wave per batch.
__global__ __launch_bounds__(256) void k_canon_len(SizeArgs a, const uint8_t* __restrict__ slice) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.nbatches) return;
  const BatchStat& st = a.bstat[b];
  if (!st.pad || !st.nkeep) return;
  const KeptRec* d = a.desc + a.rbase[b];
  if (d[0].mode != KM_ARRAY) return;
  for (uint32_t k = lane_id(); k < st.nkeep; k += 64) {
    const KeptRec r = d[k];
    const bool up = (r.pad & KF_UPPER) != 0;
    ElemRec* e = const_cast<ElemRec*>(a.elem) + (r.vpos >> 1);
    for (int32_t j = 0; j < r.ival; j++) {
      const ElemRec x = e[j];
      if (!(x.out_len >> 31)) e[j].out_len = json_canon<const uint8_t*>(slice + x.pos, x.src_len, up, nullptr);
    }
  }
}
__global__ __launch_bounds__(kWriteThreads) void k_write_canon(WriteArgs a) {
  const Plan p = *a.plan;
  const int32_t b = p.first + (int32_t)(blockIdx.x * (kWriteThreads / 64) + (threadIdx.x >> 6));
  if (p.first < 0 || b > p.last) return;
  const BatchStat st = a.bstat[b];
  if (!st.pad || !st.nkeep) return;
  const KeptRec* d = a.desc + a.rbase[b];
  if (d[0].mode != KM_ARRAY) return;
  const int64_t rel = a.seg ? 0 : a.base - st.base_offset;
  const uint64_t obase = a.seg ? 61ull * (uint64_t)(b + 1) + a.pre[b].rec_bytes
                               : 61 + (a.pre[b].rec_bytes - a.pre[p.first].rec_bytes);
  write_array_batch<true>(a, d, st.nkeep, rel, obase);
}
void launch_canon_len(const SizeArgs& a, const uint8_t* slice, hipStream_t s) {
  if (a.nbatches) hipLaunchKernelGGL(k_canon_len, dim3((a.nbatches + 3) / 4), dim3(256), 0, s, a, slice);
}
void launch_write_canon(const WriteArgs& a, uint32_t nblk, hipStream_t s) {
  if (nblk) hipLaunchKernelGGL(k_write_canon, dim3((nblk + 3) / 4), dim3(kWriteThreads), 0, s, a);
}

// k_cat — aggregate (concat) accumulator stream: cat[kCatOff..] = initial
// accumulator ++ the appended value of every aggregated record of batches
// 0..stop, in stream order (smartmodule/examples/aggregate/src/lib.rs:7-13:
// acc.push_str(value)).  One wave per batch; the initial accumulator was
// copied by the host.
__global__ __launch_bounds__(256) void k_cat(WriteArgs a, uint32_t nbatches) {
  const Plan p = *a.plan;
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nbatches || (int32_t)b > p.stop) return;
  const uint32_t lane = lane_id();
  const BatchStat st = a.bstat[b];
  const KeptRec* d = a.desc + a.rbase[b];
  if (!st.nkeep || d[0].mode != KM_CONCAT) return;
  uint8_t* cat = (uint8_t*)a.cat;
  const uint64_t base = kCatOff + a.acc_len + a.agg_pre[b].cat;
  for (uint32_t k0 = 0; k0 < st.nkeep; k0 += 64) {
    const uint32_t k = k0 + lane;
    KeptRec r = {};
    uint32_t n = 0;
    uint64_t dst = 0;
    if (k < st.nkeep) {
      r = d[k];
      n = (r.pad & KF_I32) ? dec_len_i32((int32_t)r.vlen) : r.vlen;
      dst = base + (uint32_t)r.ival - n;
      if (r.pad & KF_I32) fmt_i32((int32_t)r.vlen, cat + dst);
    }
    const uint32_t nrec = st.nkeep - k0 < 64u ? st.nkeep - k0 : 64u;
    for (uint32_t i = 0; i < nrec; i++) {
      const uint32_t rn = __builtin_amdgcn_readlane(n, i);
      const uint32_t fl = __builtin_amdgcn_readlane((uint32_t)r.pad, i);
      if (rn && !(fl & KF_I32))
        copy_seg(cat, a.slice, readlane_u64(dst, i), readlane_u64(r.vpos, i), rn, (fl & KF_UPPER) != 0);
    }
  }
}

// ---------------------------------------------------------------------------
// aggregate-json (smartmodule/examples/aggregate-json/src/lib.rs:22-36): per
// record, `accumulated + new` (`entry().and_modify(+=).or_insert()`, u32
// wrapping as in the release wasm) and the record's value = serde_json::
// to_vec_pretty of the whole map, its keys in the guest HashMap's bucket order
// (deterministic on the wasm32 target: fsg_keyed.hip k_aggj_order).  Key ids
// below are by first occurrence; the text pass lists them in that order.
//
// The fold is sequential in the reference; here it is data-parallel:
//   1. k_aggj_bcount / scan / k_aggj_flat: the folded records in stream order
//      and their entries (exclusive scans give every record its stream index
//      and its first entry index)
//   2. k_aggj_insert: every record's distinct keys into one open-addressing
//      index (CAS claim; atomicMin keeps the key's FIRST occurrence), value =
//      the key's last value in the record (a JSON object's duplicate key)
//   3. k_aggj_new / scan / k_aggj_ids / k_aggj_kid: a key's id = its rank by
//      first occurrence (insertion order), entries resolved to ids
//   4. k_aggj_bsum / k_aggj_colscan: per block of `rb` records, the sums per
//      key, then per key an exclusive scan over blocks: the map's values at
//      every block's first record
//   5. k_aggj_text: one wave per block replays its records from that row
//      (values in LDS), sizing (pass 0; the length does not depend on the key
//      order) or writing (pass 1, keys in k_aggj_order's order) each record's text
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dec_digits_u32(uint32_t v) {
  uint32_t n = 1;
  while (v >= 10u) {
    v /= 10u;
    n++;
  }
  return n;
}
__device__ __forceinline__ uint8_t key_byte(const uint8_t* p, uint32_t k, bool up) {
  const uint8_t c = p[k];
  return (up && c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
}
__device__ uint32_t aggj_hash(const uint8_t* p, uint32_t n, bool up) {  // FNV-1a
  uint32_t h = 2166136261u;
  for (uint32_t k = 0; k < n; k++) h = (h ^ key_byte(p, k, up)) * 16777619u;
  return h;
}
__device__ bool aggj_key_eq(const uint8_t* a, uint32_t an, bool aup, const uint8_t* b, uint32_t bn, bool bup) {
  if (an != bn) return false;
  for (uint32_t k = 0; k < an; k++)
    if (key_byte(a, k, aup) != key_byte(b, k, bup)) return false;
  return true;
}

// generic exclusive scan u32 -> u64 (tiles of 2048, tile totals scanned by one
// workgroup, added back); *tot = the sum
constexpr int kXsThreads = 256, kXsPer = 8, kXsTile = kXsThreads * kXsPer;
__device__ __forceinline__ uint64_t block_excl_u64(uint64_t x, uint64_t* sh, uint64_t& total) {
  const uint64_t inc = wave_incl_scan(x);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane_id() == 63) sh[w] = inc;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
  for (int i = 0; i < nw; i++) {
    const uint64_t v = sh[i];
    if (i < w) pre += v;
    tot += v;
  }
  __syncthreads();
  total = tot;
  return inc - x + pre;
}
__global__ __launch_bounds__(kXsThreads) void k_xscan_tiles(const uint32_t* in, uint64_t* out, uint64_t* tsum,
                                                           uint64_t n) {
  __shared__ uint64_t sh[kXsThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kXsTile + (uint64_t)threadIdx.x * kXsPer;
  uint32_t v[kXsPer];
  uint64_t mine = 0;
#pragma unroll
  for (int i = 0; i < kXsPer; i++) {
    v[i] = base + i < n ? in[base + i] : 0u;
    mine += v[i];
  }
  uint64_t tot;
  uint64_t run = block_excl_u64(mine, sh, tot);
#pragma unroll
  for (int i = 0; i < kXsPer; i++) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(1024) void k_xscan_top(uint64_t* tsum, uint32_t nt, unsigned long long* tot) {
  __shared__ uint64_t sh[16];
  uint64_t carry = 0;
  for (uint32_t c0 = 0; c0 < nt; c0 += 1024) {
    const uint32_t i = c0 + threadIdx.x;
    const uint64_t x = i < nt ? tsum[i] : 0ull;
    uint64_t t;
    const uint64_t ex = block_excl_u64(x, sh, t);
    if (i < nt) tsum[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) *tot = carry;
}
__global__ __launch_bounds__(256) void k_xscan_add(uint64_t* out, const uint64_t* tsum, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    out[i] += tsum[i / kXsTile];
}

// the batch of the first error bounds the fold (records after it never run)
__device__ __forceinline__ uint32_t aggj_last(const AggjArgs& a) {
  const uint32_t fe = a.mins->first_err;
  return fe != 0xFFFFFFFFu && fe < a.nbatches ? fe : (a.nbatches ? a.nbatches - 1 : 0);
}
// per batch: folded records and their entries (scal[1], scal[0])
__global__ __launch_bounds__(256) void k_aggj_bcount(AggjArgs a) {
  const uint32_t last = aggj_last(a);
  unsigned long long recs = 0, ents = 0, most = 0;
  for (uint32_t b = blockIdx.x * 256 + threadIdx.x; b < a.nbatches; b += gridDim.x * 256) {
    const BatchStat st = a.bstat[b];
    const uint32_t n = (b <= last && !(st.flags & BF_DECODE)) ? st.nkeep : 0u;
    a.bcnt[b] = n;
    const KeptRec* d = a.desc + a.rbase[b];
    for (uint32_t k = 0; k < n; k++) {
      const uint32_t e = (uint32_t)d[k].ival;
      ents += e;
      most = e > most ? e : most;
    }
    recs += n;
  }
  recs = wave_sum(recs);
  ents = wave_sum(ents);
  if (lane_id() == 0 && recs) atomicAdd(&a.scal[1], recs);
  if (lane_id() == 0 && ents) atomicAdd(&a.scal[0], ents);
  if (most) atomicMax(&a.scal[7], most);  // the most entries of one record (k_aggj_order's table sizes)
}
// one wave per batch: the stream's record table
__global__ __launch_bounds__(256) void k_aggj_flat(AggjArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.nbatches) return;
  const uint32_t n = a.bcnt[b];
  const uint64_t r0 = a.brec[b], d0 = a.rbase[b];
  for (uint32_t k = lane_id(); k < n; k += 64) {
    a.rdesc[r0 + k] = d0 + k;
    a.rne[r0 + k] = (uint32_t)a.desc[d0 + k].ival;
  }
}
struct AjKey {
  const uint8_t* p;
  uint32_t n;
  bool up;
};
__device__ __forceinline__ AjKey aggj_key_of(const AggjArgs& a, unsigned long long ref) {
  if ((ref >> 32) == 0) {  // initial key
    const uint32_t k = (uint32_t)ref - 1u;
    return {(const uint8_t*)a.kptr[k], a.klen[k], false};
  }
  const KeptRec& d = a.desc[a.rdesc[(ref >> 32) - 1]];
  const ElemRec e = a.elem[(d.vpos >> 1) + (uint32_t)ref];
  return {a.slice + e.pos, e.src_len, (d.pad & KF_UPPER) != 0};
}
// the key's slot (claimed if absent); `ref` becomes the slot's occurrence if earlier
__device__ uint32_t aggj_insert(const AggjArgs& a, unsigned long long ref, const AjKey& me) {
  uint32_t s = aggj_hash(me.p, me.n, me.up) & (a.cap - 1u);
  for (;;) {
    unsigned long long cur = __hip_atomic_load(&a.slot_ref[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0) {
      cur = atomicCAS(&a.slot_ref[s], 0ull, ref);
      if (cur == 0) return s;
    }
    const AjKey o = aggj_key_of(a, cur);
    if (aggj_key_eq(o.p, o.n, o.up, me.p, me.n, me.up)) {
      if (ref < cur) atomicMin(&a.slot_ref[s], ref);
      return s;
    }
    s = (s + 1u) & (a.cap - 1u);
  }
}
__global__ __launch_bounds__(256) void k_aggj_init(AggjArgs a) {
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < a.n_init; k += gridDim.x * 256) {
    const uint32_t s = aggj_insert(a, (unsigned long long)k + 1ull, {(const uint8_t*)a.kptr[k], a.klen[k], false});
    a.slot_id[s] = k;
  }
}
// one thread per record: its distinct keys into the index
__global__ __launch_bounds__(256) void k_aggj_insert(AggjArgs a) {
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < a.n_rec; r += (uint64_t)gridDim.x * 256) {
    const KeptRec& d = a.desc[a.rdesc[r]];
    const ElemRec* e = a.elem + (d.vpos >> 1);
    const uint32_t ne = a.rne[r];
    const uint64_t g0 = a.rent[r];
    const bool up = (d.pad & KF_UPPER) != 0;
    for (uint32_t j = 0; j < ne; j++) {
      const uint8_t* kp = a.slice + e[j].pos;
      const uint32_t kn = e[j].src_len;
      bool before = false;  // the record's own map: a key's last value, at its first position
      for (uint32_t i = 0; i < j && !before; i++) before = aggj_key_eq(a.slice + e[i].pos, e[i].src_len, up, kp, kn, up);
      if (before) {
        a.ekid[g0 + j] = kSkipEntry;
        continue;
      }
      uint32_t v = e[j].out_len;
      for (uint32_t i = j + 1; i < ne; i++)
        if (aggj_key_eq(a.slice + e[i].pos, e[i].src_len, up, kp, kn, up)) v = e[i].out_len;
      a.eval[g0 + j] = v;
      a.ekid[g0 + j] = aggj_insert(a, ((unsigned long long)(r + 1) << 32) | j, {kp, kn, up});
    }
  }
}
// keys whose first occurrence is in the record
__global__ __launch_bounds__(256) void k_aggj_new(AggjArgs a) {
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < a.n_rec; r += (uint64_t)gridDim.x * 256) {
    const uint32_t ne = a.rne[r];
    const uint64_t g0 = a.rent[r];
    uint32_t n = 0;
    for (uint32_t j = 0; j < ne; j++) {
      const uint32_t s = a.ekid[g0 + j];
      if (s != kSkipEntry && a.slot_ref[s] == (((unsigned long long)(r + 1) << 32) | j)) n++;
    }
    a.rnew[r] = n;
  }
}
__global__ __launch_bounds__(256) void k_aggj_ids(AggjArgs a) {
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < a.n_rec; r += (uint64_t)gridDim.x * 256) {
    if (!a.rnew[r]) continue;
    const KeptRec& d = a.desc[a.rdesc[r]];
    const ElemRec* e = a.elem + (d.vpos >> 1);
    const uint32_t ne = a.rne[r];
    const uint64_t g0 = a.rent[r];
    uint32_t id = a.n_init + (uint32_t)a.rnewb[r];
    for (uint32_t j = 0; j < ne; j++) {
      const uint32_t s = a.ekid[g0 + j];
      if (s == kSkipEntry || a.slot_ref[s] != (((unsigned long long)(r + 1) << 32) | j)) continue;
      a.slot_id[s] = id;
      a.tptr[id] = (uint64_t)(a.slice + e[j].pos - 1);  // the source key with its quotes: serde_json's text
      a.tlen[id] = e[j].src_len + 2u;                   // of an unescaped key
      a.kup[id] = (d.pad & KF_UPPER) ? 1u : 0u;
      id++;
    }
  }
}
__global__ __launch_bounds__(256) void k_aggj_kid(AggjArgs a, uint64_t n_ent) {
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < n_ent; g += (uint64_t)gridDim.x * 256) {
    const uint32_t s = a.ekid[g];
    if (s != kSkipEntry) a.ekid[g] = a.slot_id[s];
  }
}
// per block, the sums its records contribute per key
__global__ __launch_bounds__(256) void k_aggj_bsum(AggjArgs a) {
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < a.n_rec; r += (uint64_t)gridDim.x * 256) {
    uint32_t* row = a.state + (uint64_t)(r / a.rb) * a.nkeys;
    const uint32_t ne = a.rne[r];
    const uint64_t g0 = a.rent[r];
    for (uint32_t j = 0; j < ne; j++) {
      const uint32_t k = a.ekid[g0 + j];
      if (k != kSkipEntry) atomicAdd(&row[k], a.eval[g0 + j]);  // u32 wrapping
    }
  }
}
// one workgroup per key: exclusive scan down its column, from the initial value
__global__ __launch_bounds__(256) void k_aggj_colscan(AggjArgs a) {
  __shared__ uint64_t sh[4];
  const uint32_t k = blockIdx.x;
  uint32_t carry = k < a.n_init ? a.val_init[k] : 0u;
  for (uint32_t c0 = 0; c0 < a.nblk; c0 += 256) {
    const uint32_t b = c0 + threadIdx.x;
    uint32_t* p = a.state + (uint64_t)b * a.nkeys + k;
    const uint32_t x = b < a.nblk ? *p : 0u;
    uint64_t t;
    const uint64_t ex = block_excl_u64(x, sh, t);
    if (b < a.nblk) *p = carry + (uint32_t)ex;
    carry += (uint32_t)t;
  }
}
__device__ __forceinline__ uint32_t aggj_term(uint32_t k, uint32_t tl, uint32_t v) {
  return (k ? 4u : 3u) + tl + 2u + dec_digits_u32(v);  // (k ? ",\n  " : "\n  ") key ": " digits
}
// one wave per block of records.  kLds: the values live in LDS (K <= kAjLds),
// else in the block's own state row (agent-scope atomics: lanes of the wave
// read what other lanes wrote)
template <bool kLds>
__global__ __launch_bounds__(64) void k_aggj_text(AggjArgs a) {
  __shared__ uint32_t lds[kLds ? kAjLds : 1];
  const uint32_t b = blockIdx.x, l = lane_id();
  const uint64_t r0 = (uint64_t)b * a.rb, r1 = r0 + a.rb < a.n_rec ? r0 + a.rb : a.n_rec;
  if (r0 >= r1) return;
  uint32_t* row = a.state + (uint64_t)b * a.nkeys;
  uint32_t* V = kLds ? lds : row;
  auto vget = [&](uint32_t k) -> uint32_t {
    return kLds ? V[k] : __hip_atomic_load(&V[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto vset = [&](uint32_t k, uint32_t x) {
    if (kLds)
      V[k] = x;
    else
      __hip_atomic_store(&V[k], x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  const uint32_t nk_end = a.n_init + (uint32_t)(a.rnewb[r1 - 1] + a.rnew[r1 - 1]);
  if (kLds)
    for (uint32_t k = l; k < nk_end; k += 64) lds[k] = row[k];
  uint32_t nk = a.n_init + (uint32_t)a.rnewb[r0];
  uint64_t tot = 0;  // Σ terms of the keys so far
  if (!a.write) {
    for (uint32_t k = l; k < nk; k += 64) tot += aggj_term(k, a.tlen[k], vget(k));
    tot = wave_sum(tot);
  }
  __syncthreads();
  for (uint64_t r = r0; r < r1; r++) {
    const uint32_t ne = a.rne[r];
    const uint64_t g0 = a.rent[r];
    int64_t delta = 0;
    for (uint32_t j = l; j < ne; j += 64) {  // distinct keys within the record: no two lanes share one
      const uint32_t k = a.ekid[g0 + j];
      if (k == kSkipEntry) continue;
      const uint32_t old = k < nk ? vget(k) : 0u;
      const uint32_t nv = old + a.eval[g0 + j];
      vset(k, nv);
      if (!a.write)
        delta += k < nk ? (int64_t)dec_digits_u32(nv) - (int64_t)dec_digits_u32(old)
                        : (int64_t)aggj_term(k, a.tlen[k], nv);
    }
    nk += a.rnew[r];
    __syncthreads();
    if (!a.write) {
      tot += (uint64_t)wave_sum(delta);
      if (l == 0) a.rlen[r] = nk ? (uint32_t)(tot + 3u) : 2u;
      continue;
    }
    // the text: "{" + terms + "\n}", or "{}"
    uint8_t* o = a.cat + kCatOff + a.roff[r];
    const uint32_t len = a.rlen[r];
    if (l == 0) {
      o[0] = '{';
      o[len - 1] = '}';
      if (nk) o[len - 2] = '\n';
    }
    uint64_t q0 = 1;
    const uint32_t* order = a.ord + a.koff[r];  // the keys in the guest HashMap's bucket order (k_aggj_order)
    for (uint32_t c0 = 0; c0 < nk; c0 += 64) {
      const uint32_t p = c0 + l;
      const uint32_t k = p < nk ? order[p] : 0u;
      uint32_t v = p < nk ? vget(k) : 0u, tl = p < nk ? a.tlen[k] : 0u;
      const uint32_t t = p < nk ? aggj_term(p, tl, v) : 0u;
      const uint32_t inc = wave_incl_scan(t);
      if (p < nk) {
        uint64_t q = q0 + inc - t;
        if (p) o[q++] = ',';
        o[q++] = '\n';
        o[q++] = ' ';
        o[q++] = ' ';
        const uint8_t* tp = (const uint8_t*)a.tptr[k];
        const bool up = a.kup[k] != 0;
        for (uint32_t c = 0; c < tl; c++) o[q++] = key_byte(tp, c, up);
        o[q++] = ':';
        o[q++] = ' ';
        const uint32_t nd = dec_digits_u32(v);
        for (uint32_t c = 0; c < nd; c++) {
          o[q + nd - 1 - c] = (uint8_t)('0' + v % 10u);
          v /= 10u;
        }
      }
      q0 += __shfl(inc, 63, 64);
    }
  }
}
// records' text offsets into their descriptors; the accumulator after each batch
__global__ __launch_bounds__(256) void k_aggj_place(AggjArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < a.n_rec) {
    KeptRec& d = a.desc[a.rdesc[i]];
    d.src = kCatOff + a.roff[i];  // k_write reads the text from cat[src, src + vlen) (vpos still locates the entries)
    d.vlen = a.rlen[i];
  }
  if (i < a.nbatches) {
    const uint64_t n = a.brec[i] + a.bcnt[i];  // records folded up to and including batch i
    a.acc_off[i] = n ? kCatOff + a.roff[n - 1] : 0;
    a.acc_len[i] = n ? a.rlen[n - 1] : 0xFFFFFFFFu;
  }
}

// ---------------------------------------------------------------------------
// device framing (FileBatchIterator::next, crates/fluvio-storage/src/iterators.rs:
// 55-160, restated on the host in fsg_runtime.cpp frame()).  See FrameArgs.
// ---------------------------------------------------------------------------
// 1. candidates: one workgroup per 64 KiB chunk, 16 coalesced 16-byte rounds;
//    positions p with s[p + 16] == 2, kept in ascending order per chunk
// every 16-byte unit's loads in flight before the first use (16 per thread),
// the candidates of each round placed by wave scans and one exchange of the
// wave totals (one barrier, not two per round)
constexpr int kFrameRounds = kFrameChunk / (256 * 16);
__global__ __launch_bounds__(256) void k_frame_cand(FrameArgs a) {
  __shared__ uint32_t wt[kFrameRounds][4];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint64_t c0 = (uint64_t)blockIdx.x * kFrameChunk;
  uint4 v[kFrameRounds];
#pragma unroll
  for (int i = 0; i < kFrameRounds; i++) {
    const uint64_t u = c0 + ((uint64_t)i * 256 + t) * 16;
    v[i] = u < a.len ? *(const uint4*)(a.s + u) : make_uint4(0, 0, 0, 0);  // the slice buffer is padded (kSlicePad)
  }
  uint32_t m[kFrameRounds], ex[kFrameRounds];
#pragma unroll
  for (int i = 0; i < kFrameRounds; i++) {
    const uint64_t u = c0 + ((uint64_t)i * 256 + t) * 16;  // the 16 bytes [u, u + 16) hold magic bytes of p = u - 16 + j
    uint32_t mm = 0;
    if (u < a.len) {
      const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
      for (int d = 0; d < 4; d++) {
        const uint32_t z = zbytes(w[d] ^ 0x02020202u);
#pragma unroll
        for (int k = 0; k < 4; k++)
          if ((z >> (8 * k + 7)) & 1u) mm |= 1u << (4 * d + k);
      }
      // magic byte at u + j: candidate p = u + j - 16 (>= 0, inside the slice)
      const uint32_t lo = u < 16 ? (uint32_t)(16 - u) : 0u;
      const uint64_t lim = a.len + 16 - u;  // p < len
      mm &= (0xFFFFu << lo) & 0xFFFFu;
      if (lim < 16) mm &= (1u << lim) - 1u;
    }
    m[i] = mm;
    const uint32_t c = (uint32_t)__builtin_popcount(mm);
    const uint32_t inc = wave_incl_scan(c);
    ex[i] = inc - c;
    if (lane == 63) wt[i][wv] = inc;
  }
  __syncthreads();
  uint32_t base = 0;
#pragma unroll
  for (int i = 0; i < kFrameRounds; i++) {
    uint32_t k = base + ex[i];
    for (uint32_t w2 = 0; w2 < wv; w2++) k += wt[i][w2];
    base += wt[i][0] + wt[i][1] + wt[i][2] + wt[i][3];
    const uint64_t u = c0 + ((uint64_t)i * 256 + t) * 16;
    uint32_t mm = m[i];
    while (mm) {
      const uint32_t j = (uint32_t)__builtin_ctz(mm);
      mm &= mm - 1;
      if (k < kFrameCap) a.cbuf[(uint64_t)blockIdx.x * kFrameCap + k] = (uint16_t)(u + j - 16 - c0 + 16);
      k++;
    }
  }
  if (t == 0) {
    a.ccnt[blockIdx.x] = base < kFrameCap ? base : kFrameCap;
    if (base > kFrameCap) atomicMax(&a.scal[0], 1ull);  // too dense: host walk
  }
}
// 2. compaction: chunk offsets were stored relative to c0 - 16
__global__ __launch_bounds__(256) void k_frame_compact(FrameArgs a, uint32_t nchunks) {
  const uint32_t b = blockIdx.x;
  if (b >= nchunks) return;
  const uint32_t n = a.ccnt[b];
  const uint64_t c0 = (uint64_t)b * kFrameChunk;
  for (uint32_t k = threadIdx.x; k < n; k += 256)
    a.cand[a.coff[b] + k] = c0 + a.cbuf[(uint64_t)b * kFrameCap + k] - 16;
}
__device__ __forceinline__ uint32_t be32_at(const uint8_t* p) { return __builtin_bswap32(ld_u32_at(p)); }
// 3. each candidate's successor (the host walk's next step from it)
__global__ __launch_bounds__(256) void k_frame_next(FrameArgs a) {
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < a.ncand; c += (uint64_t)gridDim.x * 256) {
    const uint64_t p = a.cand[c];
    uint32_t nx, nrec = 0;
    if (a.len - p < 57) {
      nx = FN_IO;  // "not enough for batch header"
    } else {
      const int32_t batch_len = (int32_t)be32_at(a.s + p + 8);
      const int16_t attrs = (int16_t)(be32_at(a.s + p + 19) & 0xFFFFu);  // bytes 21..22
      const uint64_t rem = (uint64_t)(int64_t)batch_len - 45;
      if (batch_len < 45 || a.len - p - 57 < rem) {
        nx = FN_IO;
      } else if (attrs & 7) {
        nx = (attrs & 7) <= 4 ? FN_UNSUP : FN_IO;  // compressed sections: not on the GPU path yet
      } else {
        if (rem >= 4) {
          const int32_t cnt = (int32_t)be32_at(a.s + p + 57);
          uint64_t c64 = cnt > 0 ? (uint64_t)cnt : 0;
          const uint64_t mx = (rem - 4) / 7;  // a record is at least 7 bytes
          nrec = (uint32_t)(c64 < mx ? c64 : mx);
        }
        const uint64_t q = p + 57 + rem;
        if (q == a.len) {
          nx = FN_END;
        } else if (a.len - q < 57) {
          nx = FN_TAIL;  // "not enough for batch header" after this batch
        } else {  // the candidate at q, if any
          uint64_t lo = c + 1, hi = a.ncand;
          while (lo < hi) {
            const uint64_t m = (lo + hi) >> 1;
            if (a.cand[m] < q) lo = m + 1; else hi = m;
          }
          nx = lo < a.ncand && a.cand[lo] == q ? (uint32_t)lo : FN_NONCAND;
        }
      }
    }
    a.term[c] = nx;
    a.nrec[c] = nrec;
    a.jmp[c] = nx < FN_END ? nx : (uint32_t)a.ncand;  // ends -> sink
    a.mark[c] = c == 0 && p == 0 ? 1u : 0u;
    if (c == 0 && p != 0) atomicMax(&a.scal[0], 1ull);  // position 0 has no magic 2: the host walk decides
  }
}
__global__ __launch_bounds__(256) void k_frame_double(const uint32_t* src, uint32_t* dst, uint64_t n) {
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < n; c += (uint64_t)gridDim.x * 256) {
    const uint32_t x = src[c];
    dst[c] = x < n ? src[x] : x;
  }
}
// top-down: everything 2^level batches after a marked batch is on the chain
__global__ __launch_bounds__(256) void k_frame_mark(const uint32_t* jl, uint32_t* mark, uint64_t n) {
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < n; c += (uint64_t)gridDim.x * 256) {
    if (!__hip_atomic_load(&mark[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) continue;
    const uint32_t x = jl[c];
    if (x < n) __hip_atomic_store(&mark[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// 4. the chain's batches in order; tail status / fallback from its last batch
__global__ __launch_bounds__(256) void k_frame_emit(FrameArgs a) {
  unsigned long long hb = 0;
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < a.ncand; c += (uint64_t)gridDim.x * 256) {
    if (!a.mark[c]) continue;
    const uint64_t i = a.mpre[c];
    if (a.term[c] == FN_NONCAND) atomicMax(&a.scal[0], 1ull);  // a batch without magic 2 follows: host walk
    const uint64_t p = a.cand[c];
    a.bpos[i] = p;
    a.rbase[i] = a.rpre[c];
    hb += 57 + ((uint64_t)be32_at(a.s + p + 8) - 45);
  }
  hb = wave_sum(hb);
  if (lane_id() == 0 && hb) atomicAdd(&a.scal[2], hb);
}
// record counts of the chain's batches only (the ends and tails count none)
__global__ __launch_bounds__(256) void k_frame_counts(FrameArgs a) {
  for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < a.ncand; c += (uint64_t)gridDim.x * 256) {
    const uint32_t nx = a.term[c];
    const bool on = a.mark[c] != 0;
    if (on && (nx == FN_IO || nx == FN_UNSUP || nx == FN_TAIL))
      a.scal[1] = nx == FN_UNSUP ? 2ull : 1ull;  // the walk stops here (FN_TAIL: after this batch)
    if (!on || nx == FN_IO || nx == FN_UNSUP) {  // a tail position is no batch
      a.nrec[c] = 0;
      a.mark[c] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// CRC32C (reflected 0x82F63B78) over [off, off + n): chunked raw CRCs + combine
// ---------------------------------------------------------------------------
// Tables (built on the host by upload_crc_tables):
//   g_crc_z16[q][v]   raw CRC of byte v followed by q zero bytes (q = 0..15):
//                     slice-by-16 of one 16-byte block
//   g_crc_shift[k]    the linear map "append 2^k zero bytes" (x^(8*2^k) mod P),
//                     as 4 byte-indexed tables: shift(c) = ^_i T[i][(c >> 8i) & 0xff]
// The k_crc16 path: raw CRC (init 0) of the 16-byte-aligned region [16, Z) with
// the bytes before the CRC start masked to zero (leading zeros leave a raw CRC
// unchanged), every thread's blocks folded with the 4 KiB shift, per-thread
// partials shifted to the chunk end, chunk CRCs shifted to the region end and
// XOR-combined (exact: CRC is linear over GF(2)); k_crc_final appends the
// unaligned tail bytewise and applies the 0xFFFFFFFF init / final xor.
constexpr int kCrcShiftLevels = 48;
__device__ uint32_t g_crc_z16[16][256];
__device__ uint32_t g_crc_shift[kCrcShiftLevels][4][256];
constexpr int kCrcThreads = 256;
constexpr int kCrcIters = 16;                               // blocks per thread per chunk
constexpr uint32_t kCrcChunkBlocks = kCrcThreads * kCrcIters;  // 4096 x 16 B = 64 KiB

__device__ __forceinline__ uint32_t crc_shift_tab(const uint32_t (*T)[256], uint32_t c) {
  return T[0][c & 0xff] ^ T[1][(c >> 8) & 0xff] ^ T[2][(c >> 16) & 0xff] ^ T[3][c >> 24];
}
// append `n` zero bytes to a raw CRC state (global tables, any n < 2^48)
__device__ __forceinline__ uint32_t crc_shift_bytes(uint32_t c, uint64_t n) {
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1) c = crc_shift_tab(g_crc_shift[k], c);
  return c;
}

// One 64 KiB chunk per workgroup iteration; the next chunk's blocks are loaded
// (into registers) while this one is folded, and the barriers wait for LDS
// only, so the loads stay in flight.
__device__ __forceinline__ void crc16_body(const uint8_t* __restrict__ out, uint64_t skip, uint64_t nblocks,
                                           uint32_t* acc, uint32_t bid, uint32_t gdim) {
  __shared__ uint32_t z[16][256];
  __shared__ uint32_t sh[9][4][256];  // shifts by 16 B .. 4 KiB (2^4 .. 2^12 bytes)
  __shared__ uint32_t red[2][kCrcThreads / 64];
  const uint32_t t = threadIdx.x;
  const uint4* base = (const uint4*)(out + 16);
  const uint64_t nchunks = (nblocks + kCrcChunkBlocks - 1) / kCrcChunkBlocks;
  uint64_t ch = bid;
  if (ch >= nchunks) return;
  // blocks of chunk c: unconditional loads, clamped to the last block (a
  // conditional load would be waited for at once)
  auto fetch = [&](uint64_t c, uint4 (&v)[kCrcIters]) {
    const uint64_t b0 = c * kCrcChunkBlocks;
#pragma unroll
    for (int i = 0; i < kCrcIters; i++) {
      const uint64_t j = b0 + t + (uint32_t)i * kCrcThreads;
      v[i] = base[j < nblocks ? j : nblocks - 1];
    }
  };
  uint4 v[kCrcIters], nv[kCrcIters];
  fetch(ch, v);
  for (uint32_t i = t; i < 16 * 256; i += kCrcThreads) (&z[0][0])[i] = (&g_crc_z16[0][0])[i];
  for (uint32_t i = t; i < 9 * 4 * 256; i += kCrcThreads) (&sh[0][0][0])[i] = (&g_crc_shift[4][0][0])[i];
  __syncthreads();
  uint32_t par = 0;
  for (;;) {
    const uint64_t chn = ch + gdim;
    fetch(chn < nchunks ? chn : ch, nv);  // the last iteration re-reads its own chunk
    const uint64_t b0 = ch * kCrcChunkBlocks;
    const uint32_t nb = (uint32_t)(nblocks - b0 < kCrcChunkBlocks ? nblocks - b0 : kCrcChunkBlocks);
    if (b0 == 0 && t == 0) {  // bytes [16, 16 + skip) precede the CRC region
      uint32_t w[4] = {v[0].x, v[0].y, v[0].z, v[0].w};
#pragma unroll
      for (int q = 0; q < 16; q++)
        if ((uint64_t)q < skip) w[q >> 2] &= ~(0xffu << (8 * (q & 3)));
      v[0].x = w[0];
      v[0].y = w[1];
      v[0].z = w[2];
      v[0].w = w[3];
    }
    uint32_t c = 0;
    int last = -1;
#pragma unroll
    for (int i = 0; i < kCrcIters; i++) {
      const uint32_t j = t + (uint32_t)i * kCrcThreads;
      if (j < nb) {
        const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        uint32_t r = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) r ^= z[15 - q][(w[q >> 2] >> (8 * (q & 3))) & 0xff];
        c = crc_shift_tab(sh[8], c) ^ r;  // previous blocks move 4 KiB further from the end
        last = i;
      }
    }
    // shift to the chunk end: (nb - 1 - j_last) blocks of 16 B
    if (last >= 0) {
      uint32_t d = nb - 1 - (t + (uint32_t)last * kCrcThreads);
#pragma unroll
      for (int k = 0; k < 8; k++)
        if ((d >> k) & 1) c = crc_shift_tab(sh[k], c);
    }
    // workgroup XOR reduce (alternating slots: one LDS-only barrier)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o, 64);
    if ((t & 63) == 0) red[par][t >> 6] = c;
    lean_sync();
    if (t == 0) {
      uint32_t x = red[par][0] ^ red[par][1] ^ red[par][2] ^ red[par][3];
      x = crc_shift_bytes(x, (nblocks - b0 - nb) * 16ull);  // to the end of the aligned region
      atomicXor(acc, x);
    }
    par ^= 1u;
    if (chn >= nchunks) break;
    ch = chn;
#pragma unroll
    for (int i = 0; i < kCrcIters; i++) v[i] = nv[i];
  }
}
__global__ __launch_bounds__(kCrcThreads) void k_crc16(const uint8_t* __restrict__ out, uint64_t skip,
                                                        uint64_t nblocks, uint32_t* acc) {
  crc16_body(out, skip, nblocks, acc, blockIdx.x, gridDim.x);
}

// tail bytes [tail0, end) bytewise, init/xorout, big-endian CRC at out[17..21)
__global__ void k_crc_final(uint8_t* out, const uint32_t* acc, uint64_t tail0, uint64_t end, uint64_t n) {
  if (threadIdx.x != 0) return;
  uint32_t c = *acc;
  for (uint64_t i = tail0; i < end; i++) c = g_crc_z16[0][(c ^ out[i]) & 0xff] ^ (c >> 8);
  uint32_t crc = c ^ crc_shift_bytes(0xFFFFFFFFu, n) ^ 0xFFFFFFFFu;
  out[17] = (uint8_t)(crc >> 24);
  out[18] = (uint8_t)(crc >> 16);
  out[19] = (uint8_t)(crc >> 8);
  out[20] = (uint8_t)crc;
}

// ---------------------------------------------------------------------------
// k_verify_crc: CRC32C of every stored batch checked against its header on
// ingest (north_star "verify CRC32C").  The reference computes the CRC only on
// encode and never checks it (protocol record/batch.rs:398-430), so this only
// reports: process_batch never looks at the result.  One wave per batch
// (persistent over the batches) over the 16-byte-ALIGNED units covering the
// CRC range [pos + 21, end) (one dwordx4 load each; bytes outside the range
// masked to zero).  Lane j takes units j, j + 64, ... four at a time (the four
// loads in flight together), folding each with the 1 KiB shift table staged
// in LDS beside the slice-by-16 tables; its partial then moves to the aligned
// end E and the wave XORs the partials.  The raw CRC at E is the range's raw
// CRC followed by E - end zero bytes, so the stored value is compared after
// the same shift (x^8 is invertible mod the CRC32C polynomial: the comparison
// is exact).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_verify_crc(const uint8_t* __restrict__ sl, const uint64_t* __restrict__ bpos,
                                                    uint32_t nb, unsigned long long* bad, uint32_t* flags) {
  __shared__ uint32_t z[16][256];
  __shared__ uint32_t sh1k[4][256];
  for (uint32_t i = threadIdx.x; i < 16 * 256; i += 256) (&z[0][0])[i] = (&g_crc_z16[0][0])[i];
  for (uint32_t i = threadIdx.x; i < 4 * 256; i += 256) (&sh1k[0][0])[i] = (&g_crc_shift[10][0][0])[i];
  __syncthreads();
  const uint32_t l = lane_id();
  const uint32_t W = gridDim.x * 4;
  for (uint32_t b = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6)); b < nb; b += W) {
    const uint64_t pos = bpos[b];
    const uint32_t blen = __builtin_bswap32(ld_u32_at(sl + pos + 8));
    const uint32_t stored = __builtin_bswap32(ld_u32_at(sl + pos + 17));
    const uint64_t a = pos + 21, e = pos + 12 + (uint64_t)blen;  // framing checked batch_len >= 45
    const uint64_t U0 = a & ~15ull, E = (e + 15) & ~15ull;
    const uint32_t nu = (uint32_t)((E - U0) / 16);
    const uint4* units = (const uint4*)(sl + U0);
    auto crc_of = [&](uint32_t u, uint4 v) {
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
      const uint64_t x = U0 + 16ull * u;
      if (x < a || x + 16 > e) {  // the range's first / last unit
#pragma unroll
        for (int q = 0; q < 16; q++)
          if (x + q < a || x + q >= e) w[q >> 2] &= ~(0xffu << (8 * (q & 3)));
      }
      uint32_t r = 0;
#pragma unroll
      for (int q = 0; q < 16; q++) r ^= z[15 - q][(w[q >> 2] >> (8 * (q & 3))) & 0xff];
      return r;
    };
    auto fold = [&](uint32_t c) { return sh1k[0][c & 0xff] ^ sh1k[1][(c >> 8) & 0xff] ^ sh1k[2][(c >> 16) & 0xff] ^ sh1k[3][c >> 24]; };
    uint32_t acc = 0, last = 0;
    bool any = false;
    uint32_t u = l;
    for (; u + 192 < nu; u += 256) {  // four units per lane per round, loads first
      const uint4 v0 = units[u], v1 = units[u + 64], v2 = units[u + 128], v3 = units[u + 192];
      const uint32_t r0 = crc_of(u, v0), r1 = crc_of(u + 64, v1), r2 = crc_of(u + 128, v2), r3 = crc_of(u + 192, v3);
      acc = fold(fold(fold(fold(acc) ^ r0) ^ r1) ^ r2) ^ r3;
      last = u + 192;
      any = true;
    }
    for (; u < nu; u += 64) {
      acc = fold(acc) ^ crc_of(u, units[u]);  // earlier units of this lane: 1 KiB further back
      last = u;
      any = true;
    }
    if (any) acc = crc_shift_bytes(acc, 16ull * (nu - 1 - last));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
    if (l == 0) {
      const uint32_t want = crc_shift_bytes(stored ^ 0xFFFFFFFFu ^ crc_shift_bytes(0xFFFFFFFFu, e - a), E - e);
      const bool ok = acc == want;
      if (flags) flags[b] = ok ? 0u : 1u;
      if (!ok) {
        atomicAdd(&bad[0], 1ull);
        atomicMin(&bad[1], (unsigned long long)b);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// record-section decompression at ingest (fsg_codec_dev.h): sizing pass, a
// writing pass into the decompressed slice (batch header copied with
// batch_len = 45 + decompressed length, compression bits kept for the output
// header), the record counts of the new sections
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t dec_rem(const uint8_t* src, uint64_t pos) {
  return (uint64_t)__builtin_bswap32(ld_u32_at(src + pos + 8)) - 45;  // framing checked batch_len >= 45
}
__global__ __launch_bounds__(256) void k_dec_size(DecArgs a) {
  for (uint32_t b = blockIdx.x * 256 + threadIdx.x; b < a.nb; b += gridDim.x * 256) {
    const uint64_t pos = a.bpos[b], rem = dec_rem(a.src, pos);
    const uint32_t codec = a.codec[b];
    if (!codec) {
      a.dsize[b] = (int64_t)rem;
      continue;
    }
    DecOut o{nullptr, 0, 0, false};
    a.dsize[b] = dev_decompress(codec, a.src + pos + 57, rem, o, &g_crc_z16[0][0]);
  }
}
__global__ __launch_bounds__(256) void k_dec_write(DecArgs a) {
  for (uint32_t b = blockIdx.x * 256 + threadIdx.x; b < a.nb; b += gridDim.x * 256) {
    const uint32_t codec = a.codec[b];
    if (!codec) continue;
    const uint64_t pos = a.bpos[b], rem = dec_rem(a.src, pos), np = a.npos[b];
    const int64_t ds = a.dsize[b];
    uint8_t* d = a.dst + np;
    for (int k = 0; k < 57; k++) d[k] = a.src[pos + k];
    const uint32_t bl = (uint32_t)(45 + ds);
    d[8] = (uint8_t)(bl >> 24);
    d[9] = (uint8_t)(bl >> 16);
    d[10] = (uint8_t)(bl >> 8);
    d[11] = (uint8_t)bl;
    DecOut o{d + 57, 0, (uint64_t)ds, true};
    const int64_t r = dev_decompress(codec, a.src + pos + 57, rem, o, &g_crc_z16[0][0]);
    a.status[b] = r == ds ? 0 : -1;
  }
}
__global__ __launch_bounds__(256) void k_dec_copy(DecArgs a) {  // uncompressed batches, a wave each
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= a.nb || a.codec[b]) return;
  const uint64_t pos = a.bpos[b], n = 57 + dec_rem(a.src, pos), np = a.npos[b];
  for (uint64_t k = lane_id(); k < n; k += 64) a.dst[np + k] = a.src[pos + k];
}
__global__ __launch_bounds__(256) void k_dec_count(DecArgs a) {
  for (uint32_t b = blockIdx.x * 256 + threadIdx.x; b < a.nb; b += gridDim.x * 256) {
    const uint64_t np = a.npos[b], ds = (uint64_t)a.dsize[b];
    uint64_t c = 0;
    if (ds >= 4) {  // Vec<Record> count (FileBatchIterator framing's estimate)
      const int32_t v = (int32_t)__builtin_bswap32(ld_u32_at(a.dst + np + 57));
      c = v > 0 ? (uint64_t)v : 0;
      const uint64_t mx = (ds - 4) / 7;
      c = c < mx ? c : mx;
    }
    a.cnt[b] = c;
  }
}

// ---------------------------------------------------------------------------
// k_write_lean: the output of one batch of verbatim records (KM_COPY /
// KM_UPPER: filters, uppercase maps, projections) assembled in LDS and stored
// with 16-byte stores, for batches of many small records (where k_write's
// record-by-record wave copies leave the memory system idle).
//   1. wave 0, lane = record: size, wave scan, the varint fields written into
//      the staging buffer, the key / value segments into a table
//   2. all threads: segment bytes global -> LDS in 16-byte units aligned like
//      the output (interior units one LDS store, edge units bytewise), four
//      units per round with every load in flight before the first use
//   3. LDS -> HBM: interior units dwordx4 stores, the two edge units bytewise
// A batch with more than 64 survivors or more bytes than the staging buffer
// is written by the generic wave path (write_batch_wave).
// (A CRC computed from the staging buffer was measured twice and is not used:
// 64-byte pieces combined with GF(2) multiplies (round 2), and the
// slice-by-16 / shift tables read from global memory per unit (round 4: C2
// write 1.24 -> 4.70 ms, against k_crc16's 0.52 ms).)
// ---------------------------------------------------------------------------
constexpr int kWlThreads = 256;
constexpr int kObuf = 17408;  // staging bytes (one 16 KiB batch + re-encoding growth + alignment)
struct __attribute__((aligned(16))) WlLds {
  uint8_t ob[kObuf + 16];
  uint64_t s_src[128];   // segment source offsets (key and value of up to 64 records)
  uint32_t s_dst[128];   // staging offset
  uint32_t s_len[128];   // length | upper << 31
  uint32_t s_upre[129];  // exclusive prefix of the segments' 16-byte units
  uint32_t total, nunits, big;
};

// the generic writer of one batch (k_write's body), wave-wide
__device__ __forceinline__ void write_batch_wave(const WriteArgs& a, const KeptRec* d, uint32_t nkeep, int64_t rel, uint64_t obase) {
  const uint32_t lane = lane_id();
  uint8_t* out = a.out;
  uint64_t run = 0;
  for (uint32_t k0 = 0; k0 < nkeep; k0 += 64) {
    const uint32_t k = k0 + lane;
    const bool v = k < nkeep;
    KeptRec r = {};
    uint32_t sz = 0;
    if (v) {
      r = d[k];
      sz = rec_out_size(r, rel, 0, 0);
    }
    const uint64_t incl = wave_incl_scan((uint64_t)sz);
    const uint64_t my = obase + run + incl - sz;
    uint64_t kd = 0, vd = 0;
    uint32_t kl = 0, vc = 0;
    if (v) {
      uint8_t* q = out + my;
      const uint32_t vl = r.vlen;
      const uint32_t inner = 1 + vsize(r.ts) + vsize(r.od + rel) + 1 +
                             (r.has_key ? vsize((int64_t)r.klen) + r.klen : 0) + vsize((int64_t)vl) + vl + vsize(r.hdr);
      uint8_t t[16];
      uint32_t n = venc((int64_t)inner, t), w = 0;
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      q[w++] = r.attr;
      n = venc(r.ts, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      n = venc(r.od + rel, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      q[w++] = r.has_key ? 1 : 0;
      if (r.has_key) {
        n = venc((int64_t)r.klen, t);
        for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
        kd = my + w;
        kl = r.klen;
        w += r.klen;
      }
      n = venc((int64_t)vl, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
      vd = my + w;
      vc = vl;
      w += vl;
      n = venc(r.hdr, t);
      for (uint32_t i = 0; i < n; i++) q[w++] = t[i];
    }
    const uint32_t nrec = nkeep - k0 < 64u ? nkeep - k0 : 64u;
    for (uint32_t i = 0; i < nrec; i++) {
      const uint32_t rkl = __builtin_amdgcn_readlane(kl, i);
      const uint32_t rvc = __builtin_amdgcn_readlane(vc, i);
      if (rkl) copy_seg(out, a.slice, readlane_u64(kd, i), readlane_u64(r.kpos, i), rkl, false);
      if (rvc)
        copy_seg(out, a.slice, readlane_u64(vd, i), readlane_u64(r.vpos, i), rvc,
                 __builtin_amdgcn_readlane((uint32_t)r.mode, i) == KM_UPPER);
    }
    run += readlane_u64(incl, 63);
  }
}

// phase 1 on wave 0 (lane = record, `r` its descriptor when v): sizes, the
// varint fields into the staging buffer, the segment table, L.total / nunits / big
__device__ __forceinline__ void wl_phase1(WlLds& L, const KeptRec& r, bool v, int64_t rel, uint32_t d0, uint32_t nk) {
  const uint32_t lane = lane_id();
  uint32_t sz = 0;
  if (v) sz = rec_out_size(r, rel, 0, 0);
  const uint32_t incl = wave_incl_scan(sz);
  const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
  const bool big = nk > 64 || d0 + total > (uint32_t)kObuf;
  uint32_t uk = 0, uv = 0;
  if (v && !big) {
    const uint32_t off = d0 + incl - sz;
    uint8_t* q = L.ob + off;
    const uint32_t vl = r.vlen;
    const uint32_t inner = 1 + vsize(r.ts) + vsize(r.od + rel) + 1 +
                           (r.has_key ? vsize((int64_t)r.klen) + r.klen : 0) + vsize((int64_t)vl) + vl + vsize(r.hdr);
    uint32_t w = venc((int64_t)inner, q);  // varints straight into the staging buffer
    q[w++] = r.attr;
    w += venc(r.ts, q + w);
    w += venc(r.od + rel, q + w);
    q[w++] = r.has_key ? 1 : 0;
    uint32_t kdst = off + w;
    if (r.has_key) {
      w += venc((int64_t)r.klen, q + w);
      kdst = off + w;
      w += r.klen;
    }
    w += venc((int64_t)vl, q + w);
    const uint32_t vdst = off + w;
    w += vl;
    w += venc(r.hdr, q + w);
    const uint32_t kl = r.has_key ? r.klen : 0u;
    L.s_src[2 * lane] = r.kpos;
    L.s_dst[2 * lane] = kdst;
    L.s_len[2 * lane] = kl;
    L.s_src[2 * lane + 1] = r.vpos;
    L.s_dst[2 * lane + 1] = vdst;
    L.s_len[2 * lane + 1] = vl | (r.mode == KM_UPPER ? 0x80000000u : 0u);
    uk = kl ? ((kdst + kl + 15) >> 4) - (kdst >> 4) : 0u;
    uv = vl ? ((vdst + vl + 15) >> 4) - (vdst >> 4) : 0u;
  }
  const uint32_t ui = wave_incl_scan(uk + uv);
  if (v && !big) {
    L.s_upre[2 * lane] = ui - uk - uv;
    L.s_upre[2 * lane + 1] = ui - uv;
  }
  if (lane == 0) {
    L.total = total;
    L.nunits = __builtin_amdgcn_readlane(ui, 63);
    L.big = big ? 1u : 0u;
  }
  if (lane == 0 && !big) L.s_upre[2 * (nk < 64 ? nk : 64)] = __builtin_amdgcn_readlane(ui, 63);
}
// phases 2 and 3 on every thread (after phase 1 and a barrier; L.big clear)
__device__ __forceinline__ void wl_phase23(const WriteArgs& a, WlLds& L, uint64_t obase, uint32_t d0, uint32_t nk) {
  const uint32_t t = threadIdx.x;
  const uint32_t total = L.total, nunits = L.nunits, nseg = 2 * nk;
  // 2. segments -> staging, thread t copies the contiguous units [u0, u1)
  {
    const uint32_t per = (nunits + kWlThreads - 1) / kWlThreads;
    const uint32_t u0 = t * per, u1 = u0 + per < nunits ? u0 + per : nunits;
    int s = 0;
    if (u0 < u1) {  // last segment with s_upre <= u0
      int lo = 0, hi = (int)nseg - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) >> 1;
        if (L.s_upre[m] <= u0) lo = m; else hi = m - 1;
      }
      s = lo;
    }
    // four units per round: every load of the round is in flight before the first use
    for (uint32_t u = u0; u < u1; u += 4) {
      uint4 x0[4], x1[4];
      uint32_t D[4], lo[4], hi[4], sh[4], up[4];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t uu = u + i < u1 ? u + i : u1 - 1;  // a clamped duplicate does no harm (same bytes)
        while (L.s_upre[s + 1] <= uu) s++;
        const uint32_t dst = L.s_dst[s], lw = L.s_len[s];
        const uint32_t len = lw & 0x7FFFFFFFu;
        up[i] = lw >> 31;
        D[i] = ((dst >> 4) + (uu - L.s_upre[s])) << 4;      // staging unit start
        const uint64_t A = L.s_src[s] + D[i] - dst;          // source of the unit's first byte (may precede the segment)
        sh[i] = (uint32_t)(A & 15);
        lo[i] = D[i] > dst ? D[i] : dst;
        hi[i] = D[i] + 16 < dst + len ? D[i] + 16 : dst + len;
        const uint4* src = (const uint4*)(a.slice + (A & ~15ull));
        x0[i] = src[0];
        x1[i] = src[1];
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint32_t w[8] = {x0[i].x, x0[i].y, x0[i].z, x0[i].w, x1[i].x, x1[i].y, x1[i].z, x1[i].w};
        // words q .. q + 4 of w (q = sh / 4) by bit masks: a select on the
        // index would become an indexed (scratch) access
        const uint32_t m1 = 0u - ((sh[i] >> 2) & 1u), m2 = 0u - ((sh[i] >> 3) & 1u), bs = sh[i] & 3u;
        uint32_t tw[5];
#pragma unroll
        for (int j = 0; j < 5; j++) {
          const uint32_t a0 = (w[j] & ~m1) | (w[j + 1] & m1);
          const uint32_t a1 = (w[j + 2] & ~m1) | (w[j + 3] & m1);
          tw[j] = (a0 & ~m2) | (a1 & m2);
        }
        uint32_t v4[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          v4[j] = __builtin_amdgcn_alignbyte(tw[j + 1], tw[j], bs);
          if (up[i]) v4[j] = swar_upper(v4[j]);
        }
        if (lo[i] == D[i] && hi[i] == D[i] + 16) {
          *(uint4*)(L.ob + D[i]) = make_uint4(v4[0], v4[1], v4[2], v4[3]);
        } else {
#pragma unroll
          for (uint32_t j = 0; j < 16; j++)
            if (j >= lo[i] - D[i] && j < hi[i] - D[i]) L.ob[D[i] + j] = (uint8_t)(v4[j >> 2] >> (8 * (j & 3)));
        }
      }
    }
  }
  __syncthreads();
  const uint32_t E = d0 + total;
  // 3. staging -> HBM
  uint8_t* og = a.out + obase - d0;
  const uint32_t nu = (E + 15) >> 4;
  for (uint32_t u = t; u < nu; u += kWlThreads) {
    const uint32_t D = u << 4;
    if (D >= d0 && D + 16 <= E) {
      *(uint4*)(og + D) = *(const uint4*)(L.ob + D);
    } else {
      const uint32_t lo = D > d0 ? D : d0, hi = D + 16 < E ? D + 16 : E;
      for (uint32_t j = lo; j < hi; j++) og[j] = L.ob[j];
    }
  }
}

__global__ __launch_bounds__(kWlThreads) void k_write_lean(WriteArgs a) {
  __shared__ WlLds L;
  const int32_t b = a.first + (int32_t)blockIdx.x;
  if (a.first < 0 || b > a.last) return;
  const uint32_t t = threadIdx.x, lane = t & 63u;
  const BatchStat st = a.bstat[b];
  const int64_t rel = a.seg ? 0 : a.base - st.base_offset;
  const KeptRec* d = a.desc + a.rbase[b];
  const uint64_t obase = a.seg ? 61ull * (uint64_t)(b + 1) + a.pre[b].rec_bytes
                               : 61 + (a.pre[b].rec_bytes - a.pre[a.first].rec_bytes);
  const uint32_t d0 = (uint32_t)(obase & 15);
  const uint32_t nk = st.nkeep;
  if (t < 64) {  // 1. headers and segments
    const bool v = lane < nk && nk <= 64;
    KeptRec r = {};
    if (v) r = d[lane];
    wl_phase1(L, r, v, rel, d0, nk);
  }
  __syncthreads();
  if (L.big) {  // generic path for this batch
    if (t < 64) write_batch_wave(a, d, nk, rel, obase);
    return;
  }
  wl_phase23(a, L, obase, d0, nk);
}


// ---------------------------------------------------------------------------
// stateful last stages (k_sf_*): filter_look_back (examples/filter_look_back:
// keep a value above PREV, PREV = the kept value; look_back sets PREV to each
// record) and filter_hashset (examples/filter_hashset: SET.insert(value) keeps
// the record when the value was new; the BoundedHashSet holds the newest
// `limit` insertions).  k_eval validated / parsed every record reaching the
// stage and kept it; these kernels decide in stream order over the batches
// process_batch ran the stage on (sf_ran), compact the descriptors in place,
// and, after k_plan, commit the state through plan.done.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool sf_ran(const Mins& m, uint32_t b, uint32_t flags) {
  if (b >= m.first_dec || b >= m.first_unsup) return false;  // (0xFFFFFFFF = none)
  if (b < m.first_err) return true;
  return b == m.first_err && (flags & BF_LAST_STAGE);  // the error was the stage's own
}
__device__ __forceinline__ uint32_t sf_word(const uint8_t* p, uint32_t i, uint32_t n, bool upper) {
  uint32_t w = ld_u32_at(p + i);
  if (upper) w = swar_upper(w);
  if (n - i < 4) w &= (1u << (8 * (n - i))) - 1u;
  return w;
}
// hash of a value's bytes as the stage sees them (the uppercase view after a map)
__device__ uint64_t sf_hash(const uint8_t* p, uint32_t n, bool upper) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
  for (uint32_t i = 0; i < n; i += 4) {
    h = (h ^ sf_word(p, i, n, upper)) * 0x100000001B3ull;
    h ^= h >> 29;
  }
  return h | 1ull;
}
__device__ bool sf_eq(const uint8_t* p, bool pu, const uint8_t* q, bool qu, uint32_t n) {
  for (uint32_t i = 0; i < n; i += 4)
    if (sf_word(p, i, n, pu) != sf_word(q, i, n, qu)) return false;
  return true;
}

// per batch: LB: the max of the stage's values; dedup: value hashes and spans
__global__ __launch_bounds__(256) void k_sf_prep(SfArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nbatches) return;
  const BatchStat st = a.bstat[b];
  const bool ran = sf_ran(*a.mins, b, st.flags);
  const uint64_t rb = a.rbase[b];
  const uint32_t nk = ran ? st.nkeep : 0u;
  if (a.op == OP_LB_MAX) {
    int64_t m = INT64_MIN;
    for (uint32_t k = l; k < nk; k += 64) {
      const int64_t v = a.desc[rb + k].ival;
      m = v > m ? v : m;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const int64_t t = __shfl_xor(m, o, 64);
      m = t > m ? t : m;
    }
    if (l == 0) a.bval[b] = m;
    return;
  }
  for (uint32_t k = l; k < nk; k += 64) {
    const KeptRec d = a.desc[rb + k];
    a.hv[rb + k] = sf_hash(a.slice + d.vpos, d.vlen, d.mode == KM_UPPER);
    a.vref[rb + k] = d.vpos | (d.mode == KM_UPPER ? kSfEnt : 0ull);  // the value's view, past the compaction
    a.vlen[rb + k] = d.vlen;
    a.keep[rb + k] = 0;
  }
  if (l == 0) a.bn[b] = nk;
}

__global__ __launch_bounds__(256) void k_sf_clear(SfArgs a) {
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < a.cap; s += gridDim.x * 256) {
    a.sref[s] = 0ull;
    a.first[s] = 0xFFFFFFFFu;
  }
}
// the persisted entries (distinct values) back into the table
__global__ __launch_bounds__(256) void k_sf_rehash(SfArgs a) {
  const uint32_t mask = a.cap - 1;
  for (uint64_t e = blockIdx.x * 256ull + threadIdx.x; e < a.n_ent; e += gridDim.x * 256ull) {
    uint32_t s = (uint32_t)a.ent_hash[e] & mask;
    while (atomicCAS(&a.sref[s], 0ull, kSfEnt | e) != 0ull) s = (s + 1) & mask;
  }
}
// every record of the stage: find or claim the slot of its value (exact byte
// compare against the slot's entry or first claimant), note the first record
__global__ __launch_bounds__(256) void k_sf_insert(SfArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nbatches) return;
  const uint32_t n = a.bn[b];
  const uint64_t rb = a.rbase[b];
  const uint32_t mask = a.cap - 1;
  for (uint32_t k = l; k < n; k += 64) {
    const uint64_t t = rb + k;
    const uint64_t vr = a.vref[t];
    const uint32_t vl = a.vlen[t];
    const uint8_t* v = a.slice + (vr & ~kSfEnt);
    const bool up = (vr & kSfEnt) != 0;
    const uint64_t h = a.hv[t];
    uint32_t s = (uint32_t)h & mask;
    for (;;) {
      const unsigned long long cur = atomicCAS(&a.sref[s], 0ull, (unsigned long long)(t + 1));
      if (cur == 0ull) break;  // claimed
      bool same;
      if (cur & kSfEnt) {
        const uint64_t e = cur & ~kSfEnt;
        same = a.ent_hash[e] == h && a.ent_len[e] == vl && sf_eq(v, up, a.arena + a.ent_pos[e], false, vl);
      } else {
        const uint64_t t2 = cur - 1;
        const uint64_t vr2 = a.vref[t2];
        same = a.hv[t2] == h && a.vlen[t2] == vl && sf_eq(v, up, a.slice + (vr2 & ~kSfEnt), (vr2 & kSfEnt) != 0, vl);
      }
      if (same) break;
      s = (s + 1) & mask;
    }
    a.slot[t] = s;
    atomicMin(&a.first[s], (uint32_t)t);
  }
}
// no eviction can happen during the call: a record is new iff its value is
// absent at the call's start (no entry, or an entry older than the newest
// `limit` insertions) and it is the value's first record
__global__ __launch_bounds__(256) void k_sf_decide(SfArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nbatches) return;
  const uint32_t nk = a.bn[b];
  const uint64_t rb = a.rbase[b];
  uint64_t cnt = 0;
  for (uint32_t k = l; k < nk; k += 64) {
    const uint64_t t = rb + k;
    const uint32_t s = a.slot[t];
    const unsigned long long ref = a.sref[s];
    bool present = false;
    if (ref & kSfEnt) {  // last new-insertion index + 1 (0: none)
      const uint64_t last1 = a.ent_last[ref & ~kSfEnt];
      present = last1 != 0 && a.n0 - (last1 - 1) <= a.limit;
    }
    const bool kp = !present && a.first[s] == (uint32_t)t;
    a.keep[t] = kp ? 1 : 0;
    cnt += kp ? 1 : 0;
  }
  cnt = wave_sum(cnt);
  if (l == 0) a.bval[b] = (int64_t)cnt;
}
// evictions possible: the BoundedHashSet walk in stream order, one thread
// (a value is present iff its last new-insertion index is among the newest
// `limit`); cur[] starts from the entries' indices
__global__ __launch_bounds__(256) void k_sf_cur_init(SfArgs a) {
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < a.cap; s += gridDim.x * 256) {
    const unsigned long long ref = a.sref[s];
    a.cur[s] = (ref & kSfEnt) ? a.ent_last[ref & ~kSfEnt] : 0ull;
  }
}
__global__ void k_sf_seq(SfArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t N = a.n0;
  for (uint32_t b = 0; b < a.nbatches; b++) {
    const uint32_t n = a.bn[b];
    const uint64_t rb = a.rbase[b];
    int64_t cnt = 0;
    for (uint32_t k = 0; k < n; k++) {
      const uint64_t t = rb + k;
      const uint32_t s = a.slot[t];
      const uint64_t last1 = a.cur[s];
      const bool present = last1 != 0 && N - (last1 - 1) <= a.limit;
      a.keep[t] = present ? 0 : 1;
      if (!present) {
        a.cur[s] = N + 1;
        a.idx[t] = N;
        N++;
        cnt++;
      }
    }
    a.bval[b] = cnt;
  }
}
// exclusive scan of one int64 per batch (op 0: sum, 1: max) from `init`, one
// workgroup; total = the inclusive value after the last batch
__global__ __launch_bounds__(1024) void k_sf_scan(const int64_t* v, int64_t* out, uint32_t n, uint32_t op, int64_t init,
                                                   const int32_t* init32, unsigned long long* total) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry_s;
  const uint32_t t = threadIdx.x, l = t & 63u, w = t >> 6;
  auto comb = [op](int64_t x, int64_t y) { return op ? (x > y ? x : y) : x + y; };
  const int64_t ident = op ? INT64_MIN : 0;
  int64_t carry = init32 ? (int64_t)*init32 : init;  // LB: PREV from HBM
  for (uint32_t base = 0; base < n; base += 1024) {
    const uint32_t i = base + t;
    int64_t x = i < n ? v[i] : ident;
    for (int o = 1; o < 64; o <<= 1) {  // wave inclusive scan
      const int64_t y = __shfl_up(x, o, 64);
      if ((int)l >= o) x = comb(x, y);
    }
    if (l == 63) wsum[w] = x;
    __syncthreads();
    if (t == 0) {
      int64_t c = carry;
      for (int k = 0; k < 16; k++) {
        const int64_t s = wsum[k];
        wsum[k] = c;  // exclusive prefix of wave k
        c = comb(c, s);
      }
      carry_s = c;
    }
    __syncthreads();
    const int64_t ex = __shfl_up(x, 1, 64);
    const int64_t pre = l == 0 ? wsum[w] : comb(wsum[w], ex);
    if (i < n) out[i] = pre;
    carry = carry_s;
    __syncthreads();
  }
  if (t == 0 && total) *total = (unsigned long long)carry;
}
// decisions -> in-place compaction of each batch's descriptors (LB: keep a
// value above the running max of PREV and the values before it)
__global__ __launch_bounds__(256) void k_sf_compact(SfArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nbatches) return;
  BatchStat st = a.bstat[b];
  if (!sf_ran(*a.mins, b, st.flags)) return;
  const uint64_t rb = a.rbase[b];
  int64_t carry = a.bpre[b];  // LB: PREV and every value before the batch; dedup: kept before it
  uint32_t w = 0;
  for (uint32_t k0 = 0; k0 < st.nkeep; k0 += 64) {
    const uint32_t k = k0 + l;
    const bool valid = k < st.nkeep;
    KeptRec d = {};
    if (valid) d = a.desc[rb + k];
    bool kp;
    if (a.op == OP_LB_MAX) {
      int64_t x = valid ? (int64_t)d.ival : INT64_MIN;
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if ((int)l >= o) x = x > y ? x : y;
      }
      int64_t ex = __shfl_up(x, 1, 64);
      if (l == 0) ex = INT64_MIN;
      const int64_t run = ex > carry ? ex : carry;
      kp = valid && (int64_t)d.ival > run;
      const int64_t top = __shfl(x, 63, 64);
      carry = top > carry ? top : carry;
    } else {
      kp = valid && a.keep[rb + k];
      if (a.fast) {
        const uint64_t bal = ballot(kp);
        if (kp) a.idx[rb + k] = a.n0 + (uint64_t)carry + (uint64_t)__popcll(bal & ((1ull << l) - 1ull));
        carry += __popcll(bal);
      }
    }
    const uint64_t bal = ballot(kp);
    if (kp) a.desc[rb + w + __popcll(bal & ((1ull << l) - 1ull))] = d;
    w += (uint32_t)__popcll(bal);
  }
  if (l == 0) {
    a.bstat[b].nkeep = w;
    a.bstat[b].nout = w;
  }
}
// after k_plan: PREV through plan.done
__global__ void k_sf_commit_lb(SfArgs a) {
  if (threadIdx.x != 0) return;
  const int32_t done = a.plan->done;
  if (done < 0) return;
  if (a.lookback) {  // look_back: PREV = the last record's value (stops at the first error)
    const Mins m = *a.mins;
    for (int32_t b = done; b >= 0; b--) {
      const BatchStat st = a.bstat[b];
      if (sf_ran(m, (uint32_t)b, st.flags) && st.nkeep) {
        *a.prev = a.desc[a.rbase[b] + st.nkeep - 1].ival;
        return;
      }
    }
    return;
  }
  const int64_t bv = a.bval[done], bp = a.bpre[done];
  *a.prev = (int32_t)(bv > bp ? bv : bp);
}
// dedup commit 1: a value first kept in this call (through plan.done) becomes
// an entry (bytes copied to the arena as the stage saw them)
__global__ __launch_bounds__(256) void k_sf_commit_new(SfArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nbatches || (int32_t)b > a.plan->done) return;
  const uint64_t rb = a.rbase[b];
  const uint32_t n = a.bn[b];  // 0 when the stage did not run on b
  for (uint32_t k = l; k < n; k += 64) {
    const uint64_t t = rb + k;
    if (!a.keep[t]) continue;
    const uint32_t s = a.slot[t];
    if ((a.sref[s] & kSfEnt) || a.first[s] != (uint32_t)t) continue;
    const uint64_t e = atomicAdd(&a.scal[0], 1ull);
    const uint32_t len = a.vlen[t];
    const uint64_t pos = atomicAdd(&a.scal[1], (unsigned long long)len);
    const uint64_t vr = a.vref[t];
    const uint8_t* src = a.slice + (vr & ~kSfEnt);
    const bool up = (vr & kSfEnt) != 0;
    for (uint32_t i = 0; i < len; i++) {
      uint8_t c = src[i];
      if (up && c >= 'a' && c <= 'z') c -= 32;
      a.arena[pos + i] = c;
    }
    a.ent_hash[e] = a.hv[t];
    a.ent_pos[e] = pos;
    a.ent_len[e] = len;
    a.ent_last[e] = 0;
    a.sref[s] = kSfEnt | e;
  }
}
// dedup commit 2: every entry's last new-insertion index (+1) through plan.done
__global__ __launch_bounds__(256) void k_sf_commit_last(SfArgs a) {
  const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t l = lane_id();
  if (b >= a.nbatches || (int32_t)b > a.plan->done) return;
  const uint64_t rb = a.rbase[b];
  const uint32_t n = a.bn[b];
  for (uint32_t k = l; k < n; k += 64) {
    const uint64_t t = rb + k;
    if (!a.keep[t]) continue;
    const unsigned long long ref = a.sref[a.slot[t]];
    atomicMax((unsigned long long*)&a.ent_last[ref & ~kSfEnt], (unsigned long long)(a.idx[t] + 1));
  }
}
// dedup commit 3: insertions through plan.done
__global__ void k_sf_commit_n(SfArgs a) {
  if (threadIdx.x != 0) return;
  const int32_t done = a.plan->done;
  a.scal[2] = a.n0 + (done >= 0 ? (uint64_t)(a.bpre[done] + a.bval[done]) : 0ull);
}

// ---------------------------------------------------------------------------
// host-side launch wrappers (called from fsg_runtime.cpp)
// ---------------------------------------------------------------------------
}  // namespace fsg

#include "fsg_launch.h"

namespace fsg {

// g_crc_z16 / g_crc_shift exist once per device: upload per device, under a lock
static std::mutex g_tabs_mu;
static uint64_t g_tabs_ready = 0;  // bit d: tables resident on device d

hipError_t upload_crc_tables() {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(g_tabs_mu);
  if (dev < 64 && ((g_tabs_ready >> dev) & 1)) return hipSuccess;
  static uint32_t z16[16][256];
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    z16[0][i] = c;
  }
  for (int t = 1; t < 16; t++)
    for (uint32_t i = 0; i < 256; i++) z16[t][i] = (z16[t - 1][i] >> 8) ^ z16[0][z16[t - 1][i] & 0xff];
  // GF(2) multiply mod P (reflected)
  auto mm = [](uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
      if (a & m) {
        p ^= b;
        if ((a & (m - 1)) == 0) break;
      }
      m >>= 1;
      b = (b & 1) ? (b >> 1) ^ 0x82F63B78u : b >> 1;
    }
    return p;
  };
  // X[k] = x^(8 * 2^k) mod P by repeated squaring (x^(2^32) != x for this P,
  // so no exponent wrap-around is assumed)
  static uint32_t shift[kCrcShiftLevels][4][256];
  uint32_t X = 1u << 30;  // x^1
  for (int i = 0; i < 3; i++) X = mm(X, X);  // x^8
  for (int k = 0; k < kCrcShiftLevels; k++) {
    for (int b = 0; b < 4; b++)
      for (uint32_t v = 0; v < 256; v++) shift[k][b][v] = mm(X, v << (8 * b));
    X = mm(X, X);
  }
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_crc_z16), z16, sizeof z16);
  if (e != hipSuccess) return e;
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_crc_shift), shift, sizeof shift);
  if (e == hipSuccess && dev < 64) g_tabs_ready |= 1ull << dev;
  return e;
}

void launch_eval(const EvalArgs& a, uint32_t ops, int mode, hipStream_t s) {
  if (!a.nbatches) return;
  const size_t dyn = (ops & opbit(OP_REGEX)) ? kDfaDyn : 0;
  EvalArgs e = a;
  uint32_t grid = a.nbatches;
  if (mode == EVAL_ARRAY) {
    // k_arr_frame + the lean array kernel (fsg_array.hip); the exact kernel
    // takes the deferred batches' record starts from k_arr_frame where it framed them
    launch_array_lean(a, s);
    grid = a.nbatches < 2048u ? a.nbatches : 2048u;  // persistent over the deferred list
  } else if (mode == EVAL_INT) {
    // k_eval_int over every batch (starts from k_chase_w, kept with the slice), then the deferred list
    launch_eval_int(a, (ops & opbit(OP_AGG_SUM)) != 0, s);
    grid = a.nbatches < 2048u ? a.nbatches : 2048u;
  } else if (mode == EVAL_LEAN || mode == EVAL_FLAT || mode == EVAL_FJSON || mode == EVAL_RX) {
    // k_chase + k_eval_lean, or the flat substring / JSON / regex kernels (fsg_lean.hip)
    if (mode == EVAL_FLAT)
      launch_eval_flat(a, a.flat_st, s);
    else if (mode == EVAL_FJSON)
      launch_eval_fjson(a, s);
    else if (mode == EVAL_RX)
      launch_eval_rx(a, a.flat_st, s);
    else
      launch_eval_lean(a, ops, s);
    grid = a.nbatches < 2048u ? a.nbatches : 2048u;  // persistent over the deferred list
  } else {
    e.list = nullptr;
    // record starts for the exact kernel (no serial chase per window): k_chase_w
    // where batches hold few records (~2000 tiny records per batch over a few
    // hundred batches is left to the lane-0 chase through LDS; a handful of
    // batches is not worth the launch)
    if (e.rstart && a.nbatches >= 64 && a.nrec <= 256ull * a.nbatches)
      launch_chase_w(e, s);
    else
      e.rstart = nullptr, e.rend = nullptr;
  }
  if ((ops & ~kOpsContains) == 0)
    hipLaunchKernelGGL(k_eval<kOpsContains>, dim3(grid), dim3(kEvalThreads), dyn, s, e);
  else if ((ops & ~kOpsRegex) == 0)
    hipLaunchKernelGGL(k_eval<kOpsRegex>, dim3(grid), dim3(kEvalThreads), dyn, s, e);
  else if ((ops & ~kOpsJson) == 0)
    hipLaunchKernelGGL(k_eval<kOpsJson>, dim3(grid), dim3(kEvalThreads), dyn, s, e);
  else if ((ops & ~kOpsArray) == 0)
    hipLaunchKernelGGL(k_eval<kOpsArray>, dim3(grid), dim3(kEvalThreads), dyn, s, e);
  else if ((ops & ~kOpsInt) == 0)
    hipLaunchKernelGGL(k_eval<kOpsInt>, dim3(grid), dim3(kEvalThreads), dyn, s, e);
  else
    hipLaunchKernelGGL(k_eval<kOpsAll>, dim3(grid), dim3(kEvalThreads), dyn, s, e);
}
// ---------------------------------------------------------------------------
// the aggregate-sum group path (fsg_launch.h GaJob): one launch per phase
// over every chain of a group call; the per-batch phases find their job by
// a binary search of the grid offsets, the per-chain ones take a block each
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ga_job(const uint32_t* off, uint32_t n, uint32_t bid) {
  uint32_t lo = 0, hi = n - 1;  // the last job with off[j] <= bid
  while (lo < hi) {
    const uint32_t m = (lo + hi + 1) >> 1;
    if (off[m] <= bid) lo = m; else hi = m - 1;
  }
  return lo;
}
__global__ void k_ga_init(const GaJob* J, uint32_t n) {  // mins = none, no deferred batch, CRC partials 0
  const uint32_t j = blockIdx.x * 64 + threadIdx.x;
  if (j >= n) return;
  uint32_t* m = (uint32_t*)J[j].ea.mins;
  for (int k = 0; k < (int)(sizeof(Mins) / 4); k++) m[k] = 0xFFFFFFFFu;
  J[j].ea.list[0] = 0;
  *J[j].crc_acc = 0;
}
// deferred batches are not evaluated on this path: an unsupported stand-in
// keeps the later phases inside the batch's bounds; the host re-runs the chain
__global__ void k_ga_defer_mark(const GaJob* J, uint32_t n) {
  const GaJob& g = J[blockIdx.x];
  const uint32_t nd = g.ea.list[0];
  for (uint32_t i = threadIdx.x; i < nd; i += 64) {
    BatchStat st = {};
    st.flags = BF_UNSUPPORTED;
    st.err_stage = 0xFFFFFFFFu;
    g.ea.bstat[g.ea.list[1 + i]] = st;
  }
}
__global__ __launch_bounds__(256) void k_ga_mins(const GaJob* J, const uint32_t* off, uint32_t n) {
  const uint32_t j = ga_job(off, n, blockIdx.x);
  mins_body(J[j].ea.bstat, J[j].ea.nbatches, J[j].ea.mins, blockIdx.x - off[j], off[j + 1] - off[j]);
}
__global__ __launch_bounds__(256) void k_ga_size(const GaJob* J, const uint32_t* off, uint32_t n, uint32_t agg_only) {
  const uint32_t j = ga_job(off, n, blockIdx.x);
  SizeArgs a = J[j].sa;
  a.agg_only = agg_only;
  a.agg_pre = agg_only ? nullptr : J[j].aggpre;
  const uint32_t b = (blockIdx.x - off[j]) * 4 + (threadIdx.x >> 6);
  if (b < a.nbatches) size_batch(a, b);
}
__global__ __launch_bounds__(256) void k_ga_scan(const GaJob* J, uint32_t cut) {  // one tile per chain
  const GaJob& g = J[blockIdx.x];
  ScanDownArgs d{g.sa.rows, cut ? g.pre : g.aggpre, nullptr, g.sa.nbatches, cut, cut ? g.max_bytes : 0,
                 g.ea.mins, g.ea.bstat};
  scan_down_body(d, 0);
}
__global__ void k_ga_plan(const GaJob* J, GaResult* res) {  // the plan, the accumulator, the read-back row
  if (threadIdx.x != 0) return;
  const GaJob& g = J[blockIdx.x];
  plan_run(g.pa);
  const Plan p = *g.pa.plan;
  const uint32_t nd = g.ea.list[0];
  if (!nd && p.acc_touched) *g.state = (int32_t)p.acc_final;  // (k_state; a re-run chain commits there)
  res[blockIdx.x].plan = p;
  res[blockIdx.x].deferred = nd;
}
__global__ void k_ga_header(const GaJob* J) {
  if (threadIdx.x == 0 && J[blockIdx.x].out_len) header_run(J[blockIdx.x].wa.plan, J[blockIdx.x].wa.out);
}
__global__ __launch_bounds__(256) void k_ga_write(const GaJob* J, const uint32_t* off, uint32_t n) {
  const uint32_t j = ga_job(off, n, blockIdx.x);
  write_gen_body(J[j].wa, blockIdx.x - off[j]);
}
__global__ __launch_bounds__(kCrcThreads) void k_ga_crc(const GaJob* J, const uint32_t* off, uint32_t n) {
  const uint32_t j = ga_job(off, n, blockIdx.x);
  const uint64_t end = J[j].out_len, zend = end & ~15ull, nblocks = zend > 16 ? (zend - 16) / 16 : 0;
  crc16_body(J[j].wa.out, 21 - 16, nblocks, J[j].crc_acc, blockIdx.x - off[j], off[j + 1] - off[j]);
}
__global__ void k_ga_crc_final(const GaJob* J) {
  const GaJob& g = J[blockIdx.x];
  if (threadIdx.x != 0 || !g.out_len) return;
  const uint64_t end = g.out_len, zend = end & ~15ull, nblocks = zend > 16 ? (zend - 16) / 16 : 0;
  // (k_crc_final's body: tail bytes, init / xorout, the big-endian CRC at out[17..21))
  uint8_t* out = g.wa.out;
  const uint64_t n = end - 21;
  uint32_t c = *g.crc_acc;
  for (uint64_t i = nblocks ? zend : 21; i < end; i++) c = g_crc_z16[0][(c ^ out[i]) & 0xff] ^ (c >> 8);
  const uint32_t crc = c ^ crc_shift_bytes(0xFFFFFFFFu, n) ^ 0xFFFFFFFFu;
  out[17] = (uint8_t)(crc >> 24);
  out[18] = (uint8_t)(crc >> 16);
  out[19] = (uint8_t)(crc >> 8);
  out[20] = (uint8_t)crc;
}
uint32_t ga_mins_blocks(uint32_t nb) { return std::min<uint32_t>((nb + 255) / 256, 1024u); }
uint32_t ga_crc_blocks(uint64_t out_len) {
  const uint64_t zend = out_len & ~15ull, nblocks = zend > 16 ? (zend - 16) / 16 : 0;
  const uint64_t nchunks = (nblocks + kCrcChunkBlocks - 1) / kCrcChunkBlocks;
  return (uint32_t)std::min<uint64_t>(nchunks, 768);
}
void launch_ga_phase1(const GaJob* J, uint32_t n, const GaOffsets& o, GaResult* res, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_ga_init, dim3((n + 63) / 64), dim3(64), 0, s, J, n);
  launch_ga_eval_int(J, n, o.eval, o.t_eval, s);
  hipLaunchKernelGGL(k_ga_defer_mark, dim3(n), dim3(64), 0, s, J, n);
  if (o.t_mins) hipLaunchKernelGGL(k_ga_mins, dim3(o.t_mins), dim3(256), 0, s, J, o.mins, n);
  if (o.t_size) hipLaunchKernelGGL(k_ga_size, dim3(o.t_size), dim3(256), 0, s, J, o.size, n, 1u);
  hipLaunchKernelGGL(k_ga_scan, dim3(n), dim3(kScanBlock), 0, s, J, 0u);
  if (o.t_size) hipLaunchKernelGGL(k_ga_size, dim3(o.t_size), dim3(256), 0, s, J, o.size, n, 0u);
  hipLaunchKernelGGL(k_ga_scan, dim3(n), dim3(kScanBlock), 0, s, J, 1u);
  hipLaunchKernelGGL(k_ga_plan, dim3(n), dim3(64), 0, s, J, res);
}
void launch_ga_phase2(const GaJob* J, uint32_t n, const GaOffsets& o, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_ga_header, dim3(n), dim3(64), 0, s, J);
  if (o.t_write) hipLaunchKernelGGL(k_ga_write, dim3(o.t_write), dim3(256), 0, s, J, o.write, n);
  if (o.t_crc) hipLaunchKernelGGL(k_ga_crc, dim3(o.t_crc), dim3(kCrcThreads), 0, s, J, o.crc, n);
  hipLaunchKernelGGL(k_ga_crc_final, dim3(n), dim3(64), 0, s, J);
}

void launch_mins(const BatchStat* bstat, uint32_t n, Mins* mins, hipStream_t s) {
  if (!n) return;
  uint32_t g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(k_mins, dim3(g), dim3(256), 0, s, bstat, n, mins);
}
void launch_size(const SizeArgs& a, hipStream_t s) {
  if (a.nbatches) hipLaunchKernelGGL(k_size, dim3((a.nbatches + 3) / 4), dim3(256), 0, s, a);
}
uint32_t scan_tiles(uint32_t n) { return (n + kScanTile - 1) / kScanTile; }
void launch_scan(const ScanRow* rows, ScanRow* pre, ScanRow* tile_sums, ScanRow* grand, uint32_t n, bool cut,
                 uint64_t max_bytes, Mins* mins, const BatchStat* bstat, hipStream_t s) {
  if (!n) return;
  const uint32_t nt = scan_tiles(n);
  ScanDownArgs d{rows, pre, nullptr, n, cut ? 1u : 0u, max_bytes, mins, bstat};
  if (nt == 1) {  // up to kScanTile batches: one workgroup scans in place (one launch, not three)
    hipLaunchKernelGGL(k_scan_down, dim3(1), dim3(kScanBlock), 0, s, d);
    return;
  }
  hipLaunchKernelGGL(k_scan_reduce, dim3(nt), dim3(kScanBlock), 0, s, rows, n, tile_sums);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanBlock), 0, s, tile_sums, nt, grand);
  d.tile_sums = tile_sums;
  hipLaunchKernelGGL(k_scan_down, dim3(nt), dim3(kScanBlock), 0, s, d);
}
void launch_plan(const PlanArgs& a, hipStream_t s) { hipLaunchKernelGGL(k_plan, dim3(1), dim3(64), 0, s, a); }
void launch_state(const Plan* plan, int32_t* state, hipStream_t s) {
  hipLaunchKernelGGL(k_state, dim3(1), dim3(64), 0, s, plan, state);
}
void launch_header(const Plan* plan, uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_header, dim3(1), dim3(64), 0, s, plan, out);
}
void launch_cat(const WriteArgs& a, uint32_t nbatches, hipStream_t s) {
  if (nbatches) hipLaunchKernelGGL(k_cat, dim3((nbatches + 3) / 4), dim3(256), 0, s, a, nbatches);
}
static uint32_t grid_for(uint64_t n, uint32_t per = 256, uint32_t cap = 8192) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, cap));
}
void launch_xscan(const uint32_t* in, uint64_t* out, uint64_t* tsum, uint64_t n, unsigned long long* tot,
                  hipStream_t s) {
  const uint64_t nt = (n + kXsTile - 1) / kXsTile;
  if (nt) hipLaunchKernelGGL(k_xscan_tiles, dim3((uint32_t)nt), dim3(kXsThreads), 0, s, in, out, tsum, n);
  hipLaunchKernelGGL(k_xscan_top, dim3(1), dim3(1024), 0, s, tsum, (uint32_t)nt, tot);
  if (nt > 1) hipLaunchKernelGGL(k_xscan_add, dim3(grid_for(n)), dim3(256), 0, s, out, tsum, n);
}
uint64_t xscan_tiles(uint64_t n) { return (n + kXsTile - 1) / kXsTile + 1; }
// phase 0: records / entries per batch (scal[0], scal[1])
void launch_aggj_count(const AggjArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_aggj_bcount, dim3(grid_for(a.nbatches, 256, 1024)), dim3(256), 0, s, a);
}
// phase 1 (after the host sized the record / entry tables): record table, key
// index, ids; scal[2] = new keys
void launch_aggj_keys(const AggjArgs& a, uint64_t* tsum, hipStream_t s) {
  launch_xscan(a.bcnt, a.brec, tsum, a.nbatches, a.scal + 4, s);
  if (a.nbatches) hipLaunchKernelGGL(k_aggj_flat, dim3((a.nbatches + 3) / 4), dim3(256), 0, s, a);
  launch_xscan(a.rne, a.rent, tsum, a.n_rec, a.scal + 5, s);
  if (a.n_init) hipLaunchKernelGGL(k_aggj_init, dim3(grid_for(a.n_init)), dim3(256), 0, s, a);
  if (a.n_rec) {
    hipLaunchKernelGGL(k_aggj_insert, dim3(grid_for(a.n_rec)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_aggj_new, dim3(grid_for(a.n_rec)), dim3(256), 0, s, a);
  }
  launch_xscan(a.rnew, a.rnewb, tsum, a.n_rec, a.scal + 2, s);
  if (a.n_rec) {
    hipLaunchKernelGGL(k_aggj_ids, dim3(grid_for(a.n_rec)), dim3(256), 0, s, a);
  }
}
void launch_aggj_kid(const AggjArgs& a, uint64_t n_ent, hipStream_t s) {
  if (n_ent) hipLaunchKernelGGL(k_aggj_kid, dim3(grid_for(n_ent)), dim3(256), 0, s, a, n_ent);
}
// phase 2 (K known, state table zeroed): the block rows
void launch_aggj_rows(const AggjArgs& a, hipStream_t s) {
  if (!a.n_rec) return;
  hipLaunchKernelGGL(k_aggj_bsum, dim3(grid_for(a.n_rec)), dim3(256), 0, s, a);
  if (a.nkeys) hipLaunchKernelGGL(k_aggj_colscan, dim3(a.nkeys), dim3(256), 0, s, a);
}
// phase 3: pass 0 sizes, offsets, placement; scal[3] = text bytes.  With
// K > kAjLds the pass replays on the rows in place: `a.state` is then a copy
void launch_aggj_size(const AggjArgs& a, uint64_t* tsum, hipStream_t s) {
  if (a.n_rec) {
    if (a.nkeys <= kAjLds)
      hipLaunchKernelGGL(k_aggj_text<true>, dim3(a.nblk), dim3(64), 0, s, a);
    else
      hipLaunchKernelGGL(k_aggj_text<false>, dim3(a.nblk), dim3(64), 0, s, a);
  }
  launch_xscan(a.rlen, a.roff, tsum, a.n_rec, a.scal + 3, s);
  hipLaunchKernelGGL(k_aggj_place, dim3(grid_for(std::max<uint64_t>(a.n_rec, a.nbatches), 256, 1u << 30)), dim3(256),
                     0, s, a);
}
// phase 4: the texts (pass 1), replayed from the block rows
void launch_aggj_write(const AggjArgs& a, hipStream_t s) {
  if (!a.n_rec) return;
  if (a.nkeys <= kAjLds)
    hipLaunchKernelGGL(k_aggj_text<true>, dim3(a.nblk), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(k_aggj_text<false>, dim3(a.nblk), dim3(64), 0, s, a);
}
// device framing, in phases separated by host reads of FrameArgs::scal
void launch_frame_cand(const FrameArgs& a, uint32_t nchunks, uint64_t* tsum, hipStream_t s) {
  hipLaunchKernelGGL(k_frame_cand, dim3(nchunks), dim3(256), 0, s, a);
  launch_xscan(a.ccnt, a.coff, tsum, nchunks, a.scal + 3, s);  // scal[3] = candidates
}
void launch_frame_compact(const FrameArgs& a, uint32_t nchunks, hipStream_t s) {
  hipLaunchKernelGGL(k_frame_compact, dim3(nchunks), dim3(256), 0, s, a, nchunks);
}
void launch_frame_chain(const FrameArgs& a, uint32_t levels, uint64_t* tsum, hipStream_t s) {
  const uint64_t n = a.ncand;
  const uint32_t g = grid_for(n);
  hipLaunchKernelGGL(k_frame_next, dim3(g), dim3(256), 0, s, a);
  for (uint32_t j = 1; j < levels; j++)
    hipLaunchKernelGGL(k_frame_double, dim3(g), dim3(256), 0, s, a.jmp + (j - 1) * n, a.jmp + j * n, n);
  for (uint32_t j = levels; j-- > 0;) hipLaunchKernelGGL(k_frame_mark, dim3(g), dim3(256), 0, s, a.jmp + j * n, a.mark, n);
  hipLaunchKernelGGL(k_frame_counts, dim3(g), dim3(256), 0, s, a);
  launch_xscan(a.mark, a.mpre, tsum, n, a.scal + 4, s);  // batches
  launch_xscan(a.nrec, a.rpre, tsum, n, a.scal + 5, s);  // records
  hipLaunchKernelGGL(k_frame_emit, dim3(g), dim3(256), 0, s, a);
}
void launch_write(const WriteArgs& a, uint32_t nblocks, hipStream_t s) {
  // nblocks = included batches, one wave each
  if (nblocks) hipLaunchKernelGGL(k_write, dim3((nblocks + kWriteThreads / 64 - 1) / (kWriteThreads / 64)),
                                  dim3(kWriteThreads), 0, s, a);
}
void launch_write_lean(const WriteArgs& a, uint32_t nblocks, hipStream_t s) {
  // one workgroup per batch: a persistent variant that loads batch i + grid's
  // rows and descriptors while batch i is written measured slower on MI355X
  // (C2 write 1.37 -> 1.99 ms), as did round 4's LDS-DMA prefetching one
  if (nblocks) hipLaunchKernelGGL(k_write_lean, dim3(nblocks), dim3(kWlThreads), 0, s, a);
}
// CRC32C of out[off, off + n) into out[17..21); `acc` is one u32 of scratch
void launch_crc(uint8_t* out, uint64_t off, uint64_t n, uint32_t* acc, hipStream_t s) {
  const uint64_t end = off + n;
  const uint64_t zend = end & ~15ull;  // aligned blocks [16, zend); off >= 16
  const uint64_t nblocks = zend > 16 ? (zend - 16) / 16 : 0;
  (void)hipMemsetAsync(acc, 0, sizeof(uint32_t), s);
  if (nblocks) {
    const uint64_t nchunks = (nblocks + kCrcChunkBlocks - 1) / kCrcChunkBlocks;
    const uint32_t grid = (uint32_t)(nchunks < 768 ? nchunks : 768);  // 3 workgroups per CU (LDS)
    hipLaunchKernelGGL(k_crc16, dim3(grid), dim3(kCrcThreads), 0, s, (const uint8_t*)out, off - 16, nblocks, acc);
  }
  hipLaunchKernelGGL(k_crc_final, dim3(1), dim3(64), 0, s, out, (const uint32_t*)acc, nblocks ? zend : off, end, n);
}

// k_one — process() of a one-batch input in one 256-thread workgroup: the
// exact evaluation (eval_batch), then the cross-batch passes collapsed to one
// batch (minima, size row, plan, header, k_write's wave, CRC32C by one wave),
// each phase behind a workgroup-scope fence and a barrier (every byte one phase
// reads was written by this workgroup: no device-scope L2 write-back).  One launch instead of ~12, and
// no host wait between the plan and the write (the output is bounded by
// out_cap: a larger one is left unwritten for the host to redo).
__device__ void crc_wave(uint8_t* out, uint64_t end) {  // CRC32C of out[21, end) into out[17..21)
  const uint32_t l = lane_id();
  const uint64_t zend = end & ~15ull;
  const uint64_t nb = zend > 16 ? (zend - 16) / 16 : 0;  // 16-byte units from out + 16
  uint32_t c = 0;
  int64_t lastu = -1;
  for (uint64_t u = l; u < nb; u += 64) {
    const uint4 v = ((const uint4*)(out + 16))[u];
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (u == 0) w[0] = 0, w[1] &= ~0xffu;  // out[16, 21) precede the CRC region
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) r ^= g_crc_z16[15 - q][(w[q >> 2] >> (8 * (q & 3))) & 0xff];
    c = crc_shift_tab(g_crc_shift[10], c) ^ r;  // the lane's earlier units: 1 KiB back
    lastu = (int64_t)u;
  }
  if (lastu >= 0) c = crc_shift_bytes(c, (nb - 1 - (uint64_t)lastu) * 16);
  c = wave_xor(c);
  if (l == 0) {
    for (uint64_t i = nb ? zend : 21; i < end; i++) c = g_crc_z16[0][(c ^ out[i]) & 0xff] ^ (c >> 8);
    const uint32_t crc = c ^ crc_shift_bytes(0xFFFFFFFFu, end - 21) ^ 0xFFFFFFFFu;
    out[17] = (uint8_t)(crc >> 24);
    out[18] = (uint8_t)(crc >> 16);
    out[19] = (uint8_t)(crc >> 8);
    out[20] = (uint8_t)crc;
  }
}
#ifdef FSG_ONE_TIMING  // experiment builds: phase timestamps into the read-back head (bytes 416..511)
#define ONE_MARK(k) if (threadIdx.x == 0 && (k) < 12) ((uint64_t*)((uint8_t*)o.plan + 416))[k] = __builtin_amdgcn_s_memrealtime()
#else
#define ONE_MARK(k)
#endif
constexpr uint32_t kOneSerialCrc = 1024;  // outputs up to this size: the CRC by one thread from LDS
static_assert(kOneSerialCrc + 4 <= kWin + 64, "k_one's CRC copy reuses the window");
template <uint32_t kOps>
__global__ __launch_bounds__(kEvalThreads) void k_one(OneArgs o) {
  __shared__ WaveLds L;
  __shared__ uint32_t zt[1024];  // g_crc_z16[0..3] for the small-output CRC, loaded with the input
  __shared__ Plan sh_plan;
  const uint32_t t = threadIdx.x;
  const EvalArgs& a = o.ea;
  ONE_MARK(0);
  for (uint32_t i = t; i < 1024; i += kEvalThreads) zt[i] = (&g_crc_z16[0][0])[i];
  {  // the input batch from pinned host memory (over PCIe) into the device slice,
     // zeros behind it (the slice's over-read padding)
    const uint4* src = (const uint4*)o.hin;
    uint4* dst = (uint4*)a.slice;
    for (uint32_t u = t; u < o.in_len / 16; u += kEvalThreads)
      dst[u] = u < o.in_real / 16 ? src[u] : make_uint4(0, 0, 0, 0);
  }
  __threadfence_block();
  __syncthreads();
  ONE_MARK(1);
  eval_batch<kOps>(a, L, 0);
  __threadfence_block();
  __syncthreads();
  ONE_MARK(2);
  if (t == 0) {  // k_mins over the one batch
    const BatchStat st = a.bstat[0];
    Mins m = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, -1};
    if (st.flags & BF_DECODE) m.first_dec = 0;
    if (st.flags & BF_UNSUPPORTED) m.first_unsup = 0;
    if (!(st.flags & BF_DECODE)) {
      if (st.nout) m.first_keep = 0;
      if (st.flags & BF_ERR) m.first_err = 0;
    }
    *a.mins = m;
    o.pre[0] = ScanRow{};
  }
  __threadfence_block();
  __syncthreads();
  ONE_MARK(3);
  SizeArgs sa{};
  sa.bstat = a.bstat;
  sa.desc = a.desc;
  sa.rbase = a.rbase;
  sa.mins = a.mins;
  sa.rows = o.rows;
  sa.nbatches = 1;
  if (t < 64) size_batch(sa, 0);
  __threadfence_block();
  __syncthreads();
  ONE_MARK(4);
  if (t == 0) {  // one batch: the exclusive prefix is zero, no max_bytes cut
    PlanArgs pa{};
    pa.bstat = a.bstat;
    pa.rows = o.rows;
    pa.pre = o.pre;
    pa.mins = a.mins;
    pa.plan = o.plan;
    pa.nbatches = 1;
    pa.empty_chain = o.empty_chain;
    plan_run(pa);
    sh_plan = *o.plan;  // this thread's own store: the workgroup reads the plan from LDS
  }
  __threadfence_block();
  __syncthreads();
  ONE_MARK(5);
  const Plan p = sh_plan;
  const uint64_t end = 61 + p.rec_bytes;
  const bool written = p.status == 0 && end <= o.out_cap;
  if (written) {
    if (t == 0) header_run(&sh_plan, o.out);
  if (t < 64 && p.first == 0 && p.last == 0) {
    WriteArgs wa{};
    wa.slice = a.slice;
    wa.bstat = a.bstat;
    wa.desc = a.desc;
    wa.rbase = a.rbase;
    wa.pre = o.pre;
    wa.plan = o.plan;
    wa.out = o.out;
    wa.base = p.base_offset;
    write_batch(wa, p, 0);
  }
  __threadfence_block();
  __syncthreads();
  ONE_MARK(6);
  if (end <= kOneSerialCrc) {  // a small output: slice-by-4 from LDS by one thread
    uint8_t* ob = L.win;  // the output bytes (eval is done with the window)
    for (uint32_t i = t; i < (uint32_t)(end + 3) / 4; i += kEvalThreads) ((uint32_t*)ob)[i] = ((const uint32_t*)o.out)[i];
    __syncthreads();
    if (t == 0) {
      uint32_t c = 0xFFFFFFFFu;
      uint32_t i = 21;
      for (; i < end && (i & 3u); i++) c = zt[(c ^ ob[i]) & 0xffu] ^ (c >> 8);
      for (; i + 4 <= end; i += 4) {
        const uint32_t x = c ^ *(const uint32_t*)(ob + i);
        c = zt[768 + (x & 0xffu)] ^ zt[512 + ((x >> 8) & 0xffu)] ^ zt[256 + ((x >> 16) & 0xffu)] ^ zt[x >> 24];
      }
      for (; i < end; i++) c = zt[(c ^ ob[i]) & 0xffu] ^ (c >> 8);
      c ^= 0xFFFFFFFFu;
      o.out[17] = (uint8_t)(c >> 24);
      o.out[18] = (uint8_t)(c >> 16);
      o.out[19] = (uint8_t)(c >> 8);
      o.out[20] = (uint8_t)c;
    }
  } else if (t < 64) {
    crc_wave(o.out, end);
  }
  }
  __threadfence_block();
  __syncthreads();
  ONE_MARK(7);
  // the read-back block to pinned host memory (the host reads it after the wait)
  const uint32_t n = kOneHead + (written ? (uint32_t)end : 0u);
  const uint4* src = (const uint4*)o.plan;
  uint4* dst = (uint4*)o.hout;
  for (uint32_t u = t; u < (n + 15) / 16; u += kEvalThreads) dst[u] = src[u];
  // completion flag: every thread's block stores are made visible system-wide,
  // then one store of the call's sequence number releases them to the host
  __threadfence_system();
  __syncthreads();
  if (t == 0) __hip_atomic_store(o.hflag, o.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
void launch_one(const OneArgs& o, uint32_t ops, hipStream_t s) {
  const size_t dyn = (ops & opbit(OP_REGEX)) ? kDfaDyn : 0;
  if ((ops & ~kOpsContains) == 0)
    hipLaunchKernelGGL(k_one<kOpsContains>, dim3(1), dim3(kEvalThreads), dyn, s, o);
  else if ((ops & ~kOpsRegex) == 0)
    hipLaunchKernelGGL(k_one<kOpsRegex>, dim3(1), dim3(kEvalThreads), dyn, s, o);
  else if ((ops & ~kOpsJson) == 0)
    hipLaunchKernelGGL(k_one<kOpsJson>, dim3(1), dim3(kEvalThreads), dyn, s, o);
  else if ((ops & ~kOpsInt) == 0)
    hipLaunchKernelGGL(k_one<kOpsInt>, dim3(1), dim3(kEvalThreads), dyn, s, o);
  else
    hipLaunchKernelGGL(k_one<kOpsAll>, dim3(1), dim3(kEvalThreads), dyn, s, o);
}

// stateful last stage (k_sf_*), between the eval and the size passes
void launch_sf_lb(const SfArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  const uint32_t g = (a.nbatches + 3) / 4;
  hipLaunchKernelGGL(k_sf_prep, dim3(g), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_scan, dim3(1), dim3(1024), 0, s, (const int64_t*)a.bval, a.bpre, a.nbatches, 1u, (int64_t)0,
                     (const int32_t*)a.prev, (unsigned long long*)nullptr);
  if (!a.lookback) hipLaunchKernelGGL(k_sf_compact, dim3(g), dim3(256), 0, s, a);
}
void launch_sf_dedup(const SfArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  const uint32_t g = (a.nbatches + 3) / 4;
  hipLaunchKernelGGL(k_sf_prep, dim3(g), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_clear, dim3(grid_for(a.cap)), dim3(256), 0, s, a);
  if (a.n_ent) hipLaunchKernelGGL(k_sf_rehash, dim3(grid_for(a.n_ent)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_insert, dim3(g), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_decide, dim3(g), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_scan, dim3(1), dim3(1024), 0, s, (const int64_t*)a.bval, a.bpre, a.nbatches, 0u, (int64_t)0,
                     (const int32_t*)nullptr, a.scal + 3);
}
void launch_sf_dedup_seq(const SfArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  hipLaunchKernelGGL(k_sf_cur_init, dim3(grid_for(a.cap)), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_seq, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(k_sf_scan, dim3(1), dim3(1024), 0, s, (const int64_t*)a.bval, a.bpre, a.nbatches, 0u, (int64_t)0,
                     (const int32_t*)nullptr, a.scal + 3);
}
void launch_sf_compact(const SfArgs& a, hipStream_t s) {
  if (a.nbatches) hipLaunchKernelGGL(k_sf_compact, dim3((a.nbatches + 3) / 4), dim3(256), 0, s, a);
}
void launch_sf_commit(const SfArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  if (a.op == OP_LB_MAX) {
    hipLaunchKernelGGL(k_sf_commit_lb, dim3(1), dim3(64), 0, s, a);
    return;
  }
  const uint32_t g = (a.nbatches + 3) / 4;
  hipLaunchKernelGGL(k_sf_commit_new, dim3(g), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_commit_last, dim3(g), dim3(256), 0, s, a);
  hipLaunchKernelGGL(k_sf_commit_n, dim3(1), dim3(64), 0, s, a);
}
void launch_verify_crc(const uint8_t* slice, const uint64_t* bpos, uint32_t nb, unsigned long long* bad,
                       uint32_t* flags, hipStream_t s) {
  if (!nb) return;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // about 64 batches per workgroup (at least 8 workgroups per CU): blocks
  // retire while a concurrent process_batch waits for slots
  const uint32_t g = std::min<uint32_t>((nb + 3) / 4, std::max((uint32_t)std::max(1, cus) * 8u, (nb + 63) / 64));
  hipLaunchKernelGGL(k_verify_crc, dim3(g), dim3(256), 0, s, slice, bpos, nb, bad, flags);
}
void launch_decompress(const DecArgs& a, int pass, hipStream_t s) {
  if (!a.nb) return;
  const uint32_t g = std::min<uint32_t>((a.nb + 255) / 256, 4096);
  if (pass == 0) {
    hipLaunchKernelGGL(k_dec_size, dim3(g), dim3(256), 0, s, a);
  } else if (pass == 1) {
    hipLaunchKernelGGL(k_dec_write, dim3(g), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_dec_copy, dim3((a.nb + 3) / 4), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL(k_dec_count, dim3(g), dim3(256), 0, s, a);
  }
}
}  // namespace fsg
