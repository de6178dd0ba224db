// fsg_flat.hip — register-resident evaluation of substring-filter chains
// (filter_init / filter_with_param with needles of 4..64 bytes, empty needles,
// ASCII-uppercase maps: the C2 headline, smartmodule/examples/filter_init +
// map, derive filter.rs:14-40 / map.rs:17-38), one wave per stored batch.
//
// k_eval_lean stages a batch's window in LDS and walks it with two waves and
// several workgroup barriers per batch; its time goes to the serial per-batch
// path, not to HBM (SQ_WAIT_ANY 58 %, VALU 12 % on MI355X).  Here:
//   k_flat_frame  one thread per batch: the record-start chase of k_chase plus
//                 a 32-byte window descriptor (BatchWin) and the batch header's
//                 fields prefilled into BatchStat, so the evaluation issues one
//                 scalar load per batch for everything it needs to start
//   k_flat        one wave per batch, no barrier and no LDS on the scan path:
//     1. the next batch's descriptor and record starts load during this batch;
//        each record's first / last 16 bytes (lane r = record r) and then the
//        window itself (17 x 1 KiB wave loads, 16 B per lane) go straight into
//        VGPRs;
//     2. lane r decodes record r exactly (Record::decode, data.rs:534-562)
//        from its two 16-byte pieces; value spans stay in lane registers;
//     3. one pass over the 17 chunks per lane: for each stage, the needle's
//        4-grams against the aligned words (needles >= 7 B) or at every byte
//        position (4..6 B); the rare events — a chunk with a byte >= 0x80, a
//        candidate needle start — are taken one at a time from the wave's
//        ballot: every lane tests its record's value span against them (the
//        ASCII rule: then from_utf8 cannot fail in any stage), the candidate's
//        bytes are compared by readlane from the window registers;
//     4. survivors' KeptRec descriptors; nkeep / nout into the prefilled BatchStat.
// A non-ASCII value, odd framing, a long varint or > 64 records defers the
// batch to the exact kernel (k_eval, list mode), as k_eval_lean does.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "fsg_device.h"
#include "fsg_launch.h"

namespace fsg {
namespace {

constexpr uint32_t kFlatWin = 16464;  // window bytes (= k_eval_lean's kLeanWin)
constexpr int kFL = 17;               // 1 KiB wave loads per window
constexpr int kFlatMaxR = 64;         // records per batch
constexpr int kFlatWaves = 4;         // independent waves per workgroup
constexpr uint32_t kFlatNeedle = 64;  // longest needle of this path
constexpr uint32_t kFlatStages = 2;   // contains stages of this path
constexpr int kFrameT = 256;          // k_flat_frame threads per workgroup

__device__ __forceinline__ uint32_t lane() { return threadIdx.x & 63u; }

// global-memory views (generic pointers would load through FLAT, which also
// counts in lgkmcnt: every LDS / scalar wait would then wait for the window too)
template <typename T>
using gp = const __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gp<T> G(const void* p) {
  return (gp<T>)(uintptr_t)p;
}
template <typename T>
using gw = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gw<T> GW(T* p) {
  return (gw<T>)(uintptr_t)p;
}
struct alignas(16) U4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ void st16(gw<U4> d, const U4& v) {  // member-wise: the host pass rejects AS struct copies
  d->x = v.x;
  d->y = v.y;
  d->z = v.z;
  d->w = v.w;
}

// 4 bytes at any address
__device__ __forceinline__ uint32_t ld4(const uint8_t* p) {
  const uint64_t a = (uint64_t)p;
  gp<uint32_t> w = G<uint32_t>((const void*)(a & ~3ull));
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}
__device__ __forceinline__ uint64_t be64(const uint8_t* p) {
  return ((uint64_t)__builtin_bswap32(ld4(p)) << 32) | __builtin_bswap32(ld4(p + 4));
}
// 16 bytes at any address as two little-endian u64
__device__ __forceinline__ void ld16(const uint8_t* p, uint64_t& lo, uint64_t& hi) {
  const uint64_t a = (uint64_t)p;
  gp<uint32_t> w = G<uint32_t>((const void*)(a & ~3ull));
  const uint32_t s = (uint32_t)(a & 3u);
  const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
  lo = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, s) << 32);
  hi = (uint64_t)__builtin_amdgcn_alignbyte(d3, d2, s) | ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, s) << 32);
}
// drop the first n (0..15) bytes of the 16-byte little-endian buffer (lo, hi)
__device__ __forceinline__ void eat(uint64_t& lo, uint64_t& hi, uint32_t n) {
  if (n == 0) return;
  if (n >= 8) {
    lo = hi;
    hi = 0;
    n -= 8;
    if (n == 0) return;
  }
  lo = (lo >> (8 * n)) | (hi << (64 - 8 * n));
  hi >>= 8 * n;
}
// one varint (zigzag i64, varint.rs / decoder) of at most 8 bytes from the low
// bytes of x: bytes used, 0 when no terminator in the first 8
__device__ __forceinline__ uint32_t var8(uint64_t x, int64_t* out) {
  const uint64_t t = ~x & 0x8080808080808080ull;
  if (!t) return 0;
  const uint32_t n = ((uint32_t)__builtin_ctzll(t) >> 3) + 1;
  uint64_t y = n == 8 ? x : (x & ((1ull << (8 * n)) - 1ull));
  y &= 0x7F7F7F7F7F7F7F7Full;
  y = (y & 0x007F007F007F007Full) | ((y & 0x7F007F007F007F00ull) >> 1);
  y = (y & 0x00003FFF00003FFFull) | ((y & 0x3FFF00003FFF0000ull) >> 2);
  y = (y & 0x000000000FFFFFFFull) | ((y & 0x0FFFFFFF00000000ull) >> 4);
  *out = (int64_t)((y >> 1) ^ (0ull - (y & 1ull)));
  return n;
}

__device__ __forceinline__ uint32_t swar_up(uint32_t x) {  // make_ascii_uppercase per byte
  const uint32_t y = x & 0x7F7F7F7Fu;
  const uint32_t lower = (y + 0x1F1F1F1Fu) & ~(y + 0x05050505u) & ~x & 0x80808080u;
  return x - (lower >> 2);
}
// 4 bits: which bytes of a word are >= 0x80
__device__ __forceinline__ uint32_t nib4(uint32_t x) { return ((((x >> 7) & 0x01010101u) * 0x01020408u) >> 24) & 15u; }

// compile-time loop: f(integral_constant<int, K>) for K in [K0, K1) (the
// window lives in v[k]; a runtime index would move it to scratch)
template <int K0, int K1, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (K0 < K1) {
    f(std::integral_constant<int, K0>{});
    sfor<K0 + 1, K1>(f);
  }
}

// a contains stage as the scan needs it (wave-uniform)
struct FlatStage {
  uint32_t m;        // needle length (4..64)
  uint32_t upper;    // the value enters the stage uppercased (VT_SRC_UPPER)
  uint32_t rot[4];   // needle[d .. d + 4) as little-endian words
  const uint8_t* nd; // the needle bytes
};

// word i (0..3) of a uint4
__device__ __forceinline__ uint32_t comp4(const uint4& v, uint32_t i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

}  // namespace

// ---------------------------------------------------------------------------
// k_flat_frame: k_chase's record-start chase (one thread per batch, dependent
// loads of the length varints, starts staged in LDS and stored coalesced) plus
// the batch's window descriptor and its BatchStat prefilled from the header
// (file format, batch.rs:163-180): k_flat then writes only nkeep / nout.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kFrameT) void k_flat_frame(EvalArgs a) {
  __shared__ uint16_t st[kFrameT * kFlatMaxR];
  const uint32_t t = threadIdx.x;
  const uint32_t b0 = blockIdx.x * kFrameT;
  const uint32_t b = b0 + t;
  const uint32_t bl = b0 + kFrameT < a.nbatches ? b0 + kFrameT : a.nbatches;  // first batch past the block
  const uint64_t R0 = a.rbase[b0];
  const uint64_t R1 = bl < a.nbatches ? a.rbase[bl] : a.nrec;
  const bool stage = R1 - R0 <= (uint64_t)(kFrameT * kFlatMaxR);
  if (b < a.nbatches) {
    const uint64_t pos = a.bpos[b];
    const uint64_t nxt = b + 1 < a.nbatches ? a.bpos[b + 1] : a.slice_len;
    const uint64_t rb = a.rbase[b], rn = (b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb;
    const uint64_t al = pos & ~15ull;
    uint64_t wl = nxt > al ? nxt - al : 0;
    if (wl > (uint64_t)kFlatWin) wl = kFlatWin;
    const uint32_t wlen = (uint32_t)((wl + 15) & ~15ull);
    const uint8_t* base = a.slice + al;
    const uint32_t batch_len = __builtin_bswap32(ld4(a.slice + pos + 8));
    const uint64_t sec0 = pos + 57, sec_end = pos + 12 + (uint64_t)batch_len;
    const uint64_t sec_len = sec_end - sec0;
    const int32_t count = sec_len >= 4 ? (int32_t)__builtin_bswap32(ld4(a.slice + sec0)) : -1;
    uint32_t end = 0xFFFFu;
    if (sec_len >= 4 && sec_end - al <= wlen && count >= 0 && count <= kFlatMaxR && (uint64_t)count == rn) {
      const uint32_t have = (uint32_t)(sec_end - al);
      uint32_t q = (uint32_t)(sec0 + 4 - al);
      int n = 0;
      for (; n < count; n++) {
        const uint32_t x = ld4(base + q);
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
    // the window descriptor
    BatchWin w;
    w.al = al;
    w.rb = rb;
    w.wlen = wlen;
    w.nr_re = (end == 0xFFFFu ? 0xFFFFu : (uint32_t)count) | (end << 16);
    w.pad[0] = w.pad[1] = 0;
    const U4* wq = (const U4*)&w;
    gw<U4> wd = (gw<U4>)GW(a.bwin + b);
    st16(wd, wq[0]);
    st16(wd + 1, wq[1]);
    // BatchStat of a batch without errors; k_flat adds nkeep / nout (a
    // deferred batch is rewritten whole by the exact kernel)
    BatchStat s = {};
    s.base_offset = (int64_t)be64(a.slice + pos);
    s.lod_in = (int32_t)__builtin_bswap32(ld4(a.slice + pos + 23));
    s.first_ts = (int64_t)be64(a.slice + pos + 27);
    s.comp = (ld4(a.slice + pos + 20) >> 16) & 7u;  // attributes low byte (pos + 22)
    s.flags = BF_LAST_STAGE;
    s.sec_len = batch_len - 45u;  // framing validated batch_len >= 45
    s.err_stage = 0xFFFFFFFFu;
    const U4* sq = (const U4*)&s;
    gw<U4> sd = (gw<U4>)GW(a.bstat + b);
#pragma unroll
    for (int i = 0; i < (int)(sizeof(BatchStat) / 16); i++) st16(sd + i, sq[i]);
  }
  if (!stage) return;  // uniform
  __syncthreads();
  const uint64_t n = R1 - R0;
  uint16_t* dst = a.rstart + R0;
  const uint32_t head = (uint32_t)((8u - ((uintptr_t)dst & 15u) / 2u) & 7u);  // u16 slots to 16-B alignment
  for (uint64_t i = t; i < n && i < head; i += kFrameT) dst[i] = st[i];
  for (uint64_t i = head + 8ull * t; i + 8 <= n; i += 8ull * kFrameT) {
    uint4 v;
    v.x = st[i] | ((uint32_t)st[i + 1] << 16);
    v.y = st[i + 2] | ((uint32_t)st[i + 3] << 16);
    v.z = st[i + 4] | ((uint32_t)st[i + 5] << 16);
    v.w = st[i + 6] | ((uint32_t)st[i + 7] << 16);
    *(uint4*)(dst + i) = v;
  }
  const uint64_t tail0 = n > head ? head + ((n - head) & ~7ull) : n;
  for (uint64_t i = tail0 + t; i < n; i += kFrameT) dst[i] = st[i];
}

// ---------------------------------------------------------------------------
// k_flat: one wave per stored batch, persistent over b = wave + i * waves
// ---------------------------------------------------------------------------
struct FlatRec {  // one parsed record, parked in LDS between the decode and its descriptor
  uint32_t rs, ks, kl, at;  // window offsets / lengths; at = attributes | has_key << 8
  int64_t od, ts, hdr;
};
struct __attribute__((aligned(16))) FlatWave {
  FlatRec rec[kFlatMaxR];
};

#ifndef FSG_FLAT_WPE
#define FSG_FLAT_WPE 3  // waves per SIMD (the window takes 68 of 141 VGPRs)
#endif
__global__ __launch_bounds__(64 * kFlatWaves) __attribute__((amdgpu_waves_per_eu(FSG_FLAT_WPE))) void k_flat(EvalArgs a) {
  __shared__ FlatWave S[kFlatWaves];
  FlatWave& L = S[threadIdx.x >> 6];
  const uint32_t l = lane();
  const uint32_t W = gridDim.x * kFlatWaves;
  const ChainDesc& ch = *a.chain;
  const uint32_t nst = ch.nstages;
  // the contains stages (flat_eligible: at most kFlatStages with needles 4..64 B, or empty)
  FlatStage fs0 = {}, fs1 = {};  // (two named stages: an indexed array would live in scratch)
  uint32_t ncs = 0;
  for (uint32_t s = 0; s < nst; s++) {
    const StageDesc& sd = ch.st[s];
    if (sd.op != OP_CONTAINS) continue;
    if (sd.needle_len == 0) {  // contains(""): every (UTF-8) value; only the ASCII rule
      ncs |= 0x100u;
      continue;
    }
    FlatStage f;
    f.m = sd.needle_len;
    f.upper = sd.in_type == VT_SRC_UPPER ? 1u : 0u;
    f.nd = a.blob + sd.needle;
    for (uint32_t d = 0; d < 4; d++) {
      uint32_t x = 0;
      for (uint32_t t = 0; t < 4; t++)
        if (d + t < f.m) x |= (uint32_t)f.nd[d + t] << (8 * t);
      f.rot[d] = x;
    }
    if ((ncs & 0xFFu) == 0)
      fs0 = f;
    else
      fs1 = f;
    ncs++;
  }
  const bool any_contains = ncs != 0;
  ncs &= 0xFFu;
  const bool mid = (ncs > 0 && fs0.m < 7) || (ncs > 1 && fs1.m < 7);  // a 4..6-byte needle: look-ahead
  const uint32_t kmode = ch.out_type == VT_SRC_UPPER ? (uint32_t)KM_UPPER : (uint32_t)KM_COPY;

  uint32_t b = blockIdx.x * kFlatWaves + (threadIdx.x >> 6);
  if (b >= a.nbatches) return;
  BatchWin M = a.bwin[b];
  uint32_t rsv = G<uint16_t>(a.rstart)[M.rb + l];  // record starts (rstart has 64 slots of slack)
  for (;;) {
    // an opaque zero: keeps the per-chunk positions inside the loop (hoisted
    // out of it they would take a register each for the whole kernel)
    uint32_t zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    const uint32_t lo16 = l * 16u + zero;
    const uint32_t bn = b + W;
    BatchWin N = M;
    if (bn < a.nbatches) N = a.bwin[bn];  // one scalar load, used an iteration later
    const uint32_t wlen = M.wlen;
    const uint32_t nrw = M.nr_re & 0xFFFFu, re = M.nr_re >> 16;
    bool defer = nrw > (uint32_t)kFlatMaxR;  // no exact framing (k_flat_frame)
    const int nr = defer ? 0 : (int)nrw;
    const uint8_t* base = a.slice + M.al;
    // each record's first / last 16 bytes (lane r: record r), before the window
    const uint32_t rs = rsv < wlen ? rsv : 0u;
    const uint32_t r1 = __shfl_down(rs, 1, 64);
    const uint32_t lim = (int)l + 1 == nr ? re : r1;
    uint64_t lo = 0, hi = 0, tlo = 0, thi = 0;
    if ((int)l < nr) {
      ld16(base + rs, lo, hi);
      ld16(base + (lim >= 16 ? lim - 16 : 0), tlo, thi);  // the record's last 16 bytes (headers varint)
    }
    // 1. the window, straight into registers
    uint4 v[kFL];
    sfor<0, kFL>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      const uint32_t o = (uint32_t)k * 1024u + lo16;
      uint4 x = make_uint4(0, 0, 0, 0);
      if (o < wlen) {
        gp<U4> src = G<U4>(base + o);
        x = make_uint4(src->x, src->y, src->z, src->w);
      }
      v[k] = x;
    });
    // the next batch's record starts, in flight behind the window
    uint32_t rsn = 0;
    if (bn < a.nbatches) rsn = G<uint16_t>(a.rstart)[N.rb + l];
    // 2. lane r decodes record r (Record::decode, data.rs:534-562): len,
    //    attributes, timestamp_delta, offset_delta, key tag [+ key], value,
    //    headers; `rem` = valid bytes left in (lo, hi); a varint must end
    //    inside them and the record must end exactly at lim (else: exact path)
    bool bad = false;
    uint32_t vs = 0, ve = 0;
    if ((int)l < nr) {
      uint32_t q = rs;
      int rem = 16;
      auto var = [&](int64_t* out, int after) __attribute__((always_inline)) {
        const uint32_t n = var8(lo, out);
        if (n == 0 || (int)n + after > rem) return false;
        eat(lo, hi, n);
        q += n;
        rem -= (int)n;
        return true;
      };
      auto byte = [&]() __attribute__((always_inline)) {
        const uint32_t x = (uint32_t)(lo & 0xFFu);
        eat(lo, hi, 1);
        q++;
        rem--;
        return x;
      };
      auto refill = [&]() __attribute__((always_inline)) {
        if (rem < 8) {
          ld16(base + q, lo, hi);
          rem = 16;
        }
      };
      int64_t len = 0, kv = 0, vv = 0, ts = 0, od = 0, hdr = 0;
      uint32_t attr = 0, tag = 0, ks = 0, kl = 0;
      bad = !var(&len, 1) || len < 0 || (uint64_t)q + (uint64_t)len != lim;
      if (!bad) {
        attr = byte();
        bad = !var(&ts, 1) || !var(&od, 1);
      }
      if (!bad) {
        tag = byte();
        bad = tag > 1;
      }
      if (!bad && tag == 1) {
        refill();
        bad = !var(&kv, 0) || kv < 0 || (uint64_t)q + (uint64_t)kv > lim;
        ks = q;
        kl = bad ? 0u : (uint32_t)kv;
        q += kl;
        rem = 0;  // the value length follows the key bytes: reload there
      }
      if (!bad) {
        refill();
        bad = !var(&vv, 0) || vv < 0 || (uint64_t)q + (uint64_t)vv >= lim;
      }
      if (!bad) {
        vs = q;
        ve = q + (uint32_t)vv;
        // the headers varint fills [ve, lim) exactly
        const uint32_t hs = lim - ve;
        bad = hs > 8;
        if (!bad) {
          eat(tlo, thi, 16 - hs);
          bad = var8(tlo, &hdr) != hs;
        }
      }
      // parked in LDS for the descriptor (frees the registers for the scan)
      FlatRec& R = L.rec[l];
      R.rs = rs;
      R.ks = ks;
      R.kl = kl;
      R.at = attr | (tag << 8);
      R.od = od;
      R.ts = ts;
      R.hdr = hdr;
    }
    defer = defer || __ballot(bad) != 0;
    if ((int)l >= nr) vs = ve = 0xFFFFFFFFu;  // no value: never matches a position
    uint64_t alive = __ballot((int)l < nr);
    uint64_t hit0 = 0, hit1 = 0;  // records with a verified needle hit (wave-uniform)
    bool nonascii = false;        // per record lane: a byte >= 0x80 inside its value
    if (!defer && nr > 0 && any_contains) {
      // 3. one pass over the chunks
      sfor<0, kFL>([&](auto kc) __attribute__((always_inline)) {
        constexpr int k = decltype(kc)::value;
        constexpr int kn = k + 1 < kFL ? k + 1 : k;
        constexpr int kp = k > 0 ? k - 1 : k;
        const uint32_t w0[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        // (a) bytes >= 0x80: is any inside a value?  (rare: record headers' varints)
        const uint32_t hm = nib4(w0[0]) | (nib4(w0[1]) << 4) | (nib4(w0[2]) << 8) | (nib4(w0[3]) << 12);
        for (uint64_t fl = __ballot(hm != 0); fl; fl &= fl - 1) {
          const uint32_t src = (uint32_t)__builtin_ctzll(fl);
          const uint32_t hmu = __builtin_amdgcn_readlane(hm, src);
          const uint32_t cu = (uint32_t)k * 1024u + src * 16u;
          const uint32_t s0 = vs > cu ? vs : cu, e0 = ve < cu + 16 ? ve : cu + 16;
          if (s0 < e0) nonascii |= (((0xFFFFu >> (16 - (e0 - s0))) << (s0 - cu)) & hmu) != 0;
        }
        // (b) candidate needle starts, per stage
        uint32_t w4 = 0;  // the 4 bytes after the chunk (4..6-byte needles)
        if (mid) {
          w4 = __shfl_down(w0[0], 1, 64);
          const uint32_t f4 = __shfl(v[kn].x, 0, 64);
          if (l == 63) w4 = k + 1 < kFL ? f4 : 0u;
        }
        auto stage = [&](const FlatStage& st, uint64_t& hit) __attribute__((always_inline)) {
          uint32_t w[5] = {w0[0], w0[1], w0[2], w0[3], w4};
          if (st.upper) {
#pragma unroll
            for (int i = 0; i < 5; i++) w[i] = swar_up(w[i]);
          }
          uint32_t bits = 0;  // bit j: a candidate start at o - 3 + j
          if (st.m >= 7) {
            // every occurrence covers an aligned word: each word against the four 4-grams
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
              for (int d = 0; d < 4; d++) bits |= (w[i] == st.rot[d] ? 1u : 0u) << (3 + 4 * i - d);
          } else {
#pragma unroll
            for (int j = 0; j < 16; j++) {
              const uint32_t g =
                  (j & 3) ? __builtin_amdgcn_alignbyte(w[(j >> 2) + 1], w[j >> 2], (uint32_t)(j & 3)) : w[j >> 2];
              bits |= (g == st.rot[0] ? 1u : 0u) << (3 + j);
            }
          }
          for (uint64_t cl = __ballot(bits != 0); cl; cl &= cl - 1) {
            const uint32_t src = (uint32_t)__builtin_ctzll(cl);
            uint32_t bu = __builtin_amdgcn_readlane(bits, src);
            const uint32_t cu = (uint32_t)k * 1024u + src * 16u;
            while (bu) {
              const uint32_t j = (uint32_t)__builtin_ctz(bu);
              bu &= bu - 1u;
              if (cu + j < 3u) continue;  // before the window
              const uint32_t p = cu + j - 3u;
              // the record whose value holds [p, p + m) (spans in lane registers)
              const uint64_t in = __ballot(vs <= p && p + st.m <= ve);
              if (!in) continue;
              const uint32_t r = (uint32_t)__builtin_ctzll(in);
              if ((hit >> r) & 1ull) continue;  // already kept by this stage
              // the needle against the window registers (readlane; [p, p + m)
              // lies in loads k - 1 .. k + 1)
              bool eq = true;
              for (uint32_t t = 0; eq && t < st.m; t += 4) {
                const uint32_t q = p + t;
                const uint32_t qa = q & ~3u, sh = q & 3u;
                uint32_t x[2];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                  const uint32_t qq = qa + 4u * h;
                  const uint32_t ln = (qq >> 4) & 63u, wi = (qq >> 2) & 3u;
                  // a start in the last 3 bytes of load k - 1 is found by lane 0 of load k
                  const uint32_t ap = __builtin_amdgcn_readlane(comp4(v[kp], wi), ln);
                  const uint32_t a0 = __builtin_amdgcn_readlane(comp4(v[k], wi), ln);
                  const uint32_t a1 = __builtin_amdgcn_readlane(comp4(v[kn], wi), ln);
                  const uint32_t kq = qq >> 10;
                  x[h] = kq == (uint32_t)k ? a0
                         : (kq == (uint32_t)k + 1 && k + 1 < kFL) ? a1
                         : (kq + 1 == (uint32_t)k && k > 0)        ? ap
                                                                   : 0u;
                }
                uint32_t y = __builtin_amdgcn_alignbyte(x[1], x[0], sh);
                if (st.upper) y = swar_up(y);
                uint32_t nw = 0;
                for (uint32_t i = 0; i < 4 && t + i < st.m; i++) nw |= (uint32_t)st.nd[t + i] << (8 * i);
                const uint32_t km = st.m - t >= 4 ? 0xFFFFFFFFu : ((1u << (8 * (st.m - t))) - 1u);
                eq = ((y ^ nw) & km) == 0u;
              }
              if (eq) hit |= 1ull << r;
            }
          }
        };
        if (ncs > 0) stage(fs0, hit0);
        if (ncs > 1) stage(fs1, hit1);
      });
      defer = __ballot(nonascii) != 0;  // a non-ASCII value: exact UTF-8 path
      if (ncs > 0) alive &= hit0;
      if (ncs > 1) alive &= hit1;
    }
    // 4. survivors -> compaction descriptors, the batch's result
    if (defer) {
      if (l == 0) {
        const uint32_t i = atomicAdd(a.list, 1u);
        GW(a.list)[1 + i] = b;
      }
    } else {
      if ((int)l < nr && ((alive >> l) & 1ull)) {
        const FlatRec& R = L.rec[l];
        KeptRec d;
        d.src = M.al + R.rs;
        d.vpos = M.al + vs;
        d.kpos = (R.at >> 8) ? M.al + R.ks : 0;
        d.od = R.od;
        d.ts = R.ts;
        d.hdr = R.hdr;
        d.vlen = ve - vs;
        d.klen = R.kl;
        d.ival = 0;
        d.mode = (uint8_t)kmode;
        d.has_key = (uint8_t)(R.at >> 8);
        d.attr = (uint8_t)R.at;
        d.pad = 0;
        gw<U4> dst = (gw<U4>)GW(a.desc + M.rb + __popcll(alive & ((1ull << l) - 1ull)));
        const U4* q = (const U4*)&d;
#pragma unroll
        for (int i = 0; i < 4; i++) st16(dst + i, q[i]);
      }
      if (l == 0) {  // the rest of the BatchStat was prefilled by k_flat_frame
        const uint32_t nk = (uint32_t)__popcll(alive);
        GW(&a.bstat[b].nkeep)[0] = nk;
        GW(&a.bstat[b].nout)[0] = nk;
      }
    }
    if (bn >= a.nbatches) break;
    b = bn;
    M = N;
    rsv = rsn;
  }
}

// resident workgroups on the current device (CUs x occupancy)
static uint32_t flat_grid() {
  static uint32_t cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cache[dev]) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_flat, 64 * kFlatWaves, 0);
    cache[dev] = (uint32_t)(cus > 0 ? cus : 1) * (uint32_t)(per > 0 ? per : 1);
  }
  return cache[dev];
}

// contains filters (needles of 4..64 bytes, or empty; at most two) and
// uppercase maps; shorter needles (dense hits) stay on k_eval_lean
bool flat_eligible(const ChainDesc& ch, uint32_t ops) {
  if (ops & ~((1u << OP_CONTAINS) | (1u << OP_MAP_UPPER))) return false;
  uint32_t n = 0;
  for (uint32_t s = 0; s < ch.nstages; s++) {
    if (ch.st[s].op != OP_CONTAINS || ch.st[s].needle_len == 0) continue;
    if (ch.st[s].needle_len < 4 || ch.st[s].needle_len > kFlatNeedle) return false;
    n++;
  }
  return n <= kFlatStages;
}

void launch_flat(const EvalArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  hipLaunchKernelGGL(k_flat_frame, dim3((a.nbatches + kFrameT - 1) / kFrameT), dim3(kFrameT), 0, s, a);
  const uint32_t g = std::min<uint32_t>((a.nbatches + kFlatWaves - 1) / kFlatWaves, flat_grid());
  hipLaunchKernelGGL(k_flat, dim3(g), dim3(64 * kFlatWaves), 0, s, a);
}

}  // namespace fsg
