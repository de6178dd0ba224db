// fsg_array.hip — lean evaluation of array_map_json_array chains (C4:
// smartmodule/examples/array_map_json_array/src/lib.rs:38-55, derive
// generator/array_map.rs:17-42: serde_json::from_slice::<Vec<Value>> of each
// record's value, one output record per element, serde_json::to_string of it).
//
// k_eval's exact path parses every record with the full serde_json restatement
// inside a 256-thread workgroup per batch.  The lean path walks a small grammar
// of the arrays whose output is certain: flat arrays of JSON integers (no
// leading zero, <= 18 digits, not -0), strings without escapes / control /
// non-ASCII bytes, and true / false / null, with whitespace anywhere JSON
// allows it.  Every such element's serde_json::to_string is its source text.
// Anything else in a batch defers the whole batch to the exact kernel (list
// mode), as k_eval_lean does.
//
// Two passes over the source, no per-element descriptors in HBM:
//   k_arr_lean  (before the plan)  one workgroup per batch, the batch window
//               in LDS: the records framed, a thread per record through the
//               grammar DFA, element starts / ends as two bitmaps per batch
//               (2 x 2 KiB), and the counts k_size prices the output with once
//               the offset rebase is known (ArrBatch)
//   k_arr_write (after the plan)   the window and bitmaps again, every element
//               a lane: its output record (Record::new_key_value(None,
//               element)) into an LDS staging buffer, stored to HBM as aligned
//               16-byte units
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fsg_device.h"
#include "fsg_launch.h"

namespace fsg {
namespace {

template <typename T>
using gp = const __attribute__((address_space(1))) T*;
__device__ __forceinline__ uint32_t ld4g(const uint8_t* p) {
  const uint64_t a = (uint64_t)p;
  gp<uint32_t> w = (gp<uint32_t>)(uintptr_t)(a & ~3ull);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}
// 4 bytes at any LDS offset (the window holds 16 bytes of slack)
__device__ __forceinline__ uint32_t lds4(const uint8_t* W, uint32_t o) {
  const uint32_t* w = (const uint32_t*)(W + (o & ~3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], o & 3u);
}
// one zigzag varint of at most 8 bytes at window offset o (bytes used, 0 = none)
__device__ __forceinline__ uint32_t var_lds(const uint8_t* W, uint32_t o, int64_t* out) {
  const uint64_t x = (uint64_t)lds4(W, o) | ((uint64_t)lds4(W, o + 4) << 32);
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

// The lean array grammar as a byte DFA (next state | action << 5).  States:
enum ArrSt : uint32_t {
  A_BAD, A_PRE, A_VAL1, A_VAL, A_MINUS, A_ZERO, A_INT, A_STR, A_T1, A_T2, A_T3, A_F1, A_F2, A_F3, A_F4, A_N1, A_N2,
  A_N3, A_AFTER, A_POST, A_NSTATES
};
// byte classes: 0 other printable ASCII, 1 whitespace, 2 '[', 3 ']', 4 ',', 5 '"',
// 6 '-', 7 '0', 8 '1'-'9', 9 't', 10 'r', 11 'u', 12 'e', 13 'f', 14 'a', 15 'l',
// 16 's', 17 'n', 18 not allowed in a lean string (controls, '\\', >= 0x80)
constexpr __host__ __device__ uint32_t arr_class(uint32_t c) {
  if (c == ' ' || c == '\t' || c == '\n' || c == '\r') return 1;
  if (c < 0x20 || c == '\\' || c >= 0x80) return 18;
  switch (c) {
    case '[': return 2;
    case ']': return 3;
    case ',': return 4;
    case '"': return 5;
    case '-': return 6;
    case '0': return 7;
    case 't': return 9;
    case 'r': return 10;
    case 'u': return 11;
    case 'e': return 12;
    case 'f': return 13;
    case 'a': return 14;
    case 'l': return 15;
    case 's': return 16;
    case 'n': return 17;
    default: return (c >= '1' && c <= '9') ? 8 : 0;
  }
}
// next state | action << 5: 1 = an element starts with this byte, 2 = the
// element ended before this byte, 4 = the element ends with this byte
constexpr __host__ __device__ uint32_t arr_trans(uint32_t st, uint32_t cl) {
  constexpr uint32_t S = 1 << 5, EB = 2 << 5, EA = 4 << 5;
  auto value_start = [&](uint32_t c) -> uint32_t {
    switch (c) {
      case 5: return A_STR | S;
      case 6: return A_MINUS | S;
      case 7: return A_ZERO | S;
      case 8: return A_INT | S;
      case 9: return A_T1 | S;
      case 13: return A_F1 | S;
      case 17: return A_N1 | S;
      default: return A_BAD;
    }
  };
  auto lit = [&](uint32_t want, uint32_t next) -> uint32_t { return cl == want ? next : (uint32_t)A_BAD; };
  auto term = [&]() -> uint32_t {  // after a number: whitespace, ',' or ']'
    return cl == 1 ? (A_AFTER | EB) : cl == 4 ? (A_VAL | EB) : cl == 3 ? (A_POST | EB) : (uint32_t)A_BAD;
  };
  switch (st) {
    case A_PRE: return cl == 1 ? A_PRE : cl == 2 ? A_VAL1 : A_BAD;
    case A_VAL1: return cl == 1 ? A_VAL1 : cl == 3 ? A_POST : value_start(cl);
    case A_VAL: return cl == 1 ? A_VAL : value_start(cl);
    case A_MINUS: return cl == 8 ? A_INT : A_BAD;  // "-0": f64 -0.0 in serde_json (the exact kernel)
    case A_ZERO: return term();                     // a digit after 0: leading zero; '.', 'e': a float
    case A_INT: return (cl == 7 || cl == 8) ? A_INT : term();
    case A_STR: return cl == 5 ? (A_AFTER | EA) : cl == 18 ? A_BAD : A_STR;
    case A_T1: return lit(10, A_T2);
    case A_T2: return lit(11, A_T3);
    case A_T3: return lit(12, A_AFTER | EA);
    case A_F1: return lit(14, A_F2);
    case A_F2: return lit(15, A_F3);
    case A_F3: return lit(16, A_F4);
    case A_F4: return lit(12, A_AFTER | EA);
    case A_N1: return lit(11, A_N2);
    case A_N2: return lit(15, A_N3);
    case A_N3: return lit(15, A_AFTER | EA);
    case A_AFTER: return cl == 1 ? A_AFTER : cl == 4 ? A_VAL : cl == 3 ? A_POST : A_BAD;
    case A_POST: return cl == 1 ? A_POST : A_BAD;  // from_slice: trailing whitespace only
    default: return A_BAD;
  }
}
// The transition table by byte class: row c holds T[state][c] for the 20
// states as bytes (next state | action << 5).  A byte's row does not depend on
// the state, so the walk loads the rows of the next four bytes ahead and the
// per-byte dependency is only the register pick of byte `state` of the row.
constexpr uint32_t kNCls = 19;
struct ArrTab {
  uint32_t cls[64];       // byte -> class, four per word
  uint32_t row[kNCls][8]; // 20 state bytes + padding
};
constexpr ArrTab make_arr_tab() {
  ArrTab t{};
  for (uint32_t c = 0; c < 256; c++) t.cls[c / 4] |= arr_class(c) << (8 * (c % 4));
  for (uint32_t c = 0; c < kNCls; c++)
    for (uint32_t st = 0; st < A_NSTATES; st++) t.row[c][st / 4] |= arr_trans(st, c) << (8 * (st % 4));
  return t;
}
__constant__ ArrTab kArrTab = make_arr_tab();  // built at compile time
__device__ __forceinline__ void load_table(ArrTab* T) {
  const uint32_t* src = (const uint32_t*)&kArrTab;
  for (uint32_t k = threadIdx.x; k < sizeof(ArrTab) / 4; k += blockDim.x) ((uint32_t*)T)[k] = src[k];
}
struct ArrRow {
  uint4 a;
  uint32_t b;
};
__device__ __forceinline__ ArrRow arr_row(const ArrTab* T, uint32_t c) {
  const uint32_t cl = ((const uint8_t*)T->cls)[c];
  return {*(const uint4*)T->row[cl], T->row[cl][4]};
}
// byte `st` of the row: v_perm picks from each 8-byte half (selector bytes
// 0x0C are zero), so the row stays in registers
__device__ __forceinline__ uint32_t arr_pick(const ArrRow& r, uint32_t st) {
  const uint32_t sel = (st & 7u) | 0x0C0C0C00u;
  const uint32_t lo = __builtin_amdgcn_perm(r.a.y, r.a.x, sel), mid = __builtin_amdgcn_perm(r.a.w, r.a.z, sel);
  const uint32_t hi = __builtin_amdgcn_ubfe(r.b, (st & 3u) * 8, 8);
  return st < 8 ? lo : st < 16 ? mid : hi;
}
// the value bytes [v, v + n) of a record through the DFA: f(p, c, x) per byte
// (x = next state | action << 5); returns the final state
template <typename F>
__device__ __forceinline__ uint32_t arr_walk(const uint8_t* W, const ArrTab* T, uint32_t v, uint32_t n, F&& f) {
  uint32_t st = A_PRE;
  const uint32_t end = v + n;
  for (uint32_t i = v & ~3u; i < end; i += 4) {
    const uint32_t w = *(const uint32_t*)(W + i);
    ArrRow r[4];
#pragma unroll
    for (int k = 0; k < 4; k++) r[k] = arr_row(T, (w >> (8 * k)) & 0xFFu);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t p = i + k;
      if (p >= v && p < end) {
        const uint32_t x = arr_pick(r[k], st);
        f(p, (w >> (8 * k)) & 0xFFu, x);
        st = x & 31;
      }
    }
  }
  return st;
}
// varint bytes of small non-negative values (< 8192): 1 or 2
__device__ __forceinline__ uint32_t vs2(uint32_t x) { return x >= 64 ? 2u : 1u; }
// L = vsize(len) + len: an element's varint + text bytes
__device__ __forceinline__ uint32_t elem_L(uint32_t len) { return len + vs2(len); }
// elements past this L are left to the exact kernel (their record's inner
// length would reach 8192, a varint threshold the counts do not track)
constexpr uint32_t kArrMaxL = 8100;

// one record at window offsets [q0, qe): Record::decode (data.rs:534-562) down
// to the value bytes [*v, *v + *n); false = malformed (the exact kernel reports it)
__device__ bool rec_value(const uint8_t* W, uint32_t q0, uint32_t qe, uint32_t* v, uint32_t* n) {
  int64_t len = 0, ts = 0, od = 0, kl = 0, vl = 0, hdr = 0;
  uint32_t q = q0;
  uint32_t u = var_lds(W, q, &len);
  if (!u || len < 0) return false;
  q += u + 1;  // + attributes
  u = var_lds(W, q, &ts);
  if (!u) return false;
  q += u;
  u = var_lds(W, q, &od);
  if (!u) return false;
  q += u;
  const uint32_t tag = W[q++];
  if (tag > 1) return false;
  if (tag) {
    u = var_lds(W, q, &kl);
    if (!u || kl < 0 || (int64_t)q + u + kl > (int64_t)qe) return false;
    q += u + (uint32_t)kl;
  }
  u = var_lds(W, q, &vl);
  if (!u || vl < 0 || (int64_t)q + u + vl >= (int64_t)qe) return false;
  q += u;
  const uint32_t hq = q + (uint32_t)vl;
  u = var_lds(W, hq, &hdr);
  if (!u || hq + u != qe || (int64_t)q0 + vsize(len) + len != (int64_t)qe) return false;
  *v = q;
  *n = (uint32_t)vl;
  return true;
}

// the batch window [al, al + wlen) into LDS by 1 KiB LDS-DMA pieces
__device__ __forceinline__ void stage_window(const uint8_t* S, uint64_t al, uint32_t wlen, uint8_t* W) {
  const uint32_t t = threadIdx.x, l = t & 63u;
  for (uint32_t k = t >> 6; k * 1024 < wlen; k += blockDim.x / 64)
    if (k * 1024 + l * 16 < wlen)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S + al + k * 1024 + l * 16),
                                     (__attribute__((address_space(3))) void*)(W + k * 1024), 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
}

// ---------------------------------------------------------------------------
// k_arr_frame — record framing of the batches for k_arr_lean: one THREAD per
// batch (64-thread workgroups over every CU), so ~17 K independent
// length-varint chains are in flight at once
// (a wave per batch in LDS leaves too few to hide each step's latency).  Each
// step reads the record's varint from global memory and also touches the line
// 256 bytes ahead, so the chain's next steps hit L2 instead of HBM.  Starts to
// rstart, the end to rend; 0xFFFF = not framed here (the exact kernel frames it).
// ---------------------------------------------------------------------------
constexpr uint32_t kArrMaxRec = 2560;  // records per lean batch (a 17 KiB window holds ~2480 at most)
__global__ __launch_bounds__(64) void k_arr_frame(EvalArgs a) {
  const uint8_t* S = a.slice;
  for (uint32_t b = blockIdx.x * 64 + threadIdx.x; b < a.nbatches; b += gridDim.x * 64) {
    const uint64_t pos = a.bpos[b];
    const uint64_t rb = a.rbase[b];
    const uint32_t rn = (uint32_t)((b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb);
    const uint64_t al = pos & ~15ull;
    const uint8_t* base = S + al;
    const uint32_t batch_len = __builtin_bswap32(ld4g(S + pos + 8));
    const uint64_t sec_end = pos + 12 + (uint64_t)batch_len;
    uint32_t end = 0xFFFFu;
    if (sec_end - al <= (uint64_t)kWin && rn <= kArrMaxRec && batch_len >= 49 &&
        __builtin_bswap32(ld4g(S + pos + 57)) == rn) {
      const uint32_t have = (uint32_t)(sec_end - al);
      uint32_t q = (uint32_t)(pos + 61 - al), n = 0, touch = 0;
      for (; n < rn; n++) {
        const uint32_t x = ld4g(base + q);
        touch += ld4g(base + (q + 256 < have ? q + 256 : have - 4));  // the line a few records ahead
        const uint32_t term = ~x & 0x80808080u;
        const uint32_t nb = (((uint32_t)__builtin_ctz(term | 0x80000000u)) >> 3) + 1;
        const uint32_t y = nb == 4 ? x : (x & ((1u << (8 * nb)) - 1u));
        const uint32_t v = (y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u) | ((y >> 3) & 0xFE00000u);
        const uint32_t len = v >> 1;
        // no terminator in 4 bytes, past the section, a negative length, past the section
        if (!term || q + nb > have || (v & 1u) || have - (q + nb) < len) break;
        a.rstart[rb + n] = (uint16_t)q;
        q += nb + len;
      }
      if (n == rn) end = q;
      if (touch == 0x9E3779B9u && n > rn) end = 0;  // never true: keeps the look-ahead reads
    }
    a.rend[b] = (uint16_t)end;
  }
}

// ---------------------------------------------------------------------------
// k_arr_lean — pass 1, one workgroup per batch (persistent).  Wave 0 frames
// the batch's records in LDS (the length-varint chain, wave-uniform), then a
// thread per record walks its value through the DFA: element starts / ends
// into two LDS bitmaps (stored per batch for k_arr_write), and the counts
// k_size prices the batch's output with (ArrBatch).
// ---------------------------------------------------------------------------
constexpr int kArrT = 256;
struct ArrLds {
  uint8_t W[kWin + 16] __attribute__((aligned(16)));
  uint32_t bm[kArrBmBatch];  // starts, then ends
  uint16_t rs[kArrMaxRec + 1];
  ArrTab T;
  uint32_t red[kArrT / 64][4];
  uint32_t cnt[9];
};

__global__ __launch_bounds__(kArrT) void k_arr_lean(EvalArgs a) {
  __shared__ ArrLds L;
  const uint32_t t = threadIdx.x, l = t & 63u;
  load_table(&L.T);
  const uint8_t* S = a.slice;
  for (uint32_t b = blockIdx.x; b < a.nbatches; b += gridDim.x) {
    const uint64_t pos = a.bpos[b];
    const uint64_t rb = a.rbase[b];
    const uint32_t rn = (uint32_t)((b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb);
    const uint64_t al = pos & ~15ull;
    const uint32_t batch_len = __builtin_bswap32(ld4g(S + pos + 8));
    const uint64_t sec_end = pos + 12 + (uint64_t)batch_len;
    const uint32_t rend = a.rend[b];
    // a batch beyond the window / the record slots / without a record count: the exact kernel
    bool defer = sec_end - al > (uint64_t)kWin || rn > kArrMaxRec || batch_len < 49;
    __syncthreads();  // the previous batch's window, bitmaps and counters are no longer read
    if (t < 9) L.cnt[t] = 0;
    if (!defer) {
      for (uint32_t k = t; k < kArrBmBatch; k += kArrT) L.bm[k] = 0;
      stage_window(S, al, (uint32_t)((sec_end - al + 15) & ~15ull), L.W);
    }
    __syncthreads();
    if (!defer && rend == 0xFFFFu) defer = true;  // k_arr_frame could not frame it
    if (!defer)
      for (uint32_t r = t; r <= rn; r += kArrT) L.rs[r] = r < rn ? a.rstart[rb + r] : (uint16_t)rend;
    __syncthreads();
    uint32_t bne = 0, besum = 0, bc59 = 0;
    bool bad = false;
    for (uint32_t r = t; r < rn && !defer && !bad; r += kArrT) {
      uint32_t v = 0, n = 0;
      if (!rec_value(L.W, L.rs[r], L.rs[r + 1], &v, &n)) {
        bad = true;
        break;
      }
      uint32_t t0 = 0, ne = 0, esum = 0;
      const uint32_t fin = arr_walk(L.W, &L.T, v, n, [&](uint32_t p, uint32_t, uint32_t x) {
        const uint32_t act = x >> 5;
        if (act & 1) {
          t0 = p;
          atomicOr(&L.bm[p >> 5], 1u << (p & 31));
        }
        if (act & 6) {
          const uint32_t e = p + ((act >> 2) & 1u);  // exclusive end
          atomicOr(&L.bm[kArrBmWords + (e >> 5)], 1u << (e & 31));
          const uint32_t len = e - t0;
          const uint32_t el = elem_L(len);
          ne++;
          esum += el;
          if (len > 19) {  // rare: an integer beyond u64 / i64 (f64 in serde_json), a long element
            const uint32_t c = L.W[t0];
            bad |= (c == '-' || (c >= '0' && c <= '9')) || el > kArrMaxL;
            if (el >= 59)
              bc59++;
            else if (el >= 50)
              atomicAdd(&L.cnt[el - 50], 1u);
          }
        }
      });
      bad |= fin != A_POST;
      bne += ne;
      besum += esum;
    }
    defer = __syncthreads_or(defer || bad) != 0;
    if (defer) {
      if (t == 0) {
        const uint32_t i = atomicAdd(a.list, 1u);
        a.list[1 + i] = b;
      }
      continue;
    }
    // the element bitmaps of the window's words to HBM
    const uint32_t nw = (uint32_t)((sec_end - al + 31) >> 5);
    uint32_t* bmg = a.arr_bm + (uint64_t)b * kArrBmBatch;
    for (uint32_t k = t; k < nw; k += kArrT) {
      bmg[k] = L.bm[k];
      bmg[kArrBmWords + k] = L.bm[kArrBmWords + k];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      bne += __shfl_xor(bne, o, 64);
      besum += __shfl_xor(besum, o, 64);
      bc59 += __shfl_xor(bc59, o, 64);
    }
    if (l == 0) {
      L.red[t >> 6][0] = bne;
      L.red[t >> 6][1] = besum;
      L.red[t >> 6][2] = bc59;
    }
    __syncthreads();
    if (t == 0) {
      ArrBatch ab = {};
      for (int w = 0; w < kArrT / 64; w++) {
        ab.ne += L.red[w][0];
        ab.esum += L.red[w][1];
        ab.c59 += L.red[w][2];
      }
      for (int k = 0; k < 9; k++) ab.cnt[k] = L.cnt[k];
      a.arr_b[b] = ab;
      const uint8_t* h = L.W + (pos - al);
      auto be = [&](uint32_t o, int nbytes) {
        uint64_t x = 0;
        for (int k = 0; k < nbytes; k++) x = (x << 8) | h[o + k];
        return x;
      };
      BatchStat st = {};
      st.base_offset = (int64_t)be(0, 8);
      st.lod_in = (int32_t)be(23, 4);
      st.first_ts = (int64_t)be(27, 8);
      st.comp = h[22] & 7u;
      st.flags = BF_LAST_STAGE | BF_ARR_LEAN;
      st.nkeep = rn;
      st.nout = ab.ne;
      st.sec_len = batch_len - 45u;
      st.err_stage = 0xFFFFFFFFu;
      a.bstat[b] = st;
    }
  }
}

// ---------------------------------------------------------------------------
// k_arr_write — pass 2 (output), one workgroup per BF_ARR_LEAN batch of
// [plan.first, plan.last] (persistent).  No DFA: the batch's element bitmaps
// give every element's source span (the k-th start with the k-th end, by a
// workgroup popcount scan), and the elements are written a lane each, in tiles
// of 256: output size, workgroup scan, the element record (Record::
// new_key_value(None, element): inner length, attributes 0, timestamp delta 0,
// offset delta `rel`, no key, the text, no headers) into an LDS staging
// buffer, which is stored to HBM as 16-byte units when the next tile would
// not fit.  A tile larger than the buffer is written in clipped rounds.
// ---------------------------------------------------------------------------
constexpr uint32_t kStage = 8192, kEl = 2048;
constexpr uint32_t kBmPer = (kArrBmWords + kArrT - 1) / kArrT;  // bitmap words per thread
struct ArwLds {
  uint8_t W[kWin + 16] __attribute__((aligned(16)));
  uint8_t O[kStage] __attribute__((aligned(16)));
  uint32_t bm[kArrBmBatch];
  uint16_t es[kEl], ee[kEl];  // element starts / ends of the current round
  uint32_t part[kArrT / 64][2];
};

__device__ __forceinline__ void put(uint8_t* O, int32_t j, uint32_t c) {
  if ((uint32_t)j < kStage) O[j] = (uint8_t)c;
}
// a small non-negative value's zigzag varint (1 or 2 bytes, x < 8192)
__device__ __forceinline__ void put_vs2(uint8_t* O, int32_t j, uint32_t x) {
  const uint32_t z = 2 * x;
  if (x < 64) {
    put(O, j, z);
  } else {
    put(O, j, (z & 0x7Fu) | 0x80u);
    put(O, j + 1, z >> 7);
  }
}
// workgroup exclusive scan of two counters (all threads call it)
__device__ __forceinline__ void wg_scan2(uint32_t (*part)[2], uint32_t x, uint32_t y, uint32_t& xe, uint32_t& ye,
                                         uint32_t& xt, uint32_t& yt) {
  const uint32_t t = threadIdx.x, l = t & 63u;
  uint32_t xi = x, yi = y;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(xi, o, 64), b = __shfl_up(yi, o, 64);
    if (l >= (uint32_t)o) {
      xi += a;
      yi += b;
    }
  }
  if (l == 63) {
    part[t >> 6][0] = xi;
    part[t >> 6][1] = yi;
  }
  __syncthreads();
  xe = xi - x;
  ye = yi - y;
  xt = yt = 0;
  for (uint32_t w = 0; w < kArrT / 64; w++) {
    const uint32_t px = part[w][0], py = part[w][1];
    if (w < (t >> 6)) {
      xe += px;
      ye += py;
    }
    xt += px;
    yt += py;
  }
  __syncthreads();  // part is reused by the next scan
}
// staged bytes of global addresses [lo, hi) to HBM (staging index = address - B)
__device__ void stage_flush(const uint8_t* O, uint64_t B, uint64_t lo, uint64_t hi) {
  for (uint64_t X = (lo & ~15ull) + 16ull * threadIdx.x; X < hi; X += 16ull * kArrT) {
    const uint8_t* src = O + (X - B);
    if (X >= lo && X + 16 <= hi) {
      *(uint4*)(uintptr_t)X = *(const uint4*)src;
    } else {
      for (uint32_t k = 0; k < 16; k++)
        if (X + k >= lo && X + k < hi) *(uint8_t*)(uintptr_t)(X + k) = src[k];
    }
  }
}

__global__ __launch_bounds__(kArrT) void k_arr_write(ArrWriteArgs a) {
  __shared__ ArwLds L;
  const uint32_t t = threadIdx.x;
  const Plan p = *a.plan;
  if (p.first < 0 || p.last < p.first) return;
  const uint32_t nblk = (uint32_t)(p.last - p.first + 1);
  const uint8_t* S = a.slice;
  for (uint32_t j = blockIdx.x; j < nblk; j += gridDim.x) {
    const uint32_t b = (uint32_t)p.first + j;
    const BatchStat bs = a.bstat[b];
    if (!(bs.flags & BF_ARR_LEAN)) continue;  // written by k_write (the exact kernel's descriptors)
    const int64_t rel = a.seg ? 0 : p.base_offset - bs.base_offset;
    uint8_t rv[16];
    const uint32_t vr = venc(rel, rv);
    const uint64_t G = (uint64_t)(uintptr_t)a.out + (a.seg ? 61ull * (uint64_t)(b + 1) + a.pre[b].rec_bytes
                                                            : 61 + (a.pre[b].rec_bytes - a.pre[p.first].rec_bytes));
    const uint64_t pos = a.bpos[b];
    const uint64_t al = pos & ~15ull;
    const uint32_t batch_len = __builtin_bswap32(ld4g(S + pos + 8));
    const uint64_t sec_end = pos + 12 + (uint64_t)batch_len;
    const uint32_t nw = (uint32_t)((sec_end - al + 31) >> 5);
    __syncthreads();  // the previous batch's window and bitmaps are no longer read
    stage_window(S, al, (uint32_t)((sec_end - al + 15) & ~15ull), L.W);
    const uint32_t* bmg = a.arr_bm + (uint64_t)b * kArrBmBatch;
    for (uint32_t k = t; k < kArrBmWords; k += kArrT) {
      L.bm[k] = k < nw ? bmg[k] : 0u;
      L.bm[kArrBmWords + k] = k < nw ? bmg[kArrBmWords + k] : 0u;
    }
    __syncthreads();
    // this thread's bitmap words: [w0, w0 + kBmPer); element index of its first start / end
    const uint32_t w0 = t * kBmPer;
    uint32_t cs = 0, ce = 0;
    for (uint32_t k = 0; k < kBmPer; k++)
      if (w0 + k < kArrBmWords) {
        cs += __popc(L.bm[w0 + k]);
        ce += __popc(L.bm[kArrBmWords + w0 + k]);
      }
    uint32_t s_ex, e_ex, ne, ne2;
    wg_scan2(L.part, cs, ce, s_ex, e_ex, ne, ne2);
    uint64_t B = G & ~15ull, F = G, done = G;  // staging base, next byte, first byte not yet stored
    for (uint32_t k0 = 0; k0 < ne; k0 += kEl) {  // rounds of kEl elements
      const uint32_t k1 = ne - k0 < kEl ? ne - k0 : kEl;
      {  // the round's element spans from the bitmaps
        uint32_t is = s_ex, ie = e_ex;
        for (uint32_t k = 0; k < kBmPer; k++) {
          if (w0 + k >= kArrBmWords) break;
          for (uint32_t m = L.bm[w0 + k]; m; m &= m - 1, is++)
            if (is >= k0 && is < k0 + k1) L.es[is - k0] = (uint16_t)(32 * (w0 + k) + __builtin_ctz(m));
          for (uint32_t m = L.bm[kArrBmWords + w0 + k]; m; m &= m - 1, ie++)
            if (ie >= k0 && ie < k0 + k1) L.ee[ie - k0] = (uint16_t)(32 * (w0 + k) + __builtin_ctz(m));
        }
      }
      __syncthreads();
      for (uint32_t e0 = 0; e0 < k1; e0 += kArrT) {  // tiles: an element a lane
        const uint32_t e = e0 + t;
        uint32_t s0 = 0, len = 0, sz = 0;
        if (e < k1) {
          s0 = L.es[e];
          len = L.ee[e] - s0;
          const uint32_t inner = 4 + vr + len + vs2(len);
          sz = vs2(inner) + inner;
        }
        uint32_t off, z0, ttot, z1;
        wg_scan2(L.part, sz, 0, off, z0, ttot, z1);
        const uint64_t tlo = F, thi = F + ttot;
        if (thi > B + kStage && F > done) {  // the tile does not fit after what is staged: store that first
          stage_flush(L.O, B, done, F);
          __syncthreads();
          done = F;
          B = F & ~15ull;
        }
        for (uint64_t R = B;; R += kStage) {  // one round, or clipped rounds for an oversized tile
          if (sz) {
            const int32_t o = (int32_t)((int64_t)(tlo + off) - (int64_t)R);
            const uint32_t inner = 4 + vr + len + vs2(len), iv = vs2(inner), lv = vs2(len);
            put_vs2(L.O, o, inner);
            int32_t w = o + (int32_t)iv;
            put(L.O, w, 0);      // attributes
            put(L.O, w + 1, 0);  // timestamp_delta
            for (uint32_t i = 0; i < vr; i++) put(L.O, w + 2 + (int32_t)i, rv[i]);
            w += 2 + (int32_t)vr;
            put(L.O, w, 0);  // key: None
            put_vs2(L.O, w + 1, len);
            w += 1 + (int32_t)lv;
            for (uint32_t i = 0; i < len; i++) put(L.O, w + (int32_t)i, L.W[s0 + i]);
            put(L.O, w + (int32_t)len, 0);  // headers
          }
          __syncthreads();
          if (thi <= R + kStage) {
            B = R;
            break;
          }
          stage_flush(L.O, R, done, R + kStage);
          __syncthreads();
          done = R + kStage;
        }
        F = thi;
      }
      __syncthreads();  // es / ee are rewritten by the next round
    }
    if (F > done) stage_flush(L.O, B, done, F);
  }
}

template <typename K>
uint32_t resident(K kernel, int dev_threads) {
  int dev = 0, cus = 0, per = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, dev_threads, 0);
  return (uint32_t)(cus > 0 ? cus : 1) * (uint32_t)(per > 0 ? per : 1);
}
uint32_t arr_grid(uint32_t nb, int which) {  // 0: k_arr_lean, 1: k_arr_write
  static uint32_t cache[64][2];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cache[dev][which])
    cache[dev][which] = which == 1 ? resident(k_arr_write, kArrT) : resident(k_arr_lean, kArrT);
  return std::min<uint32_t>(nb, cache[dev][which]);
}

}  // namespace

// a chain of exactly one array_map_json_array stage over the source values
bool array_lean_eligible(const ChainDesc& ch, uint32_t ops) {
  return ops == (1u << OP_ARRAY_MAP) && ch.nstages == 1 && ch.st[0].in_type == VT_SRC;
}
void launch_array_lean(const EvalArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  hipLaunchKernelGGL(k_arr_frame, dim3((a.nbatches + 63) / 64), dim3(64), 0, s, a);  // spread over every CU
  hipLaunchKernelGGL(k_arr_lean, dim3(arr_grid(a.nbatches, 0)), dim3(kArrT), 0, s, a);
}
void launch_array_write(const ArrWriteArgs& a, uint32_t nblk, hipStream_t s) {
  if (!nblk) return;
  hipLaunchKernelGGL(k_arr_write, dim3(arr_grid(nblk, 1)), dim3(kArrT), 0, s, a);
}

}  // namespace fsg
