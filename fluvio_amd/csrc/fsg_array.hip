// fsg_array.hip — lean evaluation of array_map_json_array chains (C4:
// smartmodule/examples/array_map_json_array/src/lib.rs:38-55, derive
// generator/array_map.rs:17-42: serde_json::from_slice::<Vec<Value>> of each
// record's value, one output record per element, serde_json::to_string of it).
//
// k_eval's exact path parses every record with the full serde_json restatement
// inside a 256-thread workgroup per batch (instruction-bound on MI355X: C4 ~240
// records per batch).  Here one workgroup per batch, thread = record,
// records located by k_chase_x, the batch's window staged in LDS, and each
// lane walks a small grammar of the arrays whose output is
// certain: flat arrays of JSON integers (no leading zero, <= 18 digits, not
// -0), strings without escapes / control / non-ASCII bytes, and true / false /
// null, with whitespace anywhere JSON allows it.  Every such element's
// serde_json::to_string is its source text, so it is emitted verbatim
// (ElemRec with the verbatim bit).  Anything else in a batch (other values,
// errors, floats, nested arrays / objects, escapes, non-ASCII, long varints)
// defers the whole batch to the exact kernel (list mode), as k_eval_lean does.
//
// Each record's KeptRec also carries the sum of its elements' (varint + text)
// bytes (KF_ESUM): k_size then sizes the record's output records without
// reading its ElemRecs (elements shorter than 40 bytes, which is every element
// of the bench's arrays; others keep the per-element loop).
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
__device__ __forceinline__ uint32_t vsz(int64_t v) {  // zigzag varint length
  uint64_t z = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
  uint32_t n = 1;
  while (z >= 0x80) {
    z >>= 7;
    n++;
  }
  return n;
}
__device__ __forceinline__ bool is_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
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

// The lean array grammar as a byte DFA (one class lookup and one transition
// lookup per byte, both in LDS; no per-byte branches).  States:
enum ArrSt : uint32_t {
  A_BAD, A_PRE, A_VAL1, A_VAL, A_MINUS, A_ZERO, A_INT, A_STR, A_T1, A_T2, A_T3, A_F1, A_F2, A_F3, A_F4, A_N1, A_N2,
  A_N3, A_AFTER, A_POST, A_NSTATES
};
// byte classes: 0 other printable ASCII, 1 whitespace, 2 '[', 3 ']', 4 ',', 5 '"',
// 6 '-', 7 '0', 8 '1'-'9', 9 't', 10 'r', 11 'u', 12 'e', 13 'f', 14 'a', 15 'l',
// 16 's', 17 'n', 18 not allowed in a lean string (controls, '\\', >= 0x80)
constexpr uint32_t kArrCls = 32;
__device__ uint32_t arr_class(uint32_t c) {
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
// next state | action << 5: 1 = a token starts here, 2 = the element ended
// before this byte, 4 = the element ends with this byte
__device__ uint32_t arr_trans(uint32_t st, uint32_t cl) {
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

// the value bytes [v, v + n) of one record (window offsets into W; abs = the
// window's slice offset) through the DFA; elements to elem[]; false = not lean
// (the batch goes to the exact kernel)
__device__ bool lean_array(const uint8_t* W, const uint8_t* CL, const uint8_t* TR, uint32_t v, uint32_t n,
                           uint64_t abs, ElemRec* elem, uint32_t* ne_out, uint32_t* esum_out, uint32_t* big_out) {
  uint32_t st = A_PRE, ne = 0, esum = 0, big = 0, t0 = 0;
  bool isint = false, bad = false;
  ElemRec* e = elem + ((abs + v) >> 1);
  const uint32_t end = v + n;
  for (uint32_t i = v; i < end; i += 4) {
    const uint32_t w = lds4(W, i);
    const uint32_t k1 = end - i < 4 ? end - i : 4;
    for (uint32_t k = 0; k < k1; k++) {
      const uint32_t x = TR[st * kArrCls + CL[(w >> (8 * k)) & 0xFFu]];
      const uint32_t act = x >> 5;
      const uint32_t pos = i + k;
      if (act & 1) {
        t0 = pos;
        isint = (x & 31) == A_MINUS || (x & 31) == A_ZERO || (x & 31) == A_INT;
      }
      if (act & 6) {
        const uint32_t len = pos + ((act >> 2) & 1) - t0;
        bad |= isint && len > 19;  // beyond u64 / i64: f64 in serde_json
        ElemRec r;
        r.pos = abs + t0;
        r.src_len = len;
        r.out_len = len | 0x80000000u;
        e[ne++] = r;
        esum += vsz((int64_t)len) + len;
        big += len >= 40 ? 1u : 0u;
      }
      st = x & 31;
    }
  }
  *ne_out = ne;
  *esum_out = esum;
  *big_out = big;
  return st == A_POST && !bad;
}

// one workgroup per batch (persistent): the batch's window staged in LDS by
// 1 KiB LDS-DMA pieces, then thread t parses records t, t + 256, ... from LDS
constexpr int kArrT = 256;
__global__ __launch_bounds__(kArrT) void k_arr_lean(EvalArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t W[kWin + 16];
  __shared__ uint32_t red[kArrT / 64];
  __shared__ uint8_t CL[256];
  __shared__ uint8_t TR[A_NSTATES * kArrCls];
  const uint32_t t = threadIdx.x, l = t & 63u;
  CL[t] = (uint8_t)arr_class(t);
  for (uint32_t k = t; k < A_NSTATES * kArrCls; k += kArrT) TR[k] = (uint8_t)arr_trans(k / kArrCls, k % kArrCls);
  const uint8_t* S = a.slice;
  for (uint32_t b = blockIdx.x; b < a.nbatches; b += gridDim.x) {
    const uint64_t pos = a.bpos[b];
    const uint64_t rb = a.rbase[b];
    const uint32_t rn = (uint32_t)((b + 1 < a.nbatches ? a.rbase[b + 1] : a.nrec) - rb);
    const uint32_t rend = a.rend[b];
    const uint64_t al = pos & ~15ull;
    const uint32_t batch_len = __builtin_bswap32(ld4g(S + pos + 8));
    const uint64_t sec_end = pos + 12 + (uint64_t)batch_len;
    bool defer = rend == 0xFFFFu || sec_end - al > (uint64_t)kWin;  // framing / a batch beyond the window
    __syncthreads();  // the previous batch's window is no longer read
    if (!defer) {
      const uint32_t wlen = (uint32_t)((sec_end - al + 15) & ~15ull);
      const uint32_t wv = t >> 6;
      for (uint32_t k = wv; k * 1024 < wlen; k += kArrT / 64)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(S + al + k * 1024 + l * 16),
                                         (__attribute__((address_space(3))) void*)(W + k * 1024), 16, 0, 0);
      __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
    uint32_t nout = 0;
    bool bad = false;
    for (uint32_t r = t; r < rn && !defer; r += kArrT) {
      uint32_t ne = 0, esum = 0, big = 0;
      const uint32_t q0 = a.rstart[rb + r];
      const uint32_t qe = r + 1 < rn ? a.rstart[rb + r + 1] : rend;
      int64_t len = 0, ts = 0, od = 0, kl = 0, vl = 0, hdr = 0;
      uint32_t q = q0;
      uint32_t u = var_lds(W, q, &len);
      bool b1 = !u || len < 0;
      q += u;
      if (!b1) {
        q += 1;  // attributes
        u = var_lds(W, q, &ts);
        b1 = !u;
        q += u;
      }
      if (!b1) {
        u = var_lds(W, q, &od);
        b1 = !u;
        q += u;
      }
      uint32_t tag = 0;
      if (!b1) {
        tag = W[q++];
        b1 = tag > 1;
      }
      if (!b1 && tag) {
        u = var_lds(W, q, &kl);
        b1 = !u || kl < 0 || (int64_t)q + u + kl > (int64_t)qe;
        q += u + (uint32_t)(b1 ? 0 : kl);
      }
      if (!b1) {
        u = var_lds(W, q, &vl);
        b1 = !u || vl < 0 || (int64_t)q + u + vl >= (int64_t)qe;
        q += u;
      }
      if (!b1) {
        const uint32_t hq = q + (uint32_t)vl;
        u = var_lds(W, hq, &hdr);
        b1 = !u || hq + u != qe || (int64_t)q0 + vsz(len) + len != (int64_t)qe;
      }
      if (!b1) b1 = !lean_array(W, CL, TR, q, (uint32_t)vl, al, a.elem, &ne, &esum, &big);
      if (!b1) {
        KeptRec d;
        d.src = al + q0;
        d.vpos = al + q;
        d.kpos = 0;
        d.od = od;
        d.ts = esum;  // KF_ESUM: Σ (varint + text) of the elements
        d.hdr = big;  // ... and the elements of 40 bytes or more
        d.vlen = (uint32_t)vl;
        d.klen = 0;
        d.ival = (int32_t)ne;
        d.mode = KM_ARRAY;
        d.has_key = 0;
        d.attr = 0;
        d.pad = KF_ESUM;
        a.desc[rb + r] = d;
      }
      bad |= b1;
      nout += ne;
    }
    defer = __syncthreads_or(defer || bad) != 0;
    if (defer) {
      if (t == 0) {
        const uint32_t i = atomicAdd(a.list, 1u);
        a.list[1 + i] = b;
      }
      continue;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nout += __shfl_xor(nout, o, 64);
    if (l == 0) red[t >> 6] = nout;
    __syncthreads();
    if (t == 0) {
      const uint8_t* h = W + (pos - al);
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
      st.flags = BF_LAST_STAGE;
      st.nkeep = rn;
      st.nout = red[0] + red[1] + red[2] + red[3];
      st.sec_len = batch_len - 45u;
      st.err_stage = 0xFFFFFFFFu;
      a.bstat[b] = st;
    }
  }
}

uint32_t arr_grid(uint32_t nb) {
  static uint32_t cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cache[dev]) {
    int cus = 0, per = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_arr_lean, kArrT, 0);
    cache[dev] = (uint32_t)(cus > 0 ? cus : 1) * (uint32_t)(per > 0 ? per : 1);
  }
  return std::min<uint32_t>(nb, cache[dev]);
}

}  // namespace

// a chain of exactly one array_map_json_array stage over the source values
bool array_lean_eligible(const ChainDesc& ch, uint32_t ops) {
  return ops == (1u << OP_ARRAY_MAP) && ch.nstages == 1 && ch.st[0].in_type == VT_SRC;
}
void launch_array_lean(const EvalArgs& a, hipStream_t s) {
  if (!a.nbatches) return;
  hipLaunchKernelGGL(k_arr_lean, dim3(arr_grid(a.nbatches)), dim3(kArrT), 0, s, a);
}

}  // namespace fsg
