// fsg_dev_util.h — small device helpers shared by the kernel files
// (fsg_kernels.hip, fsg_lean.hip): big-endian reads, wave reductions and
// scans, the varint decoder (varint.rs:43-66), SWAR byte tests.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fsg {

__device__ __forceinline__ uint64_t rd_be(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 8) | p[i];
  return v;
}

__device__ __forceinline__ uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// wave helpers (64 lanes)
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint32_t lanemask_lt() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
  const int l = lane_id();
  for (int o = 1; o < 64; o <<= 1) {
    T t = __shfl_up(v, o, 64);
    if (l >= o) v += t;
  }
  return v;
}

// decode a varint from window bytes [q, lim); lim_sec tells whether running
// out of window bytes means "incomplete" (more section bytes) or EOF
template <typename P>
__device__ __forceinline__ int wvarint(P w, uint32_t& q, uint32_t wlim, int64_t* out) {
  uint64_t num = 0;
  uint32_t shift = 0;
  for (;;) {
    if (q >= wlim) return -1;
    uint8_t b = w[q++];
    num |= ((uint64_t)(b & 0x7f)) << (shift & 63);
    shift += 7;
    if (!(b & 0x80)) break;
  }
  int64_t sn = (int64_t)num;
  *out = (int64_t)((uint64_t)(sn >> 1) ^ (uint64_t)(-(sn & 1)));
  return 0;
}

// <i32 as FromStr>::from_str — 0 ok, 1 Empty, 2 InvalidDigit, 3 PosOverflow, 4 NegOverflow
template <typename P>
__device__ __forceinline__ int parse_i32(P s, uint32_t n, int32_t* out) {
  if (n == 0) return 1;
  uint32_t i = 0;
  bool pos = true;
  uint8_t c0 = s[0];
  if ((c0 == '+' || c0 == '-') && n == 1) return 2;
  if (c0 == '+')
    i = 1;
  else if (c0 == '-') {
    pos = false;
    i = 1;
  }
  int64_t acc = 0;
  for (; i < n; i++) {
    uint32_t c = s[i];
    if (c < '0' || c > '9') return 2;
    int d = (int)c - '0';
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

// exact zero-byte mask: 0x80 in each byte of x that is zero
__device__ __forceinline__ uint32_t zbytes(uint32_t x) {
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}

// SWAR helpers (4 bytes per u32)
__device__ __forceinline__ uint32_t swar_upper(uint32_t x) {
  // make_ascii_uppercase on each byte: 'a'..'z' -> 'A'..'Z', other bytes unchanged
  const uint32_t y = x & 0x7F7F7F7Fu;
  const uint32_t ge_a = y + 0x1F1F1F1Fu;   // high bit set where y >= 'a'
  const uint32_t gt_z = y + 0x05050505u;   // high bit set where y >= '{'
  const uint32_t lower = ge_a & ~gt_z & ~x & 0x80808080u;
  return x - (lower >> 2);
}
__device__ __forceinline__ uint32_t ld_u32_at(const uint8_t* p) {  // 4 bytes at any address
  const uint64_t a = (uint64_t)p;
  const uint32_t* w = (const uint32_t*)(a & ~3ull);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3u));
}

// Workgroup barrier over LDS only: the LDS-DMA of the next batch stays in
// flight (__syncthreads would also wait for every outstanding global access).
__device__ __forceinline__ void lean_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

}  // namespace fsg
