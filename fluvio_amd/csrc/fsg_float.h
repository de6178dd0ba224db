// fsg_float.h — the f64 arithmetic of the JSON modules, host + device.
//
// * serde_json 1.0.96 reads a JSON number that is not a u64 / i64 (a fraction,
//   an exponent, -0, or an integer beyond 64 bits) with de.rs parse_integer /
//   parse_long_integer / parse_decimal(_overflow) / parse_exponent(_overflow)
//   and f64_from_parts — the default build, without the `float_roundtrip`
//   feature (smartmodule/examples/Cargo.lock pins serde_json 1.0.96 with
//   default features): a u64 significand (digits past u64 are dropped into the
//   exponent) times / divided by POW10[|e|] (1e0 ..= 1e308), not a correctly
//   rounded parse.  Overflow to infinity is "number out of range".
// * Shortest round-trip digits: exact bignum digit generation (Steele & White
//   "free-format" with Burger & Dybvig's termination tests; the interval bounds
//   are inclusive for an even mantissa), stopping at the first digit position
//   inside the rounding interval and taking the candidate closest to the value.
//   An exact tie between the two candidates goes to the even digit for ryu
//   (d2s.rs: `vr % 2 == 0` keeps vr) and upward for Rust's Display
//   (core::num::flt2dec::strategy::dragon::format_shortest: `2r >= s` rounds up).
// * ryu 1.0.13 `Buffer::format_finite` (pretty/mod.rs format64): what
//   serde_json's Value::to_string writes for an f64 (array_map_json_array).
// * Rust `Display for f64` (shortest digits, plain decimal notation, "-0" for
//   negative zero) behind serde 1.0.160's `WithDecimalPoint` (".0" appended
//   when the text has no '.'): the `floating point `..`` of serde's
//   Unexpected::Float in "invalid type" messages.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace fsg {
namespace flt {

#define FSG_POW10_INIT {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22, 1e23, 1e24, 1e25, 1e26, 1e27, 1e28, 1e29, 1e30, 1e31, 1e32, 1e33, 1e34, 1e35, 1e36, 1e37, 1e38, 1e39, 1e40, 1e41, 1e42, 1e43, 1e44, 1e45, 1e46, 1e47, 1e48, 1e49, 1e50, 1e51, 1e52, 1e53, 1e54, 1e55, 1e56, 1e57, 1e58, 1e59, 1e60, 1e61, 1e62, 1e63, 1e64, 1e65, 1e66, 1e67, 1e68, 1e69, 1e70, 1e71, 1e72, 1e73, 1e74, 1e75, 1e76, 1e77, 1e78, 1e79, 1e80, 1e81, 1e82, 1e83, 1e84, 1e85, 1e86, 1e87, 1e88, 1e89, 1e90, 1e91, 1e92, 1e93, 1e94, 1e95, 1e96, 1e97, 1e98, 1e99, 1e100, 1e101, 1e102, 1e103, 1e104, 1e105, 1e106, 1e107, 1e108, 1e109, 1e110, 1e111, 1e112, 1e113, 1e114, 1e115, 1e116, 1e117, 1e118, 1e119, 1e120, 1e121, 1e122, 1e123, 1e124, 1e125, 1e126, 1e127, 1e128, 1e129, 1e130, 1e131, 1e132, 1e133, 1e134, 1e135, 1e136, 1e137, 1e138, 1e139, 1e140, 1e141, 1e142, 1e143, 1e144, 1e145, 1e146, 1e147, 1e148, 1e149, 1e150, 1e151, 1e152, 1e153, 1e154, 1e155, 1e156, 1e157, 1e158, 1e159, 1e160, 1e161, 1e162, 1e163, 1e164, 1e165, 1e166, 1e167, 1e168, 1e169, 1e170, 1e171, 1e172, 1e173, 1e174, 1e175, 1e176, 1e177, 1e178, 1e179, 1e180, 1e181, 1e182, 1e183, 1e184, 1e185, 1e186, 1e187, 1e188, 1e189, 1e190, 1e191, 1e192, 1e193, 1e194, 1e195, 1e196, 1e197, 1e198, 1e199, 1e200, 1e201, 1e202, 1e203, 1e204, 1e205, 1e206, 1e207, 1e208, 1e209, 1e210, 1e211, 1e212, 1e213, 1e214, 1e215, 1e216, 1e217, 1e218, 1e219, 1e220, 1e221, 1e222, 1e223, 1e224, 1e225, 1e226, 1e227, 1e228, 1e229, 1e230, 1e231, 1e232, 1e233, 1e234, 1e235, 1e236, 1e237, 1e238, 1e239, 1e240, 1e241, 1e242, 1e243, 1e244, 1e245, 1e246, 1e247, 1e248, 1e249, 1e250, 1e251, 1e252, 1e253, 1e254, 1e255, 1e256, 1e257, 1e258, 1e259, 1e260, 1e261, 1e262, 1e263, 1e264, 1e265, 1e266, 1e267, 1e268, 1e269, 1e270, 1e271, 1e272, 1e273, 1e274, 1e275, 1e276, 1e277, 1e278, 1e279, 1e280, 1e281, 1e282, 1e283, 1e284, 1e285, 1e286, 1e287, 1e288, 1e289, 1e290, 1e291, 1e292, 1e293, 1e294, 1e295, 1e296, 1e297, 1e298, 1e299, 1e300, 1e301, 1e302, 1e303, 1e304, 1e305, 1e306, 1e307, 1e308}
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __constant__ static const double kPow10[309] = FSG_POW10_INIT;
#else
static const double kPow10[309] = FSG_POW10_INIT;
#endif

// de.rs f64_from_parts (not float_roundtrip): 0 = ok, 1 = number out of range
__host__ __device__ inline int f64_from_parts(bool positive, uint64_t significand, int64_t exponent, double* out) {
  double f = (double)significand;
  for (;;) {
    const int64_t ae = exponent < 0 ? -exponent : exponent;
    if (ae <= 308) {
      if (exponent >= 0) {
        f *= kPow10[ae];
        if (__builtin_isinf(f)) return 1;
      } else {
        f /= kPow10[ae];
      }
      break;
    }
    if (f == 0.0) break;
    if (exponent >= 0) return 1;
    f /= 1e308;
    exponent += 308;
  }
  *out = positive ? f : -f;
  return 0;
}

// A syntactically valid JSON number starting at i (ParserNumber): kind 0 =
// u64 / i64 (its canonical text is its source text), 1 = f64 in *f, 2 =
// "number out of range" detected at index err.  end = index past the number.
struct NumVal {
  int kind;
  double f;
  uint32_t end, err;
};
template <class At>
__host__ __device__ inline NumVal num_value(const At& at, uint32_t i, uint32_t n) {
  NumVal r{0, 0.0, i, 0};
  auto dig = [&](uint32_t k) { return k < n && at(k) >= '0' && at(k) <= '9'; };
  const bool positive = at(i) != '-';
  if (!positive) i++;
  uint64_t sig = 0;
  int64_t exp = 0;
  bool flt = false;
  if (at(i) == '0') {
    i++;
  } else {
    while (dig(i)) {
      const uint64_t d = (uint64_t)(at(i) - '0');
      if (sig > 1844674407370955161ull || (sig == 1844674407370955161ull && d > 5)) {  // parse_long_integer
        flt = true;
        while (dig(i)) {
          i++;
          exp++;
        }
        break;
      }
      sig = sig * 10 + d;
      i++;
    }
  }
  if (i < n && at(i) == '.') {  // parse_decimal
    flt = true;
    i++;
    bool over = false;
    while (dig(i)) {
      const uint64_t d = (uint64_t)(at(i) - '0');
      if (!over && (sig > 1844674407370955161ull || (sig == 1844674407370955161ull && d > 5))) over = true;
      if (!over) {  // parse_decimal_overflow ignores every further digit
        sig = sig * 10 + d;
        exp--;
      }
      i++;
    }
  }
  if (i < n && (at(i) == 'e' || at(i) == 'E')) {  // parse_exponent
    flt = true;
    i++;
    bool pexp = true;
    if (at(i) == '+') {
      i++;
    } else if (at(i) == '-') {
      pexp = false;
      i++;
    }
    int32_t e = at(i) - '0';
    i++;
    while (dig(i)) {
      const int32_t d = at(i) - '0';
      i++;  // eaten before the overflow check
      if (e > 214748364 || (e == 214748364 && d > 7)) {  // parse_exponent_overflow
        if (sig != 0 && pexp) {
          r.kind = 2;
          r.err = i;
          while (dig(i)) i++;
          r.end = i;
          return r;
        }
        while (dig(i)) i++;
        r.kind = 1;
        r.f = positive ? 0.0 : -0.0;
        r.end = i;
        return r;
      }
      e = e * 10 + d;
    }
    exp = pexp ? exp + e : exp - e;  // i32 saturating_add / _sub
    if (exp > 2147483647) exp = 2147483647;
    if (exp < -2147483647 - 1) exp = -2147483647 - 1;
  }
  r.end = i;
  if (!flt) {
    if (positive) return r;  // U64
    if (sig != 0 && sig <= 0x8000000000000000ull) return r;  // I64
    r.kind = 1;  // -0 / below i64::MIN: -(significand as f64)
    r.f = -(double)sig;
    return r;
  }
  double f;
  if (f64_from_parts(positive, sig, exp, &f)) {
    r.kind = 2;
    r.err = i;
    return r;
  }
  r.kind = 1;
  r.f = f;
  return r;
}

// ---- exact shortest digits
struct Big {
  static constexpr int kW = 40;  // 1280 bits: r of the smallest subnormal scaled by 10^324
  uint32_t w[kW];
  int n;  // used words (no leading zero word)
  __host__ __device__ void set(uint64_t v) {
    for (int k = 0; k < kW; k++) w[k] = 0;
    w[0] = (uint32_t)v;
    w[1] = (uint32_t)(v >> 32);
    n = w[1] ? 2 : w[0] ? 1 : 0;
  }
  __host__ __device__ void shl(int b) {
    if (b <= 0 || n == 0) return;
    const int ws = b >> 5, bs = b & 31;
    for (int k = n - 1 + ws + 1; k >= 0; k--) {
      const int src = k - ws;
      uint32_t hi = (src >= 0 && src < n) ? w[src] : 0u, lo = (src - 1 >= 0 && src - 1 < n) ? w[src - 1] : 0u;
      w[k] = bs ? (hi << bs) | (lo >> (32 - bs)) : hi;
    }
    n = n + ws + 1;
    while (n > 0 && w[n - 1] == 0) n--;
  }
  __host__ __device__ void mul(uint32_t m) {
    uint64_t c = 0;
    for (int k = 0; k < n; k++) {
      const uint64_t t = (uint64_t)w[k] * m + c;
      w[k] = (uint32_t)t;
      c = t >> 32;
    }
    if (c) w[n++] = (uint32_t)c;
  }
  __host__ __device__ void mul_pow10(int k) {
    while (k >= 9) {
      mul(1000000000u);
      k -= 9;
    }
    for (; k > 0; k--) mul(10);
  }
  __host__ __device__ void add(const Big& b) {
    const int m = n > b.n ? n : b.n;
    uint64_t c = 0;
    for (int k = 0; k < m; k++) {
      const uint64_t t = (uint64_t)(k < n ? w[k] : 0u) + (k < b.n ? b.w[k] : 0u) + c;
      w[k] = (uint32_t)t;
      c = t >> 32;
    }
    n = m;
    if (c) w[n++] = (uint32_t)c;
  }
  __host__ __device__ void sub(const Big& b) {  // *this >= b
    int64_t c = 0;
    for (int k = 0; k < n; k++) {
      const int64_t t = (int64_t)w[k] - (k < b.n ? (int64_t)b.w[k] : 0) + c;
      w[k] = (uint32_t)t;
      c = t < 0 ? -1 : 0;
    }
    while (n > 0 && w[n - 1] == 0) n--;
  }
  __host__ __device__ static int cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int k = a.n - 1; k >= 0; k--)
      if (a.w[k] != b.w[k]) return a.w[k] < b.w[k] ? -1 : 1;
    return 0;
  }
};

// |v| > 0 finite -> digits d[0..len) and k: |v| ~ 0.d1 d2 .. dlen x 10^k
__host__ __device__ inline int shortest(double v, bool tie_even, uint8_t* d, int* kout) {
  uint64_t bits = (uint64_t)__builtin_bit_cast(int64_t, v) & 0x7FFFFFFFFFFFFFFFull;
  const int be = (int)(bits >> 52);
  const uint64_t fm = bits & 0xFFFFFFFFFFFFFull;
  const uint64_t f = be ? (fm | (1ull << 52)) : fm;
  const int e = be ? be - 1075 : -1074;
  const bool even = (f & 1) == 0;
  const bool asym = fm == 0 && be > 1;  // the gap below is half the gap above
  Big r, s, mp, mm;
  if (e >= 0) {
    r.set(f);
    r.shl(e + (asym ? 2 : 1));
    s.set(asym ? 4 : 2);
    mp.set(1);
    mp.shl(e + (asym ? 1 : 0));
    mm.set(1);
    mm.shl(e);
  } else {
    r.set(f);
    r.shl(asym ? 2 : 1);
    s.set(1);
    s.shl((asym ? 2 : 1) - e);
    mp.set(asym ? 2 : 1);
    mm.set(1);
  }
  // k estimate from floor(log2 v), then fixed up while the upper bound reaches 10^0
  int blen = 0;
  for (uint64_t t = f; t; t >>= 1) blen++;
  const int e2 = e + blen - 1;
  int k = (int)__builtin_ceil((double)e2 * 0.30102999566398114 - 1e-10);
  if (k >= 0) {
    s.mul_pow10(k);
  } else {
    r.mul_pow10(-k);
    mp.mul_pow10(-k);
    mm.mul_pow10(-k);
  }
  for (;;) {
    Big t = r;
    t.add(mp);
    const int c = Big::cmp(t, s);
    if (even ? c >= 0 : c > 0) {
      s.mul(10);
      k++;
    } else {
      break;
    }
  }
  int len = 0;
  for (;;) {
    r.mul(10);
    mp.mul(10);
    mm.mul(10);
    int dg = 0;
    while (Big::cmp(r, s) >= 0) {
      r.sub(s);
      dg++;
    }
    const int c1 = Big::cmp(r, mm);
    const bool tc1 = even ? c1 <= 0 : c1 < 0;
    Big t = r;
    t.add(mp);
    const int c2 = Big::cmp(t, s);
    const bool tc2 = even ? c2 >= 0 : c2 > 0;
    if (!tc1 && !tc2 && len < 17) {
      d[len++] = (uint8_t)dg;
      continue;
    }
    bool up;
    if (tc1 && tc2) {
      Big r2 = r;
      r2.shl(1);
      const int c = Big::cmp(r2, s);
      up = c > 0 || (c == 0 && (tie_even ? (dg & 1) != 0 : true));
    } else {
      up = tc2;
    }
    d[len++] = (uint8_t)(dg + (up ? 1 : 0));
    break;
  }
  *kout = k;
  return len;
}

// ryu format64 (serde_json Value::to_string of an f64); o == nullptr: length only
__host__ __device__ inline uint32_t ryu_format(double v, uint8_t* o) {
  uint32_t w = 0;
  auto put = [&](uint8_t c) {
    if (o) o[w] = c;
    w++;
  };
  if (__builtin_signbit(v)) put('-');
  if (v == 0.0) {
    put('0');
    put('.');
    put('0');
    return w;
  }
  uint8_t d[17];
  int kk;
  const int len = shortest(v, true, d, &kk);
  const int k = kk - len;  // v = digits x 10^k
  if (k >= 0 && kk <= 16) {
    for (int j = 0; j < len; j++) put((uint8_t)('0' + d[j]));
    for (int j = len; j < kk; j++) put('0');
    put('.');
    put('0');
  } else if (kk > 0 && kk <= 16) {
    for (int j = 0; j < len; j++) {
      if (j == kk) put('.');
      put((uint8_t)('0' + d[j]));
    }
  } else if (kk > -5 && kk <= 0) {
    put('0');
    put('.');
    for (int j = kk; j < 0; j++) put('0');
    for (int j = 0; j < len; j++) put((uint8_t)('0' + d[j]));
  } else {
    put((uint8_t)('0' + d[0]));
    if (len > 1) {
      put('.');
      for (int j = 1; j < len; j++) put((uint8_t)('0' + d[j]));
    }
    put('e');
    int x = kk - 1;
    if (x < 0) {
      put('-');
      x = -x;
    }
    if (x >= 100) put((uint8_t)('0' + x / 100));
    if (x >= 10) put((uint8_t)('0' + x / 10 % 10));
    put((uint8_t)('0' + x % 10));
  }
  return w;
}

// Rust `{}` of an f64 behind serde's WithDecimalPoint (".0" when no '.');
// o must hold 330 bytes
__host__ __device__ inline uint32_t display_with_point(double v, uint8_t* o) {
  uint32_t w = 0;
  if (__builtin_signbit(v)) o[w++] = '-';
  if (v == 0.0) {
    o[w++] = '0';
    o[w++] = '.';
    o[w++] = '0';
    return w;
  }
  uint8_t d[17];
  int kk;
  const int len = shortest(v, false, d, &kk);
  bool point = false;
  if (kk <= 0) {
    o[w++] = '0';
    o[w++] = '.';
    point = true;
    for (int j = kk; j < 0; j++) o[w++] = '0';
    for (int j = 0; j < len; j++) o[w++] = (uint8_t)('0' + d[j]);
  } else {
    for (int j = 0; j < len; j++) {
      if (j == kk) {
        o[w++] = '.';
        point = true;
      }
      o[w++] = (uint8_t)('0' + d[j]);
    }
    for (int j = len; j < kk; j++) o[w++] = '0';
  }
  if (!point) {
    o[w++] = '.';
    o[w++] = '0';
  }
  return w;
}

}  // namespace flt
}  // namespace fsg
