// fsg_runtime.cpp — host runtime of the MI355X SmartModule engine behind the C ABI
// (include/fsg.h).  C++ restatement of the fluvio-smartengine surface:
//
//   SmartEngine                  crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:26-41
//   SmartModuleChainBuilder      engine.rs:49-111 (+ create_transform, transforms/mod.rs:24-52)
//   SmartModuleChainInstance     engine.rs:118-218
//   SmartModuleChainMetrics      crates/fluvio-smartengine/src/engine/metrics.rs:6-41
//   SPU process_batch            crates/fluvio-spu/src/smartengine/batch.rs:41-142
//   FileBatchIterator framing    crates/fluvio-storage/src/iterators.rs:55-160
//
// The runtime owns device buffers and one HIP stream per chain instance, builds
// the chain descriptor (built-in GPU SmartModules selected at initialize()),
// frames ingested slices and launches the kernels of fsg_kernels.hip.  No record
// is transformed on the host: the only host-side record work is formatting the
// single SmartModuleTransformRuntimeError a call may return.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "fsg.h"
#include "fsg_device.h"
#include "fsg_json_dev.h"
#include "fsg_launch.h"
#include "fsg_regex.h"

using namespace fsg;

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
static thread_local std::string g_err;
static thread_local uint64_t g_store_mem[3];  // current, requested, max of the last FSG_E_STORE_MEMORY
static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
extern "C" int fsg_last_store_memory(uint64_t* current, uint64_t* requested, uint64_t* max) {
  if (current) *current = g_store_mem[0];
  if (requested) *requested = g_store_mem[1];
  if (max) *max = g_store_mem[2];
  return FSG_OK;
}
#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return fail(FSG_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

extern "C" const char* fsg_last_error_message(void) { return g_err.c_str(); }
extern "C" int fsg_abi_version(void) { return FSG_ABI_VERSION; }
extern "C" void fsg_free(void* p) { free(p); }

// ---------------------------------------------------------------------------
// small host helpers (config parsing / error formatting only)
// ---------------------------------------------------------------------------
namespace {

uint64_t rd_be(const uint8_t* p, int n) {
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 8) | p[i];
  return v;
}

// Rust from_utf8 (for config data and error hints)
bool utf8_ok(const uint8_t* s, size_t n, uint32_t* vut, uint32_t* elen) {
  size_t i = 0;
  while (i < n) {
    uint32_t f = s[i];
    if (f < 0x80) {
      i++;
      continue;
    }
    int w = (f >= 0xC2 && f <= 0xDF) ? 2 : (f >= 0xE0 && f <= 0xEF) ? 3 : (f >= 0xF0 && f <= 0xF4) ? 4 : 0;
    auto bad = [&](uint32_t l) {
      *vut = (uint32_t)i;
      *elen = l;
      return false;
    };
    if (w == 0) return bad(1);
    if (i + 1 >= n) return bad(0);
    uint32_t b1 = s[i + 1];
    if (w == 2) {
      if ((b1 & 0xC0) != 0x80) return bad(1);
      i += 2;
      continue;
    }
    bool ok1 = w == 3 ? ((f == 0xE0 && b1 >= 0xA0 && b1 <= 0xBF) || (f >= 0xE1 && f <= 0xEC && b1 >= 0x80 && b1 <= 0xBF) ||
                         (f == 0xED && b1 >= 0x80 && b1 <= 0x9F) || (f >= 0xEE && f <= 0xEF && b1 >= 0x80 && b1 <= 0xBF))
                      : ((f == 0xF0 && b1 >= 0x90 && b1 <= 0xBF) || (f >= 0xF1 && f <= 0xF3 && b1 >= 0x80 && b1 <= 0xBF) ||
                         (f == 0xF4 && b1 >= 0x80 && b1 <= 0x8F));
    if (!ok1) return bad(1);
    if (i + 2 >= n) return bad(0);
    if ((s[i + 2] & 0xC0) != 0x80) return bad(2);
    if (w == 3) {
      i += 3;
      continue;
    }
    if (i + 3 >= n) return bad(0);
    if ((s[i + 3] & 0xC0) != 0x80) return bad(3);
    i += 4;
  }
  return true;
}
std::string utf8_hint(uint32_t vut, uint32_t elen) {
  char b[96];
  if (elen)
    snprintf(b, sizeof b, "invalid utf-8 sequence of %u bytes from index %u", elen, vut);
  else
    snprintf(b, sizeof b, "incomplete utf-8 byte sequence from index %u", vut);
  return b;
}
const char* parse_hint(uint32_t kind) {
  switch (kind) {
    case 1: return "cannot parse integer from empty string";
    case 2: return "invalid digit found in string";
    case 3: return "number too large to fit in target type";
    default: return "number too small to fit in target type";
  }
}
bool is_ws(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || c == 0x20 || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}
// aggregate-sum's `acc.trim().parse::<i32>().unwrap_or(0)` on a valid UTF-8 accumulator
int32_t acc_value(const std::vector<uint8_t>& a) {
  std::vector<uint32_t> cps;
  std::vector<size_t> at;
  for (size_t i = 0; i < a.size();) {
    uint32_t f = a[i];
    int w = f < 0x80 ? 1 : f < 0xE0 ? 2 : f < 0xF0 ? 3 : 4;
    uint32_t cp = w == 1 ? f : w == 2 ? (f & 0x1F) : w == 3 ? (f & 0x0F) : (f & 0x07);
    for (int k = 1; k < w && i + k < a.size(); k++) cp = (cp << 6) | (a[i + k] & 0x3F);
    cps.push_back(cp);
    at.push_back(i);
    i += w;
  }
  size_t b = 0, e = cps.size();
  while (b < e && is_ws(cps[b])) b++;
  while (e > b && is_ws(cps[e - 1])) e--;
  const size_t bb = b < at.size() ? at[b] : a.size();
  const size_t eb = e < at.size() ? at[e] : a.size();
  if (bb >= eb) return 0;
  const uint8_t* s = a.data() + bb;
  size_t n = eb - bb, i = 0;
  bool pos = true;
  if ((s[0] == '+' || s[0] == '-') && n == 1) return 0;
  if (s[0] == '+')
    i = 1;
  else if (s[0] == '-') {
    pos = false;
    i = 1;
  }
  int64_t acc = 0;
  for (; i < n; i++) {
    if (s[i] < '0' || s[i] > '9') return 0;
    acc = pos ? acc * 10 + (s[i] - '0') : acc * 10 - (s[i] - '0');
    if (acc > 2147483647LL || acc < -2147483648LL) return 0;
  }
  return (int32_t)acc;
}

// aggregate-json's `serde_json::from_slice::<HashMap<String, u32>>(acc).unwrap_or_default()`
// (the accumulator side, host): a JSON object of strings -> u32, whitespace
// ' ' \t \n \r, string escapes decoded (UTF-8 validated), no sign / fraction /
// exponent / leading zero / overflow; anything else -> the empty map.  Keys in
// first-occurrence order, a duplicate key's last value wins.  `text` = the key
// as serde_json writes it (format_escaped_str).
struct AccMap {
  std::vector<std::string> keys, text;
  std::vector<uint32_t> vals;
  std::vector<uint32_t> seq;  // per entry in text order: its key's index, | kAjDup when the key came before
  bool dups = false;
};
// serde_json's deserialize_map calls the map visitor (which draws the map's
// RandomState) once the first non-whitespace byte is '{'
bool json_starts_map(const std::vector<uint8_t>& s) {
  size_t i = 0;
  while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
  return i < s.size() && s[i] == '{';
}
bool parse_acc_map(const std::vector<uint8_t>& s, AccMap& m) {
  size_t i = 0;
  const size_t n = s.size();
  auto ws = [&]() {
    while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++;
  };
  auto hex4 = [&](uint32_t& v) {
    if (i + 4 > n) return false;
    v = 0;
    for (int k = 0; k < 4; k++) {
      const uint8_t c = s[i++];
      const int h = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
      if (h < 0) return false;
      v = (v << 4) | (uint32_t)h;
    }
    return true;
  };
  auto put = [](std::string& o, uint32_t c) {
    if (c < 0x80) {
      o += (char)c;
    } else if (c < 0x800) {
      o += (char)(0xC0 | (c >> 6));
      o += (char)(0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      o += (char)(0xE0 | (c >> 12));
      o += (char)(0x80 | ((c >> 6) & 0x3F));
      o += (char)(0x80 | (c & 0x3F));
    } else {
      o += (char)(0xF0 | (c >> 18));
      o += (char)(0x80 | ((c >> 12) & 0x3F));
      o += (char)(0x80 | ((c >> 6) & 0x3F));
      o += (char)(0x80 | (c & 0x3F));
    }
  };
  auto str = [&](std::string& o) {  // after the opening quote
    const size_t raw0 = i;
    (void)raw0;
    for (;;) {
      if (i >= n) return false;
      const uint8_t c = s[i++];
      if (c == '"') break;
      if (c < 0x20) return false;
      if (c != '\\') {
        o += (char)c;
        continue;
      }
      if (i >= n) return false;
      const uint8_t e = s[i++];
      switch (e) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t c1;
          if (!hex4(c1)) return false;
          if (c1 >= 0xDC00 && c1 <= 0xDFFF) return false;
          if (c1 >= 0xD800 && c1 <= 0xDBFF) {
            uint32_t c2;
            if (i + 2 > n || s[i] != '\\' || s[i + 1] != 'u') return false;
            i += 2;
            if (!hex4(c2) || c2 < 0xDC00 || c2 > 0xDFFF) return false;
            c1 = (((c1 - 0xD800) << 10) | (c2 - 0xDC00)) + 0x10000;
          }
          put(o, c1);
          break;
        }
        default: return false;
      }
    }
    uint32_t vut = 0, el = 0;
    return utf8_ok((const uint8_t*)o.data(), o.size(), &vut, &el);
  };
  auto fail = [&]() {
    m = AccMap();
    return false;
  };
  ws();
  if (i >= n || s[i] != '{') return fail();
  i++;
  ws();
  if (i < n && s[i] == '}') {
    i++;
  } else {
    for (;;) {
      ws();
      if (i >= n || s[i] != '"') return fail();
      i++;
      std::string k;
      if (!str(k)) return fail();
      ws();
      if (i >= n || s[i] != ':') return fail();
      i++;
      ws();
      if (i >= n || s[i] < '0' || s[i] > '9') return fail();  // '-': negative or -0, both errors for u32
      uint64_t v = 0;
      const size_t d0 = i;
      while (i < n && s[i] >= '0' && s[i] <= '9') {
        v = v * 10 + (uint64_t)(s[i++] - '0');
        if (v > 0xFFFFFFFFull) return fail();
      }
      if (s[d0] == '0' && i - d0 > 1) return fail();  // leading zero
      if (i < n && (s[i] == '.' || s[i] == 'e' || s[i] == 'E')) return fail();  // a float: invalid type
      size_t at = 0;
      while (at < m.keys.size() && m.keys[at] != k) at++;
      if (at < m.keys.size()) {
        m.vals[at] = (uint32_t)v;
        m.seq.push_back((uint32_t)at | kAjDup);
        m.dups = true;
      } else {
        m.seq.push_back((uint32_t)m.keys.size());
        m.keys.push_back(k);
        m.vals.push_back((uint32_t)v);
      }
      ws();
      if (i < n && s[i] == ',') {
        i++;
        continue;
      }
      if (i < n && s[i] == '}') {
        i++;
        break;
      }
      return fail();
    }
  }
  ws();
  if (i != n) return fail();
  for (const auto& k : m.keys) {  // format_escaped_str (ser.rs)
    std::string t = "\"";
    for (unsigned char c : k) {
      switch (c) {
        case '"': t += "\\\""; break;
        case '\\': t += "\\\\"; break;
        case '\b': t += "\\b"; break;
        case '\f': t += "\\f"; break;
        case '\n': t += "\\n"; break;
        case '\r': t += "\\r"; break;
        case '\t': t += "\\t"; break;
        default:
          if (c < 0x20) {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", c);
            t += b;
          } else {
            t += (char)c;
          }
      }
    }
    t += "\"";
    m.text.push_back(t);
  }
  return true;
}


struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;  // owns p: no copies (a copy's destructor would free it)
  DevBuf& operator=(const DevBuf&) = delete;
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(cap, o.cap);
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t c = std::max<size_t>(n + n / 4, 4096);
    hipError_t e = hipMalloc(&p, c);
    if (e == hipSuccess) cap = c;
    return e;
  }
  template <typename T>
  T* as() const {
    return (T*)p;
  }
};

// page-locked host memory (hipHostMalloc): D2H straight from the DMA engine,
// no staging through HIP's pageable-copy path
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;  // coherent + mapped: kernels read / write it directly (k_one)
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, n, flags);
    if (e == hipSuccess) cap = n;
    return e;
  }
};

// Host-side wait for a stream: spin on hipStreamQuery for up to ~200 us (the
// one-record process() path's waits are tens of us, below the blocking
// wait's wake-up latency), then block.
hipError_t wait_stream(hipStream_t st) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    hipError_t e = hipStreamQuery(st);
    if (e != hipErrorNotReady) return e;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
  }
  return hipStreamSynchronize(st);
}

struct ModuleSpec {
  std::vector<uint8_t> bytes;
  std::map<std::string, std::string> params;  // SmartModuleExtraParams (BTreeMap)
  int16_t version = 22;                       // DEFAULT_SMARTENGINE_VERSION
  bool has_acc = false;
  std::vector<uint8_t> acc;
  int32_t lb_kind = FSG_LOOKBACK_NONE;        // SmartModuleConfig.lookback
  uint64_t lb_last = 0, lb_age_ms = 0;
};

// state of a stateful last stage, shared by the chain and its look_back-mode twin
struct SfState {
  uint64_t limit = 0xFFFFFFFEull;  // filter_hashset: usize::MAX - 1 (wasm32)
  uint64_t n_ent = 0, arena_len = 0, n = 0;
  DevBuf prev;                     // filter_look_back: PREV (i32)
  DevBuf ent_hash, ent_pos, ent_len, ent_last, arena;
};

}  // namespace

// ---------------------------------------------------------------------------
// objects
// ---------------------------------------------------------------------------
struct fsg_engine {
  int device = 0;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  hipStream_t coll = nullptr;  // collective stream (state merges)
  // aggregate-json group walks (AjGroup): created on the first group call that
  // walks and kept (a stream create + destroy per call cost ~3 ms of host time)
  std::mutex gmu;              // one group call at a time uses them
  hipStream_t gst = nullptr;
  hipEvent_t gdone = nullptr, gt0 = nullptr, gt1 = nullptr;
  void* gdlist = nullptr;
  size_t gdcap = 0;
  // the aggregate-sum group path (group_agg_fast): jobs + offsets in HBM and
  // their pinned host image, the read-back rows, phase events
  DevBuf ga_dev;
  PinBuf ga_pin;
  hipEvent_t ga_ev[5] = {};
};

struct fsg_chain_builder {
  std::vector<ModuleSpec> mods;
  size_t limit = 1000000000;  // DEFAULT_STORE_MEMORY_LIMIT (engine.rs:24)
};

struct fsg_slice {
  fsg_engine* eng = nullptr;
  DevBuf data, bpos, rbase;
  size_t len = 0;
  uint32_t nb = 0;
  uint64_t nrec = 0;
  int tail_status = 0;
  uint64_t header_bytes = 0;  // 57 B per framed batch + the record sections
  bool device_framed = false; // framed by k_frame_* (else by the host walk)
  bool decompressed = false;  // compressed sections were decompressed on the GPU at ingest
  // record starts / ends per batch (k_chase_w) for k_eval_int, computed on first
  // use and kept while the slice is unchanged (every framing resets rs_ok)
  mutable std::mutex rs_mu;
  mutable DevBuf rs_start, rs_end;
  mutable hipEvent_t rs_ev = nullptr;  // recorded after the framing: another stream waits for it
  mutable bool rs_ok = false;
  // CRC32C verify of the stored (compressed) batches, run before decompression
  uint64_t crc_bad = 0;
  int64_t crc_first = -1;
  float crc_ms = 0;
  std::vector<uint64_t> hbpos, hrbase;  // host framing (kept: the H2D copies may still be reading them)
  size_t dec_limit = 1000000000;  // largest decompressed batch (the store limit, engine.rs:24)
  // a chain segment's output (composed chains): batches whose records pass
  // through the later segments unchanged (the partial output before an error)
  DevBuf pass;
  bool has_pass = false;
  // framing / decompression scratch, grown and kept across uploads into this
  // slice (hipFree synchronises the whole device)
  DevBuf fr[12], dec[8];
  // fsg_slice_verify_crc: its stream, events and result word, kept across calls
  // (a per-call hipMalloc / hipFree of the word synchronised the device)
  mutable DevBuf vbad;
  mutable hipStream_t vst = nullptr;
  mutable hipEvent_t vev[2] = {};
  // fsg_slice_verify_crc_start: a verify in flight on vst (its result lands in
  // the pinned words vres); anything that rewrites the batch table or the
  // bytes waits for it first (verify_drain)
  mutable unsigned long long* vres = nullptr;
  mutable bool v_pending = false;
  void verify_drain() const {
    if (v_pending) (void)hipStreamSynchronize(vst);
  }
  ~fsg_slice() {
    verify_drain();
    if (vres) (void)hipHostFree(vres);
    if (rs_ev) (void)hipEventDestroy(rs_ev);
    for (auto& e : vev)
      if (e) (void)hipEventDestroy(e);
    if (vst) (void)hipStreamDestroy(vst);
  }
};

constexpr size_t kPinPlan = 256;           // pinned block: Plan, then the small output
constexpr size_t kSmallOut = 1u << 20;    // outputs up to 1 MiB come back through it

// The chains of one fsg_chain_group_process_slices call (the partitions a
// rank owns) meet once per call at aggregate-json's order pass: a walk over a
// chain's records in stream order is one workgroup's work, so the group runs
// every chain's walk in ONE launch (k_aggj_order_group) instead of one small
// launch per chain serialised on the device's few hardware queues.  Each chain
// arrives exactly once: with its walk, or empty (no aggregate-json records,
// an earlier error, a composed chain).
struct AjGroup {
  std::mutex mu;
  std::condition_variable cv;
  size_t expected = 0, arrived = 0;
  bool launched = false;
  int rc = FSG_OK;
  std::vector<AggjArgs> jobs;
  std::vector<hipEvent_t> ready;  // per job: its chain's hashes are done
  int device = 0;
  fsg_engine* eng = nullptr;  // owns the stream, events and job list below
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  hipEvent_t t0 = nullptr, t1 = nullptr;  // the walk's own duration (timed chains)
  bool timed = false;
  ~AjGroup() {
    for (auto e : ready) (void)hipEventDestroy(e);
  }
};

struct fsg_chain {
  fsg_engine* eng = nullptr;
  hipStream_t stream = nullptr;
  size_t limit = 0;
  ChainDesc hdesc{};
  std::vector<uint8_t> hblob;
  DevBuf d_desc, d_blob;
  // ingest staging of process_batch / process: reused across calls, so a call
  // pays no hipMalloc/hipFree (hipFree synchronises the device)
  fsg_slice ingest;
  std::vector<std::string> names;
  int agg_stage = -1;
  int array_stage = -1;
  std::vector<uint8_t> acc;  // aggregate accumulator bytes (SmartModuleAggregate.accumulator)
  // scratch
  DevBuf bstat, kept, rows, pre, aggpre, tiles, grand, mins, plan, out, crcparts, defer, elem, cat;
  DevBuf arr_b, arr_bm;  // lean array_map statistics and element bitmaps (per batch)
  DevBuf fbm;            // flat substring path: occurrence / high-byte bits per 16-byte chunk
  bool no_flat = getenv("FSG_NO_FLAT") != nullptr;  // A/B: the flat path off (k_eval_lean instead)
  bool no_fjson = getenv("FSG_NO_FJSON") != nullptr;  // A/B: the flat JSON path off (k_eval_lean instead)
  bool no_frx = getenv("FSG_NO_FRX") != nullptr;      // A/B: the flat regex path off (k_eval_lean instead)
  // the flat regex path for slices of records averaging at least this many
  // bytes: its per-record framing walk re-reads a line per record, which for
  // short records costs more than k_eval_lean's batch windows (C1, 256-B
  // records: k_rx_scan 0.56 + k_rx_decide 0.82 ms against k_chase +
  // k_eval_lean's 1.33 ms on MI355X)
  uint64_t frx_min_rec = getenv("FSG_FRX_MIN_REC") ? strtoull(getenv("FSG_FRX_MIN_REC"), nullptr, 10) : 512;
  bool no_int = getenv("FSG_NO_INT") != nullptr;    // A/B: integer chains through k_eval alone
  // the one-batch process() path (k_one): zeros for bpos / rbase, the device
  // block Plan | BatchStat | Mins | output batch, and coherent pinned memory
  // the kernel reads the input from and writes the block back to (no copies)
  DevBuf one_meta, one_blk;
  PinBuf one_pin;
  uint32_t one_seq = 0;  // k_one completion flag values
  void* one_dev = nullptr;        // one_pin's device address
  void* one_dev_for = nullptr;    // ... for this host allocation
  DevBuf dstate;  // aggregate-sum accumulator (i32) after the last call, in HBM
  // aggregate-json: key dictionary, index, initial keys, per-batch accumulator text
  DevBuf aj_tptr, aj_tlen, aj_kup, aj_out, aj_accoff, aj_acclen;  // aggregate-json
  DevBuf aj_bcnt, aj_brec, aj_rdesc, aj_rne, aj_rent, aj_rnew, aj_rnewb, aj_rlen, aj_roff, aj_ekid, aj_eval;
  DevBuf aj_sref, aj_sid, aj_state, aj_state2, aj_tsum;
  // the aggregate-json map between calls, in HBM (fsg_keyed.hip k_ajc_*):
  // ajs[aj_cur] holds it, the commit after a call writes the other buffer
  struct AjBuf {
    DevBuf arena, kptr, klen, tptr, tlen, val, blen, boff;
  } ajs[2];
  int aj_cur = 0;
  bool aj_dev = false;      // the state lives in ajs[aj_cur] (the initial accumulator was parsed once)
  bool aj_touched = false;  // a record was folded: the accumulator is the map's text, not c->acc
  uint32_t aj_K = 0;        // keys in the state (in the order the accumulator text lists them)
  // the guest's RandomState sequence (fsg_keyed.hip k_aggj_order): the k0 the
  // next map draws, and whether the initial accumulator draws twice (it starts
  // with '{' but does not parse: the visitor's map, then HashMap::default())
  uint64_t aj_k0 = 1;
  bool aj_e0 = false;
  DevBuf aj_iseq;           // the initial accumulator's entries with repeats (AggjArgs::iseq)
  uint32_t aj_n_iseq = 0;   // 0: no repeated key (ids in order)
  DevBuf aj_nkr, aj_koff, aj_ord, aj_hrec, aj_oscr, aj_inv;
  AjGroup* group = nullptr;  // set during a group call (fsg_chain_group_process_slices)
  bool group_arrived = false;
  uint64_t aj_bytes = 0;    // its arena bytes
  DevBuf aj_cout;           // commit scalars
  hipEvent_t kd_ev[2] = {}; // keyed collect: chain stream -> collect stream -> chain stream
  // Composed chains (stages after an array_map, an aggregate or a stateful
  // filter): the chain runs as segments, each ending at such a stage; segment
  // k's per-batch output is segment k + 1's input slice (seg_io[k]).
  std::vector<std::unique_ptr<fsg_chain>> segs;
  std::vector<uint32_t> seg_stage0;  // global index of each segment's first stage
  std::unique_ptr<fsg_slice[]> seg_io;
  // what a segment run leaves for its deferred state commit
  PlanArgs last_pa{};
  SfArgs last_sfa{};
  AggjArgs last_aj{};
  uint32_t last_aj_kmax = 0;
  bool last_has_aggj = false;
  DevBuf rstart, rend;  // k_chase (lean path record starts)
  // stateful last stage (filter_look_back / filter_hashset)
  int sf_stage = -1;
  std::shared_ptr<SfState> sf;
  fsg_lookback lookback{FSG_LOOKBACK_NONE, 0, 0, 0};
  std::unique_ptr<fsg_chain> lbc;  // the stage in look_back mode (same state)
  DevBuf sf_bval, sf_bpre, sf_bn, sf_hv, sf_vref, sf_vlen, sf_slot, sf_keep, sf_idx, sf_sref, sf_first, sf_cur,
      sf_scal;
  Plan hplan{};
  // pinned: the plan read-back and, for outputs up to kSmallOut, the output
  // batch itself (copied on the stream before run_slice's last wait)
  PinBuf hpin;
  bool out_pinned = false;
  bool timed = true;  // per-phase kernel timings (events); off for the one-record process()
  // large-output download: two pinned chunks, DMA of one overlapping the host copy of the other
  PinBuf hstage;
  hipEvent_t dl_ev[2] = {};
  hipEvent_t ev[6] = {};
  hipEvent_t ev_order[2] = {};  // around a solo aggregate-json order walk
  fsg_timings last{};
  size_t out_len = 0;
  // pipelined process_batch (process_pipelined): the host slice uploaded in
  // pieces into pipe_in while chunks of it are processed; chunk outputs
  // alternate between out and pipe_out, downloaded on pipe_dl beside the next
  // chunk's processing
  DevBuf pipe_in, pipe_out;
  fsg_slice pipe_chunk;
  PinBuf pipe_pin;
  hipStream_t pipe_upv[4] = {}, pipe_dl = nullptr;
  int pipe_up_threads = getenv("FSG_PIPE_UP") ? std::max(1, std::min(4, atoi(getenv("FSG_PIPE_UP")))) : 1;
  hipEvent_t pipe_ev[2] = {};
  bool no_pipe = getenv("FSG_NO_PIPE") != nullptr;  // A/B: the serial H2D -> process -> D2H path
  size_t pipe_bytes = getenv("FSG_PIPE_CHUNK") ? strtoull(getenv("FSG_PIPE_CHUNK"), nullptr, 10) : (size_t)128 << 20;
  ~fsg_chain() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : ev_order)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : dl_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : kd_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : pipe_ev)
      if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
    for (auto& u : pipe_upv)
      if (u) (void)hipStreamDestroy(u);
    if (pipe_dl) (void)hipStreamDestroy(pipe_dl);
  }
};

// ---------------------------------------------------------------------------
// engine
// ---------------------------------------------------------------------------
extern "C" int fsg_device_count(int* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return FSG_OK;
}

static std::atomic<int> g_engines{0};  // live engines: the last fsg_engine_free drains the host pool

extern "C" int fsg_engine_new(int device, fsg_engine** out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(FSG_E_DEVICE, "no HIP device available");
  if (device < 0 || device >= n) return fail(FSG_E_INVALID_ARG, "device index out of range");
  HIPCHK(hipSetDevice(device));
  HIPCHK(upload_crc_tables());
  hipStream_t coll = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&coll, hipStreamNonBlocking));
  auto* e = new fsg_engine();
  e->device = device;
  e->coll = coll;
  g_engines.fetch_add(1);
  *out = e;
  return FSG_OK;
}

extern "C" void fsg_engine_free(fsg_engine* e) {
  if (!e) return;
  if (e->comm) ncclCommDestroy(e->comm);
  if (e->coll) (void)hipStreamDestroy(e->coll);
  if (e->gst) (void)hipStreamDestroy(e->gst);
  if (e->gdone) (void)hipEventDestroy(e->gdone);
  if (e->gt0) (void)hipEventDestroy(e->gt0);
  if (e->gt1) (void)hipEventDestroy(e->gt1);
  if (e->gdlist) (void)hipFree(e->gdlist);
  delete e;
  if (g_engines.fetch_sub(1) == 1) fsg_host_cache_trim();
}

// ---------------------------------------------------------------------------
// builder
// ---------------------------------------------------------------------------
extern "C" int fsg_chain_builder_new(fsg_chain_builder** out) {
  *out = new fsg_chain_builder();
  return FSG_OK;
}
extern "C" void fsg_chain_builder_free(fsg_chain_builder* b) { delete b; }
extern "C" int fsg_chain_builder_set_store_memory_limit(fsg_chain_builder* b, size_t max_memory_bytes) {
  b->limit = max_memory_bytes;
  return FSG_OK;
}
extern "C" int fsg_chain_builder_add_smart_module(fsg_chain_builder* b, const fsg_param* params, size_t n_params,
                                                  int16_t version, const uint8_t* initial_acc, size_t acc_len,
                                                  int32_t has_initial_acc, const uint8_t* module, size_t module_len) {
  ModuleSpec m;
  m.bytes.assign(module, module + module_len);
  for (size_t i = 0; i < n_params; i++) m.params[params[i].key] = params[i].value;  // BTreeMap insert
  m.version = version;
  m.has_acc = has_initial_acc != 0;
  if (m.has_acc) m.acc.assign(initial_acc, initial_acc + acc_len);
  b->mods.push_back(std::move(m));
  return FSG_OK;
}

extern "C" int fsg_chain_builder_set_lookback(fsg_chain_builder* b, size_t module_index, int32_t kind, uint64_t last,
                                              uint64_t age_ms) {
  if (module_index >= b->mods.size()) return fail(FSG_E_INVALID_ARG, "no such module");
  if (kind < FSG_LOOKBACK_NONE || kind > FSG_LOOKBACK_AGE) return fail(FSG_E_INVALID_ARG, "bad lookback kind");
  ModuleSpec& m = b->mods[module_index];
  m.lb_kind = kind;
  m.lb_last = last;
  m.lb_age_ms = age_ms;
  return FSG_OK;
}

namespace {
std::string init_error(const std::string& what) { return what + "\n\nSmartModule Init Error: \n"; }

// one reference SmartModule -> one GPU stage (chain-build-time selection)
int add_stage(fsg_chain* c, const ModuleSpec& m, const std::string& name, uint8_t& vt) {
  if (c->hdesc.nstages >= (uint32_t)kMaxStages) return fail(FSG_E_UNSUPPORTED, "chain longer than 8 stages");
  if (c->agg_stage >= 0) return fail(FSG_E_UNSUPPORTED, "stages after an aggregate are not implemented on the GPU");
  if (c->array_stage >= 0) return fail(FSG_E_UNSUPPORTED, "stages after an array_map are not implemented on the GPU");
  if (c->sf_stage >= 0)
    return fail(FSG_E_UNSUPPORTED, "stages after a stateful filter (look_back) are not implemented on the GPU");
  StageDesc sd{};
  sd.in_type = vt;
  auto param = [&](const char* k) -> const std::string* {
    auto it = m.params.find(k);
    return it == m.params.end() ? nullptr : &it->second;
  };
  auto put_blob = [&](const void* p, size_t n) {
    uint32_t off = (uint32_t)c->hblob.size();
    c->hblob.insert(c->hblob.end(), (const uint8_t*)p, (const uint8_t*)p + n);
    while (c->hblob.size() % 16) c->hblob.push_back(0);
    return off;
  };
  if (name == "filter" || name == "filter_init" || name == "filter_with_param") {
    std::string needle = "a";  // examples/filter: contains('a')
    if (name != "filter") {
      const std::string* k = param("key");
      if (!k && name == "filter_init") return fail(FSG_E_INIT, init_error("Missing param key"));
      if (k) needle = *k;
    }
    sd.op = OP_CONTAINS;
    sd.kind = FSG_KIND_FILTER;
    sd.needle = put_blob(needle.data(), needle.size());
    sd.needle_len = (uint32_t)needle.size();
  } else if (name == "regex-filter" || name == "filter_regex") {
    std::string pat;
    if (name == "regex-filter") {
      const std::string* r = param("regex");
      if (!r) return fail(FSG_E_INIT, init_error("Missing param regex"));
      pat = *r;
      sd.keep_match = 1;
    } else {
      pat = "\\d{3}-\\d{2}-\\d{4}";  // examples/filter_regex: keep records without an SSN
      sd.keep_match = 0;
    }
    Dfa d, fd;
    std::string msg;
    int rc = compile_regex(pat, d, fd, msg);
    if (rc == -2) return fail(FSG_E_INIT, init_error(msg));
    if (rc) return fail(rc, msg);
    sd.op = OP_REGEX;
    sd.kind = FSG_KIND_FILTER;
    sd.dfa.nstates = d.nstates;
    sd.dfa.nclasses = d.nclasses;
    sd.dfa.s_bot = d.s_bot;
    sd.dfa.s_mid = d.s_mid;
    sd.dfa.max_len = d.max_len;
    sd.dfa.unicode_word = d.unicode_word;
    sd.dfa.classmap = put_blob(d.classmap.data(), 256);
    sd.dfa.classmap_up = put_blob(d.classmap_up.data(), 256);
    std::vector<uint8_t> t8(d.trans.begin(), d.trans.end());
    sd.dfa.trans = put_blob(t8.data(), t8.size());
    std::vector<uint8_t> acc(256, 0);
    std::copy(d.accept.begin(), d.accept.end(), acc.begin());
    sd.dfa.accept = put_blob(acc.data(), 256);
    sd.dfa.f_nstates = fd.nstates;
    sd.dfa.f_nclasses = fd.nclasses;
    sd.dfa.f_s_bot = fd.s_bot;
    sd.dfa.f_classmap = put_blob(fd.classmap.data(), 256);
    sd.dfa.f_classmap_up = put_blob(fd.classmap_up.data(), 256);
    sd.dfa.f_trans = put_blob(fd.trans.data(), fd.trans.size() * 2);
    sd.dfa.f_accept = put_blob(fd.accept.data(), fd.accept.size());
    if (fd.marked) {  // Unicode word boundaries: the marked walk classifies each code point with \w
      sd.dfa.f_marked = 1;
      const std::vector<uint32_t> wt = unicode_word_ranges();
      sd.dfa.wtab = put_blob(wt.data(), wt.size() * 4);
      sd.dfa.wtab_n = (uint32_t)(wt.size() / 2);
    }
    if (d.utab) {  // regex-syntax 0.6.27 / 0.7.1 tables differ from this build's on these
      const std::vector<uint32_t> vt = unicode_newer_ranges();
      sd.dfa.vtab = put_blob(vt.data(), vt.size() * 4);
      sd.dfa.vtab_n = (uint32_t)(vt.size() / 2);
    }
    if (d.nstates <= 16) {  // the lean kernel's byte-row tables (fsg_device.h DfaDesc)
      std::vector<uint64_t> tt(256, 0), ttu(256, 0);
      for (uint32_t b = 0; b < 256; b++)
        for (uint32_t st = 0; st < d.nstates; st++) {
          tt[b] |= (uint64_t)d.trans[st * d.nclasses + d.classmap[b]] << (4 * st);
          ttu[b] |= (uint64_t)d.trans[st * d.nclasses + d.classmap_up[b]] << (4 * st);
        }
      sd.dfa.tt = put_blob(tt.data(), tt.size() * 8);
      sd.dfa.tt_up = put_blob(ttu.data(), ttu.size() * 8);
      for (uint32_t st = 0; st < d.nstates; st++) {
        if (d.accept[st] & 1) sd.dfa.acc1 |= 1u << st;
        if (d.accept[st] & 2) sd.dfa.acc2 |= 1u << st;
      }
      sd.dfa.lean = d.max_len >= 0 ? 1 : 0;
    }
  } else if (name == "filter_json") {  // examples/filter_json: StructuredLog.level > Debug
    sd.op = OP_FILTER_JSON;
    sd.kind = FSG_KIND_FILTER;
  } else if (name == "filter_odd") {
    sd.op = OP_FILTER_ODD;
    sd.kind = FSG_KIND_FILTER;
  } else if (name == "map") {
    sd.op = OP_MAP_UPPER;
    sd.kind = FSG_KIND_MAP;
    if (vt == VT_SRC) vt = VT_SRC_UPPER;
  } else if (name == "map_double") {
    sd.op = OP_MAP_DOUBLE;
    sd.kind = FSG_KIND_MAP;
    vt = VT_I32;
  } else if (name == "filter_map") {
    sd.op = OP_FILTER_MAP;
    sd.kind = FSG_KIND_FILTER_MAP;
    vt = VT_I32;
  } else if (name == "aggregate-sum") {
    sd.op = OP_AGG_SUM;
    sd.kind = FSG_KIND_AGGREGATE;
    c->agg_stage = (int)c->hdesc.nstages;
    c->acc = m.has_acc ? m.acc : std::vector<uint8_t>();
    vt = VT_I32;
  } else if (name == "aggregate") {  // examples/aggregate: acc.push_str(from_utf8(value)?)
    sd.op = OP_AGG_CONCAT;
    sd.kind = FSG_KIND_AGGREGATE;
    c->agg_stage = (int)c->hdesc.nstages;
    c->acc = m.has_acc ? m.acc : std::vector<uint8_t>();
  } else if (name == "aggregate-json") {  // examples/aggregate-json: HashMap<String, u32> += per key (C5 keyed)
    sd.op = OP_AGG_JSON;
    sd.kind = FSG_KIND_AGGREGATE;
    c->agg_stage = (int)c->hdesc.nstages;
    c->acc = m.has_acc ? m.acc : std::vector<uint8_t>();
    vt = VT_SRC;  // the output value is the map's JSON text
  } else if (name == "map_json_project") {  // C3 field projection (parity unpinned: no reference module)
    const std::string* f = param("field");
    const std::string field = f ? *f : std::string("message");
    sd.op = OP_PROJECT;
    sd.kind = FSG_KIND_FILTER_MAP;
    sd.needle = put_blob(field.data(), field.size());
    sd.needle_len = (uint32_t)field.size();
    if (vt == VT_I32) vt = VT_SRC;  // the text of an integer is parsed (always an error)
  } else if (name == "array_map_json_array") {  // examples/array_map_json_array: explode a JSON array
    sd.op = OP_ARRAY_MAP;
    sd.kind = FSG_KIND_ARRAY_MAP;
    c->array_stage = (int)c->hdesc.nstages;
  } else if (name == "filter_look_back" || name == "filter_hashset") {
    // examples/filter_look_back (keep > PREV) / filter_hashset (dedup, BoundedHashSet)
    auto st = std::make_shared<SfState>();
    if (name == "filter_hashset") {
      const std::string* cnt = param("count");  // init: count.parse::<usize>()? (usize = u32 on wasm32)
      if (cnt) {
        const std::string& t = *cnt;
        size_t i = (!t.empty() && t[0] == '+') ? 1 : 0;
        uint64_t v = 0;
        uint32_t kind = t.empty() ? 1 : (i == t.size() ? 2 : 0);
        for (; !kind && i < t.size(); i++) {
          if (t[i] < '0' || t[i] > '9') kind = 2;
          else if ((v = v * 10 + (uint64_t)(t[i] - '0')) > 0xFFFFFFFFull) kind = 3;
        }
        if (kind) return fail(FSG_E_INIT, init_error(parse_hint(kind)));
        st->limit = v;
      }
      if (vt == VT_I32) return fail(FSG_E_UNSUPPORTED, "filter_hashset after an integer map is not implemented on the GPU");
      sd.op = OP_DEDUP;
    } else {
      sd.op = OP_LB_MAX;
    }
    sd.kind = FSG_KIND_FILTER;
    c->sf_stage = (int)c->hdesc.nstages;
    c->sf = st;
    c->lookback.kind = m.lb_kind;
    c->lookback.stage = c->hdesc.nstages;
    c->lookback.last = m.lb_last;
    c->lookback.age_ms = m.lb_age_ms;
  } else {
    return fail(FSG_E_UNKNOWN_SM, "No valid smartmodule found");
  }
  c->hdesc.st[c->hdesc.nstages++] = sd;
  c->names.push_back(name);
  return FSG_OK;
}
}  // namespace

namespace {
std::string builtin_name(const ModuleSpec& m) {
  const auto& by = m.bytes;
  if (by.size() < 4 || memcmp(by.data(), "\0fsg", 4)) return std::string();
  return std::string(by.begin() + 4, by.end());
}
// stages whose output is the input of a new segment when more stages follow
bool seg_boundary(const ModuleSpec& m) {
  const std::string name = builtin_name(m);
  return name == "array_map_json_array" || name == "aggregate-sum" || name == "aggregate" ||
         name == "aggregate-json" || name == "filter_look_back" || name == "filter_hashset";
}
// the segment ends of a chain: after every seg_boundary stage that has a
// successor, and before a filter_hashset whose input is an integer stage's
// output (map_double / filter_map: the dedup set holds the records' text, so
// that segment's output is materialized as the text records the reference's
// next stage receives, engine.rs:147-167)
std::vector<size_t> seg_ends(const std::vector<ModuleSpec>& mods) {
  std::vector<size_t> ends;
  bool int_out = false;  // the value after stage i is an i32 (VT_I32)
  for (size_t i = 0; i + 1 < mods.size(); i++) {
    const std::string name = builtin_name(mods[i]);
    if (name == "map_double" || name == "filter_map") int_out = true;
    if (seg_boundary(mods[i])) {
      ends.push_back(i);
      int_out = false;
    } else if (int_out && builtin_name(mods[i + 1]) == "filter_hashset") {
      ends.push_back(i);
      int_out = false;
    }
  }
  return ends;
}
}  // namespace

extern "C" int fsg_chain_builder_initialize(fsg_chain_builder* b, fsg_engine* e, fsg_chain** out) {
  std::unique_ptr<fsg_chain_builder> own(b);
  if (!e) return fail(FSG_E_INVALID_ARG, "null engine");
  HIPCHK(hipSetDevice(e->device));
  {  // a stage after an array_map / aggregate / stateful filter: a composed chain of segments
    std::vector<size_t> ends = seg_ends(b->mods);
    if (!ends.empty()) {
      ends.push_back(b->mods.size() - 1);
      auto c = std::make_unique<fsg_chain>();
      c->eng = e;
      c->limit = b->limit;
      size_t a0 = 0;
      for (size_t ei : ends) {
        auto* sb = new fsg_chain_builder();
        sb->limit = b->limit;
        sb->mods.assign(b->mods.begin() + a0, b->mods.begin() + ei + 1);
        fsg_chain* g = nullptr;
        int rc = fsg_chain_builder_initialize(sb, e, &g);  // takes sb
        if (rc) return rc;
        c->seg_stage0.push_back((uint32_t)a0);
        for (auto& nm : g->names) c->names.push_back(nm);
        c->segs.emplace_back(g);
        a0 = ei + 1;
      }
      c->hdesc.nstages = (uint32_t)b->mods.size();
      HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
      for (auto& ev : c->ev) HIPCHK(hipEventCreate(&ev));
      *out = c.release();
      return FSG_OK;
    }
  }
  auto c = std::make_unique<fsg_chain>();
  c->eng = e;
  c->limit = b->limit;
  uint8_t vt = VT_SRC;
  for (auto& m : b->mods) {
    const auto& by = m.bytes;
    if (by.size() >= 4 && !memcmp(by.data(), "\0asm", 4))
      return fail(FSG_E_UNKNOWN_SM, "No valid smartmodule found (wasm modules do not run on the GPU engine)");
    if (by.size() < 4 || memcmp(by.data(), "\0fsg", 4))
      return fail(FSG_E_INSTANTIATE, "Failed to instantiate: module bytes are neither wasm nor a GPU built-in descriptor");
    std::string name(by.begin() + 4, by.end());
    int rc = add_stage(c.get(), m, name, vt);
    if (rc) return rc;
  }
  c->hdesc.out_type = vt;
  c->hdesc.has_agg = c->agg_stage >= 0;
  if (c->agg_stage >= 0)
    c->hdesc.flags |= c->hdesc.st[c->agg_stage].op == OP_AGG_SUM    ? CF_AGG_SUM
                      : c->hdesc.st[c->agg_stage].op == OP_AGG_JSON ? CF_AGG_JSON
                                                                     : CF_AGG_CAT;
  if (c->array_stage >= 0) c->hdesc.flags |= CF_ARRAY;
  if (c->sf_stage >= 0) c->hdesc.flags |= CF_STATEFUL;
  if (c->agg_stage >= 0) {
    StageDesc& sd = c->hdesc.st[c->agg_stage];
    uint32_t vut = 0, el = 0;
    sd.acc_bad = !utf8_ok(c->acc.data(), c->acc.size(), &vut, &el);
    sd.acc_vut = vut;
    sd.acc_elen = el;
  }
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (auto& ev : c->ev) HIPCHK(hipEventCreate(&ev));
  if (c->hdesc.flags & CF_AGG_JSON)
    for (auto& ev : c->ev_order) HIPCHK(hipEventCreate(&ev));
  HIPCHK(c->d_desc.ensure(sizeof(ChainDesc)));
  HIPCHK(hipMemcpy(c->d_desc.p, &c->hdesc, sizeof(ChainDesc), hipMemcpyHostToDevice));
  if (c->hblob.empty()) c->hblob.resize(16, 0);
  HIPCHK(c->d_blob.ensure(c->hblob.size()));
  HIPCHK(hipMemcpy(c->d_blob.p, c->hblob.data(), c->hblob.size(), hipMemcpyHostToDevice));
  if (c->sf) {  // filter_look_back: PREV starts at 0 (static AtomicI32::new(0))
    HIPCHK(c->sf->prev.ensure(sizeof(int32_t)));
    HIPCHK(hipMemset(c->sf->prev.p, 0, sizeof(int32_t)));
  }
  if (c->hdesc.flags & CF_AGG_SUM) {  // the accumulator's i32 value, resident in HBM
    HIPCHK(c->dstate.ensure(sizeof(int32_t)));
    const int32_t a0 = acc_value(c->acc);
    HIPCHK(hipMemcpy(c->dstate.p, &a0, sizeof a0, hipMemcpyHostToDevice));
  }
  *out = c.release();
  return FSG_OK;
}

extern "C" void fsg_chain_free(fsg_chain* c) { delete c; }

// ---------------------------------------------------------------------------
// slices (ingest)
// ---------------------------------------------------------------------------
namespace {
// FileBatchIterator framing (iterators.rs:55-160): header -> batch_len -> record section
int frame(const uint8_t* s, size_t len, std::vector<uint64_t>& bpos, std::vector<uint64_t>& rbase, uint64_t& nrec,
          int& tail, uint64_t& hdr_bytes, std::vector<uint8_t>* codecs = nullptr) {
  size_t pos = 0;
  nrec = 0;
  tail = 0;
  hdr_bytes = 0;
  while (pos < len) {
    if (len - pos < 57) {
      tail = FSG_E_IO;  // "not enough for batch header"
      break;
    }
    const int32_t batch_len = (int32_t)rd_be(s + pos + 8, 4);
    const int16_t attrs = (int16_t)rd_be(s + pos + 21, 2);
    if (batch_len < 45) {
      tail = FSG_E_IO;
      break;
    }
    const size_t rem = (size_t)batch_len - 45;
    if (len - pos - 57 < rem) {
      tail = FSG_E_IO;  // "not enough for batch records"
      break;
    }
    const int comp = attrs & 7;
    // gzip / snappy / lz4 / zstd sections are decompressed on the GPU after
    // framing (decompress_slice); codes > 4 are the iterator's "unknown
    // compression value" io::Error
    if (comp > 4 || (comp != 0 && !codecs)) {
      tail = comp <= 4 ? FSG_E_UNSUPPORTED : FSG_E_IO;
      break;
    }
    if (codecs) codecs->push_back((uint8_t)comp);
    uint64_t cnt = 0;
    if (rem >= 4 && comp == 0) {
      int32_t c = (int32_t)rd_be(s + pos + 57, 4);
      cnt = c > 0 ? (uint64_t)c : 0;
      cnt = std::min<uint64_t>(cnt, (rem - 4) / 7);  // a record is at least 7 bytes
    }
    bpos.push_back(pos);
    rbase.push_back(nrec);
    nrec += cnt;
    hdr_bytes += 57 + rem;
    pos += 57 + rem;
  }
  return 0;
}

// Device framing (k_frame_*): the slice is copied as is and framed where it
// lies; 0 = framed, 1 = the host walk must decide (a batch without magic 2
// on the chain, or more than kFrameCap candidates in a 64 KiB chunk).
int frame_on_device(fsg_slice* sl, hipStream_t st, int* fallback) {
  const uint64_t len = sl->len;
  *fallback = 0;
  sl->verify_drain();
  sl->rs_ok = false;
  sl->nb = 0;
  sl->nrec = 0;
  sl->tail_status = 0;
  sl->header_bytes = 0;
  if (len == 0) return FSG_OK;
  if (len < 57) {  // "not enough for batch header" at position 0
    sl->tail_status = FSG_E_IO;
    return FSG_OK;
  }
  const uint32_t nchunks = (uint32_t)((len + kFrameChunk - 1) / kFrameChunk);
  DevBuf &cbuf = sl->fr[0], &ccnt = sl->fr[1], &coff = sl->fr[2], &tsum = sl->fr[3], &scal = sl->fr[4];
  HIPCHK(cbuf.ensure((size_t)nchunks * kFrameCap * 2));
  HIPCHK(ccnt.ensure((size_t)nchunks * 4));
  HIPCHK(coff.ensure((size_t)nchunks * 8));
  HIPCHK(scal.ensure(64));
  HIPCHK(hipMemsetAsync(scal.p, 0, 64, st));
  FrameArgs a{};
  a.s = sl->data.as<uint8_t>();
  a.len = len;
  a.cbuf = cbuf.as<uint16_t>();
  a.ccnt = ccnt.as<uint32_t>();
  a.coff = coff.as<uint64_t>();
  a.scal = scal.as<unsigned long long>();
  HIPCHK(tsum.ensure(xscan_tiles(nchunks) * 8));
  launch_frame_cand(a, nchunks, tsum.as<uint64_t>(), st);
  unsigned long long sc[8];
  HIPCHK(hipMemcpyAsync(sc, scal.p, 64, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t n = sc[3];
  if (sc[0] || n == 0 || n >= 0xFFFFFFF0ull) {
    *fallback = 1;
    return FSG_OK;
  }
  DevBuf &cand = sl->fr[5], &jmp = sl->fr[6], &term = sl->fr[7], &mark = sl->fr[8], &mpre = sl->fr[9],
         &nrec = sl->fr[10], &rpre = sl->fr[11];
  uint32_t levels = 1;
  while (levels < 40 && (1ull << (levels - 1)) < n) levels++;
  HIPCHK(cand.ensure(n * 8));
  HIPCHK(jmp.ensure((size_t)levels * n * 4));
  HIPCHK(term.ensure(n * 4));
  HIPCHK(mark.ensure(n * 4));
  HIPCHK(mpre.ensure(n * 8));
  HIPCHK(nrec.ensure(n * 4));
  HIPCHK(rpre.ensure(n * 8));
  HIPCHK(sl->bpos.ensure(n * 8));
  HIPCHK(sl->rbase.ensure(n * 8));
  HIPCHK(tsum.ensure(xscan_tiles(std::max<uint64_t>(n, nchunks)) * 8));
  a.cand = cand.as<uint64_t>();
  a.ncand = n;
  a.jmp = jmp.as<uint32_t>();
  a.term = term.as<uint32_t>();
  a.mark = mark.as<uint32_t>();
  a.mpre = mpre.as<uint64_t>();
  a.nrec = nrec.as<uint32_t>();
  a.rpre = rpre.as<uint64_t>();
  a.bpos = sl->bpos.as<uint64_t>();
  a.rbase = sl->rbase.as<uint64_t>();
  launch_frame_compact(a, nchunks, st);
  // position 0 without magic 2 (the host walk decides) is flagged in scal[0]
  // by k_frame_next, read with the chain's results: one wait, not two
  launch_frame_chain(a, levels, tsum.as<uint64_t>(), st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(sc, scal.p, 64, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (sc[0]) {
    *fallback = 1;
    return FSG_OK;
  }
  if (sc[1] == 2) {  // a compressed batch on the chain: the host walk frames, the GPU decompresses
    *fallback = 1;
    return FSG_OK;
  }
  sl->nb = (uint32_t)sc[4];
  sl->nrec = sc[5];
  sl->tail_status = sc[1] == 1 ? FSG_E_IO : 0;
  sl->header_bytes = sc[2];
  return FSG_OK;
}

// Compressed record sections (FileBatchIterator: compression.uncompress,
// iterators.rs:136-156) decompressed on the GPU into a new slice where every
// batch is stored uncompressed (header kept, batch_len = 45 + the new length,
// the compression bits kept for the output header).  A batch that fails to
// decode ends the slice there with the iterator's io::Error (zstd:
// unsupported), like the reference's Err at that batch.
int decompress_slice(fsg_slice* sl, const std::vector<uint64_t>& bpos, const std::vector<uint8_t>& codecs,
                     hipStream_t st) {
  const uint32_t nb = (uint32_t)bpos.size();
  DevBuf &dbpos = sl->dec[0], &dcodec = sl->dec[1], &dsize = sl->dec[2], &npos = sl->dec[3], &status = sl->dec[4],
         &cnt = sl->dec[5];
  HIPCHK(dbpos.ensure(std::max<size_t>(nb, 1) * 8));
  HIPCHK(dcodec.ensure(std::max<size_t>(nb, 1)));
  HIPCHK(dsize.ensure(std::max<size_t>(nb, 1) * 8));
  HIPCHK(npos.ensure(std::max<size_t>(nb, 1) * 8));
  HIPCHK(status.ensure(std::max<size_t>(nb, 1) * 4));
  HIPCHK(cnt.ensure(std::max<size_t>(nb, 1) * 8));
  HIPCHK(hipMemcpyAsync(dbpos.p, bpos.data(), nb * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(dcodec.p, codecs.data(), nb, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemsetAsync(status.p, 0, std::max<size_t>(nb, 1) * 4, st));
  DecArgs a{};
  a.src = sl->data.as<uint8_t>();
  a.bpos = dbpos.as<uint64_t>();
  a.codec = dcodec.as<uint8_t>();
  a.nb = nb;
  a.dsize = dsize.as<int64_t>();
  a.npos = npos.as<uint64_t>();
  a.status = status.as<int32_t>();
  a.cnt = cnt.as<uint64_t>();
  {  // the stored CRCs cover the compressed bytes: verify them before they go
    DevBuf& bad = sl->dec[6];
    HIPCHK(bad.ensure(16));
    const unsigned long long init[2] = {0, ~0ull};
    HIPCHK(hipMemcpyAsync(bad.p, init, sizeof init, hipMemcpyHostToDevice, st));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
    launch_verify_crc(a.src, a.bpos, nb, bad.as<unsigned long long>(), nullptr, st);
    HIPCHK(hipEventRecord(e1, st));
    unsigned long long r[2];
    HIPCHK(hipMemcpyAsync(r, bad.p, sizeof r, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipEventElapsedTime(&sl->crc_ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    sl->crc_bad = r[0];
    sl->crc_first = r[0] ? (int64_t)r[1] : -1;
  }
  launch_decompress(a, 0, st);
  std::vector<int64_t> ds(nb);
  HIPCHK(hipMemcpyAsync(ds.data(), dsize.p, nb * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  uint32_t keep = nb;
  int tail = sl->tail_status;
  for (uint32_t b = 0; b < nb; b++)
    if (ds[b] < 0 || ds[b] > 0x7FFFFFFFll - 45) {
      keep = b;
      tail = ds[b] == -2 ? FSG_E_UNSUPPORTED : FSG_E_IO;  // DEC_UNSUP: a codec without a device decoder
      break;
    }
  std::vector<uint64_t> np(nb);
  uint64_t total = 0;
  for (uint32_t b = 0; b < keep; b++) {
    np[b] = total;
    total += 57 + (uint64_t)ds[b];
  }
  // Bound what a small compressed slice may ask for before anything is
  // allocated (gzip expands up to ~1000x, lz4 ~255x).  The reference hands one
  // decompressed batch at a time to a guest whose memory is capped by the store
  // limit (engine.rs:24, limiter.rs:18-35): a batch larger than the limit is
  // StoreMemoryExceeded, exactly as there.  Here the whole decompressed slice
  // is also resident: a slice that does not fit in the device's free memory
  // (with half kept for the chain's scratch) is a device shortfall outside the
  // reference's behaviour: FSG_E_DEVICE, not a StoreMemoryExceeded the
  // reference would never raise for batches under the limit.
  {
    uint64_t big = 0;
    for (uint32_t b = 0; b < keep; b++) big = std::max<uint64_t>(big, (uint64_t)ds[b]);
    if (big > sl->dec_limit) {
      char b[200];
      snprintf(b, sizeof b, "Requested memory %llub exceeded max allowed %llub (decompressed record sections)",
               (unsigned long long)big, (unsigned long long)sl->dec_limit);
      g_store_mem[0] = 0;
      g_store_mem[1] = big;
      g_store_mem[2] = sl->dec_limit;
      return fail(FSG_E_STORE_MEMORY, b);
    }
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) fr = 0;
    if (total + kSlicePad + kWin > fr / 2) {
      char b[200];
      snprintf(b, sizeof b, "decompressed slice of %llu bytes does not fit the device's free memory (%zu bytes)",
               (unsigned long long)total, fr);
      return fail(FSG_E_DEVICE, b);
    }
  }
  DevBuf& nd = sl->dec[7];  // swapped with the compressed slice below: both stay for the next upload
  const size_t alloc = ((total + 15) & ~(size_t)15) + kSlicePad + kWin;
  HIPCHK(nd.ensure(alloc));
  HIPCHK(hipMemsetAsync(nd.p, 0, alloc, st));
  HIPCHK(hipMemcpyAsync(npos.p, np.data(), std::max<size_t>(keep, 1) * 8, hipMemcpyHostToDevice, st));
  a.nb = keep;
  a.dst = nd.as<uint8_t>();
  launch_decompress(a, 1, st);
  launch_decompress(a, 2, st);
  HIPCHK(hipGetLastError());
  std::vector<int32_t> stv(std::max<uint32_t>(keep, 1));
  std::vector<uint64_t> cv(std::max<uint32_t>(keep, 1));
  HIPCHK(hipMemcpyAsync(stv.data(), status.p, keep * 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(cv.data(), cnt.p, keep * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  for (uint32_t b = 0; b < keep; b++)
    if (stv[b]) {  // a checksum (or stream) error found while writing
      keep = b;
      tail = FSG_E_IO;
      total = np[b];
      break;
    }
  std::vector<uint64_t> rb(std::max<uint32_t>(keep, 1));
  uint64_t nrec = 0;
  for (uint32_t b = 0; b < keep; b++) {
    rb[b] = nrec;
    nrec += cv[b];
  }
  HIPCHK(sl->bpos.ensure(std::max<size_t>(keep, 1) * 8));
  HIPCHK(sl->rbase.ensure(std::max<size_t>(keep, 1) * 8));
  if (keep) {
    HIPCHK(hipMemcpyAsync(sl->bpos.p, np.data(), keep * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(sl->rbase.p, rb.data(), keep * 8, hipMemcpyHostToDevice, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  std::swap(sl->data.p, nd.p);
  std::swap(sl->data.cap, nd.cap);
  sl->len = total;
  sl->rs_ok = false;
  sl->nb = keep;
  sl->nrec = nrec;
  sl->tail_status = tail;
  sl->header_bytes = total;
  sl->decompressed = true;
  return FSG_OK;
}

// device_frame: frame on the device (fsg_slice_upload, process_batch); the
// host walk frames the one-batch slices process() builds itself
size_t slice_alloc(size_t len) { return ((len + 15) & ~(size_t)15) + kSlicePad + kWin; }

// sync=false: the caller keeps `s` alive and synchronises the stream itself;
// padded: `s` already holds slice_alloc(len) bytes, zeros behind the slice
int upload_slice(fsg_engine* e, const uint8_t* s, size_t len, fsg_slice* sl, hipStream_t stream,
                 bool device_frame = true, bool sync = true, bool padded = false) {
  sl->verify_drain();
  sl->v_pending = false;  // the verified bytes are being replaced
  sl->eng = e;
  sl->len = len;
  sl->rs_ok = false;
  sl->nb = 0;
  sl->nrec = 0;
  sl->tail_status = 0;
  sl->header_bytes = 0;
  sl->device_framed = false;
  sl->decompressed = false;
  sl->crc_bad = 0;
  sl->crc_first = -1;
  sl->crc_ms = 0;
  const size_t alloc = slice_alloc(len);
  HIPCHK(sl->data.ensure(alloc));
  if (padded) {  // one copy carries the slice and its zero padding
    HIPCHK(hipMemcpyAsync(sl->data.p, s, alloc, hipMemcpyHostToDevice, stream));
  } else {
    HIPCHK(hipMemsetAsync((uint8_t*)sl->data.p + (len & ~(size_t)15), 0, alloc - (len & ~(size_t)15), stream));
    if (len) HIPCHK(hipMemcpyAsync(sl->data.p, s, len, hipMemcpyHostToDevice, stream));
  }
  int fallback = 1;
  if (device_frame) {
    int rc = frame_on_device(sl, stream, &fallback);
    if (rc) return rc;
    sl->device_framed = !fallback;
  }
  if (fallback) {
    sl->device_framed = false;
    std::vector<uint64_t>& bpos = sl->hbpos;
    std::vector<uint64_t>& rbase = sl->hrbase;
    bpos.clear();
    rbase.clear();
    std::vector<uint8_t> codecs;
    frame(s, len, bpos, rbase, sl->nrec, sl->tail_status, sl->header_bytes, &codecs);
    if (std::any_of(codecs.begin(), codecs.end(), [](uint8_t c) { return c != 0; }))
      return decompress_slice(sl, bpos, codecs, stream);
    sl->nb = (uint32_t)bpos.size();
    HIPCHK(sl->bpos.ensure(std::max<size_t>(1, bpos.size()) * 8));
    HIPCHK(sl->rbase.ensure(std::max<size_t>(1, rbase.size()) * 8));
    if (!bpos.empty()) {
      HIPCHK(hipMemcpyAsync(sl->bpos.p, bpos.data(), bpos.size() * 8, hipMemcpyHostToDevice, stream));
      HIPCHK(hipMemcpyAsync(sl->rbase.p, rbase.data(), rbase.size() * 8, hipMemcpyHostToDevice, stream));
    }
  }
  HIPCHK(sl->bpos.ensure(8));
  HIPCHK(sl->rbase.ensure(8));
  if (sync) HIPCHK(hipStreamSynchronize(stream));
  return FSG_OK;
}
}  // namespace

extern "C" int fsg_slice_upload(fsg_engine* e, const uint8_t* s, size_t len, fsg_slice** out) {
  HIPCHK(hipSetDevice(e->device));
  auto sl = std::make_unique<fsg_slice>();
  int rc = upload_slice(e, s, len, sl.get(), 0);
  if (rc) return rc;
  *out = sl.release();
  return FSG_OK;
}
extern "C" int fsg_slice_device_framed(const fsg_slice* s) { return s->device_framed ? 1 : 0; }
// frame the slice's resident bytes again on the device, as a freshly fetched
// slice is framed (FileBatchIterator, iterators.rs:55-160): the fetch-shaped
// measurement re-runs framing + CRC verify + process on HBM-resident bytes
extern "C" int fsg_slice_reframe(fsg_slice* s) {
  HIPCHK(hipSetDevice(s->eng->device));
  if (s->decompressed) return fail(FSG_E_UNSUPPORTED, "the slice was decompressed at ingest: its stored bytes are gone");
  // a host-framed slice stays as it is: device framing would reset its batch
  // table before finding that it needs the host walk again
  if (!s->device_framed) return fail(FSG_E_UNSUPPORTED, "this slice needs the host framing walk (no magic-2 framing)");
  int fallback = 0;
  int rc = frame_on_device(s, 0, &fallback);
  if (rc) return rc;
  if (fallback) return fail(FSG_E_UNSUPPORTED, "this slice needs the host framing walk (no magic-2 framing)");
  s->device_framed = true;
  HIPCHK(hipStreamSynchronize(0));
  return FSG_OK;
}
// CRC32C of every framed batch against its header (report only: the reference
// never verifies, protocol record/batch.rs:398-430, so nothing else changes)
// Started on the slice's own stream, so a fetch can verify while the chain
// processes the same batches (both only read the stored bytes); the result is
// collected by fsg_slice_verify_crc.
extern "C" int fsg_slice_verify_crc_start(const fsg_slice* s) {
  if (s->decompressed) return FSG_OK;  // checked on the stored bytes at ingest
  HIPCHK(hipSetDevice(s->eng->device));
  s->verify_drain();
  // (default priority: a low-priority stream measured no faster here, and the
  // runtime then placed LATER streams of the process on its low-priority
  // hardware queue: c5-agg-sum 8.7 -> 14.3 ms after a fetch-shaped run)
  if (!s->vst) HIPCHK(hipStreamCreateWithFlags(&s->vst, hipStreamNonBlocking));
  for (auto& e : s->vev)
    if (!e) HIPCHK(hipEventCreate(&e));
  if (!s->vres) HIPCHK(hipHostMalloc((void**)&s->vres, 16, hipHostMallocDefault));
  hipStream_t st = s->vst;
  HIPCHK(s->vbad.ensure(16));
  HIPCHK(hipMemsetAsync(s->vbad.p, 0, 8, st));  // [0] mismatches, [1] first mismatching batch (min)
  HIPCHK(hipMemsetAsync((uint8_t*)s->vbad.p + 8, 0xFF, 8, st));
  HIPCHK(hipEventRecord(s->vev[0], st));
  launch_verify_crc((const uint8_t*)s->data.p, s->bpos.as<uint64_t>(), s->nb, s->vbad.as<unsigned long long>(), nullptr, st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(s->vev[1], st));
  HIPCHK(hipMemcpyAsync(s->vres, s->vbad.p, 16, hipMemcpyDeviceToHost, st));
  s->v_pending = true;
  return FSG_OK;
}
extern "C" int fsg_slice_verify_crc(const fsg_slice* s, uint64_t* n_bad, int64_t* first_bad, float* ms) {
  if (s->decompressed) {  // checked on the stored bytes at ingest, before decompression
    if (n_bad) *n_bad = s->crc_bad;
    if (first_bad) *first_bad = s->crc_first;
    if (ms) *ms = s->crc_ms;
    return FSG_OK;
  }
  if (!s->v_pending) {
    int rc = fsg_slice_verify_crc_start(s);
    if (rc) return rc;
  }
  HIPCHK(hipSetDevice(s->eng->device));
  HIPCHK(hipStreamSynchronize(s->vst));
  s->v_pending = false;
  float t = 0;
  HIPCHK(hipEventElapsedTime(&t, s->vev[0], s->vev[1]));
  if (n_bad) *n_bad = s->vres[0];
  if (first_bad) *first_bad = s->vres[0] ? (int64_t)s->vres[1] : -1;
  if (ms) *ms = t;
  return FSG_OK;
}
extern "C" int fsg_slice_info(const fsg_slice* s, uint64_t* n_batches, uint64_t* n_records, uint64_t* bytes) {
  if (n_batches) *n_batches = s->nb;
  if (n_records) *n_records = s->nrec;
  if (bytes) *bytes = s->header_bytes;
  return FSG_OK;
}
extern "C" void fsg_slice_free(fsg_slice* s) { delete s; }

// ---------------------------------------------------------------------------
// process_batch over a resident slice
// ---------------------------------------------------------------------------
namespace {

void free_error(fsg_runtime_error& e) {
  free((void*)e.hint);
  free((void*)e.key);
  free((void*)e.value);
  memset(&e, 0, sizeof e);
}

// serde_json::Error Display for the descriptor k_eval found (fsg_json_dev.h):
// "<message> at line L column C" with serde's custom messages
// (serde/src/de/mod.rs: invalid_type / invalid_length / unknown_variant /
// duplicate_field / missing_field).  The GPU did the parse; this renders text
// from its code, reader index and spans.  Returns false outside the restatement.
static void json_unescape(const std::vector<uint8_t>& v, uint32_t a, uint32_t b, std::string& out) {
  auto hexv = [](int c) {
    return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10;
  };
  auto put = [&](uint32_t c) {
    if (c < 0x80) {
      out += (char)c;
    } else if (c < 0x800) {
      out += (char)(0xC0 | (c >> 6));
      out += (char)(0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      out += (char)(0xE0 | (c >> 12));
      out += (char)(0x80 | ((c >> 6) & 0x3F));
      out += (char)(0x80 | (c & 0x3F));
    } else {
      out += (char)(0xF0 | (c >> 18));
      out += (char)(0x80 | ((c >> 12) & 0x3F));
      out += (char)(0x80 | ((c >> 6) & 0x3F));
      out += (char)(0x80 | (c & 0x3F));
    }
  };
  for (uint32_t i = a; i < b && i < v.size();) {
    if (v[i] != '\\') {
      out += (char)v[i++];
      continue;
    }
    const uint8_t e = v[i + 1];
    i += 2;
    switch (e) {
      case 'b': out += '\b'; break;
      case 'f': out += '\f'; break;
      case 'n': out += '\n'; break;
      case 'r': out += '\r'; break;
      case 't': out += '\t'; break;
      case 'u': {
        uint32_t c = 0;
        for (int k = 0; k < 4; k++) c = (c << 4) | (uint32_t)hexv(v[i + k]);
        i += 4;
        if (c >= 0xD800 && c <= 0xDBFF) {  // validated pair \uD8xx\uDCxx
          uint32_t c2 = 0;
          for (int k = 0; k < 4; k++) c2 = (c2 << 4) | (uint32_t)hexv(v[i + 2 + k]);
          i += 6;
          c = (((c - 0xD800) << 10) | (c2 - 0xDC00)) + 0x10000;
        }
        put(c);
        break;
      }
      default: out += (char)e; break;  // " \\ /
    }
  }
}

bool json_hint(uint32_t code_word, uint32_t pos, uint32_t a, uint32_t b, const std::vector<uint8_t>& v,
               std::string& out) {
  static const char* const kSyntax[] = {
      "", "EOF while parsing a list", "EOF while parsing an object", "EOF while parsing a string",
      "EOF while parsing a value", "expected `:`", "expected `,` or `]`", "expected `,` or `}`", "expected ident",
      "expected value", "invalid escape", "invalid number", "invalid unicode code point",
      "control character (\\u0000-\\u001F) found while parsing a string", "key must be a string",
      "lone leading surrogate in hex escape", "trailing comma", "trailing characters",
      "unexpected end of hex escape", "recursion limit exceeded"};
  static const char* const kFields[] = {"level", "message"};
  const uint32_t code = (code_word >> 8) & 0xFF, sub = (code_word >> 16) & 0xFF;
  std::string msg;
  if (code >= JE_EOF_LIST && code <= JE_RECURSION) {
    msg = kSyntax[code];
  } else if (code == JE_DUP_FIELD) {
    msg = std::string("duplicate field `") + kFields[a & 1] + "`";
  } else if (code == JE_MISSING_FIELD) {
    msg = std::string("missing field `") + kFields[a & 1] + "`";
  } else if (code == JE_INVALID_LENGTH) {
    msg = "invalid length " + std::to_string(a) + ", expected struct StructuredLog with 2 elements";
  } else if (code == JE_UNKNOWN_VARIANT) {
    std::string val;
    json_unescape(v, a, b, val);
    msg = "unknown variant `" + val + "`, expected one of `debug`, `info`, `warn`, `error`";
  } else if (code == JE_RANGE) {
    msg = "number out of range";
  } else if (code == JE_INVALID_VALUE) {  // the u32 visitor (aggregate-json): visit_u64 / visit_i64 out of range
    msg = std::string("invalid value: integer `") + ((sub & 15) == JU_NINT ? "-" : "") +
          std::string(v.begin() + a, v.begin() + b) + "`, expected u32";
  } else if (code == JE_INVALID_TYPE) {
    static const char* const kExp[] = {"struct StructuredLog", "a string", "variant identifier", "unit",
                                       "a sequence", "a map", "u32", ""};
    std::string un;
    switch (sub & 15) {
      case JU_UNIT: un = "unit value"; break;
      case JU_TRUE: un = "boolean `true`"; break;
      case JU_FALSE: un = "boolean `false`"; break;
      case JU_UINT: un = "integer `" + std::string(v.begin() + a, v.begin() + b) + "`"; break;
      case JU_NINT: un = "integer `-" + std::string(v.begin() + a, v.begin() + b) + "`"; break;
      case JU_STR: {
        std::string raw;
        json_unescape(v, a, b, raw);
        un = "string ";
        if (!rust_str_debug(raw, un)) return false;
        break;
      }
      case JU_SEQ: un = "sequence"; break;
      case JU_MAP: un = "map"; break;
      case JU_FLOAT: {  // serde Unexpected::Float: Rust Display behind WithDecimalPoint
        const bool neg = a > 0 && a <= v.size() && v[a - 1] == '-';
        const uint32_t st = neg ? a - 1 : a;
        auto acc = [&](uint32_t k) -> int { return k < b && k < v.size() ? v[k] : -1; };
        const flt::NumVal nv = flt::num_value(acc, st, b);
        if (nv.kind != 1) return false;
        uint8_t txt[400];
        const uint32_t tl = flt::display_with_point(nv.f, txt);
        un = "floating point `" + std::string((const char*)txt, tl) + "`";
        break;
      }
      default: return false;
    }
    msg = "invalid type: " + un + ", expected " + kExp[(sub >> 4) & 7];
  } else {
    return false;  // JE_DEEP
  }
  size_t line = 1, col = 0;
  for (uint32_t i = 0; i < pos && i < v.size(); i++) {
    if (v[i] == '\n') {
      line++;
      col = 0;
    } else {
      col++;
    }
  }
  out = msg + " at line " + std::to_string(line) + " column " + std::to_string(col);
  return true;  // (a NUL inside, from "unknown variant" of a raw string, crosses with hint_len)
}

// Build SmartModuleTransformRuntimeError (link/smartmodule.rs:26-43) for the
// error record of batch eb: hint, offset = base_offset + offset_delta, kind,
// and the record's key/value as they entered the failing stage.
int build_error(fsg_chain* c, const fsg_slice* s, const BatchStat& st, fsg_runtime_error& err) {
  memset(&err, 0, sizeof err);
  // fetch the failing record's bytes (header first, then the full record)
  uint8_t head[16] = {0};
  const size_t avail = s->len - st.err_pos;
  HIPCHK(hipMemcpy(head, (uint8_t*)s->data.p + st.err_pos, std::min<size_t>(16, avail), hipMemcpyDeviceToHost));
  uint64_t num = 0;
  unsigned shift = 0;
  size_t i = 0;
  for (;;) {
    uint8_t bb = head[i++];
    num |= (uint64_t)(bb & 0x7f) << (shift & 63);
    shift += 7;
    if (!(bb & 0x80) || i >= 10) break;
  }
  const int64_t len = (int64_t)((num >> 1) ^ (~(num & 1) + 1));
  const size_t rlen = std::min<size_t>(avail, i + (size_t)std::max<int64_t>(len, 0) + 16);
  std::vector<uint8_t> rec(rlen);
  HIPCHK(hipMemcpy(rec.data(), (uint8_t*)s->data.p + st.err_pos, rlen, hipMemcpyDeviceToHost));
  // parse the record fields (Record::decode) to recover key and value
  size_t q = 0;
  auto var = [&](int64_t* v) {
    uint64_t n = 0;
    unsigned sh = 0;
    for (;;) {
      if (q >= rec.size()) return false;
      uint8_t bb = rec[q++];
      n |= (uint64_t)(bb & 0x7f) << (sh & 63);
      sh += 7;
      if (!(bb & 0x80)) break;
    }
    *v = (int64_t)((n >> 1) ^ (~(n & 1) + 1));
    return true;
  };
  int64_t t;
  var(&t);   // len
  q++;       // attributes
  var(&t);   // timestamp_delta
  var(&t);   // offset_delta
  const uint8_t tag = q < rec.size() ? rec[q++] : 0;
  std::vector<uint8_t> key, val;
  if (tag == 1) {
    int64_t kl;
    var(&kl);
    size_t take = std::min<size_t>((size_t)kl, rec.size() - q);
    key.assign(rec.begin() + q, rec.begin() + q + take);
    q += take;
  }
  int64_t vl;
  var(&vl);
  size_t take = std::min<size_t>((size_t)vl, rec.size() - q);
  val.assign(rec.begin() + q, rec.begin() + q + take);
  const StageDesc& sd = c->hdesc.st[st.err_stage];
  if (sd.in_type != VT_I32) {  // the value's view as it entered the stage (a projection narrows it)
    val.resize(st.err_vlen);
    if (st.err_vlen)
      HIPCHK(hipMemcpy(val.data(), (uint8_t*)s->data.p + st.err_vpos, st.err_vlen, hipMemcpyDeviceToHost));
  }
  if (sd.in_type == VT_SRC_UPPER)
    for (auto& ch : val)
      if (ch >= 'a' && ch <= 'z') ch -= 32;
  if (sd.in_type == VT_I32) {
    char b[16];
    int n = snprintf(b, sizeof b, "%d", st.err_ival);
    val.assign(b, b + n);
  }
  std::string hint;
  if ((st.err_code & 0xFF) == EC_JSON) {
    if (!json_hint(st.err_code, st.err_aux, st.err_aux2, st.err_aux3, val, hint))
      return fail(FSG_E_UNSUPPORTED, "serde_json error text outside the GPU restatement (deep ignored nesting)");
  } else if (st.err_code == EC_UTF8 || st.err_code == EC_ACC_UTF8) {
    hint = utf8_hint(st.err_aux, st.err_aux2);
  } else if (st.err_code == EC_PARSE) {
    hint = parse_hint(st.err_aux);
    if (sd.op == OP_FILTER_ODD)
      hint = "Oops something went wrong\n\nCaused by:\n   0: Failed to parse int\n   1: " + hint;
  }
  err.hint = (const char*)malloc(hint.size() + 1);
  memcpy((void*)err.hint, hint.c_str(), hint.size() + 1);
  err.hint_len = hint.size();
  err.offset = st.base_offset + st.err_od;
  err.kind = sd.kind;
  err.has_key = tag == 1;
  if (tag == 1) {
    err.key = (const uint8_t*)malloc(std::max<size_t>(1, key.size()));
    memcpy((void*)err.key, key.data(), key.size());
    err.key_len = key.size();
  }
  err.value = (const uint8_t*)malloc(std::max<size_t>(1, val.size()));
  memcpy((void*)err.value, val.data(), val.size());
  err.value_len = val.size();
  return FSG_OK;
}

// grow a persistent device buffer keeping its first `used` bytes
hipError_t grow_keep(DevBuf& b, size_t need, size_t used, hipStream_t st) {
  if (need <= b.cap) return hipSuccess;
  void* np = nullptr;
  const size_t cap = std::max<size_t>(need + need / 2, 4096);
  hipError_t e = hipMalloc(&np, cap);
  if (e != hipSuccess) return e;
  if (used) {
    e = hipMemcpyAsync(np, b.p, used, hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      (void)hipFree(np);
      return e;
    }
  }
  if (b.p) (void)hipFree(b.p);
  b.p = np;
  b.cap = cap;
  return hipSuccess;
}

// the stateful last stage (k_sf_*): decisions in stream order over the batches
// it ran on, descriptors compacted; the commit follows k_plan (sf_commit)
int sf_run(fsg_chain* c, const fsg_slice* s, const EvalArgs& ea, SfArgs& sa, hipStream_t st) {
  SfState& S = *c->sf;
  const StageDesc& sd = c->hdesc.st[c->sf_stage];
  const uint32_t nb = s->nb;
  const size_t nr = std::max<uint64_t>(s->nrec, 1);
  sa = SfArgs{};
  sa.slice = ea.slice;
  sa.bstat = ea.bstat;
  sa.desc = ea.desc;
  sa.rbase = ea.rbase;
  sa.mins = ea.mins;
  sa.plan = c->plan.as<Plan>();
  sa.nbatches = nb;
  sa.op = sd.op;
  sa.lookback = sd.keep_match;
  HIPCHK(c->sf_bval.ensure(std::max<uint32_t>(nb, 1) * 8));
  HIPCHK(c->sf_bpre.ensure(std::max<uint32_t>(nb, 1) * 8));
  sa.bval = c->sf_bval.as<int64_t>();
  sa.bpre = c->sf_bpre.as<int64_t>();
  sa.prev = S.prev.as<int32_t>();
  if (sd.op == OP_LB_MAX) {
    launch_sf_lb(sa, st);
    return FSG_OK;
  }
  // filter_hashset: the table holds the entries and this call's records
  uint32_t cap = 1024;
  while (cap < 2 * (S.n_ent + s->nrec) + 16) cap <<= 1;
  const size_t state = (size_t)(S.n_ent + s->nrec) * 28 + S.arena_len + s->len;
  const size_t scratch = nr * 41 + (size_t)cap * 20 + (size_t)std::max<uint32_t>(nb, 1) * 20;
  if (state + scratch > c->limit) {
    char b[160];
    snprintf(b, sizeof b, "Requested memory %zub exceeded max allowed %zub", state + scratch, c->limit);
    g_store_mem[0] = (size_t)S.n_ent * 28 + S.arena_len;
    g_store_mem[1] = state + scratch;
    g_store_mem[2] = c->limit;
    return fail(FSG_E_STORE_MEMORY, b);
  }
  HIPCHK(grow_keep(S.ent_hash, (S.n_ent + nr) * 8, S.n_ent * 8, st));
  HIPCHK(grow_keep(S.ent_pos, (S.n_ent + nr) * 8, S.n_ent * 8, st));
  HIPCHK(grow_keep(S.ent_len, (S.n_ent + nr) * 4, S.n_ent * 4, st));
  HIPCHK(grow_keep(S.ent_last, (S.n_ent + nr) * 8, S.n_ent * 8, st));
  HIPCHK(grow_keep(S.arena, S.arena_len + s->len + 64, S.arena_len, st));
  HIPCHK(c->sf_bn.ensure(std::max<uint32_t>(nb, 1) * 4));
  HIPCHK(c->sf_hv.ensure(nr * 8));
  HIPCHK(c->sf_vref.ensure(nr * 8));
  HIPCHK(c->sf_vlen.ensure(nr * 4));
  HIPCHK(c->sf_slot.ensure(nr * 4));
  HIPCHK(c->sf_keep.ensure(nr));
  HIPCHK(c->sf_idx.ensure(nr * 8));
  HIPCHK(c->sf_sref.ensure((size_t)cap * 8));
  HIPCHK(c->sf_first.ensure((size_t)cap * 4));
  HIPCHK(c->sf_cur.ensure((size_t)cap * 8));
  HIPCHK(c->sf_scal.ensure(64));
  sa.bn = c->sf_bn.as<uint32_t>();
  sa.hv = c->sf_hv.as<uint64_t>();
  sa.vref = c->sf_vref.as<uint64_t>();
  sa.vlen = c->sf_vlen.as<uint32_t>();
  sa.slot = c->sf_slot.as<uint32_t>();
  sa.keep = c->sf_keep.as<uint8_t>();
  sa.idx = c->sf_idx.as<uint64_t>();
  sa.sref = c->sf_sref.as<unsigned long long>();
  sa.first = c->sf_first.as<uint32_t>();
  sa.cur = c->sf_cur.as<uint64_t>();
  sa.cap = cap;
  sa.ent_hash = S.ent_hash.as<uint64_t>();
  sa.ent_pos = S.ent_pos.as<uint64_t>();
  sa.ent_len = S.ent_len.as<uint32_t>();
  sa.ent_last = S.ent_last.as<uint64_t>();
  sa.arena = S.arena.as<uint8_t>();
  sa.n_ent = S.n_ent;
  sa.n0 = S.n;
  sa.limit = S.limit;
  sa.scal = c->sf_scal.as<unsigned long long>();
  const unsigned long long sc0[4] = {S.n_ent, S.arena_len, S.n, 0};
  HIPCHK(hipMemcpyAsync(sa.scal, sc0, sizeof sc0, hipMemcpyHostToDevice, st));
  launch_sf_dedup(sa, st);
  unsigned long long kept = 0;
  HIPCHK(hipMemcpyAsync(&kept, sa.scal + 3, sizeof kept, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // no value leaves the set during the call when the set (the newest `limit`
  // insertions) has room for every insertion the parallel pass found
  const uint64_t live = std::min<uint64_t>(S.n, S.limit);
  sa.fast = live + kept <= S.limit ? 1u : 0u;
  if (!sa.fast) launch_sf_dedup_seq(sa, st);
  launch_sf_compact(sa, st);
  return FSG_OK;
}

// aggregate-json state in HBM.  The first call (or a keyed collect before any
// call) parses the initial accumulator once (unwrap_or_default, as the guest's
// serde_json::from_slice) into ajs[aj_cur]: per key its match bytes and its
// serialized text in one arena, and its value.
int aj_state_init(fsg_chain* c) {
  if (c->aj_dev) return FSG_OK;
  AccMap am;
  const bool ok = parse_acc_map(c->acc, am);
  c->aj_e0 = !ok && json_starts_map(c->acc);
  const uint32_t n = (uint32_t)am.keys.size();
  if (am.dups) {  // HashMap::insert reserves before it finds a repeated key: the layout sees it
    HIPCHK(c->aj_iseq.ensure(am.seq.size() * 4));
    HIPCHK(hipMemcpy(c->aj_iseq.p, am.seq.data(), am.seq.size() * 4, hipMemcpyHostToDevice));
    c->aj_n_iseq = (uint32_t)am.seq.size();
  }
  std::vector<uint8_t> arena;
  std::vector<uint64_t> ko(n), to(n);
  std::vector<uint32_t> kl(n), tl(n);
  for (uint32_t k = 0; k < n; k++) {
    ko[k] = arena.size();
    arena.insert(arena.end(), am.keys[k].begin(), am.keys[k].end());
    to[k] = arena.size();
    arena.insert(arena.end(), am.text[k].begin(), am.text[k].end());
    kl[k] = (uint32_t)am.keys[k].size();
    tl[k] = (uint32_t)am.text[k].size();
  }
  fsg_chain::AjBuf& S = c->ajs[c->aj_cur];
  const size_t n1 = std::max<uint32_t>(n, 1);
  HIPCHK(S.arena.ensure(arena.size() + 16));
  HIPCHK(S.kptr.ensure(n1 * 8));
  HIPCHK(S.klen.ensure(n1 * 4));
  HIPCHK(S.tptr.ensure(n1 * 8));
  HIPCHK(S.tlen.ensure(n1 * 4));
  HIPCHK(S.val.ensure(n1 * 4));
  const uint64_t base = (uint64_t)S.arena.p;
  for (uint32_t k = 0; k < n; k++) {
    ko[k] += base;
    to[k] += base;
  }
  hipStream_t st = c->stream;
  if (n) {
    HIPCHK(hipMemcpyAsync(S.arena.p, arena.data(), arena.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.kptr.p, ko.data(), n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.tptr.p, to.data(), n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.klen.p, kl.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.tlen.p, tl.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(S.val.p, am.vals.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // the host vectors go out of scope
  }
  c->aj_K = n;
  c->aj_bytes = arena.size();
  c->aj_dev = true;
  return FSG_OK;
}

// the map after the stop batch into the other state buffer (two phases: the
// arena is sized by a scan), then it becomes the state
int aj_commit(fsg_chain* c, const AggjArgs& aj, int32_t stop, uint32_t kmax) {
  hipStream_t st = c->stream;
  fsg_chain::AjBuf& D = c->ajs[1 - c->aj_cur];
  const size_t k1 = std::max<uint32_t>(kmax, 1);
  HIPCHK(D.kptr.ensure(k1 * 8));
  HIPCHK(D.klen.ensure(k1 * 4));
  HIPCHK(D.tptr.ensure(k1 * 8));
  HIPCHK(D.tlen.ensure(k1 * 4));
  HIPCHK(D.val.ensure(k1 * 4));
  HIPCHK(D.blen.ensure(k1 * 4));
  HIPCHK(D.boff.ensure(k1 * 8));
  HIPCHK(D.arena.ensure(16));
  HIPCHK(c->aj_cout.ensure(64));
  HIPCHK(c->aj_tsum.ensure(xscan_tiles(k1) * 8));
  HIPCHK(c->aj_inv.ensure(k1 * 4));
  AjCommitArgs ca{};
  ca.a = aj;
  ca.stop = stop;
  ca.kmax = kmax;
  ca.inv = c->aj_inv.as<uint32_t>();
  ca.out = c->aj_cout.as<unsigned long long>();
  ca.dst.arena = D.arena.as<uint8_t>();
  ca.dst.kptr = D.kptr.as<uint64_t>();
  ca.dst.klen = D.klen.as<uint32_t>();
  ca.dst.tptr = D.tptr.as<uint64_t>();
  ca.dst.tlen = D.tlen.as<uint32_t>();
  ca.dst.val = D.val.as<uint32_t>();
  ca.dst.blen = D.blen.as<uint32_t>();
  ca.dst.boff = D.boff.as<uint64_t>();
  launch_aggj_commit(ca, c->aj_tsum.as<uint64_t>(), 0, st);
  unsigned long long o[5] = {0, 0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(o, ca.out, sizeof o, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  // the RandomStates the guest drew through the stop batch: two per folded
  // record from k0_base (which counts the initial accumulator's extra draw),
  // and at a final aggregate error its accumulator map plus, when the value
  // starts with '{', the record's map
  if (o[1] + o[3] > 0) c->aj_k0 = aj.k0_base + 2ull * o[1] + (o[3] ? 1ull + o[4] : 0ull);
  if (o[1] == 0) return FSG_OK;  // no record folded through the stop batch: the state stands
  HIPCHK(D.arena.ensure(o[2] + 16));
  ca.dst.arena = D.arena.as<uint8_t>();
  launch_aggj_commit(ca, c->aj_tsum.as<uint64_t>(), 1, st);
  HIPCHK(hipGetLastError());
  c->aj_cur = 1 - c->aj_cur;
  c->aj_K = (uint32_t)o[0];
  c->aj_bytes = o[2];
  c->aj_touched = true;  // the accumulator is now the last output text: no repeats, parses
  c->aj_n_iseq = 0;
  return FSG_OK;
}

// serde_json::to_vec_pretty of the state (the text the guest's last record
// carried): "{}" or "{\n  key: v,\n  ...\n}", keys in the state's order (that text's)
int aj_render(fsg_chain* c, std::vector<uint8_t>& out) {
  const fsg_chain::AjBuf& S = c->ajs[c->aj_cur];
  const uint32_t K = c->aj_K;
  HIPCHK(hipSetDevice(c->eng->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  std::vector<uint64_t> tp(K);
  std::vector<uint32_t> tl(K), v(K);
  std::vector<uint8_t> ar(c->aj_bytes);
  if (K) {
    HIPCHK(hipMemcpy(tp.data(), S.tptr.p, (size_t)K * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(tl.data(), S.tlen.p, (size_t)K * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(v.data(), S.val.p, (size_t)K * 4, hipMemcpyDeviceToHost));
    if (!ar.empty()) HIPCHK(hipMemcpy(ar.data(), S.arena.p, ar.size(), hipMemcpyDeviceToHost));
  }
  out.clear();
  out.push_back('{');
  for (uint32_t k = 0; k < K; k++) {
    const char* sep = k ? ",\n  " : "\n  ";
    out.insert(out.end(), sep, sep + strlen(sep));
    const uint64_t off = tp[k] - (uint64_t)S.arena.p;
    out.insert(out.end(), ar.begin() + off, ar.begin() + off + tl[k]);
    char b[16];
    const int n = snprintf(b, sizeof b, ": %u", v[k]);
    out.insert(out.end(), b, b + n);
  }
  if (K) out.push_back('\n');
  out.push_back('}');
  return FSG_OK;
}

// segment mode of run_slice (composed chains): the segment's per-batch output
// becomes `out`, a slice of batches [0, stop] with the source headers; the
// state commits wait for the final segment's stop (commit_deferred)
struct SegOut {
  fsg_slice* out;
  int tail;        // the status of a failure right after the output's last batch (0: none)
  int fail_batch;  // that batch (its process() call failed), -1: the input's own tail
};

// the host copy of an aggregate-sum / concat accumulator after a call that touched it
int acc_update(fsg_chain* c, const Plan& p, bool cat) {
  if (cat) {
    std::vector<uint8_t> na(c->acc.size() + p.cat_final);
    HIPCHK(hipMemcpy(na.data(), c->cat.as<uint8_t>() + kCatOff, na.size(), hipMemcpyDeviceToHost));
    c->acc.swap(na);
  } else {
    char b[16];
    int n = snprintf(b, sizeof b, "%d", (int32_t)p.acc_final);
    c->acc.assign(b, b + n);
  }
  return FSG_OK;
}

int run_composed(fsg_chain* c, const fsg_slice* s, uint64_t max_bytes, fsg_metrics* m, fsg_batch_output* res);
// one chunk of a pipelined fsg_chain_process_batch (process_pipelined): the
// output batch an earlier chunk started (its base offset, compression bits)
// and the max_bytes budget the earlier chunks used; out: the chunk output's
// CRC32C over [21, out_len) (its own header, then its records)
struct Carry {
  bool cont = false;
  int64_t base = -1;
  int32_t comp = 0;
  uint64_t spent = 0;
  uint32_t crc = 0;
};

// the group's walks, once every chain has arrived (the last arrival launches)
int group_launch(AjGroup* g) {
  const size_t n = g->jobs.size();
  if (!n) return FSG_OK;  // nothing walks: no chain waits for the group
  HIPCHK(hipSetDevice(g->device));
  fsg_engine* e = g->eng;
  if (!e->gst) HIPCHK(hipStreamCreateWithFlags(&e->gst, hipStreamNonBlocking));
  if (!e->gdone) HIPCHK(hipEventCreateWithFlags(&e->gdone, hipEventDisableTiming));
  g->st = e->gst;
  g->done = e->gdone;
  const size_t need = n * sizeof(AggjArgs);
  if (need > e->gdcap) {  // grow-only (the previous group's walk was waited for by its chains)
    if (e->gdlist) HIPCHK(hipFree(e->gdlist));
    e->gdlist = nullptr;
    e->gdcap = 0;
    HIPCHK(hipMalloc(&e->gdlist, need));
    e->gdcap = need;
  }
  for (auto ev : g->ready) HIPCHK(hipStreamWaitEvent(g->st, ev, 0));
  HIPCHK(hipMemcpyAsync(e->gdlist, g->jobs.data(), need, hipMemcpyHostToDevice, g->st));
  if (g->timed) {
    if (!e->gt0) HIPCHK(hipEventCreate(&e->gt0));
    if (!e->gt1) HIPCHK(hipEventCreate(&e->gt1));
    g->t0 = e->gt0;
    g->t1 = e->gt1;
    HIPCHK(hipEventRecord(g->t0, g->st));
  }
  launch_aggj_order_group((const AggjArgs*)e->gdlist, (uint32_t)n, g->st);
  HIPCHK(hipGetLastError());
  if (g->timed) HIPCHK(hipEventRecord(g->t1, g->st));
  HIPCHK(hipEventRecord(g->done, g->st));
  return FSG_OK;
}
// a chain's arrival (job = nullptr: nothing to walk); returns once the group's
// launch is queued, with `st` ordered after it
int group_arrive(fsg_chain* c, const AggjArgs* job, hipStream_t st) {
  AjGroup* g = c->group;
  if (!g || c->group_arrived) return FSG_OK;
  std::unique_lock<std::mutex> lk(g->mu);
  // the arrival always counts, even when queueing this chain's walk fails:
  // every other walker waits for the count to reach `expected`
  int rc = FSG_OK;
  if (job) {
    hipEvent_t e = nullptr;
    hipError_t he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventRecord(e, st);
    if (he != hipSuccess) {
      if (e) (void)hipEventDestroy(e);
      rc = fail(FSG_E_DEVICE, std::string("group_arrive: ") + hipGetErrorString(he));
      job = nullptr;
    } else {
      if (c->timed) g->timed = true;
      g->jobs.push_back(*job);
      g->ready.push_back(e);
    }
  }
  c->group_arrived = true;
  if (++g->arrived == g->expected) {
    g->rc = group_launch(g);
    g->launched = true;
    g->cv.notify_all();
  } else if (job) {
    g->cv.wait(lk, [&] { return g->launched; });
  }
  if (rc) return rc;
  if (job) {
    if (g->rc) return g->rc;
    HIPCHK(hipStreamWaitEvent(st, g->done, 0));
  }
  return FSG_OK;
}
int group_order(fsg_chain* c, const AggjArgs* aj, hipStream_t st) {
  return group_arrive(c, aj->n_rec ? aj : nullptr, st);
}

int run_slice(fsg_chain* c, const fsg_slice* s, uint64_t max_bytes, fsg_metrics* m, fsg_batch_output* res,
              bool empty_chain_io, SegOut* so = nullptr, Carry* cy = nullptr) {
  if (!c->segs.empty()) return run_composed(c, s, max_bytes, m, res);
  hipStream_t st = c->stream;
  const uint32_t nb = s->nb;
  memset(res, 0, sizeof *res);
  if (so) max_bytes = ~0ull;  // the SPU's max_bytes applies to the final segment's output only
  // scratch (StoreMemoryExceeded past the store limit, limiter.rs:18-35)
  const bool has_array = c->array_stage >= 0;
  const bool has_aggj = (c->hdesc.flags & CF_AGG_JSON) != 0;
  const size_t elem_cap = (has_array || has_aggj) ? (s->len / 2 + 2) : 0;  // ElemRec slots (fsg_device.h)
  const size_t need = (size_t)std::max<uint32_t>(nb, 1) * (sizeof(BatchStat) + 3 * sizeof(ScanRow)) +
                      (size_t)std::max<uint64_t>(s->nrec, 1) * sizeof(KeptRec) + elem_cap * sizeof(ElemRec);
  // (the lean array path's per-batch element bitmaps are device scratch of
  // this engine, not guest memory: sized below only when that path is taken)
  if (need > c->limit) {
    char b[160];
    snprintf(b, sizeof b, "Requested memory %zub exceeded max allowed %zub", need, c->limit);
    g_store_mem[0] = 0;  // nothing of this call is allocated yet
    g_store_mem[1] = need;
    g_store_mem[2] = c->limit;
    return fail(FSG_E_STORE_MEMORY, b);
  }
  HIPCHK(c->bstat.ensure(std::max<uint32_t>(nb, 1) * sizeof(BatchStat)));
  HIPCHK(c->kept.ensure(std::max<uint64_t>(s->nrec, 1) * sizeof(KeptRec)));
  HIPCHK(c->rows.ensure(std::max<uint32_t>(nb, 1) * sizeof(ScanRow)));
  HIPCHK(c->pre.ensure(std::max<uint32_t>(nb, 1) * sizeof(ScanRow)));
  HIPCHK(c->aggpre.ensure(std::max<uint32_t>(nb, 1) * sizeof(ScanRow)));
  HIPCHK(c->defer.ensure(((size_t)nb + 1) * sizeof(uint32_t)));
  HIPCHK(c->tiles.ensure(std::max<uint32_t>(scan_tiles(nb), 1) * sizeof(ScanRow)));
  HIPCHK(c->grand.ensure(sizeof(ScanRow)));
  HIPCHK(c->mins.ensure(sizeof(Mins)));
  HIPCHK(c->plan.ensure(sizeof(Plan)));
  if (has_array || has_aggj) HIPCHK(c->elem.ensure(elem_cap * sizeof(ElemRec)));
  const bool has_agg = c->agg_stage >= 0;
  const bool has_cat = has_agg && (c->hdesc.flags & CF_AGG_CAT);
  const int64_t acc0 = has_agg && !has_cat && !has_aggj ? acc_value(c->acc) : 0;

  HIPCHK(hipMemsetAsync(c->mins.p, 0xFF, sizeof(Mins), st));
  if (cy && cy->cont) {  // a continuation: every batch counts, records rebase to the carried base
    Mins m0;
    memset(&m0, 0xFF, sizeof m0);
    m0.first_keep = 0;
    m0.carry = (uint32_t)cy->comp & 7u;
    m0.carry_base = cy->base;
    HIPCHK(hipMemcpyAsync(c->mins.p, &m0, sizeof m0, hipMemcpyHostToDevice, st));
  }
  if (cy) max_bytes -= cy->spent;  // the budget the earlier chunks left (they stayed within it)
  if (c->timed) HIPCHK(hipEventRecord(c->ev[0], st));
  EvalArgs ea{};
  ea.slice = (const uint8_t*)s->data.p;
  ea.slice_len = s->len;
  ea.bpos = s->bpos.as<uint64_t>();
  ea.rbase = s->rbase.as<uint64_t>();
  ea.nbatches = nb;
  ea.chain = c->d_desc.as<ChainDesc>();
  ea.blob = c->d_blob.as<uint8_t>();
  ea.bstat = c->bstat.as<BatchStat>();
  ea.desc = c->kept.as<KeptRec>();
  ea.mins = c->mins.as<Mins>();
  ea.list = c->defer.as<uint32_t>();
  ea.elem = (has_array || has_aggj) ? c->elem.as<ElemRec>() : nullptr;
  ea.arr_b = nullptr;
  ea.arr_bm = nullptr;
  ea.rows = c->rows.as<ScanRow>();  // (rows is sized above; k_size fills what the flat decides leave)
  ea.nrec = s->nrec;
  uint32_t ops = 0;
  bool lean_stages = true;  // every stage has a lean form
  bool projected = false;  // a projection seen: only uppercase maps may follow on the lean path
  for (uint32_t k = 0; k < c->hdesc.nstages; k++) {
    const StageDesc& sd = c->hdesc.st[k];
    ops |= 1u << sd.op;
    if (projected && sd.op != OP_MAP_UPPER) lean_stages = false;
    if (sd.op == OP_CONTAINS && sd.needle_len > 128) lean_stages = false;  // kLeanNeedle
    if (sd.op == OP_REGEX && !sd.dfa.lean) lean_stages = false;
    if ((sd.op == OP_FILTER_JSON || sd.op == OP_PROJECT) && sd.in_type != VT_SRC) lean_stages = false;
    if (sd.op == OP_PROJECT) {
      projected = true;
      if (sd.needle_len > 128) lean_stages = false;  // kLeanNeedle
    }
  }
  // substring / bounded regex / filter_json filters, a final field projection
  // and uppercase maps: the lean kernel first, the batches it defers then go
  // through the exact kernel (list mode)
  const bool lean = (ops & ~((1u << OP_CONTAINS) | (1u << OP_MAP_UPPER) | (1u << OP_REGEX) |
                             (1u << OP_FILTER_JSON) | (1u << OP_PROJECT))) == 0 &&
                    !has_agg && lean_stages && nb > 1 &&  // one batch: the exact kernel alone (1 launch, not 3)
                    !s->has_pass;                         // pass-through batches: the exact kernel knows them
  ea.pass = s->has_pass ? s->pass.as<uint8_t>() : nullptr;
  // record starts per batch (k_chase for the lean kernel, k_chase_w for the exact and array ones)
  HIPCHK(c->rstart.ensure(((size_t)s->nrec + 64) * sizeof(uint16_t)));  // + a wave of over-read
  HIPCHK(c->rend.ensure(((size_t)nb + 1) * sizeof(uint16_t)));
  ea.rstart = c->rstart.as<uint16_t>();
  ea.rend = c->rend.as<uint16_t>();
  // array_map alone: the lean array kernel, unsupported shapes deferred to k_eval
  bool arr = !lean && nb > 1 && !s->has_pass && array_lean_eligible(c->hdesc, ops);
  if (arr) {  // the lean array path's element statistics (fsg_array.hip); no room: the exact kernel
    arr = c->arr_b.ensure((size_t)nb * sizeof(ArrBatch)) == hipSuccess &&
          c->arr_bm.ensure((size_t)nb * kArrBmBatch * 4) == hipSuccess;
    (void)hipGetLastError();
    if (arr) {
      ea.arr_b = c->arr_b.as<ArrBatch>();
      ea.arr_bm = c->arr_bm.as<uint32_t>();
    }
  }
  // one substring stage: the flat path (the slice streamed once as bytes,
  // per-16-byte-chunk occurrence / high-byte bits, then one wave per batch decides)
  const int fst = lean ? flat_stage(c->hdesc, ops) : -1;
  // filter_json / projection (with at most one substring stage): the flat JSON path
  const int fjf = lean && fst < 0 && !c->no_fjson ? fjson_flags(c->hdesc, ops) : -1;
  // one bounded regex stage: the flat regex path
  const int rxs = lean && fst < 0 && fjf < 0 && !c->no_frx && s->len >= c->frx_min_rec * std::max<uint64_t>(s->nrec, 1)
                      ? rx_flat_stage(c->hdesc, ops) : -1;
  bool flat = false, fjson = false, frx = false;
  if ((fst >= 0 || fjf >= 0 || rxs >= 0) && !c->no_flat) {
    ea.fbm_words = (s->len + 1023) / 1024;
    // (two words per 1 KiB round; + the rounds past the last)
    const bool have = c->fbm.ensure((size_t)ea.fbm_words * 16 + 64) == hipSuccess;
    (void)hipGetLastError();
    if (have) {
      ea.fbm = c->fbm.as<unsigned long long>();
      if (fst >= 0) {
        flat = true;
        ea.flat_st = (uint32_t)fst | (c->hdesc.st[fst].needle_len << 8);
      } else if (fjf >= 0) {
        fjson = true;
        ea.flat_st = (uint32_t)fjf;
      } else {
        frx = true;
        ea.flat_st = (uint32_t)rxs;
        ea.chain_host_max_len = c->hdesc.st[rxs].dfa.max_len;
      }
    }
  }
  // integer stages over decimal values (filter_odd / map_double / filter_map /
  // aggregate-sum): k_eval_int with the slice's record starts (k_chase_w once per slice)
  bool ints = !lean && !arr && nb > 1 && !s->has_pass && !c->no_int && int_lean_eligible(c->hdesc, ops);
  if (ints) {  // (chains of one group call may share the slice: one framing, the others wait for its event)
    std::lock_guard<std::mutex> lk(s->rs_mu);
    if (!s->rs_ok) {
      ints = s->rs_start.ensure(((size_t)s->nrec + 64) * sizeof(uint16_t)) == hipSuccess &&
             s->rs_end.ensure(((size_t)nb + 1) * sizeof(uint16_t)) == hipSuccess &&
             (s->rs_ev || hipEventCreateWithFlags(&s->rs_ev, hipEventDisableTiming) == hipSuccess);
      (void)hipGetLastError();
      if (ints) {
        EvalArgs ca = ea;
        ca.rstart = s->rs_start.as<uint16_t>();
        ca.rend = s->rs_end.as<uint16_t>();
        launch_chase_w(ca, st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(s->rs_ev, st));
        s->rs_ok = true;
      }
    } else {
      HIPCHK(hipStreamWaitEvent(st, s->rs_ev, 0));
    }
    if (ints) {
      ea.rstart = s->rs_start.as<uint16_t>();
      ea.rend = s->rs_end.as<uint16_t>();
    }
  }
  if (lean || arr || ints) HIPCHK(hipMemsetAsync(ea.list, 0, sizeof(uint32_t), st));
  launch_eval(ea, ops,
              flat ? EVAL_FLAT : fjson ? EVAL_FJSON : frx ? EVAL_RX : lean ? EVAL_LEAN : arr ? EVAL_ARRAY
              : ints ? EVAL_INT : EVAL_EXACT,
              st);
  HIPCHK(hipGetLastError());
  if (c->timed) HIPCHK(hipEventRecord(c->ev[1], st));
  launch_mins(ea.bstat, nb, ea.mins, st);
  SfArgs sfa{};
  const bool has_sf = (c->hdesc.flags & CF_STATEFUL) != 0;
  if (has_sf) {  // stateful last stage: decide + compact, then the minima again (first surviving batch)
    int rc = sf_run(c, s, ea, sfa, st);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(c->mins.p, 0xFF, sizeof(Mins), st));
    launch_mins(ea.bstat, nb, ea.mins, st);
  }
  // aggregate-json: fold the entries in stream order, size every record's map text
  AggjArgs aj{};
  uint64_t aj_nnew = 0;
  if (has_aggj) {
    int rc0 = aj_state_init(c);  // the initial accumulator, parsed once (unwrap_or_default)
    if (rc0) return rc0;
    const uint32_t n_init = c->aj_K;
    const fsg_chain::AjBuf& S = c->ajs[c->aj_cur];
    const size_t nbb = std::max<uint32_t>(nb, 1);
    HIPCHK(c->aj_out.ensure(64));
    HIPCHK(c->aj_bcnt.ensure(nbb * 4));
    HIPCHK(c->aj_brec.ensure(nbb * 8));
    HIPCHK(c->aj_accoff.ensure(nbb * 8));
    HIPCHK(c->aj_acclen.ensure(nbb * 4));
    HIPCHK(hipMemsetAsync(c->aj_out.p, 0, 64, st));
    aj.slice = ea.slice;
    aj.bstat = ea.bstat;
    aj.desc = ea.desc;
    aj.rbase = ea.rbase;
    aj.elem = ea.elem;
    aj.mins = ea.mins;
    aj.nbatches = nb;
    aj.bcnt = c->aj_bcnt.as<uint32_t>();
    aj.brec = c->aj_brec.as<uint64_t>();
    aj.scal = c->aj_out.as<unsigned long long>();
    aj.acc_off = c->aj_accoff.as<uint64_t>();
    aj.acc_len = c->aj_acclen.as<uint32_t>();
    aj.n_init = n_init;
    launch_aggj_count(aj, st);
    unsigned long long sc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(sc, c->aj_out.p, sizeof sc, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t nent = sc[0], nrec = sc[1], most_ent = sc[7];
    uint32_t cap = 16;
    while (cap < 2 * (n_init + nent) + 1) cap <<= 1;
    const size_t nkmax = (size_t)n_init + nent + 1;
    const size_t dict = (size_t)nrec * 44 + (size_t)nent * 8 + (size_t)cap * 12 + nkmax * 28;
    if (dict > c->limit) {
      char b[160];
      snprintf(b, sizeof b, "Requested memory %zub exceeded max allowed %zub", dict, c->limit);
      g_store_mem[0] = 0;
      g_store_mem[1] = dict;
      g_store_mem[2] = c->limit;
      return fail(FSG_E_STORE_MEMORY, b);
    }
    const size_t nr1 = std::max<uint64_t>(nrec, 1), ne1 = std::max<uint64_t>(nent, 1);
    HIPCHK(c->aj_rdesc.ensure(nr1 * 8));
    HIPCHK(c->aj_rne.ensure(nr1 * 4));
    HIPCHK(c->aj_rent.ensure(nr1 * 8));
    HIPCHK(c->aj_rnew.ensure(nr1 * 4));
    HIPCHK(c->aj_rnewb.ensure(nr1 * 8));
    HIPCHK(c->aj_rlen.ensure(nr1 * 4));
    HIPCHK(c->aj_roff.ensure(nr1 * 8));
    HIPCHK(c->aj_ekid.ensure(ne1 * 4));
    HIPCHK(c->aj_eval.ensure(ne1 * 4));
    HIPCHK(c->aj_hrec.ensure(ne1 * 4));
    HIPCHK(c->aj_nkr.ensure(nr1 * 4));
    HIPCHK(c->aj_koff.ensure(nr1 * 8));
    HIPCHK(c->aj_sref.ensure((size_t)cap * 8));
    HIPCHK(c->aj_sid.ensure((size_t)cap * 4));
    HIPCHK(c->aj_tptr.ensure(nkmax * 8));
    HIPCHK(c->aj_tlen.ensure(nkmax * 4));
    HIPCHK(c->aj_kup.ensure(nkmax * 4));
    HIPCHK(c->aj_tsum.ensure(xscan_tiles(std::max<uint64_t>(nrec, std::max<uint64_t>(nent, nb))) * 8));
    HIPCHK(hipMemsetAsync(c->aj_sref.p, 0, (size_t)cap * 8, st));
    if (n_init) {  // the state's keys (match bytes, text, values) straight from HBM
      HIPCHK(hipMemcpyAsync(c->aj_tptr.p, S.tptr.p, (size_t)n_init * 8, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpyAsync(c->aj_tlen.p, S.tlen.p, (size_t)n_init * 4, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemsetAsync(c->aj_kup.p, 0, (size_t)n_init * 4, st));
    }
    aj.kptr = S.kptr.as<uint64_t>();
    aj.klen = S.klen.as<uint32_t>();
    aj.val_init = S.val.as<uint32_t>();
    aj.n_rec = nrec;
    aj.rdesc = c->aj_rdesc.as<uint64_t>();
    aj.rne = c->aj_rne.as<uint32_t>();
    aj.rent = c->aj_rent.as<uint64_t>();
    aj.rnew = c->aj_rnew.as<uint32_t>();
    aj.rnewb = c->aj_rnewb.as<uint64_t>();
    aj.rlen = c->aj_rlen.as<uint32_t>();
    aj.roff = c->aj_roff.as<uint64_t>();
    aj.ekid = c->aj_ekid.as<uint32_t>();
    aj.eval = c->aj_eval.as<uint32_t>();
    aj.slot_ref = c->aj_sref.as<unsigned long long>();
    aj.slot_id = c->aj_sid.as<uint32_t>();
    aj.cap = cap;
    aj.tptr = c->aj_tptr.as<uint64_t>();
    aj.tlen = c->aj_tlen.as<uint32_t>();
    aj.kup = c->aj_kup.as<uint32_t>();
    // the output order's inputs (k_aggj_order): RandomState k0 of the first
    // record's accumulator map, the initial accumulator's entries with repeats
    aj.nkr = c->aj_nkr.as<uint32_t>();
    aj.koff = c->aj_koff.as<uint64_t>();
    aj.hrec = c->aj_hrec.as<uint32_t>();
    aj.k0_base = c->aj_k0 + (!c->aj_touched && c->aj_e0 ? 1u : 0u);
    aj.iseq = !c->aj_touched && c->aj_n_iseq ? c->aj_iseq.as<uint32_t>() : nullptr;
    aj.n_iseq = aj.iseq ? c->aj_n_iseq : 0u;
    aj.agg_stage = (uint32_t)c->agg_stage;
    aj.in_i32 = c->hdesc.st[c->agg_stage].in_type == VT_I32 ? 1u : 0u;
    launch_aggj_keys(aj, c->aj_tsum.as<uint64_t>(), st);
    launch_aggj_kid(aj, nent, st);
    unsigned long long nnew = 0;
    HIPCHK(hipMemcpyAsync(&nnew, aj.scal + 2, sizeof nnew, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t K = n_init + nnew;
    aj_nnew = nnew;
    // blocks of rb records: ~4096 blocks (one wave each), the row table
    // nblk x K bounded to 64 Mi values
    uint64_t rb = std::max<uint64_t>(32, (nrec + 4095) / 4096);
    while (((nrec + rb - 1) / rb) * K > (64ull << 20) && rb < nrec) rb *= 2;
    const uint64_t nblk = nrec ? (nrec + rb - 1) / rb : 0;
    const size_t rows = (size_t)std::max<uint64_t>(nblk * K, 1) * 4;
    const size_t need_rows = dict + rows * (K > kAjLds ? 2 : 1);  // a copy of the rows when K > kAjLds
    if (need_rows > c->limit) {
      char b[160];
      snprintf(b, sizeof b, "Requested memory %zub exceeded max allowed %zub", need_rows, c->limit);
      g_store_mem[0] = dict;
      g_store_mem[1] = need_rows;
      g_store_mem[2] = c->limit;
      return fail(FSG_E_STORE_MEMORY, b);
    }
    HIPCHK(c->aj_state.ensure(rows));
    HIPCHK(hipMemsetAsync(c->aj_state.p, 0, rows, st));
    aj.nkeys = (uint32_t)K;
    aj.rb = (uint32_t)rb;
    aj.nblk = (uint32_t)nblk;
    aj.state = c->aj_state.as<uint32_t>();
    launch_aggj_rows(aj, st);
    AggjArgs a0 = aj;
    if (K > kAjLds) {  // pass 0 replays in place: on a copy of the rows
      HIPCHK(c->aj_state2.ensure(rows));
      HIPCHK(hipMemcpyAsync(c->aj_state2.p, c->aj_state.p, rows, hipMemcpyDeviceToDevice, st));
      a0.state = c->aj_state2.as<uint32_t>();
    }
    a0.write = 0;
    launch_aggj_size(a0, c->aj_tsum.as<uint64_t>(), st);
    launch_aggj_nk(aj, c->aj_tsum.as<uint64_t>(), st);
    // general-path tables of k_aggj_order: the most keys / entries one map
    // holds, one growth past it (a repeated key can reserve at capacity)
    const uint64_t most = std::max<uint64_t>(std::max<uint64_t>(K, most_ent), aj.n_iseq);
    uint32_t ob = 0;
    if (most > kAjRegKeys) {
      uint64_t b = 4;
      while ((b <= 8 ? b - 1 : b / 8 * 7) < most + 1) b *= 2;
      if (2 * b > (1ull << 31)) return fail(FSG_E_UNSUPPORTED, "aggregate-json map past 2^30 keys");
      ob = (uint32_t)(2 * b);
    }
    aj.obmax = ob;
    aj.oscr = nullptr;
    if (ob > kAjLdsBuckets) {
      HIPCHK(c->aj_oscr.ensure((size_t)4 * (ob / 32 + ob) * 4));
      aj.oscr = c->aj_oscr.as<uint32_t>();
    }
  }
  SizeArgs sa{};
  sa.bstat = ea.bstat;
  sa.desc = ea.desc;
  sa.rbase = ea.rbase;
  sa.mins = ea.mins;
  sa.rows = c->rows.as<ScanRow>();
  sa.nbatches = nb;
  sa.acc0 = acc0;
  sa.elem = ea.elem;
  sa.acc_len = has_cat ? c->acc.size() : 0;
  sa.seg = so ? 1u : 0u;
  sa.arr_b = ea.arr_b;
  if (has_array) launch_canon_len(sa, ea.slice, st);
  if (has_agg) {
    sa.agg_only = 1;
    launch_size(sa, st);
    launch_scan(sa.rows, c->aggpre.as<ScanRow>(), c->tiles.as<ScanRow>(), c->grand.as<ScanRow>(), nb, false, 0,
                ea.mins, ea.bstat, st);
    sa.agg_only = 0;
    sa.agg_pre = c->aggpre.as<ScanRow>();
  }
  launch_size(sa, st);
  launch_scan(sa.rows, c->pre.as<ScanRow>(), c->tiles.as<ScanRow>(), c->grand.as<ScanRow>(), nb, true, max_bytes,
              ea.mins, ea.bstat, st);
  PlanArgs pa{};
  pa.bstat = ea.bstat;
  pa.rows = sa.rows;
  pa.pre = c->pre.as<ScanRow>();
  pa.mins = ea.mins;
  pa.plan = c->plan.as<Plan>();
  pa.nbatches = nb;
  pa.tail_status = s->tail_status;
  pa.empty_chain = empty_chain_io ? 1 : 0;
  pa.has_agg = has_agg;
  pa.seg = so ? 1 : 0;
  pa.acc0 = acc0;
  launch_plan(pa, st);
  c->last_pa = pa;
  c->last_sfa = sfa;
  if (!so) {  // a segment's state commits wait for the final segment (commit_deferred)
    if (c->hdesc.flags & CF_AGG_SUM) launch_state(pa.plan, c->dstate.as<int32_t>(), st);
    if (has_sf) launch_sf_commit(sfa, st);  // the stage's state through plan.done
  }
  HIPCHK(hipGetLastError());
  if (c->timed) HIPCHK(hipEventRecord(c->ev[2], st));
  HIPCHK(c->hpin.ensure(kPinPlan + kSmallOut));
  HIPCHK(hipMemcpyAsync(c->hpin.p, c->plan.p, sizeof(Plan), hipMemcpyDeviceToHost, st));
  static_assert(sizeof(Plan) + sizeof(uint32_t) <= kPinPlan, "pinned plan block");
  if (lean || arr || ints)
    HIPCHK(hipMemcpyAsync((uint8_t*)c->hpin.p + sizeof(Plan), ea.list, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  unsigned long long sfs[3] = {0, 0, 0};
  const bool dedup = has_sf && sfa.op == OP_DEDUP && nb && !so;
  if (dedup) HIPCHK(hipMemcpyAsync(sfs, sfa.scal, sizeof sfs, hipMemcpyDeviceToHost, st));
  HIPCHK(wait_stream(st));
  memcpy(&c->hplan, c->hpin.p, sizeof(Plan));
  c->last.eval_path = flat ? FSG_EVAL_FLAT : fjson ? FSG_EVAL_FJSON : frx ? FSG_EVAL_RX : lean ? FSG_EVAL_LEAN
                    : arr ? FSG_EVAL_ARRAY
                    : ints ? FSG_EVAL_INT : FSG_EVAL_EXACT;
  c->last.deferred = 0;
  if (lean || arr || ints) memcpy(&c->last.deferred, (const uint8_t*)c->hpin.p + sizeof(Plan), sizeof(uint32_t));
  if (dedup) {
    c->sf->n_ent = sfs[0];
    c->sf->arena_len = sfs[1];
    c->sf->n = sfs[2];
  }
  if (so && c->hplan.status != 0) {
    // a segment: batches up to the failing one go on; the failure becomes the
    // output slice's tail (the final segment reports it if it gets that far)
    so->tail = c->hplan.status;
    so->fail_batch = c->hplan.done + 1 < (int32_t)nb ? c->hplan.done + 1 : -1;
    pa.nbatches = (uint32_t)(c->hplan.done + 1);
    pa.tail_status = 0;
    launch_plan(pa, st);
    c->last_pa = pa;
    HIPCHK(hipMemcpyAsync(c->hpin.p, c->plan.p, sizeof(Plan), hipMemcpyDeviceToHost, st));
    HIPCHK(wait_stream(st));
    memcpy(&c->hplan, c->hpin.p, sizeof(Plan));
  }
  const Plan p = c->hplan;
  if (m) {
    m->bytes_in += p.bytes_in;
    m->invocation_count += p.invocations;
    if (c->hdesc.nstages) m->records_out += p.records_out;  // the empty chain adds none (engine.rs:179-184)
  }
  if (p.status != 0 && !so && p.done >= 0) {
    // process() completed for batches 0..done before the failing one: their
    // state stands (the reference's chain instance keeps it), as on success
    int rc = FSG_OK;
    if (has_aggj) {
      // the commit lists the keys in the last folded record's output order:
      // this chain's order walk alone (a group call's walks do not wait for it)
      unsigned long long sc[4] = {0, 0, 0, 0};  // scal[6] ord slots
      HIPCHK(hipMemcpy(sc, aj.scal + 3, sizeof sc, hipMemcpyDeviceToHost));
      HIPCHK(c->aj_ord.ensure(std::max<uint64_t>(sc[3], 1) * 4));
      aj.ord = c->aj_ord.as<uint32_t>();
      launch_aggj_hash(aj, st);
      launch_aggj_order(aj, st);
      HIPCHK(hipGetLastError());
      rc = aj_commit(c, aj, p.done, (uint32_t)(aj.n_init + aj_nnew));
    } else if (has_agg && p.acc_touched) {
      if (has_cat) {  // the accumulator stream through `done` (k_cat reads plan.stop = done)
        HIPCHK(c->cat.ensure(kCatOff + c->acc.size() + p.cat_final + 64));
        if (!c->acc.empty())
          HIPCHK(hipMemcpyAsync(c->cat.as<uint8_t>() + kCatOff, c->acc.data(), c->acc.size(), hipMemcpyHostToDevice, st));
        WriteArgs wc{};
        wc.slice = ea.slice;
        wc.bstat = ea.bstat;
        wc.desc = ea.desc;
        wc.rbase = ea.rbase;
        wc.pre = pa.pre;
        wc.agg_pre = c->aggpre.as<ScanRow>();
        wc.plan = pa.plan;
        wc.acc_len = sa.acc_len;
        wc.cat = c->cat.as<uint8_t>();
        launch_cat(wc, nb, st);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(st));
      }
      rc = acc_update(c, p, has_cat);
    }
    if (rc) return rc;
  }
  if (p.status != 0) {
    const char* why = p.status == FSG_E_UNSUPPORTED ? "input needs a feature the GPU path does not implement"
                      : p.status == FSG_E_IO        ? "io error while decoding batches"
                                                    : "failed to decode SmartModule base input";
    return fail(p.status, why);
  }
  // output batch: 61-byte header + records (a segment: 61 bytes per batch + records)
  const uint32_t seg_nb = so && p.stop >= 0 ? (uint32_t)p.stop + 1 : 0u;
  const size_t out_len = so ? 61ull * seg_nb + p.rec_bytes : 61 + p.rec_bytes;
  DevBuf& obuf = so ? so->out->data : c->out;
  if (so) {
    const size_t alloc = slice_alloc(out_len);
    HIPCHK(obuf.ensure(alloc));
    HIPCHK(hipMemsetAsync((uint8_t*)obuf.p + (out_len & ~(size_t)15), 0, alloc - (out_len & ~(size_t)15), st));
  } else {
    HIPCHK(c->out.ensure(out_len + 64));
  }
  HIPCHK(c->crcparts.ensure(sizeof(uint32_t)));
  WriteArgs wa{};
  wa.slice = ea.slice;
  wa.bstat = ea.bstat;
  wa.desc = ea.desc;
  wa.rbase = ea.rbase;
  wa.pre = pa.pre;
  wa.agg_pre = has_agg ? c->aggpre.as<ScanRow>() : nullptr;
  wa.plan = pa.plan;
  wa.out = obuf.as<uint8_t>();
  wa.seg = so ? 1u : 0u;
  wa.acc0 = acc0;
  wa.elem = ea.elem;
  wa.acc_len = sa.acc_len;
  wa.first = p.first;
  wa.last = p.last;
  wa.base = p.base_offset;
  if (has_cat) {  // the accumulator stream: initial accumulator ++ appended values (k_cat)
    HIPCHK(c->cat.ensure(kCatOff + c->acc.size() + p.cat_final + 64));
    if (!c->acc.empty())
      HIPCHK(hipMemcpyAsync(c->cat.as<uint8_t>() + kCatOff, c->acc.data(), c->acc.size(), hipMemcpyHostToDevice, st));
    wa.cat = c->cat.as<uint8_t>();
    launch_cat(wa, nb, st);
  }
  if (has_aggj) {  // pass 1: the map texts into cat (sized by pass 0), keys in the guest's order
    unsigned long long sc[4] = {0, 0, 0, 0};  // scal[3] text bytes, scal[6] ord slots
    HIPCHK(hipMemcpy(sc, aj.scal + 3, sizeof sc, hipMemcpyDeviceToHost));
    const uint64_t aj_total = sc[0], n_ord = sc[3];
    if (aj_total + kCatOff > c->limit) {
      char b[160];
      snprintf(b, sizeof b, "Requested memory %zub exceeded max allowed %zub", (size_t)(aj_total + kCatOff), c->limit);
      g_store_mem[0] = 0;
      g_store_mem[1] = aj_total + kCatOff;
      g_store_mem[2] = c->limit;
      return fail(FSG_E_STORE_MEMORY, b);
    }
    HIPCHK(c->cat.ensure(kCatOff + aj_total + 64));
    HIPCHK(c->aj_ord.ensure(std::max<uint64_t>(n_ord, 1) * 4));  // Σ keys <= text bytes / 8
    aj.ord = c->aj_ord.as<uint32_t>();
    launch_aggj_hash(aj, st);
    if (c->group) {
      int rc = group_order(c, &aj, st);
      if (rc) return rc;
    } else {
      if (c->timed) HIPCHK(hipEventRecord(c->ev_order[0], st));
      launch_aggj_order(aj, st);
      if (c->timed) HIPCHK(hipEventRecord(c->ev_order[1], st));
    }
    aj.cat = c->cat.as<uint8_t>();
    aj.write = 1;
    launch_aggj_write(aj, st);
    wa.cat = aj.cat;
  }
  if (!so) launch_header(pa.plan, wa.out, st);
  if (c->timed) HIPCHK(hipEventRecord(c->ev[3], st));
  const uint32_t nblk = p.last >= p.first && p.first >= 0 ? (uint32_t)(p.last - p.first + 1) : 0u;
  // verbatim records (filters, uppercase, projections): staged in LDS
  // (k_write_lean; a batch beyond its staging buffer or 64 survivors takes the
  // wave path inside it); measured on MI355X: C2 1 KB records write 1.33 -> 1.23
  // ms, C2-json 1.89 -> 1.39 ms against k_write's record-by-record wave copies
  const bool verbatim = !has_agg && !has_array && c->hdesc.out_type != VT_I32;
  // generated integer values (map_double / filter_map outputs, aggregate-sum's
  // running sums): staged per batch in LDS (k_write_gen)
  const bool gen_int = !has_array && !has_aggj && !has_cat &&
                       (c->hdesc.out_type == VT_I32 || (c->hdesc.flags & CF_AGG_SUM));
  if (verbatim && nblk && p.n_records)
    launch_write_lean(wa, nblk, st);
  else if (gen_int && nblk && p.n_records)
    launch_write_gen(wa, nblk, st);
  else
    launch_write(wa, nblk, st);
  if (arr) {  // the lean batches' element records (k_write skips them)
    ArrWriteArgs aw{};
    aw.slice = ea.slice;
    aw.bpos = ea.bpos;
    aw.rbase = ea.rbase;
    aw.nbatches = nb;
    aw.seg = wa.seg;
    aw.nrec = s->nrec;
    aw.bstat = ea.bstat;
    aw.arr_bm = ea.arr_bm;
    aw.pre = pa.pre;
    aw.plan = pa.plan;
    aw.out = wa.out;
    launch_array_write(aw, nblk, st);
  }
  if (has_array) launch_write_canon(wa, nblk, st);
  HIPCHK(hipGetLastError());
  if (c->timed) HIPCHK(hipEventRecord(c->ev[4], st));
  if (so) {  // the next segment's input: headers, positions, record-count prefix, pass-through flags
    fsg_slice* o = so->out;
    HIPCHK(o->bpos.ensure(std::max<size_t>(seg_nb, 1) * 8));
    HIPCHK(o->rbase.ensure(std::max<size_t>(seg_nb, 1) * 8));
    HIPCHK(o->pass.ensure(std::max<size_t>(seg_nb, 1)));
    SegArgs ga{};
    ga.src = ea.slice;
    ga.bpos = ea.bpos;
    ga.rows = sa.rows;
    ga.pre = pa.pre;
    ga.nb = seg_nb;
    ga.pass_batch = p.err_batch;
    ga.pass_in = ea.pass;
    ga.dst = obuf.as<uint8_t>();
    ga.dbpos = o->bpos.as<uint64_t>();
    ga.drbase = o->rbase.as<uint64_t>();
    ga.dpass = o->pass.as<uint8_t>();
    launch_seg_headers(ga, st);
    o->eng = c->eng;
    o->len = out_len;
    o->rs_ok = false;
    o->nb = seg_nb;
    o->nrec = p.n_records;
    o->header_bytes = out_len;
    o->tail_status = p.err_batch >= 0 ? 0 : so->tail;  // an error batch ends the slice
    o->device_framed = true;
    o->decompressed = s->decompressed;
    o->has_pass = p.err_batch >= 0 || s->has_pass;
  } else {
    launch_crc(wa.out, 21, out_len - 21, c->crcparts.as<uint32_t>(), st);
  }
  HIPCHK(hipGetLastError());
  if (c->timed) HIPCHK(hipEventRecord(c->ev[5], st));
  c->out_pinned = !so && out_len <= kSmallOut;
  if (c->out_pinned)
    HIPCHK(hipMemcpyAsync((uint8_t*)c->hpin.p + kPinPlan, wa.out, out_len, hipMemcpyDeviceToHost, st));
  HIPCHK(wait_stream(st));
  c->out_len = out_len;
  if (cy) {  // CRC32C of [21, out_len) as k_crc_final stored it (big-endian at 17)
    uint8_t b4[4];
    HIPCHK(hipMemcpy(b4, wa.out + 17, 4, hipMemcpyDeviceToHost));
    cy->crc = (uint32_t)b4[0] << 24 | (uint32_t)b4[1] << 16 | (uint32_t)b4[2] << 8 | b4[3];
  }
  // timings
  float t[5] = {0};
  if (c->timed)
    for (int k = 0; k < 5; k++) HIPCHK(hipEventElapsedTime(&t[k], c->ev[k], c->ev[k + 1]));
  c->last.eval_ms = t[0];
  c->last.plan_ms = t[1];
  c->last.write_ms = t[3];
  c->last.crc_ms = t[4];
  c->last.text_ms = t[2];
  c->last.total_ms = t[0] + t[1] + t[2] + t[3] + t[4];
  c->last.order_ms = 0;
  c->last.chunks = 0;
  if (has_aggj && aj.n_rec) {  // the order walk alone (the group's launch for a group call: timed when its first chain is)
    AjGroup* g = c->group;
    if (g && g->timed && g->t0 && g->t1)
      HIPCHK(hipEventElapsedTime(&c->last.order_ms, g->t0, g->t1));
    else if (!g && c->timed)
      HIPCHK(hipEventElapsedTime(&c->last.order_ms, c->ev_order[0], c->ev_order[1]));
  }
  c->last.in_bytes = s->header_bytes;
  c->last.out_bytes = out_len;
  c->last.n_batches = nb;
  c->last.n_records_in = s->nrec;
  // result
  res->base_offset = p.base_offset;
  res->last_offset_delta = p.lod;
  res->n_records = (uint32_t)p.n_records;
  if (p.err_batch >= 0) {
    BatchStat bs;
    HIPCHK(hipMemcpy(&bs, ea.bstat + p.err_batch, sizeof bs, hipMemcpyDeviceToHost));
    int rc = build_error(c, s, bs, res->error);
    if (rc) return rc;
    res->has_error = 1;
  }
  c->last_aj = aj;
  c->last_aj_kmax = (uint32_t)(aj.n_init + aj_nnew);
  c->last_has_aggj = has_aggj;
  if (so) return FSG_OK;  // state commits: commit_deferred, once the final segment's stop is known
  if (has_aggj && p.stop >= 0) {  // the map after the last processed batch stays in HBM
    int rc = aj_commit(c, aj, p.stop, (uint32_t)(aj.n_init + aj_nnew));
    if (rc) return rc;
  }
  if (has_agg && !has_aggj && p.acc_touched) return acc_update(c, p, has_cat);
  return FSG_OK;
}

// the state commits of segment `c` of a composed chain through `done` (the
// last batch whose process() call completed, as the final segment decided):
// k_plan again with the cut at `done`, then the commits run_slice skipped
int commit_deferred(fsg_chain* c, int32_t done) {
  const bool has_agg = c->agg_stage >= 0, has_sf = (c->hdesc.flags & CF_STATEFUL) != 0;
  if ((!has_agg && !has_sf) || done < 0) return FSG_OK;
  hipStream_t st = c->stream;
  HIPCHK(c->aj_cout.ensure(64));
  const uint32_t cut = (uint32_t)done;
  HIPCHK(hipMemcpyAsync(&c->mins.as<Mins>()->cut, &cut, sizeof cut, hipMemcpyHostToDevice, st));
  launch_plan(c->last_pa, st);
  if (c->hdesc.flags & CF_AGG_SUM) launch_state(c->last_pa.plan, c->dstate.as<int32_t>(), st);
  const SfArgs& sfa = c->last_sfa;
  const bool dedup = has_sf && sfa.op == OP_DEDUP && sfa.nbatches;
  if (has_sf) launch_sf_commit(sfa, st);
  HIPCHK(hipGetLastError());
  unsigned long long sfs[3] = {0, 0, 0};
  if (dedup) HIPCHK(hipMemcpyAsync(sfs, sfa.scal, sizeof sfs, hipMemcpyDeviceToHost, st));
  Plan p;
  HIPCHK(hipMemcpyAsync(&p, c->last_pa.plan, sizeof p, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (dedup) {
    c->sf->n_ent = sfs[0];
    c->sf->arena_len = sfs[1];
    c->sf->n = sfs[2];
  }
  if (p.status != 0) return FSG_OK;
  if (c->last_has_aggj) return p.stop >= 0 ? aj_commit(c, c->last_aj, p.stop, c->last_aj_kmax) : FSG_OK;
  if (has_agg && p.acc_touched) return acc_update(c, p, (c->hdesc.flags & CF_AGG_CAT) != 0);
  return FSG_OK;
}

// a composed chain: segment k's per-batch output (one batch per input batch,
// the source headers) is segment k + 1's input, as the reference feeds each
// stage's successes to the next one per SmartModuleInput (engine.rs:147-167).
// A segment's error batch passes through the later segments unchanged (the
// reference returns that stage's partial output at once) and its error is the
// chain's if the final segment gets that far; the SPU's max_bytes and stop
// rules run on the final segment's output; state commits run once the final
// stop is known; metrics count the original input (engine.rs:139-141).
int run_composed(fsg_chain* c, const fsg_slice* s, uint64_t max_bytes, fsg_metrics* m, fsg_batch_output* res) {
  const size_t n = c->segs.size();
  if (!c->seg_io) c->seg_io.reset(new fsg_slice[n - 1]);
  HIPCHK(hipStreamSynchronize(c->stream));  // the input was uploaded on the outer chain's stream
  const fsg_slice* in = s;
  fsg_runtime_error pend{};
  int32_t pend_batch = -1;
  int fail_status = 0, fail_batch = -1;
  for (size_t k = 0; k + 1 < n; k++) {
    fsg_chain* g = c->segs[k].get();
    g->timed = c->timed;
    SegOut so{&c->seg_io[k], 0, -1};
    fsg_batch_output r;
    int rc = run_slice(g, in, ~0ull, nullptr, &r, false, &so);
    if (rc) {
      free_error(r.error);
      free_error(pend);
      return rc;
    }
    if (r.has_error) {  // ends this segment's output; an earlier pending error lay beyond it
      free_error(pend);
      pend = r.error;
      pend_batch = g->hplan.err_batch;
    } else {
      free_error(r.error);
    }
    if (so.tail && so.fail_batch >= 0) {
      fail_status = so.tail;
      fail_batch = so.fail_batch;
    }
    in = &c->seg_io[k];
  }
  fsg_chain* f = c->segs.back().get();
  f->timed = c->timed;
  int rc = run_slice(f, in, max_bytes, nullptr, res, false);
  const Plan pf = f->hplan;
  // metrics of the original input: per process() call its raw bytes (segment 0's rows)
  if (m) {
    uint64_t inv = pf.invocations;
    if (rc && fail_batch >= 0 && pf.status == fail_status && inv == (uint64_t)fail_batch) inv++;  // the failing call
    uint64_t bin = 0;
    if (inv) {
      ScanRow r2[2];
      fsg_chain* g0 = c->segs[0].get();
      HIPCHK(hipMemcpy(&r2[0], g0->pre.as<ScanRow>() + (inv - 1), sizeof(ScanRow), hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(&r2[1], g0->rows.as<ScanRow>() + (inv - 1), sizeof(ScanRow), hipMemcpyDeviceToHost));
      bin = r2[0].bytes_in + r2[1].bytes_in;
    }
    m->bytes_in += bin;
    m->invocation_count += inv;
    m->records_out += pf.records_out;
  }
  if (rc) {
    free_error(pend);
    return rc;
  }
  if (pend_batch >= 0 && pf.stop == pend_batch && !res->has_error) {
    res->error = pend;
    res->has_error = 1;
    pend = fsg_runtime_error{};
  }
  free_error(pend);
  for (size_t k = 0; k + 1 < n; k++) {
    rc = commit_deferred(c->segs[k].get(), pf.done);
    if (rc) return rc;
  }
  return FSG_OK;
}

// Host buffers for downloaded batches.  Large ones (>= 4 MiB) are 2 MiB aligned,
// advised onto transparent huge pages and recycled: host_free parks a large
// buffer in a small process-wide cache and host_alloc takes it back for the
// next output that fits, so a repeated multi-GB process_batch reuses memory
// that is already faulted in (first touch zero-fills every page, which costs
// as much as the D2H copy itself).
constexpr size_t kHuge = 2u << 20;
constexpr int kHostCache = 2;  // parked buffers, process-wide
struct HostPool {
  std::mutex mu;
  std::map<void*, size_t> live;              // large buffers handed out -> capacity
  std::vector<std::pair<void*, size_t>> parked;
};
HostPool& host_pool() {
  static HostPool* p = new HostPool;  // never destroyed: frees may run at exit
  return *p;
}

uint8_t* host_alloc(size_t n) {
  if (n < 2 * kHuge) return (uint8_t*)malloc(std::max<size_t>(n, 1));
  HostPool& hp = host_pool();
  {
    std::lock_guard<std::mutex> g(hp.mu);
    for (size_t i = 0; i < hp.parked.size(); i++) {
      if (hp.parked[i].second >= n && hp.parked[i].second <= 2 * n) {
        auto b = hp.parked[i];
        hp.parked.erase(hp.parked.begin() + i);
        hp.live[b.first] = b.second;
        return (uint8_t*)b.first;
      }
    }
  }
  const size_t cap = (n + kHuge - 1) & ~(kHuge - 1);
  void* p = nullptr;
  if (posix_memalign(&p, kHuge, cap)) return nullptr;
  (void)madvise(p, cap, MADV_HUGEPAGE);
  std::lock_guard<std::mutex> g(hp.mu);
  hp.live[p] = cap;
  return (uint8_t*)p;
}

void host_free(const void* q) {
  if (!q) return;
  void* p = const_cast<void*>(q);
  HostPool& hp = host_pool();
  {
    std::lock_guard<std::mutex> g(hp.mu);
    auto it = hp.live.find(p);
    if (it != hp.live.end()) {
      const size_t cap = it->second;
      hp.live.erase(it);
      hp.parked.emplace_back(p, cap);
      if ((int)hp.parked.size() <= kHostCache) return;
      p = hp.parked.front().first;  // evict the oldest parked buffer
      hp.parked.erase(hp.parked.begin());
    }
  }
  free(p);
}

}  // namespace

// frees every parked output buffer (buffers still held by the caller are untouched)
extern "C" void fsg_host_cache_trim(void) {
  HostPool& hp = host_pool();
  std::vector<std::pair<void*, size_t>> v;
  {
    std::lock_guard<std::mutex> g(hp.mu);
    v.swap(hp.parked);
  }
  for (auto& b : v) free(b.first);
}

namespace {
constexpr size_t kDlChunk = 32u << 20;
constexpr size_t kDlStaged = 128u << 20;  // outputs from here on take the staged download
constexpr int kDlThreads = 4;

// host copy of one staged chunk, split over kDlThreads threads
void copy_out(uint8_t* dst, const uint8_t* src, size_t n) {
  std::thread th[kDlThreads - 1];
  const size_t part = (n / kDlThreads + 4095) & ~(size_t)4095;
  for (int t = 1; t < kDlThreads; t++) {
    const size_t a = std::min(n, part * t), b = std::min(n, part * (t + 1));
    th[t - 1] = std::thread([=] {
      if (b > a) memcpy(dst + a, src + a, b - a);
    });
  }
  memcpy(dst, src, std::min(n, part));
  for (auto& x : th) x.join();
}

// device -> pinned chunk k (alternating buffers) -> caller memory: the DMA of
// chunk k+1 runs while the host copies chunk k out of the other buffer
hipError_t staged_copy(PinBuf& pin, hipEvent_t* ev, hipStream_t st, uint8_t* dst, const uint8_t* src, size_t n) {
  hipError_t e = pin.ensure(2 * kDlChunk);
  for (int k = 0; k < 2 && e == hipSuccess; k++)
    if (!ev[k]) e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
  if (e != hipSuccess) return e;
  uint8_t* buf[2] = {(uint8_t*)pin.p, (uint8_t*)pin.p + kDlChunk};
  const size_t nch = (n + kDlChunk - 1) / kDlChunk;
  auto issue = [&](size_t k) -> hipError_t {
    const size_t off = k * kDlChunk, len = std::min(kDlChunk, n - off);
    hipError_t r = hipMemcpyAsync(buf[k & 1], src + off, len, hipMemcpyDeviceToHost, st);
    return r == hipSuccess ? hipEventRecord(ev[k & 1], st) : r;
  };
  for (size_t k = 0; k < std::min<size_t>(2, nch) && e == hipSuccess; k++) e = issue(k);
  for (size_t k = 0; k < nch && e == hipSuccess; k++) {
    e = hipEventSynchronize(ev[k & 1]);
    if (e != hipSuccess) break;
    const size_t off = k * kDlChunk;
    copy_out(dst + off, buf[k & 1], std::min(kDlChunk, n - off));
    if (k + 2 < nch) e = issue(k + 2);
  }
  if (e != hipSuccess) (void)hipStreamSynchronize(st);  // nothing left in flight into the pinned chunks
  return e;
}
hipError_t staged_download(fsg_chain* c, uint8_t* dst, const uint8_t* src, size_t n) {
  return staged_copy(c->hstage, c->dl_ev, c->stream, dst, src, n);
}

// the chain holding the output of the last call (a composed chain: its final segment)
fsg_chain* fin(fsg_chain* c) { return c->segs.empty() ? c : c->segs.back().get(); }

int download_output(fsg_chain* c0, fsg_batch_output* res) {
  fsg_chain* c = fin(c0);
  uint8_t* h = host_alloc(c->out_len);
  if (!h) return fail(FSG_E_DEVICE, "host allocation failed");
  hipError_t e = hipSuccess;
  if (c->out_pinned)
    memcpy(h, (const uint8_t*)c->hpin.p + kPinPlan, c->out_len);
  else if (c->out_len >= kDlStaged)
    e = staged_download(c, h, (const uint8_t*)c->out.p, c->out_len);
  else
    e = hipMemcpy(h, c->out.p, c->out_len, hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    host_free(h);
    return fail(FSG_E_DEVICE, hipGetErrorString(e));
  }
  res->batch = h;
  res->batch_len = c->out_len;
  return FSG_OK;
}

}  // namespace

extern "C" int fsg_chain_process_slice(fsg_chain* c, const fsg_slice* s, uint64_t max_bytes, fsg_metrics* m,
                                       fsg_batch_output** out) {
  HIPCHK(hipSetDevice(c->eng->device));
  auto res = std::make_unique<fsg_batch_output>();
  int rc = run_slice(c, s, max_bytes, m, res.get(), c->hdesc.nstages == 0);
  if (rc) {
    free_error(res->error);
    return rc;
  }
  if (out) {
    rc = download_output(c, res.get());
    if (rc) {
      free_error(res->error);
      return rc;
    }
    *out = res.release();
  } else {
    free_error(res->error);
  }
  return FSG_OK;
}

// The aggregate-sum group path: chains that are one aggregate-sum stage over
// a resident slice of decimal records (k_eval_int's chains, C5) run as ONE
// launch per phase over the whole group (fsg_launch.h GaJob): jobs uploaded
// once, phase 1 (eval, minima, sizes, scans, plan, accumulator) and its
// read-back with one wait, the host sizes the outputs, phase 2 (header,
// records, CRC32C) with one wait.  A chain whose batches the integer kernel
// defers, or whose call ends in an error, is re-run on the general path (its
// accumulator depends only on the host accumulator and its input, so the
// re-run commits the same state).  Returns the indices left to the general path.
int group_agg_fast(fsg_chain* const* chains, const fsg_slice* const* slices, size_t n, uint64_t max_bytes,
                   fsg_metrics* metrics, fsg_batch_output** outs, int* rcs, std::vector<size_t>& rest) {
  std::vector<size_t> fast;
  rest.clear();
  static const bool disabled = getenv("FSG_NO_GROUP_FAST") != nullptr;
  for (size_t i = 0; i < n; i++) {
    fsg_chain* c = chains[i];
    const fsg_slice* s = slices[i];
    const ChainDesc& h = c->hdesc;
    const bool ok = !disabled && c->segs.empty() && h.nstages == 1 && h.st[0].op == OP_AGG_SUM && (h.flags & CF_AGG_SUM) &&
                    !h.st[0].acc_bad && h.st[0].in_type == VT_SRC && !c->no_int && s->nb > 1 &&
                    scan_tiles(s->nb) == 1 && !s->has_pass && s->rs_ok && c->dstate.p &&
                    (size_t)s->nb * (sizeof(BatchStat) + 3 * sizeof(ScanRow)) + (size_t)s->nrec * sizeof(KeptRec) <=
                        c->limit;
    (ok ? fast : rest).push_back(i);
  }
  if (fast.size() < 2) {  // one chain: the general path
    if (!fast.empty()) rest.insert(rest.begin(), fast[0]);
    return FSG_OK;
  }
  auto bail = [&](const char*) {  // an allocation failed: every chain takes the general path
    rest.resize(n);
    for (size_t i = 0; i < n; i++) rest[i] = i;
    (void)hipGetLastError();
    return FSG_OK;
  };
  fsg_engine* e = chains[0]->eng;
  if (!e->gst && hipStreamCreateWithFlags(&e->gst, hipStreamNonBlocking) != hipSuccess) return bail("stream");
  for (auto& ev : e->ga_ev)
    if (!ev && hipEventCreate(&ev) != hipSuccess) return bail("event");
  hipStream_t gs = e->gst;
  const uint32_t m = (uint32_t)fast.size();
  // buffers of each chain (grow-only; after the first call nothing is allocated)
  for (size_t i : fast) {
    fsg_chain* c = chains[i];
    const fsg_slice* s = slices[i];
    const uint32_t nb = s->nb;
    if (c->bstat.ensure(nb * sizeof(BatchStat)) || c->kept.ensure(std::max<uint64_t>(s->nrec, 1) * sizeof(KeptRec)) ||
        c->rows.ensure(nb * sizeof(ScanRow)) || c->pre.ensure(nb * sizeof(ScanRow)) ||
        c->aggpre.ensure(nb * sizeof(ScanRow)) || c->defer.ensure(((size_t)nb + 1) * sizeof(uint32_t)) ||
        c->mins.ensure(sizeof(Mins)) || c->plan.ensure(sizeof(Plan)) || c->crcparts.ensure(sizeof(uint32_t)))
      return bail("buffers");
  }
  // jobs | 5 offset tables | read-back rows
  const size_t jb = (size_t)m * sizeof(GaJob), ob = (size_t)5 * (m + 1) * sizeof(uint32_t);
  const size_t rb_off = (jb + ob + 255) & ~(size_t)255, total = rb_off + (size_t)m * sizeof(GaResult);
  if (e->ga_dev.ensure(total) || e->ga_pin.ensure(total)) return bail("job buffers");
  uint8_t* hp = (uint8_t*)e->ga_pin.p;
  GaJob* J = (GaJob*)hp;
  uint32_t* off = (uint32_t*)(hp + jb);
  uint32_t* oe = off, *om = off + (m + 1), *os = off + 2 * (m + 1), *ow = off + 3 * (m + 1), *oc = off + 4 * (m + 1);
  oe[0] = om[0] = os[0] = ow[0] = oc[0] = 0;
  // the chains' earlier work (a collect, the record starts) before the group stream reads their buffers
  for (size_t i : fast) {
    fsg_chain* c = chains[i];
    if (hipStreamQuery(c->stream) == hipErrorNotReady) (void)hipStreamSynchronize(c->stream);
    if (slices[i]->rs_ev) (void)hipEventSynchronize(slices[i]->rs_ev);
  }
  (void)hipGetLastError();
  for (uint32_t k = 0; k < m; k++) {
    fsg_chain* c = chains[fast[k]];
    const fsg_slice* s = slices[fast[k]];
    const uint32_t nb = s->nb;
    GaJob g{};
    EvalArgs& ea = g.ea;
    ea.slice = (const uint8_t*)s->data.p;
    ea.slice_len = s->len;
    ea.bpos = s->bpos.as<uint64_t>();
    ea.rbase = s->rbase.as<uint64_t>();
    ea.nbatches = nb;
    ea.chain = c->d_desc.as<ChainDesc>();
    ea.blob = c->d_blob.as<uint8_t>();
    ea.bstat = c->bstat.as<BatchStat>();
    ea.desc = c->kept.as<KeptRec>();
    ea.mins = c->mins.as<Mins>();
    ea.list = c->defer.as<uint32_t>();
    ea.nrec = s->nrec;
    ea.rstart = s->rs_start.as<uint16_t>();
    ea.rend = s->rs_end.as<uint16_t>();
    const int64_t acc0 = acc_value(c->acc);
    SizeArgs& sa = g.sa;
    sa.bstat = ea.bstat;
    sa.desc = ea.desc;
    sa.rbase = ea.rbase;
    sa.mins = ea.mins;
    sa.rows = c->rows.as<ScanRow>();
    sa.nbatches = nb;
    sa.acc0 = acc0;
    g.aggpre = c->aggpre.as<ScanRow>();
    g.pre = c->pre.as<ScanRow>();
    g.max_bytes = max_bytes;
    PlanArgs& pa = g.pa;
    pa.bstat = ea.bstat;
    pa.rows = sa.rows;
    pa.pre = g.pre;
    pa.mins = ea.mins;
    pa.plan = c->plan.as<Plan>();
    pa.nbatches = nb;
    pa.tail_status = s->tail_status;
    pa.has_agg = 1;
    pa.acc0 = acc0;
    g.state = c->dstate.as<int32_t>();
    g.crc_acc = c->crcparts.as<uint32_t>();
    J[k] = g;
    oe[k + 1] = oe[k] + nb;
    om[k + 1] = om[k] + ga_mins_blocks(nb);
    os[k + 1] = os[k] + (nb + 3) / 4;
  }
  GaJob* dJ = e->ga_dev.as<GaJob>();
  const uint32_t* doff = (const uint32_t*)((uint8_t*)e->ga_dev.p + jb);
  GaResult* dres = (GaResult*)((uint8_t*)e->ga_dev.p + rb_off);
  GaOffsets o{doff, doff + (m + 1), doff + 2 * (m + 1), doff + 3 * (m + 1), doff + 4 * (m + 1),
              oe[m], om[m], os[m], 0, 0};
  const bool timed = chains[fast[0]]->timed;
  HIPCHK(hipMemcpyAsync(e->ga_dev.p, hp, jb + ob, hipMemcpyHostToDevice, gs));
  if (timed) HIPCHK(hipEventRecord(e->ga_ev[0], gs));
  launch_ga_phase1(dJ, m, o, dres, gs);
  if (timed) HIPCHK(hipEventRecord(e->ga_ev[1], gs));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(hp + rb_off, dres, (size_t)m * sizeof(GaResult), hipMemcpyDeviceToHost, gs));
  HIPCHK(wait_stream(gs));
  const GaResult* R = (const GaResult*)(hp + rb_off);
  // the plans: outputs sized, abnormal chains back to the general path
  std::vector<uint8_t> done(m, 0);
  for (uint32_t k = 0; k < m; k++) {
    fsg_chain* c = chains[fast[k]];
    const Plan& p = R[k].plan;
    if (R[k].deferred || p.status != 0 || p.err_batch >= 0) {
      J[k].out_len = 0;
      J[k].wa = WriteArgs{};
      J[k].wa.first = -1;
      ow[k + 1] = ow[k];
      oc[k + 1] = oc[k];
      continue;
    }
    done[k] = 1;
    const size_t out_len = 61 + p.rec_bytes;
    if (c->out.ensure(out_len + 64)) return bail("output");
    WriteArgs& wa = J[k].wa;
    wa = WriteArgs{};
    wa.slice = J[k].ea.slice;
    wa.bstat = J[k].ea.bstat;
    wa.desc = J[k].ea.desc;
    wa.rbase = J[k].ea.rbase;
    wa.pre = J[k].pre;
    wa.agg_pre = J[k].aggpre;
    wa.plan = J[k].pa.plan;
    wa.out = c->out.as<uint8_t>();
    wa.acc0 = J[k].pa.acc0;
    wa.first = p.first;
    wa.last = p.last;
    wa.base = p.base_offset;
    J[k].out_len = out_len;
    const uint32_t nblk = p.last >= p.first && p.first >= 0 && p.n_records ? (uint32_t)(p.last - p.first + 1) : 0u;
    ow[k + 1] = ow[k] + nblk;
    oc[k + 1] = oc[k] + ga_crc_blocks(out_len);
  }
  o.t_write = ow[m];
  o.t_crc = oc[m];
  HIPCHK(hipMemcpyAsync(e->ga_dev.p, hp, jb + ob, hipMemcpyHostToDevice, gs));
  launch_ga_phase2(dJ, m, o, gs);
  if (timed) {
    HIPCHK(hipEventRecord(e->ga_ev[2], gs));
    HIPCHK(hipEventRecord(e->ga_ev[3], gs));
  }
  HIPCHK(hipGetLastError());
  HIPCHK(wait_stream(gs));
  float t1 = 0, t2 = 0;
  if (timed) {
    HIPCHK(hipEventElapsedTime(&t1, e->ga_ev[0], e->ga_ev[1]));
    HIPCHK(hipEventElapsedTime(&t2, e->ga_ev[1], e->ga_ev[2]));
  }
  for (uint32_t k = 0; k < m; k++) {
    const size_t i = fast[k];
    fsg_chain* c = chains[i];
    const fsg_slice* s = slices[i];
    if (!done[k]) {
      rest.push_back(i);
      continue;
    }
    const Plan& p = R[k].plan;
    c->hplan = p;
    c->last_pa = J[k].pa;
    c->out_len = J[k].out_len;
    c->out_pinned = false;
    c->last_has_aggj = false;
    fsg_timings& t = c->last;
    t = fsg_timings{};
    if (k == 0) {  // the group's phase times on its first chain (the phases are one launch each for every chain)
      t.eval_ms = t1;
      t.write_ms = t2;
      t.total_ms = t1 + t2;
    }
    t.in_bytes = s->header_bytes;
    t.out_bytes = J[k].out_len;
    t.n_batches = s->nb;
    t.n_records_in = s->nrec;
    t.eval_path = FSG_EVAL_INT;
    if (metrics) {
      metrics[i].bytes_in += p.bytes_in;
      metrics[i].invocation_count += p.invocations;
      metrics[i].records_out += p.records_out;
    }
    rcs[i] = FSG_OK;
    if (p.acc_touched) (void)acc_update(c, p, false);
    if (outs) {
      auto res = std::make_unique<fsg_batch_output>();
      res->base_offset = p.base_offset;
      res->last_offset_delta = p.lod;
      res->n_records = (uint32_t)p.n_records;
      const int rc = download_output(c, res.get());
      if (rc) {
        rcs[i] = rc;
        continue;
      }
      outs[i] = res.release();
    }
  }
  return FSG_OK;
}

extern "C" int fsg_chain_group_process_slices(fsg_chain* const* chains, const fsg_slice* const* slices, size_t n,
                                              uint64_t max_bytes, fsg_metrics* metrics, fsg_batch_output** outs,
                                              int* rcs) {
  if (!chains || !slices || !rcs || n > 4096) return fail(FSG_E_INVALID_ARG, "fsg_chain_group_process_slices: bad arguments");
  if (!n) return FSG_OK;
  for (size_t i = 0; i < n; i++) {
    if (!chains[i] || !slices[i]) return fail(FSG_E_INVALID_ARG, "fsg_chain_group_process_slices: null chain / slice");
    for (size_t j = 0; j < i; j++)
      if (chains[j] == chains[i]) return fail(FSG_E_INVALID_ARG, "fsg_chain_group_process_slices: a chain twice");
    if (chains[i]->eng->device != chains[0]->eng->device)
      return fail(FSG_E_INVALID_ARG, "fsg_chain_group_process_slices: chains on different devices");
  }
  std::unique_lock<std::mutex> glk(chains[0]->eng->gmu);
  HIPCHK(hipSetDevice(chains[0]->eng->device));
  if (outs)
    for (size_t i = 0; i < n; i++) outs[i] = nullptr;
  // aggregate-sum chains over decimal records: one launch per phase for all of them
  std::vector<size_t> todo;
  const int frc = group_agg_fast(chains, slices, n, max_bytes, metrics, outs, rcs, todo);
  if (frc) return frc;
  AjGroup g;
  g.device = chains[0]->eng->device;
  g.eng = chains[0]->eng;
  g.expected = todo.size();
  std::vector<size_t> walkers, others;
  for (size_t i : todo) {
    fsg_chain* c = chains[i];
    // only plain aggregate-json chains walk in the group; the others arrive at once
    const bool walks = (c->hdesc.flags & CF_AGG_JSON) && c->segs.empty();
    c->group = &g;
    c->group_arrived = false;
    if (!walks) (void)group_arrive(c, nullptr, nullptr);
    (walks ? walkers : others).push_back(i);
  }
  std::vector<std::string> errs(n);
  std::vector<std::array<uint64_t, 3>> smem(n);  // g_store_mem is thread-local too
  // per-phase timing events on the first chain only: ~8 event calls per chain
  // and call contend for the runtime's locks with every other chain's launches
  std::vector<uint8_t> was_timed(n);
  for (size_t i = 0; i < n; i++) {
    was_timed[i] = chains[i]->timed ? 1 : 0;
    if (i) chains[i]->timed = false;
  }
  auto one = [&](size_t i) {
    fsg_chain* c = chains[i];
    if (outs) outs[i] = nullptr;
    rcs[i] = fsg_chain_process_slice(c, slices[i], max_bytes, metrics ? metrics + i : nullptr, outs ? outs + i : nullptr);
    if (rcs[i]) {
      errs[i] = g_err;
      smem[i] = {g_store_mem[0], g_store_mem[1], g_store_mem[2]};
    }
    (void)group_arrive(c, nullptr, nullptr);  // a chain that failed before its walk
  };
  // a walker blocks at the rendezvous until every walker has arrived: one
  // thread each; the other chains share a pool (host launch and sync work
  // does not scale past ~16 threads)
  std::vector<std::thread> th;
  th.reserve(walkers.size() + 16);
  for (size_t i : walkers) th.emplace_back(one, i);
  std::atomic<size_t> next{0};
  static const size_t kPool = getenv("FSG_GROUP_THREADS") ? std::max(1, atoi(getenv("FSG_GROUP_THREADS"))) : 16;
  const size_t pool = std::min<size_t>(others.size(), kPool);
  for (size_t k = 0; k < pool; k++)
    th.emplace_back([&] {
      for (size_t j = next++; j < others.size(); j = next++) one(others[j]);
    });
  for (auto& t : th) t.join();
  int rc = FSG_OK;
  for (size_t i = 0; i < n; i++) {
    chains[i]->group = nullptr;
    chains[i]->timed = was_timed[i] != 0;
    if (rcs[i] && rc == FSG_OK) {
      rc = rcs[i];
      g_err = errs[i];
      for (int k = 0; k < 3; k++) g_store_mem[k] = smem[i][k];
    }
  }
  HIPCHK(hipSetDevice(g.device));
  if (g.st) HIPCHK(hipStreamSynchronize(g.st));  // the job list is rewritten by the next group call
  return rc;
}

extern "C" int fsg_chain_output_device(fsg_chain* c0, const void** dptr, size_t* len) {
  fsg_chain* c = fin(c0);
  *dptr = c->out.p;
  *len = c->out_len;
  return FSG_OK;
}


// ---------------------------------------------------------------------------
// Pipelined process_batch: for a host slice of at least two chunks, H2D of
// the slice (64 MiB pieces, an upload thread on its own stream), processing of
// chunk k (whole batches, framed on the device) and D2H of chunk k - 1's
// records (a download thread: pinned pieces, copied out) overlap.  The output
// is the one batch the serial path returns: chunk k > 0 continues the batch an
// earlier chunk started (Mins::carry: records rebase to its base offset, the
// max_bytes budget goes on), the host writes the 61-byte header, and the
// CRC32C is combined from the chunks' (GF(2) shift of the CRC so far by the
// next chunk's length).  Stateless chains of verbatim / uppercased /
// projected records (their output stays within len + 10 B per record), and
// only when the call wants the output; 1 = not taken.
// ---------------------------------------------------------------------------
uint32_t crc32c_host(const uint8_t* p, size_t n) {  // standard init / xorout, bitwise (a header's 40 bytes)
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}
// a GF(2) 32 x 32 matrix (word k = the image of bit k) applied to v
uint32_t gf2_apply(const uint32_t* mat, uint32_t v) {
  uint32_t r = 0;
  for (int k = 0; v; k++, v >>= 1)
    if (v & 1u) r ^= mat[k];
  return r;
}
void gf2_sq(uint32_t* out, const uint32_t* mat) {
  for (int k = 0; k < 32; k++) out[k] = gf2_apply(mat, mat[k]);
}
// CRC32C of A ++ B from crc(A), crc(B) and |B|: crc(A) moved past |B| zero
// bytes (the one-zero-bit operator squared up to bytes, then by the bits of
// |B|), xor crc(B); the init / xorout terms cancel
uint32_t crc32c_combine(uint32_t a, uint32_t b, uint64_t nb) {
  if (nb == 0) return a ^ b;
  uint32_t odd[32], even[32];
  odd[0] = 0x82F63B78u;
  for (int k = 1; k < 32; k++) odd[k] = 1u << (k - 1);
  gf2_sq(even, odd);  // two zero bits
  gf2_sq(odd, even);  // four
  for (;;) {
    gf2_sq(even, odd);  // eight, then 32, 128 ...
    if (nb & 1) a = gf2_apply(even, a);
    nb >>= 1;
    if (!nb) break;
    gf2_sq(odd, even);
    if (nb & 1) a = gf2_apply(odd, a);
    nb >>= 1;
    if (!nb) break;
  }
  return a ^ b;
}
// the output batch header k_header writes (Batch::default() + base offset, lod, count)
void host_header(uint8_t* h, int64_t base, uint64_t rec_bytes, int32_t comp, int32_t lod, uint64_t nrec) {
  auto be = [&](int off, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) h[off + i] = (uint8_t)(v >> (8 * (nb - 1 - i)));
  };
  be(0, (uint64_t)base, 8);
  be(8, (uint32_t)(45 + 4 + rec_bytes), 4);
  be(12, (uint32_t)-1, 4);
  h[16] = 2;
  be(17, 0, 4);
  be(21, (uint32_t)comp & 7u, 2);
  be(23, (uint32_t)lod, 4);
  be(27, (uint64_t)-1, 8);
  be(35, (uint64_t)-1, 8);
  be(43, (uint64_t)-1, 8);
  be(51, (uint16_t)-1, 2);
  be(53, (uint32_t)-1, 4);
  be(57, (uint32_t)nrec, 4);
}

bool pipe_eligible(const fsg_chain* c) {
  if (c->no_pipe || !c->segs.empty() || c->agg_stage >= 0 || c->array_stage >= 0 || c->sf_stage >= 0) return false;
  if ((c->hdesc.flags & (CF_AGG_JSON | CF_STATEFUL | CF_ARRAY | CF_AGG_SUM)) || c->hdesc.out_type == VT_I32) return false;
  for (uint32_t k = 0; k < c->hdesc.nstages; k++) {
    const uint32_t op = c->hdesc.st[k].op;
    if (op != OP_CONTAINS && op != OP_REGEX && op != OP_FILTER_JSON && op != OP_MAP_UPPER && op != OP_PROJECT)
      return false;
  }
  return true;
}

// chunk bytes [src, src + n) of the resident slice into `sl` (zero padding
// behind them) and framed on the device; *fallback: the host walk would decide
int load_chunk(fsg_engine* e, fsg_slice* sl, const uint8_t* src, size_t n, hipStream_t st, int* fallback) {
  sl->verify_drain();
  sl->v_pending = false;
  sl->eng = e;
  sl->len = n;
  sl->rs_ok = false;
  sl->nb = 0;
  sl->nrec = 0;
  sl->tail_status = 0;
  sl->header_bytes = 0;
  sl->device_framed = false;
  sl->decompressed = false;
  sl->has_pass = false;
  const size_t alloc = slice_alloc(n);
  HIPCHK(sl->data.ensure(alloc));
  HIPCHK(hipMemsetAsync((uint8_t*)sl->data.p + (n & ~(size_t)15), 0, alloc - (n & ~(size_t)15), st));
  HIPCHK(hipMemcpyAsync(sl->data.p, src, n, hipMemcpyDeviceToDevice, st));
  int rc = frame_on_device(sl, st, fallback);
  if (rc) return rc;
  sl->device_framed = !*fallback;
  HIPCHK(sl->bpos.ensure(8));
  HIPCHK(sl->rbase.ensure(8));
  return FSG_OK;
}

int process_pipelined(fsg_chain* c, const uint8_t* s, size_t len, uint64_t max_bytes, fsg_metrics* m,
                      fsg_batch_output** out) {
  const size_t C = std::max<size_t>(c->pipe_bytes, 1 << 16);
  if (!out || len < 2 * C || !pipe_eligible(c)) return 1;
  constexpr size_t kPiece = 64u << 20;
  const int dev = c->eng->device;
  hipStream_t st = c->stream;
  for (int t = 0; t < c->pipe_up_threads; t++)
    if (!c->pipe_upv[t]) HIPCHK(hipStreamCreateWithFlags(&c->pipe_upv[t], hipStreamNonBlocking));
  if (!c->pipe_dl) HIPCHK(hipStreamCreateWithFlags(&c->pipe_dl, hipStreamNonBlocking));
  HIPCHK(c->pipe_in.ensure(len + 64));
  // the output: header + records within len + 10 B per record (>= 7 B each)
  const size_t bound = 61 + len + 10 * (len / 7) + 64;
  uint8_t* h = host_alloc(bound);
  if (!h) return fail(FSG_E_DEVICE, "host allocation failed");
  // upload thread: pieces in order, progress = bytes resident
  std::mutex mu;
  std::condition_variable cv;
  size_t up_done = 0;
  bool up_fin = false, stop = false;
  hipError_t up_err = hipSuccess;
  uint8_t* big = c->pipe_in.as<uint8_t>();
  // (pieces k = t mod T on upload thread t, each on its own stream; up_done =
  // the bytes of the resident prefix of pieces)
  const int T = c->pipe_up_threads;
  const size_t npieces = (len + kPiece - 1) / kPiece;
  std::vector<uint8_t> pdone(npieces, 0);
  size_t upk = 0;
  int up_exited = 0;
  auto upf = [&](int t) {
    hipError_t e = hipSetDevice(dev);
    for (size_t k = (size_t)t; k < npieces && e == hipSuccess; k += (size_t)T) {
      {
        std::lock_guard<std::mutex> g(mu);
        if (stop) break;
      }
      const size_t off = k * kPiece, n = std::min(kPiece, len - off);
      e = hipMemcpyAsync(big + off, s + off, n, hipMemcpyHostToDevice, c->pipe_upv[t]);
      if (e == hipSuccess) e = hipStreamSynchronize(c->pipe_upv[t]);
      std::lock_guard<std::mutex> g(mu);
      if (e == hipSuccess) {
        pdone[k] = 1;
        while (upk < npieces && pdone[upk]) upk++;
        up_done = std::min(len, upk * kPiece);
      }
      cv.notify_all();
    }
    std::lock_guard<std::mutex> g(mu);
    if (e != hipSuccess) up_err = e;
    if (++up_exited == T) up_fin = true;
    cv.notify_all();
  };
  std::vector<std::thread> ups;
  for (int t = 0; t < T; t++) ups.emplace_back(upf, t);
  // download thread: jobs (device records -> h + offset) in order
  struct Job {
    const uint8_t* src;
    uint8_t* dst;
    size_t n;
  };
  std::vector<Job> jobs;
  size_t dl_next = 0, dl_done = 0;
  bool dl_quit = false;
  hipError_t dl_err = hipSuccess;
  std::thread dl([&] {
    hipError_t e = hipSetDevice(dev);
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return dl_next < jobs.size() || dl_quit; });
        if (dl_next >= jobs.size()) break;
        j = jobs[dl_next++];
      }
      if (e == hipSuccess && j.n) e = staged_copy(c->pipe_pin, c->pipe_ev, c->pipe_dl, j.dst, j.src, j.n);
      std::lock_guard<std::mutex> g(mu);
      dl_done++;
      if (e != hipSuccess) dl_err = e;
      cv.notify_all();
    }
  });
  auto finish = [&]() {  // both threads drained and joined (every exit path)
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
      dl_quit = true;
    }
    cv.notify_all();
    for (auto& u : ups) u.join();
    dl.join();
  };
  fsg_metrics mloc{};
  Carry cy;
  fsg_batch_output res{};
  uint64_t rec_total = 0, nrec_total = 0, in_bytes = 0;
  int32_t lod = -1, comp = 0;
  int64_t base = -1;
  uint32_t crc_rec = 0;
  size_t X = 0, want = std::min(len, C);
  int rc = FSG_OK;
  bool fell_back = false;
  // chunk outputs alternate between two device buffers (c->out is the one
  // run_slice writes; physical buffer `cur`); buf_job: the download reading each
  const size_t NOJOB = ~(size_t)0;
  size_t buf_job[2] = {NOJOB, NOJOB};
  int cur = 0;
  uint32_t nchunk = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return up_done >= want || up_fin; });
      if (up_done < want) {
        rc = fail(FSG_E_DEVICE, up_err != hipSuccess ? hipGetErrorString(up_err) : "upload stopped");
        break;
      }
    }
    bool last = want == len;
    int fb = 0;
    rc = load_chunk(c->eng, &c->pipe_chunk, big + X, want - X, st, &fb);
    if (rc) break;
    if (fb) {  // the host walk decides this slice (no magic 2, compressed batches): the serial path
      fell_back = true;
      break;
    }
    fsg_slice& cs = c->pipe_chunk;
    const uint64_t E = cs.header_bytes;
    if (!last && E < want - X) {
      // framing stopped inside the chunk: a batch the chunk's end cuts (the
      // full slice holds it: the next chunk starts there), or the framing
      // failure the serial path meets at the same position
      const size_t q = X + E, rem = len - q;
      bool cut_batch = false;
      if (rem >= 57) {
        const int32_t bl = (int32_t)rd_be(s + q + 8, 4);
        const int comp_q = (int)(rd_be(s + q + 21, 2) & 7);
        if (bl >= 45 && rem - 57 >= (size_t)bl - 45) {
          if (comp_q != 0) {  // compressed: the serial path decompresses it
            fell_back = true;
            break;
          }
          cut_batch = true;
        }
      }
      if (cut_batch) {
        cs.tail_status = 0;
        if (E == 0) {  // no whole batch yet: a longer chunk
          want = std::min(len, want + C);
          continue;
        }
      } else {
        last = true;
      }
    }
    const int tgt = (int)(nchunk & 1u);
    if (cur != tgt) {
      c->out.swap(c->pipe_out);
      cur = tgt;
    }
    if (buf_job[tgt] != NOJOB) {  // its previous chunk's records are downloaded first
      std::unique_lock<std::mutex> g(mu);
      cv.wait(g, [&] { return dl_done > buf_job[tgt]; });
      buf_job[tgt] = NOJOB;
    }
    fsg_batch_output rk{};
    rc = run_slice(c, &cs, max_bytes, &mloc, &rk, c->hdesc.nstages == 0, nullptr, &cy);
    in_bytes += cs.header_bytes;
    if (rc) {
      free_error(rk.error);
      break;
    }
    nchunk++;
    const Plan p = c->hplan;
    if (p.first >= 0) {
      if (!cy.cont) {
        cy.cont = true;
        cy.base = base = p.base_offset;
        cy.comp = comp = p.comp;
        lod = p.lod;
      } else {
        lod += p.lod + 1;
      }
      if (p.rec_bytes) {
        uint8_t hc[61];
        host_header(hc, p.base_offset, p.rec_bytes, p.comp, p.lod, p.n_records);
        // the chunk's records: crc(header ++ records) with the header's CRC taken out
        const uint32_t crc_k = crc32c_combine(crc32c_host(hc + 21, 40), cy.crc, p.rec_bytes);
        crc_rec = rec_total ? crc32c_combine(crc_rec, crc_k, p.rec_bytes) : crc_k;
        if (61 + rec_total + p.rec_bytes > bound) {
          rc = fail(FSG_E_DEVICE, "pipelined output past its bound");
          free_error(rk.error);
          break;
        }
        {
          std::lock_guard<std::mutex> g(mu);
          jobs.push_back({c->out.as<uint8_t>() + 61, h + 61 + rec_total, p.rec_bytes});
          buf_job[tgt] = jobs.size() - 1;
        }
        cv.notify_all();
      }
      rec_total += p.rec_bytes;
      nrec_total += p.n_records;
      cy.spent += p.rec_bytes + 4ull * (uint64_t)p.nonempty;
    }
    // an error batch, or the max_bytes cut (last < stop; at the chunk's last batch too)
    const bool stopped = rk.has_error || p.stop + 1 < (int32_t)cs.nb || (p.first >= 0 && p.last < p.stop);
    if (rk.has_error) {
      res.has_error = 1;
      res.error = rk.error;
    } else {
      free_error(rk.error);
    }
    if (stopped || last) break;
    X += E;
    want = std::min(len, X + C);
  }
  // the downloads before the header goes in
  {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return dl_done >= jobs.size(); });
  }
  const hipError_t de = dl_err;
  finish();
  if (rc == FSG_OK && !fell_back && de != hipSuccess) rc = fail(FSG_E_DEVICE, hipGetErrorString(de));
  if (rc != FSG_OK || fell_back) {
    if (res.has_error) free_error(res.error);
    host_free(h);
    if (rc != FSG_OK) {  // a status error: the metrics of the batches before it stand, as on the serial path
      if (m) {
        m->bytes_in += mloc.bytes_in;
        m->invocation_count += mloc.invocation_count;
        m->records_out += mloc.records_out;
      }
      return rc;
    }
    return 1;  // nothing of this call is visible: the serial path runs it
  }
  host_header(h, base, rec_total, comp, lod, nrec_total);
  const uint32_t crc = crc32c_combine(crc32c_host(h + 21, 40), crc_rec, rec_total);
  h[17] = (uint8_t)(crc >> 24);
  h[18] = (uint8_t)(crc >> 16);
  h[19] = (uint8_t)(crc >> 8);
  h[20] = (uint8_t)crc;
  if (m) {
    m->bytes_in += mloc.bytes_in;
    m->invocation_count += mloc.invocation_count;
    m->records_out += mloc.records_out;
  }
  c->out_len = 0;  // the device holds only the last chunk's output
  c->last.chunks = nchunk;
  c->last.in_bytes = in_bytes;
  c->last.out_bytes = 61 + rec_total;
  auto r = std::make_unique<fsg_batch_output>(res);
  r->batch = h;
  r->batch_len = 61 + rec_total;
  r->base_offset = base;
  r->last_offset_delta = lod;
  r->n_records = (uint32_t)nrec_total;
  *out = r.release();
  return FSG_OK;
}

extern "C" int fsg_chain_process_batch(fsg_chain* c, const uint8_t* slice, size_t len, uint64_t max_bytes,
                                       fsg_metrics* m, fsg_batch_output** out) {
  HIPCHK(hipSetDevice(c->eng->device));
  const int pr = process_pipelined(c, slice, len, max_bytes, m, out);
  if (pr != 1) return pr;
  c->ingest.dec_limit = c->limit;
  int rc = upload_slice(c->eng, slice, len, &c->ingest, c->stream);
  if (rc) return rc;
  return fsg_chain_process_slice(c, &c->ingest, max_bytes, m, out);
}

// SmartModuleChainInstance::process: one SmartModuleInput{base_offset, raw_bytes,
// base_timestamp} is one batch of the same pipeline (no offset fix-up applies).
namespace {
// process() of a stateless chain in one launch (k_one): upload, k_one, one
// read-back of plan + batch result + output, one wait.  1 = not taken (the
// general path runs: a stateful / aggregate / array chain, a composed chain,
// an output beyond the block).
int process_one(fsg_chain* c, const uint8_t* raw, size_t len, int64_t base_offset, int64_t base_timestamp,
                fsg_metrics* m, fsg_output** out) {
  if (!c->segs.empty() || c->agg_stage >= 0 || c->array_stage >= 0 || c->sf_stage >= 0 ||
      (c->hdesc.flags & (CF_AGG_JSON | CF_STATEFUL | CF_ARRAY)))
    return 1;
  static_assert(sizeof(Plan) <= 192 && sizeof(BatchStat) <= 192 && sizeof(Mins) <= 64, "k_one read-back head");
  const size_t in_len = 57 + len, alloc = slice_alloc(in_len);
  const size_t cap = 128 + 4 * len;  // stateless outputs stay within the input's size plus the i32 digits
  if (alloc > kSmallOut || kOneHead + cap > kSmallOut) return 1;
  c->one_pin.flags = hipHostMallocMapped | hipHostMallocCoherent;
  HIPCHK(c->one_pin.ensure(2 * kSmallOut + 64));  // input | read-back block | completion flag
  HIPCHK(c->ingest.data.ensure(alloc));
  HIPCHK(c->one_blk.ensure(kOneHead + cap));
  HIPCHK(c->kept.ensure(std::max<size_t>(len / 7 + 1, 1) * sizeof(KeptRec)));
  HIPCHK(c->rows.ensure(sizeof(ScanRow)));
  HIPCHK(c->pre.ensure(sizeof(ScanRow)));
  if (!c->one_meta.p) {
    HIPCHK(c->one_meta.ensure(16));
    HIPCHK(hipMemsetAsync(c->one_meta.p, 0, 16, c->stream));
  }
  // the batch (Batch::default() + base offset / timestamp, the records as given)
  // in pinned memory, one copy up
  uint8_t* b = (uint8_t*)c->one_pin.p;
  const size_t in_real = (in_len + 15) & ~(size_t)15;  // k_one reads these, zero-fills the rest on the device
  memset(b, 0, 57);
  memset(b + in_len, 0, in_real - in_len);
  auto be = [&](size_t off, uint64_t v, int n) {
    for (int i = 0; i < n; i++) b[off + i] = (uint8_t)(v >> (8 * (n - 1 - i)));
  };
  be(0, (uint64_t)base_offset, 8);
  be(8, (uint32_t)(45 + len), 4);
  be(12, (uint32_t)-1, 4);
  b[16] = 2;
  be(27, (uint64_t)base_timestamp, 8);
  if (len) memcpy(b + 57, raw, len);
  uint64_t nrec = 0;  // frame(): the count, clamped by the bytes a record needs at least
  if (len >= 4) {
    const int32_t cnt = (int32_t)rd_be(raw, 4);
    nrec = std::min<uint64_t>(cnt > 0 ? (uint64_t)cnt : 0, (len - 4) / 7);
  }
  hipStream_t st = c->stream;
  uint8_t* blk = c->one_blk.as<uint8_t>();
  uint8_t* hb = (uint8_t*)c->one_pin.p + kSmallOut;  // the read-back block lands here
  // the pinned buffer's device address (k_one reads the input, writes the block
  // and the flag through it), looked up once per allocation
  if (c->one_dev_for != c->one_pin.p) {
    HIPCHK(hipHostGetDevicePointer(&c->one_dev, c->one_pin.p, 0));
    c->one_dev_for = c->one_pin.p;
  }
  void* din = c->one_dev;
  void* dout = (uint8_t*)c->one_dev + kSmallOut;
  OneArgs o{};
  EvalArgs& ea = o.ea;
  ea.slice = c->ingest.data.as<uint8_t>();
  ea.slice_len = in_len;
  ea.bpos = c->one_meta.as<uint64_t>();
  ea.rbase = c->one_meta.as<uint64_t>() + 1;
  ea.nbatches = 1;
  ea.chain = c->d_desc.as<ChainDesc>();
  ea.blob = c->d_blob.as<uint8_t>();
  ea.bstat = (BatchStat*)(blk + 192);
  ea.desc = c->kept.as<KeptRec>();
  ea.mins = (Mins*)(blk + 384);
  ea.nrec = nrec;
  o.rows = c->rows.as<ScanRow>();
  o.pre = c->pre.as<ScanRow>();
  o.plan = (Plan*)blk;
  o.out = blk + kOneHead;
  o.out_cap = cap;
  o.hin = (const uint8_t*)din;
  o.hout = (uint8_t*)dout;
  o.in_len = (uint32_t)alloc;
  o.in_real = (uint32_t)in_real;
  o.empty_chain = c->hdesc.nstages == 0 ? 1 : 0;
  volatile uint32_t* flag = (volatile uint32_t*)((uint8_t*)c->one_pin.p + 2 * kSmallOut);
  *flag = 0;
  o.hflag = (uint32_t*)((uint8_t*)c->one_dev + 2 * kSmallOut);
  o.seq = ++c->one_seq ? c->one_seq : ++c->one_seq;  // never 0
  uint32_t ops = 0;
  for (uint32_t k = 0; k < c->hdesc.nstages; k++) ops |= 1u << c->hdesc.st[k].op;
  launch_one(o, ops, st);  // one launch: input over PCIe, process(), the block back to pinned memory
  HIPCHK(hipGetLastError());
  // the kernel's last act is the flag store (after a system-scope fence): poll
  // host memory, no runtime call on the fast path; the stream is waited for
  // only if the flag is late (an error or a slow device surfaces there)
  {
    const auto t0 = std::chrono::steady_clock::now();
    bool seen = false;
    while (!seen) {
      seen = __atomic_load_n(flag, __ATOMIC_ACQUIRE) == o.seq;
      if (!seen && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(500)) break;
    }
    if (!seen) HIPCHK(wait_stream(st));
  }
  Plan p;
  BatchStat bs;
  memcpy(&p, hb, sizeof p);
  memcpy(&bs, hb + 192, sizeof bs);
#ifdef FSG_ONE_TIMING
  {
    const uint64_t* tm = (const uint64_t*)(hb + 416);
    static int calls = 0;
    if (++calls % 500 == 0) {
      fprintf(stderr, "k_one phases (10 ns ticks):");
      for (int k = 1; k < 10 && tm[k]; k++) fprintf(stderr, " %d:%llu", k, (unsigned long long)(tm[k] - tm[k - 1]));
      fprintf(stderr, "\n");
    }
  }
#endif
  if (p.status != 0) {
    if (m) {
      m->bytes_in += p.bytes_in;
      m->invocation_count += p.invocations;
    }
    const char* why = p.status == FSG_E_UNSUPPORTED ? "input needs a feature the GPU path does not implement"
                      : p.status == FSG_E_IO        ? "io error while decoding batches"
                                                    : "failed to decode SmartModule base input";
    return fail(p.status, why);
  }
  const uint64_t out_len = 61 + p.rec_bytes;
  if (out_len > cap) return 1;  // nothing was written: the general path redoes the call
  if (m) {
    m->bytes_in += p.bytes_in;
    m->invocation_count += p.invocations;
    if (c->hdesc.nstages) m->records_out += p.records_out;
  }
  auto o2 = std::make_unique<fsg_output>();
  memset(o2.get(), 0, sizeof(fsg_output));
  const size_t rl = out_len - 57;  // u32 count + records
  uint8_t* h = host_alloc(rl);
  if (!h) return fail(FSG_E_DEVICE, "host allocation failed");
  memcpy(h, hb + kOneHead + 57, rl);
  o2->records = h;
  o2->records_len = rl;
  o2->n_records = (uint32_t)p.n_records;
  if (p.err_batch >= 0) {
    c->ingest.eng = c->eng;
    c->ingest.len = in_len;
    c->ingest.nb = 1;
    c->ingest.nrec = nrec;
    int rc = build_error(c, &c->ingest, bs, o2->error);
    if (rc) {
      host_free(h);
      return rc;
    }
    o2->has_error = 1;
  }
  c->out_len = out_len;
  c->last = fsg_timings{};
  c->last.in_bytes = in_len;
  c->last.out_bytes = out_len;
  c->last.n_batches = 1;
  c->last.n_records_in = nrec;
  *out = o2.release();
  return FSG_OK;
}
}  // namespace

extern "C" int fsg_chain_process(fsg_chain* c, const uint8_t* raw, size_t len, int64_t base_offset,
                                 int64_t base_timestamp, fsg_metrics* m, fsg_output** out) {
  HIPCHK(hipSetDevice(c->eng->device));
  {
    const int rc = process_one(c, raw, len, base_offset, base_timestamp, m, out);
    if (rc != 1) return rc;
  }
  std::vector<uint8_t> b(slice_alloc(57 + len));  // zero-padded: uploaded in one copy
  auto be = [&](size_t off, uint64_t v, int n) {
    for (int i = 0; i < n; i++) b[off + i] = (uint8_t)(v >> (8 * (n - 1 - i)));
  };
  be(0, (uint64_t)base_offset, 8);
  be(8, (uint32_t)(45 + len), 4);
  be(12, (uint32_t)-1, 4);
  b[16] = 2;
  be(21, 0, 2);
  be(23, 0, 4);
  be(27, (uint64_t)base_timestamp, 8);
  if (len) memcpy(b.data() + 57, raw, len);
  // no sync after the upload: `b` lives to the end of this call, which run_slice synchronises
  int rc = upload_slice(c->eng, b.data(), 57 + len, &c->ingest, c->stream, false, false, true);
  if (rc) return rc;
  fsg_batch_output r;
  c->timed = false;  // 11 event calls are a tenth of a one-record call's latency
  rc = run_slice(c, &c->ingest, ~0ull, m, &r, c->hdesc.nstages == 0);
  c->timed = true;
  if (rc) {
    (void)hipStreamSynchronize(c->stream);  // an early error return may leave the upload in flight
    free_error(r.error);
    return rc;
  }
  auto o = std::make_unique<fsg_output>();
  memset(o.get(), 0, sizeof(fsg_output));
  c = fin(c);
  const size_t rl = c->out_len - 57;  // u32 count + records
  uint8_t* h = host_alloc(rl);
  if (!h) {
    free_error(r.error);
    return fail(FSG_E_DEVICE, "host allocation failed");
  }
  hipError_t e = hipSuccess;
  if (c->out_pinned)
    memcpy(h, (const uint8_t*)c->hpin.p + kPinPlan + 57, rl);
  else
    e = hipMemcpy(h, (uint8_t*)c->out.p + 57, rl, hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    host_free(h);
    free_error(r.error);
    return fail(FSG_E_DEVICE, hipGetErrorString(e));
  }
  o->records = h;
  o->records_len = rl;
  o->n_records = r.n_records;
  o->has_error = r.has_error;
  o->error = r.error;
  *out = o.release();
  return FSG_OK;
}

extern "C" void fsg_runtime_error_free(fsg_runtime_error* e) {
  if (e) free_error(*e);
}

namespace {
// the stateful stage alone, in look_back mode (StageDesc::keep_match = 1),
// sharing the chain's state
int make_lookback_chain(fsg_chain* c) {
  if (c->lbc) return FSG_OK;
  auto l = std::make_unique<fsg_chain>();
  l->eng = c->eng;
  l->limit = c->limit;
  StageDesc sd = c->hdesc.st[c->sf_stage];
  sd.in_type = VT_SRC;  // look_back reads the records themselves
  sd.keep_match = 1;
  l->hdesc.nstages = 1;
  l->hdesc.st[0] = sd;
  l->hdesc.out_type = VT_SRC;
  l->hdesc.flags = CF_STATEFUL;
  l->hblob = c->hblob;
  l->names.push_back(c->names[c->sf_stage]);
  l->sf_stage = 0;
  l->sf = c->sf;
  HIPCHK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
  for (auto& ev : l->ev) HIPCHK(hipEventCreate(&ev));
  HIPCHK(l->d_desc.ensure(sizeof(ChainDesc)));
  HIPCHK(hipMemcpy(l->d_desc.p, &l->hdesc, sizeof(ChainDesc), hipMemcpyHostToDevice));
  HIPCHK(l->d_blob.ensure(l->hblob.size()));
  HIPCHK(hipMemcpy(l->d_blob.p, l->hblob.data(), l->hblob.size(), hipMemcpyHostToDevice));
  c->lbc = std::move(l);
  return FSG_OK;
}
}  // namespace

// SmartModuleChainInstance::look_back (engine.rs:187-218): a stage with a
// look_back export (instance.rs:92-95) and a Lookback gets read_fn's records as
// one SmartModuleInput (try_from_records: base offset 0), metrics.add_bytes_in,
// and its look_back over them (derive generator/look_back.rs: stops at the
// first Err with SmartModuleLookbackRuntimeError).
namespace {
// a composed chain's segment holding global stage `stage` (local index in *local)
fsg_chain* seg_of(fsg_chain* c, size_t stage, size_t* local) {
  for (size_t k = c->segs.size(); k-- > 0;)
    if (stage >= c->seg_stage0[k]) {
      *local = stage - c->seg_stage0[k];
      return c->segs[k].get();
    }
  *local = stage;
  return c;
}
}  // namespace

extern "C" int fsg_chain_look_back(fsg_chain* c, fsg_read_fn read_fn, void* user, fsg_metrics* m,
                                   fsg_runtime_error* error) {
  if (error) memset(error, 0, sizeof *error);
  if (!c->segs.empty()) {  // every segment's stateful stage with a Lookback, in chain order
    for (auto& g : c->segs) {
      int rc = fsg_chain_look_back(g.get(), read_fn, user, m, error);
      if (rc) return rc;
    }
    return FSG_OK;
  }
  if (c->sf_stage < 0 || c->lookback.kind == FSG_LOOKBACK_NONE) return FSG_OK;
  if (!read_fn) return fail(FSG_E_INVALID_ARG, "look_back needs a read_fn");
  HIPCHK(hipSetDevice(c->eng->device));
  const uint8_t* recs = nullptr;
  size_t len = 0;
  if (read_fn(user, &c->lookback, &recs, &len) != 0) return fail(FSG_E_IO, "look_back read_fn failed");
  if (m) {
    m->bytes_in += len;
    m->invocation_count += 1;
  }
  int rc = make_lookback_chain(c);
  if (rc) return rc;
  fsg_output* o = nullptr;
  rc = fsg_chain_process(c->lbc.get(), recs, len, 0, -1, nullptr, &o);
  if (rc) return rc;
  if (o->has_error) {
    if (error) {
      *error = o->error;
      memset(&o->error, 0, sizeof o->error);
    }
    fsg_output_free(o);
    return fail(FSG_E_LOOKBACK, "look_back: SmartModule Lookback Error");
  }
  fsg_output_free(o);
  return FSG_OK;
}

extern "C" int fsg_chain_get_accumulator(fsg_chain* c0, size_t stage0, uint8_t** acc, size_t* len) {
  size_t stage = stage0;
  fsg_chain* c = seg_of(c0, stage0, &stage);
  if ((int)stage != c->agg_stage) return fail(FSG_E_INVALID_ARG, "stage is not an aggregate");
  std::vector<uint8_t> txt;
  const std::vector<uint8_t>* a = &c->acc;
  if ((c->hdesc.flags & CF_AGG_JSON) && c->aj_touched) {  // rendered from the state in HBM
    int rc = aj_render(c, txt);
    if (rc) return rc;
    a = &txt;
  }
  *acc = (uint8_t*)malloc(std::max<size_t>(1, a->size()));
  if (!*acc) return fail(FSG_E_DEVICE, "host allocation failed");
  if (!a->empty()) memcpy(*acc, a->data(), a->size());
  *len = a->size();
  return FSG_OK;
}

extern "C" int fsg_chain_last_timings(fsg_chain* c, fsg_timings* t) {
  *t = fin(c)->last;
  if (!c->segs.empty()) {  // phases summed over the segments; the input as segment 0 saw it
    const fsg_timings& t0 = c->segs[0]->last;
    for (size_t k = 0; k + 1 < c->segs.size(); k++) {
      const fsg_timings& g = c->segs[k]->last;
      t->eval_ms += g.eval_ms;
      t->plan_ms += g.plan_ms;
      t->write_ms += g.write_ms;
      t->crc_ms += g.crc_ms;
      t->total_ms += g.total_ms;
    }
    t->in_bytes = t0.in_bytes;
    t->n_batches = t0.n_batches;
    t->n_records_in = t0.n_records_in;
  }
  return FSG_OK;
}

extern "C" void fsg_output_free(fsg_output* o) {
  if (!o) return;
  host_free(o->records);
  free_error(o->error);
  delete o;
}
extern "C" void fsg_batch_output_free(fsg_batch_output* o) {
  if (!o) return;
  host_free(o->batch);
  free_error(o->error);
  delete o;
}

// ---------------------------------------------------------------------------
// RCCL: aggregate state merge across GPUs (partitions sharded p -> GPU p mod n)
// ---------------------------------------------------------------------------
extern "C" int fsg_comm_unique_id(uint8_t id[FSG_UNIQUE_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) == FSG_UNIQUE_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return fail(FSG_E_DEVICE, "ncclGetUniqueId failed");
  memcpy(id, &u, sizeof u);
  return FSG_OK;
}
extern "C" int fsg_engine_comm_init(fsg_engine* e, const uint8_t id[FSG_UNIQUE_ID_BYTES], int nranks, int rank) {
  HIPCHK(hipSetDevice(e->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclResult_t r = ncclCommInitRank(&e->comm, nranks, u, rank);
  if (r != ncclSuccess) return fail(FSG_E_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  e->nranks = nranks;
  e->rank = rank;
  return FSG_OK;
}
namespace {
bool nccl_type(int dtype, ncclDataType_t* t, size_t* sz) {
  switch (dtype) {
    case FSG_DTYPE_I32: *t = ncclInt32; *sz = 4; return true;
    case FSG_DTYPE_U32: *t = ncclUint32; *sz = 4; return true;
    case FSG_DTYPE_I64: *t = ncclInt64; *sz = 8; return true;
    case FSG_DTYPE_U64: *t = ncclUint64; *sz = 8; return true;
    case FSG_DTYPE_F64: *t = ncclFloat64; *sz = 8; return true;
    default: return false;
  }
}
int allreduce_on(fsg_engine* e, void* dev, size_t count, int dtype, hipStream_t st) {
  if (!e->comm) return fail(FSG_E_INVALID_ARG, "engine has no communicator (fsg_engine_comm_init)");
  ncclDataType_t t;
  size_t sz;
  if (!nccl_type(dtype, &t, &sz)) return fail(FSG_E_INVALID_ARG, "unknown state dtype");
  HIPCHK(hipSetDevice(e->device));
  // integer sums wrap in two's complement, like the wasm guest's release-mode adds
  ncclResult_t r = ncclAllReduce(dev, dev, count, t, ncclSum, e->comm, st);
  if (r != ncclSuccess) return fail(FSG_E_DEVICE, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  HIPCHK(hipStreamSynchronize(st));
  return FSG_OK;
}
}  // namespace

extern "C" int fsg_allreduce_state(fsg_engine* e, void* dev_state, size_t count, int dtype) {
  return allreduce_on(e, dev_state, count, dtype, e->coll);
}
extern "C" int fsg_chain_allreduce_state(fsg_chain* c, void* dev_state, size_t count, int dtype) {
  return allreduce_on(c->eng, dev_state, count, dtype, c->stream);
}

// ---------------------------------------------------------------------------
// per-partition aggregate state vector in HBM
// ---------------------------------------------------------------------------
struct fsg_state {
  fsg_engine* eng = nullptr;
  std::mutex mu;
  DevBuf buf;
  size_t count = 0, esize = 4;
  int dtype = FSG_DTYPE_I32;
};

extern "C" int fsg_state_new(fsg_engine* e, size_t count, int dtype, fsg_state** out) {
  ncclDataType_t t;
  size_t sz;
  if (!nccl_type(dtype, &t, &sz)) return fail(FSG_E_INVALID_ARG, "unknown state dtype");
  HIPCHK(hipSetDevice(e->device));
  auto s = std::make_unique<fsg_state>();
  s->eng = e;
  s->count = count;
  s->esize = sz;
  s->dtype = dtype;
  HIPCHK(s->buf.ensure(std::max<size_t>(count, 1) * sz));
  HIPCHK(hipMemsetAsync(s->buf.p, 0, std::max<size_t>(count, 1) * sz, e->coll));
  HIPCHK(hipStreamSynchronize(e->coll));
  *out = s.release();
  return FSG_OK;
}
extern "C" int fsg_state_collect(fsg_state* s, size_t slot, fsg_chain* c) {
  for (auto& g : c->segs)  // a composed chain: its aggregate-sum segment
    if (g->hdesc.flags & CF_AGG_SUM) return fsg_state_collect(s, slot, g.get());
  if (slot >= s->count) return fail(FSG_E_INVALID_ARG, "state slot out of range");
  if (!(c->hdesc.flags & CF_AGG_SUM) || s->dtype != FSG_DTYPE_I32)
    return fail(FSG_E_INVALID_ARG, "collect needs an aggregate-sum chain and an i32 state vector");
  if (c->eng->device != s->eng->device) return fail(FSG_E_INVALID_ARG, "chain and state on different devices");
  HIPCHK(hipSetDevice(s->eng->device));
  // device to device on the chain's stream, after its last k_state; chains of
  // different partitions may collect from different host threads at once.  The
  // merge stream waits for the copy on the device (no host wait per collect).
  HIPCHK(hipMemcpyAsync((uint8_t*)s->buf.p + slot * s->esize, c->dstate.p, 4, hipMemcpyDeviceToDevice, c->stream));
  if (!c->kd_ev[0]) HIPCHK(hipEventCreateWithFlags(&c->kd_ev[0], hipEventDisableTiming));
  if (!c->kd_ev[1]) HIPCHK(hipEventCreateWithFlags(&c->kd_ev[1], hipEventDisableTiming));
  std::lock_guard<std::mutex> g(s->mu);  // hipStreamWaitEvent on the shared merge stream
  HIPCHK(hipEventRecord(c->kd_ev[0], c->stream));
  HIPCHK(hipStreamWaitEvent(s->eng->coll, c->kd_ev[0], 0));
  return FSG_OK;
}
extern "C" int fsg_state_allreduce(fsg_state* s) {
  return allreduce_on(s->eng, s->buf.p, s->count, s->dtype, s->eng->coll);
}
extern "C" int fsg_state_read(fsg_state* s, void* host, size_t bytes) {
  HIPCHK(hipSetDevice(s->eng->device));
  HIPCHK(hipStreamSynchronize(s->eng->coll));
  HIPCHK(hipMemcpy(host, s->buf.p, std::min(bytes, s->count * s->esize), hipMemcpyDeviceToHost));
  return FSG_OK;
}
extern "C" int fsg_state_device(fsg_state* s, void** dptr) {
  *dptr = s->buf.p;
  return FSG_OK;
}
extern "C" void fsg_state_free(fsg_state* s) { delete s; }

// ---------------------------------------------------------------------------
// topic-wide keyed totals of aggregate-json states (C5 keyed, SURVEY §8 e)
// ---------------------------------------------------------------------------
struct fsg_keyed {
  fsg_engine* eng = nullptr;
  hipStream_t st = nullptr;
  // rank-local table (KdTable)
  DevBuf arena, koff, klen, val, slot, cnt;
  uint32_t cap = 0;           // slots
  uint64_t kcap = 0, acap = 0;  // key / arena capacity
  uint64_t nb = 0, bb = 0;      // upper bounds of the keys / bytes in the table
  // the merge
  DevBuf gcnt, ldesc, gdesc, garena, uslot, gslot, first, idpre, gid, ulen, uoff, uarena, dense, tsum, tot;
  uint64_t K = 0, ubytes = 0;
  bool merged = false;
  ~fsg_keyed() {
    if (st) (void)hipStreamDestroy(st);
  }
  KdTable table() {
    KdTable t;
    t.arena = arena.as<uint8_t>();
    t.koff = koff.as<uint64_t>();
    t.klen = klen.as<uint32_t>();
    t.val = val.as<uint32_t>();
    t.slot = slot.as<uint32_t>();
    t.cap = cap;
    t.cnt = cnt.as<unsigned long long>();
    return t;
  }
};

namespace {
// table slots: a power of two >= n (callers bound n to 2^31, the u32 slot range)
uint32_t pow2_at_least(uint64_t n) {
  uint64_t c = 16;
  while (c < n) c <<= 1;
  return (uint32_t)c;
}
// room for `nk` more keys and `nbytes` more key bytes (grows and rehashes; rare)
int kd_reserve(fsg_keyed* k, uint64_t nk, uint64_t nbytes) {
  const uint64_t need_k = k->nb + nk, need_b = k->bb + nbytes;
  if (need_k <= k->kcap && need_b + 16 <= k->acap && 2 * need_k <= k->cap) return FSG_OK;
  hipStream_t st = k->st;
  unsigned long long c[2] = {0, 0};
  if (k->cnt.p) HIPCHK(hipMemcpyAsync(c, k->cnt.p, sizeof c, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t kc = std::max<uint64_t>(2 * need_k, 1024), ac = std::max<uint64_t>(2 * need_b, 1 << 16);
  DevBuf na, nko, nkl, nv, ns;
  HIPCHK(na.ensure(ac + 16));
  HIPCHK(nko.ensure(kc * 8));
  HIPCHK(nkl.ensure(kc * 4));
  HIPCHK(nv.ensure(kc * 4));
  if (2 * kc > (1ull << 31)) return fail(FSG_E_UNSUPPORTED, "keyed table past 2^30 keys");
  const uint32_t cap = pow2_at_least(2 * kc);
  HIPCHK(ns.ensure((size_t)cap * 4));
  HIPCHK(hipMemsetAsync(ns.p, 0, (size_t)cap * 4, st));
  if (c[0]) {
    HIPCHK(hipMemcpyAsync(na.p, k->arena.p, c[1], hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(nko.p, k->koff.p, c[0] * 8, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(nkl.p, k->klen.p, c[0] * 4, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(nv.p, k->val.p, c[0] * 4, hipMemcpyDeviceToDevice, st));
  }
  HIPCHK(k->cnt.ensure(16));
  if (!k->kcap) HIPCHK(hipMemsetAsync(k->cnt.p, 0, 16, st));
  HIPCHK(hipStreamSynchronize(st));
  std::swap(k->arena.p, na.p);
  std::swap(k->arena.cap, na.cap);
  std::swap(k->koff.p, nko.p);
  std::swap(k->koff.cap, nko.cap);
  std::swap(k->klen.p, nkl.p);
  std::swap(k->klen.cap, nkl.cap);
  std::swap(k->val.p, nv.p);
  std::swap(k->val.cap, nv.cap);
  std::swap(k->slot.p, ns.p);
  std::swap(k->slot.cap, ns.cap);
  k->cap = cap;
  k->kcap = kc;
  k->acap = ac + 16;
  launch_kd_rehash(k->table(), (uint32_t)c[0], st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));  // the old buffers are freed on return
  return FSG_OK;
}
int kd_gather(fsg_keyed* k, const void* send, void* recv, size_t count, ncclDataType_t t, size_t esize) {
  fsg_engine* e = k->eng;
  if (!e->comm) {  // one rank without a communicator: the gather is a copy
    if (count) HIPCHK(hipMemcpyAsync(recv, send, count * esize, hipMemcpyDeviceToDevice, k->st));
    return FSG_OK;
  }
  ncclResult_t r = ncclAllGather(send, recv, count, t, e->comm, k->st);
  if (r != ncclSuccess) return fail(FSG_E_DEVICE, std::string("ncclAllGather: ") + ncclGetErrorString(r));
  return FSG_OK;
}
}  // namespace

extern "C" int fsg_keyed_new(fsg_engine* e, fsg_keyed** out) {
  HIPCHK(hipSetDevice(e->device));
  auto k = std::make_unique<fsg_keyed>();
  k->eng = e;
  HIPCHK(hipStreamCreateWithFlags(&k->st, hipStreamNonBlocking));
  int rc = kd_reserve(k.get(), 1024, 1 << 16);
  if (rc) return rc;
  *out = k.release();
  return FSG_OK;
}

extern "C" int fsg_keyed_reset(fsg_keyed* k) {
  HIPCHK(hipSetDevice(k->eng->device));
  HIPCHK(hipMemsetAsync(k->cnt.p, 0, 16, k->st));
  HIPCHK(hipMemsetAsync(k->slot.p, 0, (size_t)k->cap * 4, k->st));
  k->nb = k->bb = 0;
  k->merged = false;
  return FSG_OK;
}

extern "C" int fsg_keyed_collect(fsg_keyed* k, fsg_chain* c0, size_t stage0) {
  size_t stage = stage0;
  fsg_chain* c = seg_of(c0, stage0, &stage);
  if ((int)stage != c->agg_stage || !(c->hdesc.flags & CF_AGG_JSON))
    return fail(FSG_E_INVALID_ARG, "stage is not an aggregate-json aggregate");
  if (c->eng->device != k->eng->device) return fail(FSG_E_INVALID_ARG, "chain and keyed table on different devices");
  HIPCHK(hipSetDevice(k->eng->device));
  int rc = aj_state_init(c);  // a chain that has not processed anything yet: its initial accumulator
  if (rc) return rc;
  const uint32_t n = c->aj_K;
  rc = kd_reserve(k, n, c->aj_bytes);
  if (rc) return rc;
  k->nb += n;
  k->bb += c->aj_bytes;
  k->merged = false;
  for (auto& ev : c->kd_ev)
    if (!ev) HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  // the chain's state after its queued work; the chain's next commit waits
  // for the collect (it may overwrite the other state buffer, never this one,
  // but the one after it would)
  HIPCHK(hipEventRecord(c->kd_ev[0], c->stream));
  HIPCHK(hipStreamWaitEvent(k->st, c->kd_ev[0], 0));
  const fsg_chain::AjBuf& S = c->ajs[c->aj_cur];
  launch_kd_collect(k->table(), S.kptr.as<uint64_t>(), S.klen.as<uint32_t>(), S.val.as<uint32_t>(), n, k->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->kd_ev[1], k->st));
  HIPCHK(hipStreamWaitEvent(c->stream, c->kd_ev[1], 0));
  return FSG_OK;
}

// the other ranks' send buffers, supplied by the caller (fsg_keyed_allreduce_sim)
struct KdSim {
  const uint64_t* n;
  const uint64_t* const* desc;
  const uint8_t* const* arena;
  const uint64_t* arena_len;
  const uint32_t* const* vals;
};

// The topic dictionary: every rank's key list all-gathered, the union built on
// every rank (ids by first occurrence in rank order), then one all-reduce of
// the dense K-slot u32 table.  World 1 (no communicator): the same steps with
// device copies in place of the collectives.  `sim`: this rank is `me` of `nr`
// and the other ranks' gathered inputs come from the caller (uploads in place
// of the all-gathers, their dense scatters summed in place of the all-reduce).
static int kd_allreduce(fsg_keyed* k, int nr, int me, const KdSim* sim, size_t* n_keys, size_t* key_bytes) {
  fsg_engine* e = k->eng;
  HIPCHK(hipSetDevice(e->device));
  hipStream_t st = k->st;
  const bool nccl = e->comm && !sim;
  HIPCHK(k->gcnt.ensure((size_t)nr * 16));
  HIPCHK(k->tot.ensure(64));
  std::vector<unsigned long long> gc((size_t)nr * 2);
  int rc = FSG_OK;
  if (sim) {
    HIPCHK(hipMemcpyAsync(gc.data() + 2 * me, k->cnt.p, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int r = 0; r < nr; r++)
      if (r != me) {
        gc[2 * r] = sim->n[r];
        gc[2 * r + 1] = sim->arena_len[r];
      }
  } else {
    rc = kd_gather(k, k->cnt.p, k->gcnt.p, 2, ncclUint64, 8);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(gc.data(), k->gcnt.p, gc.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  uint64_t maxn = 1, maxb = 16;
  for (int r = 0; r < nr; r++) {
    maxn = std::max<uint64_t>(maxn, gc[2 * r]);
    maxb = std::max<uint64_t>(maxb, gc[2 * r + 1]);
  }
  maxb = (maxb + 15) & ~15ull;
  const uint64_t nloc = gc[2 * me];
  if (maxn * (uint64_t)nr >= 0xFFFFFFF0ull) return fail(FSG_E_INVALID_ARG, "too many keys for the merge");
  const uint32_t nitems = (uint32_t)(maxn * nr);
  // the send buffers must hold maxn / maxb entries (all-gather counts are equal on every rank)
  rc = kd_reserve(k, maxn > k->nb ? maxn - k->nb : 0, maxb > k->bb ? maxb - k->bb : 0);
  if (rc) return rc;
  HIPCHK(k->ldesc.ensure(maxn * 8));
  HIPCHK(k->gdesc.ensure((size_t)nitems * 8));
  HIPCHK(k->garena.ensure((size_t)nr * maxb + 16));
  launch_kd_desc(k->table(), (uint32_t)nloc, (uint32_t)maxn, k->ldesc.as<uint64_t>(), st);
  std::vector<uint64_t> hdesc;
  std::vector<uint8_t> harena;
  if (sim) {  // this rank's buffers at its slot, the others' uploaded padded to maxn / maxb
    hdesc.assign((size_t)nr * maxn, kKdLenDeadDesc);
    harena.assign((size_t)nr * maxb, 0);
    for (int r = 0; r < nr; r++) {
      if (r == me) continue;
      for (uint64_t i = 0; i < sim->n[r]; i++) hdesc[(size_t)r * maxn + i] = sim->desc[r][i];
      if (sim->arena_len[r]) memcpy(harena.data() + (size_t)r * maxb, sim->arena[r], sim->arena_len[r]);
    }
    HIPCHK(hipMemcpyAsync(k->gdesc.p, hdesc.data(), hdesc.size() * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(k->garena.p, harena.data(), harena.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(k->gdesc.as<uint64_t>() + (size_t)me * maxn, k->ldesc.p, maxn * 8,
                          hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(k->garena.as<uint8_t>() + (size_t)me * maxb, k->arena.p, maxb, hipMemcpyDeviceToDevice,
                          st));
  } else {
    if (e->comm) ncclGroupStart();
    rc = kd_gather(k, k->ldesc.p, k->gdesc.p, maxn, ncclUint64, 8);
    if (!rc) rc = kd_gather(k, k->arena.p, k->garena.p, maxb, ncclUint8, 1);
    if (e->comm) ncclGroupEnd();
    if (rc) return rc;
  }
  if (2ull * nitems > (1ull << 31)) return fail(FSG_E_UNSUPPORTED, "keyed merge past 2^30 gathered keys");
  const uint32_t ucap = pow2_at_least(2ull * nitems);
  HIPCHK(k->uslot.ensure((size_t)ucap * 4));
  HIPCHK(hipMemsetAsync(k->uslot.p, 0, (size_t)ucap * 4, st));
  HIPCHK(k->gslot.ensure((size_t)nitems * 4));
  HIPCHK(k->first.ensure((size_t)nitems * 4));
  HIPCHK(k->idpre.ensure((size_t)nitems * 8));
  HIPCHK(k->gid.ensure((size_t)nitems * 4));
  HIPCHK(k->tsum.ensure(xscan_tiles(nitems) * 8));
  KdUnionArgs u{};
  u.gdesc = k->gdesc.as<uint64_t>();
  u.garena = k->garena.as<uint8_t>();
  u.maxb = maxb;
  u.maxn = (uint32_t)maxn;
  u.nitems = nitems;
  u.me = (uint32_t)me;
  u.lval = k->val.as<uint32_t>();
  u.slot = k->uslot.as<uint32_t>();
  u.cap = ucap;
  u.gslot = k->gslot.as<uint32_t>();
  u.first = k->first.as<uint32_t>();
  u.idpre = k->idpre.as<uint64_t>();
  u.gid = k->gid.as<uint32_t>();
  u.tsum = k->tsum.as<uint64_t>();
  u.tot = k->tot.as<unsigned long long>();
  launch_kd_union(u, st);
  unsigned long long K = 0;
  HIPCHK(hipMemcpyAsync(&K, u.tot, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const size_t K1 = std::max<uint64_t>(K, 1);
  HIPCHK(k->ulen.ensure(K1 * 4));
  HIPCHK(k->uoff.ensure(K1 * 8));
  HIPCHK(k->uarena.ensure((size_t)nr * maxb + 16));
  HIPCHK(k->dense.ensure(K1 * 4));
  HIPCHK(k->tsum.ensure(xscan_tiles(std::max<uint64_t>(nitems, K1)) * 8));
  HIPCHK(hipMemsetAsync(k->dense.p, 0, K1 * 4, st));
  u.ulen = k->ulen.as<uint32_t>();
  u.uoff = k->uoff.as<uint64_t>();
  u.uarena = k->uarena.as<uint8_t>();
  u.dense = k->dense.as<uint32_t>();
  u.tsum = k->tsum.as<uint64_t>();
  launch_kd_ids(u, st);
  launch_kd_place(u, K, st);
  HIPCHK(hipGetLastError());
  DevBuf sv;
  if (sim && K) {  // the all-reduce: every other rank's values scattered by the same union ids
    HIPCHK(sv.ensure((size_t)nr * maxn * 4));
    std::vector<uint32_t> hv((size_t)nr * maxn, 0);
    for (int r = 0; r < nr; r++)
      if (r != me)
        for (uint64_t i = 0; i < sim->n[r]; i++) hv[(size_t)r * maxn + i] = sim->vals[r][i];
    HIPCHK(hipMemcpyAsync(sv.p, hv.data(), hv.size() * 4, hipMemcpyHostToDevice, st));
    for (int r = 0; r < nr; r++) {
      if (r == me) continue;
      KdUnionArgs o = u;
      o.me = (uint32_t)r;
      o.lval = sv.as<uint32_t>() + (size_t)r * maxn;
      launch_kd_place(o, K, st);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));  // sv and the host vectors go out of scope
  }
  if (nccl && K) {  // u32 sums wrap, like the guest's release-mode adds
    ncclResult_t r = ncclAllReduce(k->dense.p, k->dense.p, K, ncclUint32, ncclSum, e->comm, st);
    if (r != ncclSuccess) return fail(FSG_E_DEVICE, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  }
  unsigned long long ub = 0;
  HIPCHK(hipMemcpyAsync(&ub, u.tot + 1, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  k->K = K;
  k->ubytes = ub;
  k->merged = true;
  if (n_keys) *n_keys = K;
  if (key_bytes) *key_bytes = ub;
  return FSG_OK;
}

extern "C" int fsg_keyed_allreduce(fsg_keyed* k, size_t* n_keys, size_t* key_bytes) {
  fsg_engine* e = k->eng;
  return kd_allreduce(k, e->comm ? e->nranks : 1, e->comm ? e->rank : 0, nullptr, n_keys, key_bytes);
}

// the merge over simulated gathered lists (C++ linkage, not part of the C ABI:
// its C entry lives in the test-hook library libfsg_hooks.so, fsg_hooks.cpp)
namespace fsg {
int keyed_allreduce_sim(fsg_keyed* k, uint32_t nranks, uint32_t me, const uint64_t* rank_n,
                        const uint64_t* const* rank_desc, const uint8_t* const* rank_arena,
                        const uint64_t* rank_arena_len, const uint32_t* const* rank_vals, size_t* n_keys,
                        size_t* key_bytes) {
  if (!nranks || me >= nranks || nranks > 1024 || !rank_n || !rank_desc || !rank_arena || !rank_arena_len ||
      !rank_vals)
    return fail(FSG_E_INVALID_ARG, "fsg_keyed_allreduce_sim: bad rank arguments");
  const KdSim sim{rank_n, rank_desc, rank_arena, rank_arena_len, rank_vals};
  return kd_allreduce(k, (int)nranks, (int)me, &sim, n_keys, key_bytes);
}
}  // namespace fsg

extern "C" int fsg_keyed_read(fsg_keyed* k, uint8_t* keys, size_t key_bytes, uint64_t* offs, uint32_t* vals,
                              size_t n) {
  if (!k->merged) return fail(FSG_E_INVALID_ARG, "fsg_keyed_allreduce has not run since the last collect");
  if (n < k->K || key_bytes < k->ubytes) return fail(FSG_E_INVALID_ARG, "buffers smaller than the merged table");
  HIPCHK(hipSetDevice(k->eng->device));
  HIPCHK(hipStreamSynchronize(k->st));
  if (k->K) {
    HIPCHK(hipMemcpy(offs, k->uoff.p, k->K * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(vals, k->dense.p, k->K * 4, hipMemcpyDeviceToHost));
  }
  if (offs) offs[k->K] = k->ubytes;
  if (k->ubytes) HIPCHK(hipMemcpy(keys, k->uarena.p, k->ubytes, hipMemcpyDeviceToHost));
  return FSG_OK;
}

extern "C" int fsg_keyed_device(fsg_keyed* k, const uint8_t** keys, const uint64_t** offs, const uint32_t** vals) {
  if (!k->merged) return fail(FSG_E_INVALID_ARG, "fsg_keyed_allreduce has not run since the last collect");
  HIPCHK(hipSetDevice(k->eng->device));
  HIPCHK(hipStreamSynchronize(k->st));
  if (keys) *keys = k->uarena.as<uint8_t>();
  if (offs) *offs = k->uoff.as<uint64_t>();
  if (vals) *vals = k->dense.as<uint32_t>();
  return FSG_OK;
}

extern "C" void fsg_keyed_free(fsg_keyed* k) { delete k; }
