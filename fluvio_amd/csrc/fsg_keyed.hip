// fsg_keyed.hip — aggregate-json state kept in HBM between calls, and the
// topic-wide keyed merge of the partitions' states (C5 keyed, SURVEY §8 e).
//
// 1. k_ajc_*: after a call of an aggregate-json chain the map as it stands
//    after the last record folded through the stop batch (the accumulator the
//    next record would read: aggregate-json/src/lib.rs:22-36, the SDK's
//    aggregate loop carrying `accumulator` from record to record) is written
//    into the chain's other state buffer (AjState).  The next call takes it as
//    its initial keys: no accumulator text is copied to the host and nothing
//    is re-parsed there.
// 2. k_kd_*: the rank-local table of exact keys (fsg_keyed_collect adds a
//    chain's state into it), the union dictionary of the all-gathered key lists
//    (ids by first occurrence in rank order, so every rank builds the same one)
//    and the dense K-slot u32 table that one ncclAllReduce sums.
#include <hip/hip_runtime.h>

#include "fsg_device.h"
#include "fsg_launch.h"

namespace fsg {
namespace {

__device__ __forceinline__ uint8_t up_byte(uint8_t c, bool up) {
  return (up && c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c;
}
__device__ __forceinline__ uint32_t grid_tid() { return blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint32_t grid_n() { return gridDim.x * blockDim.x; }

// ---------------------------------------------------------------------------
// 1. aggregate-json commit
// ---------------------------------------------------------------------------
__global__ void k_ajc_head(AjCommitArgs c) {
  if (threadIdx.x || blockIdx.x) return;
  const AggjArgs& a = c.a;
  const uint64_t n = a.brec[c.stop] + a.bcnt[c.stop];  // records folded through the stop batch
  uint32_t K = a.n_init;
  if (n) K = a.n_init + (uint32_t)(a.rnewb[n - 1] + a.rnew[n - 1]);
  c.out[0] = K;
  c.out[1] = n;
}
__global__ __launch_bounds__(256) void k_ajc_len(AjCommitArgs c) {
  const AggjArgs& a = c.a;
  const uint32_t K = (uint32_t)c.out[0];
  for (uint32_t k = grid_tid(); k < c.kmax; k += grid_n()) {
    if (k >= K) {
      c.dst.blen[k] = 0;
      continue;
    }
    const uint32_t tl = a.tlen[k];
    const uint32_t ml = k < a.n_init ? a.klen[k] : tl - 2u;  // a new key: its source bytes between the quotes
    c.dst.blen[k] = ml + tl;
    c.dst.val[k] = k < a.n_init ? a.val_init[k] : 0u;
  }
}
__global__ __launch_bounds__(256) void k_ajc_copy(AjCommitArgs c) {
  const AggjArgs& a = c.a;
  const uint32_t K = (uint32_t)c.out[0];
  for (uint32_t k = grid_tid(); k < K; k += grid_n()) {
    const bool init = k < a.n_init;
    const uint32_t tl = a.tlen[k];
    const uint8_t* t = (const uint8_t*)a.tptr[k];
    const uint8_t* m = init ? (const uint8_t*)a.kptr[k] : t + 1;
    const uint32_t ml = init ? a.klen[k] : tl - 2u;
    const bool up = !init && a.kup[k];  // committed keys are stored as the stage saw them
    uint8_t* d = c.dst.arena + c.dst.boff[k];
    for (uint32_t i = 0; i < ml; i++) d[i] = up_byte(m[i], up);
    for (uint32_t i = 0; i < tl; i++) d[ml + i] = up_byte(t[i], up);
    c.dst.kptr[k] = (uint64_t)d;
    c.dst.klen[k] = ml;
    c.dst.tptr[k] = (uint64_t)(d + ml);
    c.dst.tlen[k] = tl;
  }
}
// the values: the initial ones plus every entry of the records folded through
// the stop batch (u32 wrapping, as the release wasm adds)
__global__ __launch_bounds__(256) void k_ajc_vals(AjCommitArgs c) {
  const AggjArgs& a = c.a;
  const uint64_t n = c.out[1];
  for (uint64_t r = grid_tid(); r < n; r += grid_n()) {
    const uint32_t ne = a.rne[r];
    const uint64_t g0 = a.rent[r];
    for (uint32_t j = 0; j < ne; j++) {
      const uint32_t k = a.ekid[g0 + j];
      if (k != kSkipEntry) atomicAdd(&c.dst.val[k], a.eval[g0 + j]);
    }
  }
}

// ---------------------------------------------------------------------------
// 2. keyed tables
// ---------------------------------------------------------------------------
__device__ uint32_t kd_hash(const uint8_t* p, uint32_t n) {
  uint32_t h = 2166136261u;  // FNV-1a, then a finaliser (slots are taken from the low bits)
  for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 16777619u;
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  return h;
}
// bytes another workgroup published (slot CAS after a release fence): read
// at agent scope, past this CU's vector cache
__device__ __forceinline__ uint8_t ld_coherent(const uint8_t* p) {
  const uint32_t* w = (const uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
  const uint32_t x = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint8_t)(x >> (8 * ((uintptr_t)p & 3)));
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a chain's keys into the rank-local table (values added).  The source keys of
// one launch are distinct; a key already in the table (an earlier collect on
// this stream) gets the value added.  A new key is copied into the arena and
// published by a slot CAS; a thread that loses the slot to an equal key marks
// its copy dead.
__global__ __launch_bounds__(256) void k_kd_collect(KdTable t, const uint64_t* sptr, const uint32_t* slen,
                                                    const uint32_t* sval, uint32_t n) {
  for (uint32_t i = grid_tid(); i < n; i += grid_n()) {
    const uint8_t* p = (const uint8_t*)sptr[i];
    const uint32_t len = slen[i];
    const uint32_t v = sval[i];
    uint32_t s = kd_hash(p, len) & (t.cap - 1u);
    uint32_t mine = kKdDead;
    for (;;) {
      uint32_t cur = ld_agent(&t.slot[s]);
      if (cur == 0) {
        if (mine == kKdDead) {
          mine = (uint32_t)atomicAdd(&t.cnt[0], 1ull);
          const uint64_t off = atomicAdd(&t.cnt[1], (unsigned long long)len);
          for (uint32_t q = 0; q < len; q++) t.arena[off + q] = p[q];
          t.koff[mine] = off;
          t.klen[mine] = len;
          t.val[mine] = 0;
          __threadfence();  // the key before the slot that publishes it
        }
        cur = atomicCAS(&t.slot[s], 0u, mine + 1u);
        if (cur == 0) {
          atomicAdd(&t.val[mine], v);
          break;
        }
      }
      const uint32_t k = cur - 1u;
      const uint32_t kl = ld_agent(&t.klen[k]);
      bool eq = kl == len;
      if (eq) {
        const uint8_t* q = t.arena + ld_agent(&t.koff[k]);
        for (uint32_t j = 0; j < len && eq; j++) eq = ld_coherent(q + j) == p[j];
      }
      if (eq) {
        atomicAdd(&t.val[k], v);
        if (mine != kKdDead) t.klen[mine] = kKdDead;
        break;
      }
      s = (s + 1u) & (t.cap - 1u);
    }
  }
}
// the live keys of `src` into a fresh table `dst` (growth)
__global__ __launch_bounds__(256) void k_kd_rehash(KdTable dst, uint32_t n) {
  for (uint32_t i = grid_tid(); i < n; i += grid_n()) {
    if (dst.klen[i] == kKdDead) continue;
    uint32_t s = kd_hash(dst.arena + dst.koff[i], dst.klen[i]) & (dst.cap - 1u);
    while (atomicCAS(&dst.slot[s], 0u, i + 1u) != 0u) s = (s + 1u) & (dst.cap - 1u);
  }
}

// the union of the gathered key lists: item g = rank * maxn + i; gdesc[g] =
// arena offset | len << 40 (kKdDesc dead / absent), bytes in garena[rank * maxb ..]
__device__ __forceinline__ const uint8_t* kd_item(const uint8_t* garena, uint64_t maxb, uint32_t maxn, uint64_t d,
                                                  uint32_t g) {
  return garena + (uint64_t)(g / maxn) * maxb + (d & ((1ull << 40) - 1ull));
}
constexpr uint64_t kKdLenDead = 0xFFFFFFull;
__global__ __launch_bounds__(256) void k_kd_union(uint32_t* slot, uint32_t cap, const uint64_t* gdesc,
                                                  const uint8_t* garena, uint64_t maxb, uint32_t maxn, uint32_t nitems,
                                                  uint32_t* gslot) {
  for (uint32_t g = grid_tid(); g < nitems; g += grid_n()) {
    const uint64_t d = gdesc[g];
    const uint32_t len = (uint32_t)(d >> 40);
    if (len == kKdLenDead) {
      gslot[g] = kKdDead;
      continue;
    }
    const uint8_t* p = kd_item(garena, maxb, maxn, d, g);
    uint32_t s = kd_hash(p, len) & (cap - 1u);
    for (;;) {
      uint32_t cur = ld_agent(&slot[s]);
      if (cur == 0) {
        cur = atomicCAS(&slot[s], 0u, g + 1u);
        if (cur == 0) break;
      }
      // an equal key holds the slot: the earliest item (rank-major) keeps it.
      // Every item with this key has the same bytes, so the comparison does not
      // depend on which of them the slot names at the moment.
      const uint32_t o = cur - 1u;
      const uint64_t od = gdesc[o];
      bool eq = (uint32_t)(od >> 40) == len;
      if (eq) {
        const uint8_t* q = kd_item(garena, maxb, maxn, od, o);
        for (uint32_t j = 0; j < len && eq; j++) eq = q[j] == p[j];
      }
      if (eq) {
        if (g + 1u < cur) atomicMin(&slot[s], g + 1u);
        break;
      }
      s = (s + 1u) & (cap - 1u);
    }
    gslot[g] = s;
  }
}
__global__ __launch_bounds__(256) void k_kd_first(const uint32_t* slot, const uint32_t* gslot, uint32_t nitems,
                                                  uint32_t* first) {
  for (uint32_t g = grid_tid(); g < nitems; g += grid_n())
    first[g] = (gslot[g] != kKdDead && slot[gslot[g]] == g + 1u) ? 1u : 0u;
}
// per item: the union id of its key; the union's key lengths by id
__global__ __launch_bounds__(256) void k_kd_ids(const uint32_t* slot, const uint32_t* gslot, const uint64_t* idpre,
                                                const uint64_t* gdesc, uint32_t nitems, uint32_t* gid, uint32_t* ulen) {
  for (uint32_t g = grid_tid(); g < nitems; g += grid_n()) {
    if (gslot[g] == kKdDead) {
      gid[g] = kKdDead;
      continue;
    }
    const uint32_t f = slot[gslot[g]] - 1u;
    const uint32_t id = (uint32_t)idpre[f];
    gid[g] = id;
    if (f == g) ulen[id] = (uint32_t)(gdesc[g] >> 40);
  }
}
// the union's keys in id order (the first occurrence copies them); this
// rank's values into the dense table (a rank's keys are distinct)
__global__ __launch_bounds__(256) void k_kd_place(const uint32_t* slot, const uint32_t* gslot, const uint32_t* gid,
                                                  const uint64_t* gdesc, const uint8_t* garena, uint64_t maxb,
                                                  uint32_t maxn, uint32_t nitems, const uint64_t* uoff, uint8_t* uarena,
                                                  uint32_t me, const uint32_t* lval, uint32_t* dense) {
  for (uint32_t g = grid_tid(); g < nitems; g += grid_n()) {
    const uint32_t id = gid[g];
    if (id == kKdDead) continue;
    if (g / maxn == me) dense[id] += lval[g % maxn];
    if (slot[gslot[g]] != g + 1u) continue;
    const uint64_t d = gdesc[g];
    const uint32_t len = (uint32_t)(d >> 40);
    const uint8_t* p = kd_item(garena, maxb, maxn, d, g);
    uint8_t* q = uarena + uoff[id];
    for (uint32_t j = 0; j < len; j++) q[j] = p[j];
  }
}
// the local table's key descriptors for the all-gather (off | len << 40)
__global__ __launch_bounds__(256) void k_kd_desc(KdTable t, uint32_t n, uint32_t maxn, uint64_t* desc) {
  for (uint32_t i = grid_tid(); i < maxn; i += grid_n())
    desc[i] = i < n && t.klen[i] != kKdDead ? (t.koff[i] | ((uint64_t)t.klen[i] << 40)) : (kKdLenDead << 40);
}

uint32_t grid1(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (uint32_t)(g < 1 ? 1 : g > 4096 ? 4096 : g);
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers (fsg_launch.h)
// ---------------------------------------------------------------------------
void launch_aggj_commit(const AjCommitArgs& c, uint64_t* tsum, int pass, hipStream_t s) {
  if (pass == 0) {  // keys / records through the stop batch, arena bytes (out[0..2])
    hipLaunchKernelGGL(k_ajc_head, dim3(1), dim3(64), 0, s, c);
    if (c.kmax) hipLaunchKernelGGL(k_ajc_len, dim3(grid1(c.kmax)), dim3(256), 0, s, c);
    launch_xscan(c.dst.blen, c.dst.boff, tsum, c.kmax, c.out + 2, s);
    return;
  }
  if (c.kmax) hipLaunchKernelGGL(k_ajc_copy, dim3(grid1(c.kmax)), dim3(256), 0, s, c);
  if (c.a.n_rec) hipLaunchKernelGGL(k_ajc_vals, dim3(grid1(c.a.n_rec)), dim3(256), 0, s, c);
}
void launch_kd_collect(const KdTable& t, const uint64_t* sptr, const uint32_t* slen, const uint32_t* sval, uint32_t n,
                       hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_kd_collect, dim3(grid1(n)), dim3(256), 0, s, t, sptr, slen, sval, n);
}
void launch_kd_rehash(const KdTable& t, uint32_t n, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_kd_rehash, dim3(grid1(n)), dim3(256), 0, s, t, n);
}
void launch_kd_desc(const KdTable& t, uint32_t n, uint32_t maxn, uint64_t* desc, hipStream_t s) {
  if (maxn) hipLaunchKernelGGL(k_kd_desc, dim3(grid1(maxn)), dim3(256), 0, s, t, n, maxn, desc);
}
void launch_kd_union(const KdUnionArgs& u, hipStream_t s) {
  if (!u.nitems) return;
  const uint32_t g = grid1(u.nitems);
  hipLaunchKernelGGL(k_kd_union, dim3(g), dim3(256), 0, s, u.slot, u.cap, u.gdesc, u.garena, u.maxb, u.maxn, u.nitems,
                     u.gslot);
  hipLaunchKernelGGL(k_kd_first, dim3(g), dim3(256), 0, s, u.slot, u.gslot, u.nitems, u.first);
  launch_xscan(u.first, u.idpre, u.tsum, u.nitems, u.tot + 0, s);  // tot[0] = K
}
void launch_kd_ids(const KdUnionArgs& u, hipStream_t s) {
  if (!u.nitems) return;
  hipLaunchKernelGGL(k_kd_ids, dim3(grid1(u.nitems)), dim3(256), 0, s, u.slot, u.gslot, u.idpre, u.gdesc, u.nitems,
                     u.gid, u.ulen);
}
void launch_kd_place(const KdUnionArgs& u, uint64_t nkeys, hipStream_t s) {
  launch_xscan(u.ulen, u.uoff, u.tsum, nkeys, u.tot + 1, s);  // tot[1] = union arena bytes
  if (!u.nitems) return;
  hipLaunchKernelGGL(k_kd_place, dim3(grid1(u.nitems)), dim3(256), 0, s, u.slot, u.gslot, u.gid, u.gdesc, u.garena,
                     u.maxb, u.maxn, u.nitems, u.uoff, u.uarena, u.me, u.lval, u.dense);
}

}  // namespace fsg
