// fsg_hooks.cpp — GPU test hooks outside the C ABI of libfsg.so: the
// topic-wide keyed merge run over simulated gathered key lists of 2..N ranks on
// one GPU (the same kd_desc -> kd_union -> kd_ids -> kd_place kernels the RCCL
// merge runs).  Built as libfsg_hooks.so, linked against libfsg.so; no process
// call goes through it.
#include <cstddef>
#include <cstdint>

#include "fsg.h"

namespace fsg {
int keyed_allreduce_sim(fsg_keyed* k, uint32_t nranks, uint32_t me, const uint64_t* rank_n,
                        const uint64_t* const* rank_desc, const uint8_t* const* rank_arena,
                        const uint64_t* rank_arena_len, const uint32_t* const* rank_vals, size_t* n_keys,
                        size_t* key_bytes);
}

// every rank's send buffers (count, u64 descriptors, key arena, values), entry
// `me` ignored (the local table); the all-reduce is the sum of every rank's
// dense scatter
extern "C" int fsg_keyed_allreduce_sim(fsg_keyed* k, uint32_t nranks, uint32_t me, const uint64_t* rank_n,
                                       const uint64_t* const* rank_desc, const uint8_t* const* rank_arena,
                                       const uint64_t* rank_arena_len, const uint32_t* const* rank_vals,
                                       size_t* n_keys, size_t* key_bytes) {
  return fsg::keyed_allreduce_sim(k, nranks, me, rank_n, rank_desc, rank_arena, rank_arena_len, rank_vals, n_keys,
                                  key_bytes);
}
