/*
 * fsg.h — C ABI of the MI355X SmartModule engine (libfsg.so).
 *
 * Drop-in boundary for Fluvio's SmartModule record-transform path.  Each entry
 * point replaces one reference interface (paths relative to the reference
 * deem0n/fluvio tree):
 *
 *   fsg_engine_new                      SmartEngine::new
 *                                         crates/fluvio-smartengine/src/engine/wasmtime/engine.rs:31
 *   fsg_chain_builder_new               SmartModuleChainBuilder::default            engine.rs:94-103
 *   fsg_chain_builder_set_store_memory_limit
 *                                       SmartModuleChainBuilder::set_store_memory_limit  engine.rs:60
 *   fsg_chain_builder_add_smart_module  SmartModuleChainBuilder::add_smart_module   engine.rs:56
 *                                         (+ SmartModuleConfig, config.rs:33-74)
 *   fsg_chain_builder_initialize        SmartModuleChainBuilder::initialize         engine.rs:65-91
 *                                         (+ create_transform, transforms/mod.rs:24-52)
 *   fsg_chain_process                   SmartModuleChainInstance::process           engine.rs:135-185
 *   fsg_chain_look_back                 SmartModuleChainInstance::look_back         engine.rs:187-218
 *                                         (read_fn = the SPU's read_records, smartengine/context.rs:46-60,117-160)
 *   fsg_chain_builder_set_lookback      SmartModuleConfigBuilder::lookback          config.rs:45-73
 *   fsg_chain_process_batch             fluvio-spu process_batch                    crates/fluvio-spu/src/smartengine/batch.rs:41-142
 *                                         over a FileBatchIterator slice           crates/fluvio-storage/src/iterators.rs:55-160
 *   fsg_chain_get_accumulator           SmartModuleAggregate accumulator            transforms/aggregate.rs:22-25,95
 *   fsg_metrics                         SmartModuleChainMetrics                     crates/fluvio-smartengine/src/engine/metrics.rs:6-41
 *   fsg_runtime_error                   SmartModuleTransformRuntimeError            crates/fluvio-protocol/src/link/smartmodule.rs:12-43
 *   fsg_last_store_memory               EngineError::StoreMemoryExceeded{current,requested,max}
 *                                         crates/fluvio-smartengine/src/engine/error.rs:2-13
 *   fsg_state_* / fsg_allreduce_state   per-partition aggregate state (SmartModuleAggregate.accumulator,
 *                                         transforms/aggregate.rs:22-25) kept in HBM and merged across GPUs;
 *                                         no reference counterpart (partitions never exchange state there:
 *                                         crates/fluvio-spu/src/smartengine/context.rs:25-30)
 *
 * SmartModule selection happens at chain-build time: `module` bytes are either a
 * wasm binary ("\0asm" magic -> FSG_E_UNKNOWN_SM: this library runs no wasm) or a
 * built-in descriptor "\0fsg" + <reference module name>, e.g. "\0fsgregex-filter".
 * Transform configuration travels in `params` exactly as the reference passes it
 * to `init` (wasmtime/instance.rs:69-78): key="..." for filter_init, regex="..."
 * for regex-filter, etc.
 *
 * Conventions: the caller owns input buffers (borrowed for the call); the
 * library owns output objects until the matching *_free.  Every function
 * returns 0 on success or a negative FSG_E_* code; fsg_last_error_message()
 * gives the text of the last failure on the calling thread.  A record-level
 * SmartModule error is data (has_error in the output), not a return code,
 * exactly like SmartModuleOutput.error.  A chain is single-threaded (&mut self
 * in the reference); an engine may be shared by chains.  Everything runs on the
 * GPU: there is no CPU fallback, and with no usable HIP device fsg_engine_new
 * fails with FSG_E_DEVICE.
 */
#ifndef FSG_H
#define FSG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FSG_ABI_VERSION 6 /* 6: fsg_timings gained chunks; 5: fsg_timings gained text_ms / order_ms; 4: eval_path / deferred, fsg_keyed_*, fsg_host_cache_trim */

/* ---- status codes (mirror EngineError and the guest status enums) ---- */
#define FSG_OK 0
#define FSG_E_UNKNOWN -1             /* SmartModuleTransformErrorStatus::UnknownError (error.rs:20) */
#define FSG_E_INIT -2                /* SmartModuleInitErrorStatus::InitError (error.rs:41) */
#define FSG_E_DECODING_BASE_INPUT -11 /* SmartModuleTransformErrorStatus::DecodingBaseInput */
#define FSG_E_DECODING_RECORDS -22
#define FSG_E_ENCODING_OUTPUT -33
#define FSG_E_UNKNOWN_SM -100        /* EngineError::UnknownSmartModule (error.rs:3) */
#define FSG_E_INSTANTIATE -101       /* EngineError::Instantiate */
#define FSG_E_STORE_MEMORY -102      /* EngineError::StoreMemoryExceeded */
#define FSG_E_UNSUPPORTED -103       /* valid for the reference, not implemented on the GPU path */
#define FSG_E_IO -104                /* io::Error from batch framing / empty-chain record decode */
#define FSG_E_INVALID_ARG -105
#define FSG_E_LOOKBACK -106          /* Err(SmartModuleLookbackRuntimeError) from look_back (link/smartmodule.rs:150-176) */
#define FSG_E_DEVICE -200            /* HIP runtime failure / no device */

/* SmartModuleKind tags (link/smartmodule.rs:80-95) */
#define FSG_KIND_FILTER 0
#define FSG_KIND_MAP 1
#define FSG_KIND_ARRAY_MAP 2
#define FSG_KIND_AGGREGATE 3
#define FSG_KIND_FILTER_MAP 4

/* Lookback (config.rs:45-49): Last(n) / Age{age, last} */
#define FSG_LOOKBACK_NONE 0
#define FSG_LOOKBACK_LAST 1
#define FSG_LOOKBACK_AGE 2

typedef struct fsg_engine fsg_engine;
typedef struct fsg_chain_builder fsg_chain_builder;
typedef struct fsg_chain fsg_chain;
typedef struct fsg_slice fsg_slice;

typedef struct fsg_param {
  const char *key;
  const char *value;
} fsg_param;

typedef struct fsg_metrics {
  uint64_t bytes_in;
  uint64_t records_out;
  uint64_t invocation_count;
  uint64_t fuel_used; /* always 0: no fuel metering on the GPU */
} fsg_metrics;

typedef struct fsg_runtime_error {
  const char *hint; /* UTF-8, hint_len bytes (not NUL-terminated in general) */
  size_t hint_len;
  int64_t offset;
  int32_t kind;     /* FSG_KIND_* */
  int32_t has_key;
  const uint8_t *key;
  size_t key_len;
  const uint8_t *value;
  size_t value_len;
} fsg_runtime_error;

/* SmartModuleOutput: successes encoded as Vec<Record> (u32 BE count + records) */
typedef struct fsg_output {
  const uint8_t *records;
  size_t records_len;
  uint32_t n_records;
  int32_t has_error;
  fsg_runtime_error error;
} fsg_output;

/* the Lookback a stage asks its look_back records for */
typedef struct fsg_lookback {
  int32_t kind;    /* FSG_LOOKBACK_LAST / FSG_LOOKBACK_AGE */
  uint32_t stage;  /* chain position of the stage */
  uint64_t last;
  uint64_t age_ms;
} fsg_lookback;
/* look_back's read_fn: the records to feed (encoded Vec<Record>: u32 BE count +
 * records), valid until read_fn is called again or look_back returns; nonzero
 * return = the read failed (look_back returns FSG_E_IO) */
typedef int (*fsg_read_fn)(void *user, const fsg_lookback *lb, const uint8_t **records, size_t *len);

/* (Batch, Option<SmartModuleTransformRuntimeError>) returned by SPU process_batch.
 * `batch` is the file-format encoding (12-byte preamble + 45-byte header + u32
 * count + records) with CRC32C computed, as Batch::encode writes it. */
typedef struct fsg_batch_output {
  const uint8_t *batch;
  size_t batch_len;
  int64_t base_offset;
  int32_t last_offset_delta;
  uint32_t n_records;
  int32_t has_error;
  fsg_runtime_error error;
} fsg_batch_output;

/* per-call device timings of the last process call (HIP events on the chain stream) */
typedef struct fsg_timings {
  float eval_ms;    /* decode + transform kernel */
  float plan_ms;    /* size + scan + plan kernels */
  float write_ms;   /* compaction / re-encode kernel */
  float crc_ms;     /* CRC32C kernels */
  float total_ms;   /* first kernel start to last kernel end */
  uint64_t in_bytes;      /* algorithmic bytes read (batch headers + record sections) */
  uint64_t out_bytes;     /* algorithmic bytes written (output batch) */
  uint64_t n_batches;
  uint64_t n_records_in;
  uint32_t eval_path;     /* FSG_EVAL_*: the first evaluation kernel */
  uint32_t deferred;      /* batches that kernel handed to the exact kernel (non-ASCII, odd framing, ...) */
  float text_ms;          /* plan end to write start: aggregate texts, the aggregate-json order walk, the header */
  float order_ms;         /* the aggregate-json order walk kernel alone (a group call: the group's one launch) */
  uint32_t chunks;        /* fsg_chain_process_batch pipelined over this many slice chunks (0: serial); the
                             per-phase times and eval_path are then the last chunk's */
  uint32_t reserved;
} fsg_timings;
#define FSG_EVAL_EXACT 0 /* k_eval over every batch */
#define FSG_EVAL_LEAN 1  /* k_eval_lean (LDS windows), deferred batches through k_eval */
/* 2: retired (an opt-in register-resident substring path, slower than k_eval_lean on MI355X) */
#define FSG_EVAL_ARRAY 3 /* k_arr_lean (array_map lane per record), deferred batches through k_eval */
#define FSG_EVAL_FLAT 4  /* one substring stage: the slice streamed as bytes (k_flat_scan), a wave per batch
                            decides (k_flat_decide), deferred batches through k_eval */
#define FSG_EVAL_INT 5   /* integer stages over decimal values: k_eval_int (workgroup per batch, record starts
                            kept with the slice), deferred batches through k_eval */
#define FSG_EVAL_FJSON 6 /* filter_json / field projection (+ one substring stage): the slice streamed as bytes
                            (k_flat_scan<., kJson>: JSON-interesting chunks), a thread per batch parses the
                            records' values as flat objects (k_fj_decide), deferred batches through k_eval */
#define FSG_EVAL_RX 7    /* one bounded regex stage: the DFA over every 16-byte chunk's window of the flat slice
                            (k_rx_scan), a thread per batch decides from the bits and the values' edges
                            (k_rx_decide), deferred batches through k_eval */

const char *fsg_last_error_message(void);
int fsg_abi_version(void);
/* the numbers of the last FSG_E_STORE_MEMORY on the calling thread
 * (EngineError::StoreMemoryExceeded{current, requested, max}) */
int fsg_last_store_memory(uint64_t *current, uint64_t *requested, uint64_t *max);

/* ---- engine ------------------------------------------------------------ */
int fsg_device_count(int *count);
int fsg_engine_new(int device, fsg_engine **out);
void fsg_engine_free(fsg_engine *engine);

/* ---- chain builder ----------------------------------------------------- */
int fsg_chain_builder_new(fsg_chain_builder **out);
int fsg_chain_builder_set_store_memory_limit(fsg_chain_builder *b, size_t max_memory_bytes);
/* SmartModuleConfig{params, version, initial_data} + module bytes.
 * has_initial_acc=0 means SmartModuleInitialData::None. */
int fsg_chain_builder_add_smart_module(fsg_chain_builder *b, const fsg_param *params, size_t n_params,
                                       int16_t version, const uint8_t *initial_acc, size_t acc_len,
                                       int32_t has_initial_acc, const uint8_t *module, size_t module_len);
/* SmartModuleConfig.lookback of the module added `module_index`-th (0-based) */
int fsg_chain_builder_set_lookback(fsg_chain_builder *b, size_t module_index, int32_t kind, uint64_t last,
                                   uint64_t age_ms);
/* consumes the builder (initialize(self)) whether or not it succeeds */
int fsg_chain_builder_initialize(fsg_chain_builder *b, fsg_engine *engine, fsg_chain **out);
void fsg_chain_builder_free(fsg_chain_builder *b);

/* ---- chain ------------------------------------------------------------- */
int fsg_chain_process(fsg_chain *c, const uint8_t *raw_records, size_t len, int64_t base_offset,
                      int64_t base_timestamp, fsg_metrics *metrics, fsg_output **out);
/* process_batch over a host slice.  A slice of at least two chunks (128 MiB;
 * FSG_PIPE_CHUNK bytes) through a stateless chain of filters / uppercase maps /
 * projections, with `out` given, runs pipelined: the slice is uploaded in
 * pieces on one thread while whole-batch chunks of it are processed and the
 * previous chunk's records are downloaded on another; the result is the same
 * one output batch (fsg_timings.chunks says how many chunks; the device copy
 * of fsg_chain_output_device is then not kept).  FSG_NO_PIPE=1: serial. */
int fsg_chain_process_batch(fsg_chain *c, const uint8_t *slice, size_t len, uint64_t max_bytes,
                            fsg_metrics *metrics, fsg_batch_output **out);
/* look_back (engine.rs:187-218): for every stage with a look_back function
 * (filter_look_back, filter_hashset) and a Lookback, read_fn gives the records and
 * the stage's look_back runs over them on the GPU (metrics: bytes_in + one
 * invocation per stage).  A record error returns FSG_E_LOOKBACK with *error set
 * (free with fsg_runtime_error_free); no such stage: Ok without calling read_fn. */
int fsg_chain_look_back(fsg_chain *c, fsg_read_fn read_fn, void *user, fsg_metrics *metrics,
                        fsg_runtime_error *error);
void fsg_runtime_error_free(fsg_runtime_error *e);
int fsg_chain_get_accumulator(fsg_chain *c, size_t stage, uint8_t **acc, size_t *len);
int fsg_chain_last_timings(fsg_chain *c, fsg_timings *t);
void fsg_chain_free(fsg_chain *c);
/* Release an output.  Large output buffers (>= 4 MiB) are parked for reuse by the
 * next large output (at most two, process-wide) instead of being unmapped; a
 * parked buffer still holds earlier output bytes past its batch_len. */
void fsg_output_free(fsg_output *o);
void fsg_batch_output_free(fsg_batch_output *o);
void fsg_free(void *p);
/* Unmap every parked output buffer now (the last fsg_engine_free does it too).
 * No reference counterpart: the host memory policy of this library. */
void fsg_host_cache_trim(void);

/* ---- HBM-resident path (batches ingested once, processed many times) --- */
/* Ingest: copies the slice to HBM and frames its batches (FileBatchIterator). */
int fsg_slice_upload(fsg_engine *engine, const uint8_t *slice, size_t len, fsg_slice **out);
int fsg_slice_info(const fsg_slice *s, uint64_t *n_batches, uint64_t *n_records, uint64_t *bytes);
/* 1 if the slice was framed on the device (k_frame_*: magic-2 candidates,
 * pointer doubling from position 0), 0 if the host walk framed it (a batch
 * without magic 2 on the chain, or candidates too dense).  Same result either
 * way (FileBatchIterator::next, crates/fluvio-storage/src/iterators.rs:55-160). */
int fsg_slice_device_framed(const fsg_slice *s);
/* Frame the slice's HBM-resident bytes again on the device (a freshly fetched
 * slice: FileBatchIterator framing, iterators.rs:55-160); FSG_E_UNSUPPORTED
 * for slices that needed the host walk or were decompressed at ingest. */
int fsg_slice_reframe(fsg_slice *s);
/* CRC32C (Castagnoli) of every framed batch, computed on the GPU over header
 * bytes 21.. + records and compared with the stored crc: *n_bad mismatches,
 * *first_bad the first such batch (-1 none), *ms the kernel time.  Reports
 * only — the reference never verifies (crates/fluvio-protocol/src/record/
 * batch.rs:398-430 computes the CRC on encode only), so processing ignores it.
 * For a slice with compressed batches the check runs on the stored bytes at
 * ingest (before decompression) and this returns that result. */
int fsg_slice_verify_crc(const fsg_slice *s, uint64_t *n_bad, int64_t *first_bad, float *ms);
/* Starts the same check on the slice's own stream and returns at once, so a
 * fetch verifies while fsg_chain_process_slice runs on the same (read-only)
 * bytes; the next fsg_slice_verify_crc returns its result.  Reframing or
 * re-uploading the slice waits for it first.  The slice must be fully framed
 * when this is called: nothing on the device orders the verify after the
 * framing, which holds because fsg_slice_upload and fsg_slice_reframe return
 * only once their framing (and the batch table it writes) is complete. */
int fsg_slice_verify_crc_start(const fsg_slice *s);
void fsg_slice_free(fsg_slice *s);
/* process_batch over a resident slice; the output batch stays in HBM until
 * fsg_chain_download_output (out may be NULL to keep it resident). */
int fsg_chain_process_slice(fsg_chain *c, const fsg_slice *s, uint64_t max_bytes, fsg_metrics *metrics,
                            fsg_batch_output **out);
/* process_slice of several chains at once: the partitions a rank owns, one
 * chain instance each (crates/fluvio-spu/src/smartengine/context.rs:25-30),
 * each over its own resident slice.  The chains run concurrently on their own
 * streams; what walks a chain's records in stream order (aggregate-json's map
 * order) runs as one launch over all of them.  metrics: n entries or NULL;
 * outs: n entries or NULL (NULL keeps every output in HBM, as process_slice);
 * rcs[i] = chain i's status (the call returns the first failure, its message
 * in fsg_last_error_message). */
int fsg_chain_group_process_slices(fsg_chain *const *chains, const fsg_slice *const *slices, size_t n,
                                   uint64_t max_bytes, fsg_metrics *metrics, fsg_batch_output **outs, int *rcs);
/* device pointer + size of the last resident output batch (valid until the next call) */
int fsg_chain_output_device(fsg_chain *c, const void **dptr, size_t *len);

/* ---- multi-GPU aggregate state merge (RCCL over xGMI) ------------------- */
#define FSG_UNIQUE_ID_BYTES 128
/* element types of aggregate state (sums wrap like the release-mode wasm guest) */
#define FSG_DTYPE_I32 0
#define FSG_DTYPE_U32 1
#define FSG_DTYPE_I64 2
#define FSG_DTYPE_U64 3
#define FSG_DTYPE_F64 4
int fsg_comm_unique_id(uint8_t id[FSG_UNIQUE_ID_BYTES]);
int fsg_engine_comm_init(fsg_engine *engine, const uint8_t id[FSG_UNIQUE_ID_BYTES], int nranks, int rank);
/* all-reduce (sum) of `count` dtype elements of aggregate state in HBM across the
 * engine's communicator, on the engine's collective stream; returns when done */
int fsg_allreduce_state(fsg_engine *engine, void *dev_state, size_t count, int dtype);
/* the same on a chain's stream (ordered after the chain's kernels) */
int fsg_chain_allreduce_state(fsg_chain *c, void *dev_state, size_t count, int dtype);

/* Per-partition aggregate state vector in HBM (one slot per topic partition;
 * partitions sharded p -> GPU p mod N).  collect copies a chain's aggregate-sum
 * accumulator (i32, written by the GPU after every call) into a slot, device to
 * device; allreduce merges the vectors of all ranks (slots owned by other ranks
 * are zero locally, so the sum is the topic-wide table). */
typedef struct fsg_state fsg_state;
int fsg_state_new(fsg_engine *engine, size_t count, int dtype, fsg_state **out);
int fsg_state_collect(fsg_state *s, size_t slot, fsg_chain *c);
int fsg_state_allreduce(fsg_state *s);
int fsg_state_read(fsg_state *s, void *host, size_t bytes);
int fsg_state_device(fsg_state *s, void **dptr);
void fsg_state_free(fsg_state *s);

/* ---- topic-wide keyed totals of aggregate-json states (C5 keyed) ---------
 * Each partition's chain keeps its aggregate-json map in HBM between calls
 * (SmartModuleAggregate.accumulator, context.rs:25-30; the map of
 * smartmodule/examples/aggregate-json/src/lib.rs:22-35).  A keyed table sums
 * the maps of the chains collected into it by exact key bytes (u32 wrapping);
 * fsg_keyed_allreduce builds the topic key dictionary across ranks (RCCL
 * all-gather of every rank's key list; the union in rank order, so every rank
 * holds the same dictionary) and sums one dense K-slot u32 table with an RCCL
 * all-reduce.  Without a communicator (one rank) the same steps run locally.
 * The key order of the result is the union's (first occurrence by rank, then
 * by collect); no reference counterpart: each partition's own accumulator is
 * the reference's (fsg_chain_get_accumulator). */
typedef struct fsg_keyed fsg_keyed;
int fsg_keyed_new(fsg_engine *engine, fsg_keyed **out);
int fsg_keyed_reset(fsg_keyed *k);                                  /* empty the local table */
int fsg_keyed_collect(fsg_keyed *k, fsg_chain *c, size_t stage);     /* add the chain's map (device side, async) */
int fsg_keyed_allreduce(fsg_keyed *k, size_t *n_keys, size_t *key_bytes);
/* keys: the union's key bytes (key i = keys[offs[i] .. offs[i + 1])), offs: n + 1 entries, vals: n */
int fsg_keyed_read(fsg_keyed *k, uint8_t *keys, size_t key_bytes, uint64_t *offs, uint32_t *vals, size_t n);
int fsg_keyed_device(fsg_keyed *k, const uint8_t **keys, const uint64_t **offs, const uint32_t **vals);
void fsg_keyed_free(fsg_keyed *k);
/* (The merge over simulated ranks, fsg_keyed_allreduce_sim, is a GPU test hook
 * in libfsg_hooks.so, outside this ABI.) */

#ifdef __cplusplus
}
#endif
#endif /* FSG_H */
