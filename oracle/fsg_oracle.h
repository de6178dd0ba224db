/*
 * fsg_oracle.h — CPU ORACLE for the SmartModule record-transform path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C restatement of the reference
 * algorithm (deem0n/fluvio: fluvio-protocol codec, fluvio-smartmodule derive
 * semantics, fluvio-smartengine chain, fluvio-spu process_batch).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / the timed CPU baseline — never as the product path.
 *
 * Parity pinning: see oracle/README.md and tests/golden/ (KATs transcribed
 * from the reference's own tests; reference is Rust, unbuildable here).
 */
#ifndef FSG_ORACLE_H
#define FSG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes — same numeric space as include/fsg.h */
#define ORC_OK 0
#define ORC_E_UNKNOWN -1                 /* SmartModuleTransformErrorStatus::UnknownError */
#define ORC_E_INIT -2                    /* SmartModuleInitErrorStatus::InitError */
#define ORC_E_DECODING_BASE_INPUT -11
#define ORC_E_DECODING_RECORDS -22
#define ORC_E_ENCODING_OUTPUT -33
#define ORC_E_UNKNOWN_SM -100            /* EngineError::UnknownSmartModule */
#define ORC_E_INSTANTIATE -101
#define ORC_E_STORE_MEMORY -102
#define ORC_E_UNSUPPORTED -103
#define ORC_E_IO -104                    /* io::Error surfaced by FileBatchIterator / empty-chain decode */
#define ORC_E_INVALID_ARG -105

typedef struct orc_result {
  int status;
  /* process(): encoded Vec<Record> (u32 BE count + records)
   * process_batch(): encoded Batch (file format: 12-B preamble + 45-B header + records, CRC32C set) */
  uint8_t *bytes;
  size_t bytes_len;
  uint32_t n_records;
  int64_t base_offset;
  int32_t last_offset_delta;
  /* Option<SmartModuleTransformRuntimeError> */
  int has_error;
  char *hint;
  size_t hint_len;
  int64_t err_offset;
  int32_t err_kind;
  int has_key;
  uint8_t *key;
  size_t key_len;
  uint8_t *value;
  size_t value_len;
  /* infra error message (init errors etc.) */
  char *message;
  /* metrics deltas of this call */
  uint64_t m_bytes_in, m_records_out, m_invocations;
} orc_result;

typedef struct orc_chain orc_chain;

uint32_t orc_crc32c(const uint8_t *p, size_t n);
size_t orc_varint_encode(int64_t v, uint8_t *out);
size_t orc_varint_size(int64_t v);
int orc_varint_decode(const uint8_t *p, size_t n, int64_t *v, size_t *used);
/* 1: Rust's str Debug (toolchain 1.75) writes code point cp as \u{..}: not printable or Grapheme_Extend */
int orc_u_dbg_escaped(uint32_t cp);

orc_chain *orc_chain_new(void);
void orc_chain_free(orc_chain *c);
/* add a built-in SmartModule by reference module name; runs init().
 * returns ORC_OK or an error (message in *msg_out, malloc'd, may be NULL) */
int orc_chain_add(orc_chain *c, const char *module, const char **keys, const char **vals,
                  size_t n_params, const uint8_t *acc, size_t acc_len, int has_acc, char **msg_out);
int orc_chain_process(orc_chain *c, const uint8_t *raw, size_t raw_len, int64_t base_offset,
                      int64_t base_ts, orc_result *out);
int orc_process_batch(orc_chain *c, const uint8_t *slice, size_t slice_len, uint64_t max_bytes,
                      orc_result *out);
int orc_chain_accumulator(orc_chain *c, size_t stage, uint8_t **acc, size_t *len);
/* SmartModuleChainInstance::look_back for one stage: out->has_error carries the
 * SmartModuleLookbackRuntimeError (hint, err_offset, key, value) */
int orc_chain_look_back(orc_chain *c, size_t stage, const uint8_t *raw, size_t raw_len, orc_result *out);
void orc_result_free(orc_result *r);
void orc_free(void *p);

/* record-section codecs (fsg_codec.c): Compression::uncompress for codec
 * 1 gzip, 2 snappy, 3 lz4 (0 ok, -1 decode error, ORC_E_UNSUPPORTED zstd) and
 * the test-data encoders */
int orc_decompress(int codec, const uint8_t *s, size_t n, uint8_t **out, size_t *out_len);
int orc_compress(int codec, const uint8_t *s, size_t n, int flags, uint8_t **out, size_t *out_len);
uint32_t orc_xxh32(const uint8_t *p, size_t n, uint32_t seed);

/* regex oracle exposed for cross-checks with an independent engine */
int orc_regex_is_match(const char *pattern, const uint8_t *text, size_t n, int *is_match);

/* serde_json 1.0.96 from_slice::<StructuredLog> (fsg_json.c): 0 ok (*level =
 * 0 debug .. 3 error), 1 error (*msg / *msg_len: Display text, free with
 * orc_free), ORC_E_UNSUPPORTED */
int orc_json_structured_log(const uint8_t *s, size_t n, int *level, char **msg, size_t *msg_len);
/* generic derive(Deserialize) struct: fields "name" (String) or "name=a|b|c"
 * (unit enum, rename_all lowercase names), for the reference's other fixtures */
/* serde_json from_slice::<Vec<Value>> + to_string per element (array_map_json_array):
* 0 ok (elems / lens: count malloc'd canonical strings; free each + arrays with orc_free),
 * 1 error (*msg Display text), ORC_E_UNSUPPORTED (floats) */
int orc_json_array_map(const uint8_t *s, size_t n, uint8_t ***elems, size_t **lens, size_t *count, char **msg,
                       size_t *msg_len);
/* map_json_project: Map<String, Value> from_slice, to_string of the field's value.
 * 0 ok (*found; *out canonical value when found), 1 error (*msg), ORC_E_UNSUPPORTED */
/* aggregate-json: HashMap<String, u32> of one value (entries in text order) */
int orc_json_map_u32(const uint8_t *s, size_t n, uint8_t ***keys, size_t **klens, uint32_t **vals, size_t *count,
                     char **msg, size_t *msg_len);
/* SipHash-c-d (64-bit output) of m[0..n) under (k0, k1): SipHash-1-3 is std's
 * DefaultHasher, which fixes aggregate-json's HashMap order (fsg_oracle.c hb_*) */
uint64_t orc_siphash(int c_rounds, int d_rounds, uint64_t k0, uint64_t k1, const uint8_t *m, size_t n);
void orc_json_pretty_map(uint8_t *const *keys, const size_t *klens, const uint32_t *vals, size_t n, uint8_t **out,
                         size_t *out_len);
int orc_json_project(const uint8_t *s, size_t n, const char *field, uint8_t **out, size_t *out_len, int *found,
                     char **msg, size_t *msg_len);
int orc_json_struct(const uint8_t *s, size_t n, const char *name, const char **fields, int nfields, int *vals,
                    char **msg, size_t *msg_len);

#ifdef __cplusplus
}
#endif
#endif
