// fsg_device.h — data layout shared by the host runtime and the CDNA4 kernels.
//
// HBM layout of one process_batch call (see DESIGN.md "Data layout"):
//   slice     : the stored batches exactly as FileBatchIterator reads them
//               (57-byte file header + record section per batch), padded to
//               a 16-byte multiple plus kSlicePad bytes of zeros
//   bpos[]    : u64 byte offset of each batch in the slice (ingest framing)
//   rbase[]   : u64 exclusive prefix of the record counts (descriptor base)
//   bstat[]   : BatchStat per batch (written by k_eval)
//   desc[]    : KeptRec per kept record, at rbase[b] + k
//   rows[]    : ScanRow per batch (k_size), scanned in place
//   out       : the output batch (61-byte header + records)
#pragma once
#include <stdint.h>

namespace fsg {

constexpr int kWave = 64;
constexpr int kWin = 17408;     // LDS record window per wave (bytes)
constexpr int kMaxR = 128;      // records per window
constexpr int kMaxStages = 8;
constexpr int kSlicePad = 256;  // zero padding behind the slice (over-read guard)
constexpr int kCrcChunk = 65536;

// stage operations (built-in GPU SmartModules)
enum StageOp : uint8_t {
  OP_CONTAINS = 0,     // filter / filter_init / filter_with_param: from_utf8 + contains(needle)
  OP_REGEX = 1,        // regex-filter (keep match) / filter_regex (keep non-match)
  OP_FILTER_ODD = 2,   // filter_odd: from_utf8 + parse::<i32> + keep even
  OP_MAP_UPPER = 3,    // map: make_ascii_uppercase
  OP_MAP_DOUBLE = 4,   // map_double: from_utf8 + parse::<i32> * 2
  OP_FILTER_MAP = 5,   // filter_map: from_utf8_lossy + parse::<i32>, even -> /2
  OP_AGG_SUM = 6,      // aggregate-sum (last stage only)
  OP_FILTER_JSON = 7,  // filter_json: serde_json::from_slice::<StructuredLog>, keep level > Debug
  OP_ARRAY_MAP = 8,    // array_map_json_array: Vec<serde_json::Value> -> one record per element (last stage)
  OP_AGG_CONCAT = 9,   // aggregate: String accumulator ++ value (last stage)
  OP_PROJECT = 10,     // map_json_project: the value narrows to one JSON field's text (FilterMap)
  OP_AGG_JSON = 11,    // aggregate-json: HashMap<String, u32> += per key, pretty JSON accumulator (last stage)
  OP_LB_MAX = 12,      // filter_look_back: from_utf8 + parse::<i32>, keep > PREV (stateful, last stage)
  OP_DEDUP = 13,       // filter_hashset: from_utf8, keep values new to a BoundedHashSet (stateful, last stage)
};

// value representation entering a stage (static per chain position)
enum ValType : uint8_t { VT_SRC = 0, VT_SRC_UPPER = 1, VT_I32 = 2 };

// error detail codes stored in BatchStat::err_code
enum ErrCode : uint32_t {
  EC_NONE = 0,
  EC_UTF8 = 1,        // aux = valid_up_to, aux2 = error_len (0 = None)
  EC_PARSE = 2,       // aux = ParseIntError kind (1 Empty, 2 InvalidDigit, 3 PosOverflow, 4 NegOverflow)
  EC_ACC_UTF8 = 3,    // aggregate accumulator is not UTF-8 (aux/aux2 as EC_UTF8)
  EC_UNSUP = 4,       // the record needs a feature the GPU path lacks (reached in stream order)
  EC_JSON = 5,        // serde_json error: bits 8..15 JsonErr, 16..23 sub; aux = reader index,
                      // aux2 / aux3 = span (fsg_json_dev.h)
};

struct DfaDesc {
  // ASCII DFA: every class restricted to ASCII; exact on ASCII-only values.
  // <= 255 states, u8 transitions, staged in LDS when it fits.
  uint32_t nstates;
  uint32_t nclasses;
  uint32_t s_bot;      // start state at value start (^ satisfied)
  uint32_t s_mid;      // restart state inside a value
  int32_t max_len;     // longest match in bytes, -1 = unbounded
  uint32_t classmap;   // blob offset: u8[256]
  uint32_t classmap_up;// blob offset: u8[256], classmap of toupper(byte)
  uint32_t trans;      // blob offset: u8[nstates * nclasses]
  uint32_t accept;     // blob offset: u8[256] (bit0 accept, bit1 accept at end of value)
  // full Unicode DFA for values with non-ASCII bytes: u16 transitions (global)
  uint32_t f_nstates;
  uint32_t f_nclasses;
  uint32_t f_s_bot;
  uint32_t f_classmap;
  uint32_t f_classmap_up;
  uint32_t f_trans;    // blob offset: u16[f_nstates * f_nclasses]
  uint32_t f_accept;   // blob offset: u8[f_nstates]
  uint32_t unicode_word;
  // f_marked: the full DFA expects a marker byte before every code point
  // (0xFC word / 0xFD other / 0xFE \n: Unicode word boundaries); wtab: blob
  // offset of the Unicode \w ranges (u32 lo, hi pairs), wtab_n of them
  uint32_t f_marked;
  uint32_t wtab;
  uint32_t wtab_n;
  // register-resident form for the lean kernel (ASCII DFA with <= 16 states):
  // tt[b] = the row of byte b, next state of s in bits [4s, 4s+4); acc1/acc2 =
  // states with accept bit0 / bit1
  uint32_t lean;       // 1: tt / tt_up / acc1 / acc2 are valid
  uint32_t tt;         // blob offset: u64[256]
  uint32_t tt_up;      // blob offset: u64[256], rows of toupper(byte)
  uint32_t acc1;
  uint32_t acc2;
  // version-uncertain code points (fsg_unicode.h fsg_u_newer): blob offset of
  // (lo, hi) u32 pairs, vtab_n of them; 0 when the pattern uses no
  // version-dependent table (a value holding one is then FSG_E_UNSUPPORTED)
  uint32_t vtab;
  uint32_t vtab_n;
};

struct StageDesc {
  uint8_t op;
  uint8_t kind;        // SmartModuleKind tag (FSG_KIND_*)
  uint8_t in_type;     // ValType
  uint8_t keep_match;  // OP_REGEX: 1 keep matching, 0 keep non-matching; OP_LB_MAX / OP_DEDUP: 1 = look_back mode
  uint32_t needle;     // blob offset (OP_CONTAINS)
  uint32_t needle_len;
  uint32_t acc_bad;    // OP_AGG_SUM: initial accumulator is invalid UTF-8
  uint32_t acc_vut;    //   its Utf8Error valid_up_to
  uint32_t acc_elen;   //   its Utf8Error error_len
  DfaDesc dfa;
};

// ChainDesc::flags: what the last stage is
enum ChainFlags : uint32_t { CF_AGG_SUM = 1u, CF_AGG_CAT = 2u, CF_ARRAY = 4u, CF_AGG_JSON = 8u, CF_STATEFUL = 16u };
struct ChainDesc {
  uint32_t nstages;
  uint32_t out_type;   // ValType of the value after the last stage
  uint32_t has_agg;
  uint32_t flags;      // ChainFlags
  StageDesc st[kMaxStages];
};

// per-batch result of k_eval
enum BatchFlags : uint32_t {
  BF_ERR = 1u,         // a record-level SmartModule error (SmartModuleTransformRuntimeError)
  BF_DECODE = 2u,      // Vec<Record> decode failed -> the process() call returns Err
  BF_UNSUPPORTED = 4u, // input needs a feature the GPU path does not implement
  BF_LAST_STAGE = 8u,  // the error (if any) happened in the last stage -> records_out counted
  BF_ARR_LEAN = 16u,   // array_map batch of k_arr_lean: sized from ArrBatch, written by k_arr_write
  BF_ROWDONE = 64u,    // the flat decide wrote the batch's ScanRow for first_keep = 0 (k_size skips it then)
  BF_COMPACT = 32u,    // the batch's descriptors are 16-byte KeptC (k_eval_int's aggregate-sum batches)
};

// varint size with the encoder quirk (varint.rs:68-80)
__device__ __forceinline__ uint32_t vsize(int64_t num) {
  int64_t v = (int64_t)(((uint64_t)num << 1) ^ (uint64_t)(num >> 31));
  uint32_t n = 1;
  while (v & (int64_t)0xffffff80) {
    n++;
    v >>= 7;
  }
  return n;
}
// variant_encode (varint.rs:43-66); returns bytes written
__device__ __forceinline__ uint32_t venc(int64_t num, uint8_t* out) {
  int64_t v = (int64_t)(((uint64_t)num << 1) ^ (uint64_t)(num >> 31));
  uint32_t k = 0;
  while (v & (int64_t)0xffffff80) {
    out[k++] = (uint8_t)((v & 0x7f) | 0x80);
    v >>= 7;
  }
  out[k++] = (uint8_t)v;
  return k;
}

// k_arr_lean's per-batch element statistics (array_map, fsg_array.hip).  An
// element's output record is 5 + vsize(rel) + L + [L >= 60 - vsize(rel)]
// bytes, L = vsize(len) + len, so the batch's bytes follow from these counts
// once k_size knows the offset rebase `rel`.
struct ArrBatch {
  uint32_t ne;         // elements
  uint32_t esum;       // Σ L
  uint32_t c59;        // elements with L >= 59
  uint32_t cnt[9];     // elements with L = 50 .. 58
};
// per lean array batch, two bitmaps over its window offsets: element starts,
// then element ends (exclusive); the k-th start pairs with the k-th end
constexpr uint32_t kArrBmWords = kWin / 32;                // u32 words per bitmap
constexpr uint32_t kArrBmBatch = 2 * kArrBmWords;          // per batch

struct BatchStat {
  int64_t base_offset;
  int64_t first_ts;
  int32_t lod_in;      // header.last_offset_delta
  uint32_t flags;
  uint32_t nkeep;      // records in the stage output (before the error record)
  uint32_t sec_len;    // record-section length = bytes_in of this process() call
  uint32_t err_stage;
  uint32_t err_code;
  uint64_t err_pos;    // absolute slice offset of the failing record
  int64_t err_od;      // its offset_delta
  int32_t err_ival;    // VT_I32 value entering the failing stage
  uint32_t err_aux;
  uint32_t err_aux2;
  uint32_t err_aux3;
  int64_t agg_sum;     // wrapping i32 sum of the aggregate inputs of this batch
  uint32_t nout;       // output records of the stage output (array_map: elements; else nkeep)
  uint32_t pad;
  uint64_t cat_sum;    // aggregate (concat): bytes appended to the accumulator by this batch
  uint64_t err_vpos;   // the failing record's value as it entered the failing stage (byte views:
  uint32_t err_vlen;   //   a projection narrows the view)
  uint32_t comp;       // header attributes & 7 (the output batch takes the first surviving batch's)
};

// one kept output record (a compaction descriptor, 64 bytes): enough to
// re-encode the record canonically without re-parsing the source
enum KeepMode : uint8_t { KM_COPY = 0, KM_UPPER = 1, KM_I32 = 2, KM_AGG = 3, KM_ARRAY = 4, KM_CONCAT = 5,
                         KM_AGGJ = 6 };  // KM_AGGJ: value = cat[vpos, vpos + vlen) (k_aggj's map text)
// KeptRec::pad bits for KM_ARRAY / KM_CONCAT
enum KeepFlags : uint8_t { KF_UPPER = 1, KF_I32 = 2,
                           KF_ESUM = 4 };  // KM_ARRAY from k_arr_lean: ts = Σ (varint + text) bytes of the
                                           // elements, hdr = elements of >= 40 bytes (fsg_array.hip)
struct KeptRec {
  uint64_t src;        // absolute slice offset of the source record (its length varint)
  uint64_t vpos;       // absolute slice offset of the source value bytes
  uint64_t kpos;       // absolute slice offset of the key bytes
  int64_t od;          // source offset_delta
  int64_t ts;          // timestamp_delta
  int64_t hdr;         // headers varint
  uint32_t vlen;       // source value length (KM_COPY / KM_UPPER / KM_CONCAT), i32 bits with KF_I32
  uint32_t klen;
  int32_t ival;        // KM_I32 value / KM_AGG batch-local inclusive sum / KM_ARRAY element count /
                       // KM_CONCAT batch-local inclusive byte count
  uint8_t mode;        // KeepMode
  uint8_t has_key;
  uint8_t attr;
  uint8_t pad;         // KeepFlags
};
static_assert(sizeof(KeptRec) == 64, "KeptRec is one 64-byte line");
// output size of a verbatim kept record (KM_COPY / KM_UPPER) after the offset
// fix-up: k_size's rec_out_size for those modes (the flat decides' rows)
__device__ __forceinline__ uint32_t copy_out_size(const KeptRec& d, int64_t rel) {
  const uint32_t inner = 1 + vsize(d.ts) + vsize(d.od + rel) + 1 +
                         (d.has_key ? vsize((int64_t)d.klen) + d.klen : 0) + vsize((int64_t)d.vlen) + d.vlen +
                         vsize(d.hdr);
  return vsize((int64_t)inner) + inner;
}
// the compact descriptor of a generated-integer record without key or headers
// and with 32-bit deltas (k_eval_int's aggregate-sum batches, BF_COMPACT): a
// quarter of the KeptRec traffic its eval, size and write passes move; the
// batch's KeptC array starts where its KeptRec array would
struct KeptC {
  int32_t od;
  int32_t ts;
  int32_t ival;
  uint8_t mode;
  uint8_t attr;
  uint16_t pad;
};
static_assert(sizeof(KeptC) == 16, "KeptC is 16 bytes");
__device__ __forceinline__ KeptRec kept_at(const KeptRec* d, uint32_t k, bool compact) {
  if (!compact) return d[k];
  const KeptC c = ((const KeptC*)d)[k];
  KeptRec r = {};
  r.od = c.od;
  r.ts = c.ts;
  r.ival = c.ival;
  r.mode = c.mode;
  r.attr = c.attr;
  return r;
}

// one array_map output element: the source span of a JSON array element and
// the length of its serde_json::to_string form.  The elements of a record with
// value at slice offset v live at elem[(v >> 1) + j] (an element needs >= 2
// value bytes with its separator, so records never overlap).
struct ElemRec {
  uint64_t pos;        // absolute slice offset of the element's first byte
  uint32_t src_len;    // source span (whitespace inside included)
  uint32_t out_len;    // canonical length; bit 31 = canonical bytes == source bytes
};
static_assert(sizeof(ElemRec) == 16, "ElemRec is 16 bytes");

// per-batch row of the cross-batch scan (in place: exclusive prefix afterwards)
struct ScanRow {
  uint64_t rec_bytes;  // Σ output record sizes of this batch (after offset fix-up)
  uint64_t nonempty;   // 1 if the batch contributes records
  uint64_t lod;        // input last_offset_delta + 1 for batches >= first surviving batch
  uint64_t nrec;       // records contributed
  uint64_t bytes_in;   // record-section bytes (metrics.bytes_in)
  uint64_t recs_out;   // last-stage output records (metrics.records_out)
  int64_t agg;         // aggregate sum (wrapping i32 in the low bits)
  uint64_t cat;        // aggregate (concat): accumulator bytes appended
};

// cross-batch minima found with atomics (reset to 0xFFFFFFFF per call)
struct Mins {
  uint32_t first_keep;
  uint32_t first_err;
  uint32_t first_dec;
  uint32_t first_unsup;
  uint32_t cut;
  // a continuation (fsg_chain_process_batch's pipelined chunks): the output
  // batch was started by an earlier chunk, so every batch of this one counts
  // from its first (first_keep = 0) and records rebase to carry_base; carry =
  // that batch's compression bits, 0xFFFFFFFF (the 0xFF fill) = none
  uint32_t carry;
  int64_t carry_base;
};

struct Plan {
  int32_t status;      // 0, FSG_E_DECODING_BASE_INPUT, FSG_E_IO, FSG_E_UNSUPPORTED
  int32_t err_batch;   // batch whose error is returned, -1 none
  int32_t first;       // first surviving batch, -1 none
  int32_t last;        // last batch whose records are included
  int32_t stop;        // last processed batch (-1 none)
  int32_t lod;
  int64_t base_offset;
  uint64_t n_records;
  uint64_t rec_bytes;
  uint64_t bytes_in;
  uint64_t invocations;
  uint64_t records_out;
  int64_t agg_prefix_first;  // aggregate prefix (exclusive) at `first` — unused unless has_agg
  int64_t acc_final;         // aggregate accumulator after the stop batch
  int32_t acc_touched;       // accumulator changed by this call
  int32_t done;              // last batch whose process() call completed (-1 none): state commits through it
  int32_t comp;              // compression bits of the first surviving batch (set_compression, batch.rs:144-153)
  int32_t nonempty;          // batches of [first, last] with records (each adds 4 to records.write_size)
  uint64_t cat_final;        // aggregate (concat): accumulator bytes appended through the stop batch
};

struct EvalArgs {
  const uint8_t* slice;
  uint64_t slice_len;
  const uint64_t* bpos;
  const uint64_t* rbase;
  uint32_t nbatches;
  uint32_t flat_st;    // EVAL_FLAT: the substring stage of the flat path | its needle length << 8
  int32_t chain_host_max_len;  // EVAL_RX: the regex stage's max_len (host copy for the launch)
  const ChainDesc* chain;
  const uint8_t* blob;
  BatchStat* bstat;
  KeptRec* desc;
  Mins* mins;
  uint32_t* list;      // deferred batches: list[0] = count, list[1..] = indices (k_eval_lean -> k_eval)
  ElemRec* elem;       // array_map element descriptors (nullptr without an array_map stage)
  uint64_t nrec;       // records of the slice (rbase's total)
  uint16_t* rstart;    // k_chase: record n of batch b starts at window offset rstart[rbase[b] + n] ...
  uint16_t* rend;      // ... and the last one ends at rend[b] (0xFFFF: no lean framing, exact path)
  const uint8_t* pass; // per batch, 1: the records pass through unchanged (no stage runs on them:
                       // an earlier segment's partial output before its error), nullptr: none
  ArrBatch* arr_b;     // array_map lean path: per batch element statistics ...
  uint32_t* arr_bm;    // ... and element bitmaps (kArrBmBatch words per batch)
  unsigned long long* fbm;  // flat substring path (fsg_lean.hip): a bit per 16-byte chunk of the slice,
                            // per 1 KiB round the occurrence-start word then the bytes >= 0x80 word
  uint64_t fbm_words;
  struct ScanRow* rows;     // the flat decides' rows for a first surviving batch 0 (BF_ROWDONE), nullptr: none
};

struct SizeArgs {
  const BatchStat* bstat;
  const KeptRec* desc;
  const uint64_t* rbase;
  const Mins* mins;
  const ScanRow* agg_pre;  // exclusive aggregate prefix (nullptr if no aggregate)
  ScanRow* rows;
  uint32_t nbatches;
  uint32_t agg_only;       // 1: only fill rows[].agg (first pass of an aggregate chain)
  int64_t acc0;
  const ElemRec* elem;
  uint64_t acc_len;        // aggregate (concat): initial accumulator bytes
  uint32_t seg;            // 1: segment output (no offset rebase: rel = 0)
  const ArrBatch* arr_b;   // BF_ARR_LEAN batches: element statistics
};

struct PlanArgs {
  const BatchStat* bstat;
  const ScanRow* rows;
  const ScanRow* pre;
  const Mins* mins;
  Plan* plan;
  uint32_t nbatches;
  int32_t tail_status;  // framing status of the batch after the last framed one (0 = clean end)
  int32_t empty_chain;
  int32_t has_agg;
  int32_t seg;  // a segment of a composed chain: `done` locates the failure for the next segment
  int64_t acc0;
};

struct WriteArgs {
  const uint8_t* slice;
  const BatchStat* bstat;
  const KeptRec* desc;
  const uint64_t* rbase;
  const ScanRow* pre;
  const ScanRow* agg_pre;
  const Plan* plan;
  uint8_t* out;
  int64_t acc0;
  const ElemRec* elem;
  const uint8_t* cat;      // aggregate (concat): kCatOff + accumulator stream
  uint64_t acc_len;
  uint32_t seg;            // 1: segment output: batch b's records at 61 * (b + 1) + pre[b], rel = 0
  int32_t first, last;     // plan.first / plan.last as the host read them (k_write_lean: no plan load
                           // ahead of the batch rows)
  int64_t base;            // plan.base_offset as the host read it: records rebase to it (batch.rs:95-100)
};
// k_arr_write: the output records of the BF_ARR_LEAN batches of [plan.first,
// plan.last], re-walked from the source window (fsg_array.hip)
struct ArrWriteArgs {
  const uint8_t* slice;
  const uint64_t* bpos;
  const uint64_t* rbase;
  uint32_t nbatches;
  uint32_t seg;            // WriteArgs::seg
  uint64_t nrec;
  const BatchStat* bstat;
  const uint32_t* arr_bm;
  const ScanRow* pre;
  const Plan* plan;
  uint8_t* out;
};
// k_one: the whole process() of a one-batch input in one workgroup (the
// producer's one-record path, f3): eval, minima, size, plan, header, write,
// CRC32C.  Stateless chains only; an output past out_cap is left to the
// host (the plan says how big it is).
struct OneArgs {
  EvalArgs ea;       // nbatches = 1; ea.bstat / ea.mins point into the read-back block
  ScanRow* rows;     // [1]
  ScanRow* pre;      // [1]
  Plan* plan;        // the read-back block: Plan at +0, BatchStat at +192, Mins at +384 ...
  uint8_t* out;      // ... the output batch at +kOneHead (out_cap bytes)
  uint64_t out_cap;
  const uint8_t* hin;  // the input batch in pinned host memory (copied into ea.slice first), in_len bytes
  uint8_t* hout;       // pinned host memory: the read-back block is copied here last
  uint32_t in_len;     // the device slice's allocation (zeros behind the input)
  uint32_t in_real;    // input bytes to read from hin (a multiple of 16)
  int32_t empty_chain;
  uint32_t seq;        // written to *hflag (pinned) once the read-back block is in host memory
  uint32_t* hflag;     // the host polls it instead of the stream
};
constexpr uint32_t kOneHead = 512;  // Plan | BatchStat | Mins, then the output batch
// a chain segment's output as the next segment's input slice (k_seg_headers):
// batch b in [0, nb) = the source batch's 57-byte header (base offset, last
// offset delta, timestamps, attributes) with batch_len / the record count of
// the records the segment produced for it, at 61 * b + pre[b].rec_bytes
struct SegArgs {
  const uint8_t* src;      // the segment's input slice
  const uint64_t* bpos;    // its batch positions
  const ScanRow* rows;     // per batch: rec_bytes / nrec of the segment's output
  const ScanRow* pre;      // ... exclusive prefix
  uint32_t nb;             // batches of the output slice
  int32_t pass_batch;      // this segment's error batch (passes through the next segments), -1 none
  const uint8_t* pass_in;  // the input slice's pass-through flags (nullptr: none)
  uint8_t* dst;            // the output slice
  uint64_t* dbpos;         // its batch positions ...
  uint64_t* drbase;        // ... record-count prefix ...
  uint8_t* dpass;          // ... and pass-through flags
};
constexpr uint64_t kCatOff = 64;  // the concat stream starts this far into its buffer (copy_seg margin)

// aggregate-json (k_aggj_*): the folded records in stream order (records of
// batches up to the first error batch), their entries, the key dictionary
// (ids by first occurrence) with an open-addressing index in HBM, and the
// per-block state table (the map's values at every block's first record).
// Keys point at their bytes: the slice for keys met in records, the uploaded
// initial accumulator otherwise.
struct AggjArgs {
  const uint8_t* slice;
  const BatchStat* bstat;
  KeptRec* desc;
  const uint64_t* rbase;
  const ElemRec* elem;
  const Mins* mins;
  uint32_t nbatches;
  uint32_t write;          // text pass: 0 sizes, 1 writes the map text into cat
  uint8_t* cat;            // text buffer (kCatOff margin)
  // per batch
  uint32_t* bcnt;          // folded records of batch b
  uint64_t* brec;          // ... exclusive prefix (stream index of its first record)
  // per folded record
  uint64_t n_rec;
  uint64_t* rdesc;         // KeptRec index
  uint32_t* rne;           // entries (json_map_u32 pairs) of the record
  uint64_t* rent;          // ... exclusive prefix (entry index of its first pair)
  uint32_t* rnew;          // keys the record inserts into the map
  uint64_t* rnewb;         // ... exclusive prefix
  uint32_t* rlen;          // map text bytes after the record
  uint64_t* roff;          // ... exclusive prefix (offset in cat after kCatOff)
  // per entry: key id (kSkipEntry for a key the same record names again
  // earlier) and the value the record contributes (the key's last value in it)
  uint32_t* ekid;
  uint32_t* eval;
  // dictionary
  unsigned long long* slot_ref;  // 0 empty; else the key's first occurrence: init key k -> k + 1,
                                 // record r entry j -> (r + 1) << 32 | j
  uint32_t* slot_id;
  uint32_t cap;            // slots (power of two)
  uint32_t n_init;         // keys of the initial accumulator (ids 0 .. n_init - 1)
  const uint64_t* kptr;    // initial keys: match bytes
  const uint32_t* klen;
  const uint32_t* val_init;
  uint64_t* tptr;          // per key id: text as serialized ("..." with escapes)
  uint32_t* tlen;
  uint32_t* kup;           // 1: read through the ASCII-uppercase view
  uint32_t nkeys;          // K: keys after the call (host-known once the ids exist)
  // blocks of `rb` consecutive records: state[b * K + k] = key k's value
  // before block b's first record
  uint32_t rb;
  uint32_t nblk;
  uint32_t* state;
  unsigned long long* scal;  // [0] entries [1] records [2] new keys [3] text bytes [4] [5] scan totals
                             // [6] Σ keys over the records' maps (ord slots) [7] most entries of a record
  uint64_t* acc_off;       // per batch: the accumulator text after it (offset in cat) ...
  uint32_t* acc_len;       // ... and its length (0xFFFFFFFF: no record aggregated yet)
  // the output key order (fsg_keyed.hip k_aggj_hash / k_aggj_order): record
  // i's map is the guest's HashMap<String, u32> built from record i - 1's
  // output text under RandomState k0 = k0_base + 2 i, plus the record's own
  // map (k0 + 1) added in that map's bucket order; its text lists the keys in
  // bucket order
  uint32_t* nkr;           // per folded record: keys in the map after it
  uint64_t* koff;          // ... exclusive prefix: the record's slots in `ord`
  uint32_t* ord;           // per record, by key id: hash under its accumulator map's keys; then, by
                           //   position: the key ids in output order (k_aggj_order writes in place)
  uint32_t* hrec;          // per entry: its key's hash under the record map's keys
  uint64_t k0_base;        // RandomState k0 of the first folded record's accumulator map
  const uint32_t* iseq;    // record 0's accumulator keys in text order, kAjDup on a repeated key;
  uint32_t n_iseq;         //   nullptr: the ids 0 .. n_init - 1
  uint32_t agg_stage;      // the aggregate's stage index in this chain (its error draws a RandomState)
  uint32_t in_i32;         // the stage reads an i32 view (never '{')
  uint32_t* oscr;          // k_aggj_order: tables of maps past the register path (4 x obmax buckets)
  uint32_t obmax;          // ... buckets per table (a power of two), 0: none
};
constexpr uint32_t kAjRegKeys = 55;  // k_aggj_order's register path: <= 55 keys / entries keep a map
                                     // within 64 buckets (capacity 56: no reserve grows past it)
constexpr uint32_t kAjDup = 0x80000000u;  // AggjArgs::iseq: the key appeared earlier in the text
constexpr uint32_t kAjLdsBuckets = 2048;  // the general path's tables in LDS up to this many buckets
// device framing of a stored slice (FileBatchIterator, iterators.rs:55-160):
// every position whose magic byte (offset 16) is 2 is a candidate batch start;
// each candidate's successor (pos + 57 + batch_len - 45) is found among the
// candidates, pointer doubling marks the chain from position 0.  A chain that
// reaches a non-candidate (a batch without magic 2) goes back to the host walk.
constexpr uint32_t kFrameChunk = 65536;  // bytes per candidate-collection workgroup
constexpr uint32_t kFrameCap = 1024;     // candidates per chunk (more: host walk)
// FN_END: the slice ends after this batch; FN_TAIL: a batch, then fewer than 57 bytes
// (IO tail); FN_IO / FN_UNSUP: no batch here, the walk stops with that status
enum FrameNext : uint32_t { FN_END = 0xFFFFFFF0u, FN_TAIL, FN_IO, FN_UNSUP, FN_NONCAND };
struct FrameArgs {
  const uint8_t* s;
  uint64_t len;
  uint16_t* cbuf;        // per chunk: candidate offsets in the chunk
  uint32_t* ccnt;        // per chunk: candidates
  uint64_t* coff;        // ... exclusive prefix
  uint64_t* cand;        // candidate positions, ascending
  uint64_t ncand;
  uint32_t* jmp;         // levels x ncand: successor after 2^level batches (sink = ncand)
  uint32_t* term;        // per candidate: FrameNext when the walk ends there, else its successor
  uint32_t* mark;        // per candidate: on the chain from position 0
  uint64_t* mpre;        // ... exclusive prefix (batch index)
  uint32_t* nrec;        // per candidate: record count as framed
  uint64_t* rpre;        // ... exclusive prefix (rbase)
  uint64_t* bpos;        // out: batch positions
  uint64_t* rbase;       // out
  unsigned long long* scal;  // [0] overflow / fallback, [1] tail status, [2] header bytes, [3..] scan totals
};
// stateful last stages (k_sf_*): filter_look_back (running max, PREV) and
// filter_hashset (BoundedHashSet<String>: FIFO of distinct values, `limit`).
// The stage runs on the records that reach it in batches b that
// process_batch evaluates up to the stage (sf_ran); decisions in stream order,
// descriptors compacted in place, state committed through plan.done.
// Dedup state: entries (hash, arena bytes, last new-insertion index) persist
// across calls; an open-addressing table over entries + this call's records is
// rebuilt per call.  A value is in the set iff its last new-insertion index is
// among the newest `limit` (the set holds the newest `limit` insertions).
constexpr unsigned long long kSfEnt = 1ull << 63;  // table ref: entry id (else record index + 1)
constexpr uint64_t kSfNone = ~0ull;
struct SfArgs {
  const uint8_t* slice;
  BatchStat* bstat;
  KeptRec* desc;
  const uint64_t* rbase;
  const Mins* mins;
  const Plan* plan;
  uint32_t nbatches;
  uint32_t op;             // OP_LB_MAX / OP_DEDUP
  uint32_t lookback;       // 1: look_back mode (no decisions, no compaction)
  uint32_t fast;           // dedup: 1 = no eviction during this call (parallel decisions)
  int64_t* bval;           // per batch: LB max of the values / dedup kept count
  int64_t* bpre;           // ... exclusive prefix (LB: max with PREV, dedup: sum)
  int32_t* prev;           // LB: PREV in HBM
  // dedup
  uint32_t* bn;            // per batch: records reaching the stage (0 where it did not run)
  uint64_t* hv;            // per record (rbase index): value hash
  uint64_t* vref;          // per record: value offset in the slice | kSfEnt for the uppercase view
  uint32_t* vlen;          // per record: value length
  uint32_t* slot;          // per record: table slot
  uint8_t* keep;           // per record: decision
  uint64_t* idx;           // per record: new-insertion index when kept
  unsigned long long* sref;  // table: 0 empty, kSfEnt | entry, record index + 1
  uint32_t* first;         // per slot: first record of this call
  uint64_t* cur;           // per slot: last new-insertion index + 1 during the sequential walk
  uint32_t cap;
  uint64_t* ent_hash;
  uint64_t* ent_pos;       // arena offset
  uint32_t* ent_len;
  uint64_t* ent_last;      // last new-insertion index + 1 (0: none)
  uint8_t* arena;
  uint64_t n_ent;          // entries at call start
  uint64_t n0;             // new insertions before this call
  uint64_t limit;
  unsigned long long* scal;  // [0] entries after commit [1] arena bytes [2] N after commit [3] keeps
};
// record-section decompression at ingest (fsg_codec_dev.h, k_dec_*)
struct DecArgs {
  const uint8_t* src;     // the slice as stored
  const uint64_t* bpos;   // its batches
  const uint8_t* codec;   // attributes & 7 per batch (0, 1 gzip, 2 snappy, 3 lz4)
  uint32_t nb;
  int64_t* dsize;         // decompressed section length / DEC_BAD / DEC_UNSUP
  uint8_t* dst;           // the decompressed slice
  const uint64_t* npos;   // batch positions in dst
  int32_t* status;        // writing pass: 0 ok, -1 decode / checksum error
  uint64_t* cnt;          // record count estimate of each new section
};
constexpr uint32_t kSkipEntry = 0xFFFFFFFFu;
constexpr uint32_t kAjLds = 4096;  // k_aggj_text keeps up to this many values in LDS

// aggregate-json state kept in HBM between calls (fsg_keyed.hip k_ajc_*): after
// a call, the map as it stands after the last record folded through the stop
// batch (process_batch's last processed batch) is rewritten into the chain's
// other state buffer: per key, in the order the last record's text lists them, its match bytes and its
// serialized text in one arena, and its u32 value.  The next call reads it as
// its initial keys, so no accumulator text crosses PCIe and nothing is parsed
// on the host after the first call.
struct AjState {
  uint8_t* arena;        // per key: match bytes, then text bytes
  uint64_t* kptr;        // match bytes (device address)
  uint32_t* klen;
  uint64_t* tptr;        // serialized text ("..." with escapes)
  uint32_t* tlen;
  uint32_t* val;
  uint32_t* blen;        // scratch: match + text bytes per key
  uint64_t* boff;        // ... exclusive prefix
};
struct AjCommitArgs {
  AggjArgs a;            // this call's dictionary, records, entries
  int32_t stop;          // the last processed batch (plan.stop, >= 0)
  uint32_t kmax;         // key ids of this call (n_init + new keys): the grid bound
  AjState dst;           // keys in the output order of the last folded record (= its text's order)
  uint32_t* inv;         // scratch: key id -> position in dst
  unsigned long long* out;  // [0] keys after the stop batch [1] records folded through it [2] arena bytes
                            // [3] the stop batch ends at an aggregate error [4] ... whose value starts with '{'
};

// Topic-wide keyed totals (fsg_keyed_*, C5 keyed): a rank-local table of exact
// keys (bytes in an arena, open addressing over key indices), values summed
// u32-wrapping from the chains' aggregate-json states; the merge across ranks
// all-gathers the key lists, builds the union dictionary (ids by first
// occurrence in rank order: identical on every rank) and all-reduces a dense
// K-slot u32 table.
struct KdTable {
  uint8_t* arena;
  uint64_t* koff;        // key i: arena offset ...
  uint32_t* klen;        // ... and length (kKdDead: a lost duplicate)
  uint32_t* val;
  uint32_t* slot;        // slot -> key index + 1 (0 empty)
  uint32_t cap;          // slots (power of two)
  unsigned long long* cnt;  // [0] keys [1] arena bytes
};
constexpr uint32_t kKdDead = 0xFFFFFFFFu;
// gathered key descriptors (k_kd_desc): arena offset | length << 40; this
// length marks an entry with no key (a lost duplicate, or padding to maxn)
constexpr uint64_t kKdLenDead = 0xFFFFFFull;
constexpr uint64_t kKdLenDeadDesc = kKdLenDead << 40;
struct KdUnionArgs {
  const uint64_t* gdesc;   // all-gathered descriptors: rank r's key i at r * maxn + i
  const uint8_t* garena;   // all-gathered arenas: rank r's at r * maxb
  uint64_t maxb;
  uint32_t maxn, nitems;   // nitems = nranks * maxn
  uint32_t me;             // this rank
  const uint32_t* lval;    // this rank's local values (by local key index)
  uint32_t* slot;          // union table
  uint32_t cap;
  uint32_t* gslot;         // per item: its slot
  uint32_t* first;         // per item: 1 at a key's first occurrence
  uint64_t* idpre;         // ... exclusive prefix = the union id
  uint32_t* gid;           // per item: union id
  uint32_t* ulen;          // per union id: key bytes
  uint64_t* uoff;          // ... exclusive prefix
  uint8_t* uarena;         // union keys, id order
  uint32_t* dense;         // K-slot u32 table (this rank's values; summed by the all-reduce)
  uint64_t* tsum;          // scan scratch
  unsigned long long* tot; // [0] K [1] union arena bytes
};


}  // namespace fsg
