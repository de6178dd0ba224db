// fsg_launch.h — host-side launch wrappers of the kernels in fsg_kernels.hip
#pragma once
#include <hip/hip_runtime.h>

#include "fsg_device.h"

namespace fsg {
hipError_t upload_crc_tables();
// ops: bit per StageOp in the chain.  mode: EVAL_EXACT = k_eval over every
// batch; EVAL_LEAN = k_chase + k_eval_lean, then k_eval over its deferred list;
// EVAL_ARRAY = k_arr_frame + k_arr_lean (fsg_array.hip), then k_eval over its deferred list
// EVAL_FLAT = k_chase + k_flat_scan + k_flat_decide (a.flat_st, a.fbm), then k_eval over the deferred list
// EVAL_INT = k_eval_int over every batch (record starts in a.rstart / a.rend from k_chase_w), then k_eval over
// its deferred list
// EVAL_FJSON = k_flat_scan<., kJson> + k_fj_decide (a.flat_st = fjson_flags, a.fbm), then k_eval over the deferred list
// EVAL_RX = k_rx_scan + k_rx_decide (a.flat_st = the regex stage, a.fbm), then k_eval over the deferred list
enum EvalMode { EVAL_EXACT = 0, EVAL_LEAN = 1, EVAL_ARRAY = 3, EVAL_FLAT = 4, EVAL_INT = 5, EVAL_FJSON = 6, EVAL_RX = 7 };
void launch_eval(const EvalArgs& a, uint32_t ops, int mode, hipStream_t s);
// k_chase + k_eval_lean (fsg_lean.hip), the kernel variant picked by the chain's stage ops
void launch_eval_lean(const EvalArgs& a, uint32_t ops, hipStream_t s);
// the flat substring path (fsg_lean.hip): the chain's one substring stage (needle 4..128 bytes, with
// only uppercase maps beside it) or -1; k_chase + k_flat_scan + k_flat_decide over a.fbm
int flat_stage(const ChainDesc& ch, uint32_t ops);
void launch_eval_flat(const EvalArgs& a, uint32_t flat_st, hipStream_t s);
// the flat JSON path (fsg_lean.hip): filter_json / a field projection with at most one substring stage
// (needle 4..128 bytes) and uppercase maps beside them; its launch flags for a.flat_st, or -1
int fjson_flags(const ChainDesc& ch, uint32_t ops);
void launch_eval_fjson(const EvalArgs& a, hipStream_t s);
// the flat regex path (fsg_lean.hip): one bounded regex stage (ASCII DFA <= 16 states, max_len <= 17) and
// uppercase maps; the stage or -1
int rx_flat_stage(const ChainDesc& ch, uint32_t ops);
void launch_eval_rx(const EvalArgs& a, uint32_t stage, hipStream_t s);
// integer-stage chains (filter_odd, map_double, filter_map, a final aggregate-sum) over decimal values (fsg_lean.hip)
bool int_lean_eligible(const ChainDesc& ch, uint32_t ops);
void launch_eval_int(const EvalArgs& a, bool agg, hipStream_t s);
// array_map_json_array alone over the source values (fsg_array.hip)
bool array_lean_eligible(const ChainDesc& ch, uint32_t ops);
void launch_array_lean(const EvalArgs& a, hipStream_t s);
// the output records of its BF_ARR_LEAN batches among the nblk of the plan
void launch_array_write(const ArrWriteArgs& a, uint32_t nblk, hipStream_t s);
// record starts / ends of every batch (k_chase_w)
void launch_chase_w(const EvalArgs& a, hipStream_t s);
void launch_mins(const BatchStat* bstat, uint32_t n, Mins* mins, hipStream_t s);
// ---------------------------------------------------------------------------
// The aggregate-sum group path (fsg_chain_group_process_slices): one launch
// per phase over every chain of the group instead of ~13 launches and two
// host waits per chain.  GaJob = one chain's arguments; the grid offsets of
// the per-batch phases (job j owns the virtual blocks [off[j], off[j + 1]))
// live beside the jobs in device memory.
struct GaJob {
  EvalArgs ea;        // k_eval_int<1> over the batches (record starts kept with the slice)
  SizeArgs sa;        // k_size, agg_only set by the phase
  ScanRow* aggpre;    // exclusive aggregate prefix (first scan)
  ScanRow* pre;       // exclusive output prefix + max_bytes cut (second scan)
  uint64_t max_bytes;
  PlanArgs pa;
  int32_t* state;     // the accumulator in HBM (k_state)
  uint32_t* crc_acc;
  WriteArgs wa;       // phase 2: k_header, k_write_gen over [wa.first, wa.last]
  uint64_t out_len;
};
struct GaResult {     // per job, read back after phase 1
  Plan plan;
  uint32_t deferred;  // batches k_eval_int left to the exact kernel (the chain is re-run on the general path)
  uint32_t pad[3];
};
struct GaOffsets {    // device pointers to the n + 1 grid offsets per phase, and the totals
  const uint32_t *eval, *mins, *size, *write, *crc;
  uint32_t t_eval, t_mins, t_size, t_write, t_crc;
};
uint32_t ga_mins_blocks(uint32_t nb);
uint32_t ga_crc_blocks(uint64_t out_len);
void launch_ga_phase1(const GaJob* jobs, uint32_t n, const GaOffsets& o, GaResult* res, hipStream_t s);
void launch_ga_phase2(const GaJob* jobs, uint32_t n, const GaOffsets& o, hipStream_t s);
void launch_ga_eval_int(const GaJob* jobs, uint32_t n, const uint32_t* off, uint32_t total, hipStream_t s);
void launch_size(const SizeArgs& a, hipStream_t s);
uint32_t scan_tiles(uint32_t n);
void launch_scan(const ScanRow* rows, ScanRow* pre, ScanRow* tile_sums, ScanRow* grand, uint32_t n, bool cut,
                 uint64_t max_bytes, Mins* mins, const BatchStat* bstat, hipStream_t s);
void launch_plan(const PlanArgs& a, hipStream_t s);
void launch_state(const Plan* plan, int32_t* state, hipStream_t s);
void launch_header(const Plan* plan, uint8_t* out, hipStream_t s);
// a chain segment's output as the next segment's input slice (SegArgs)
void launch_seg_headers(const SegArgs& a, hipStream_t s);
void launch_write(const WriteArgs& a, uint32_t nblocks, hipStream_t s);
// array elements whose canonical text differs from their source (json_canon):
// lengths before k_size, payloads after k_write, in the batches k_eval flagged
void launch_canon_len(const SizeArgs& a, const uint8_t* slice, hipStream_t s);
void launch_write_canon(const WriteArgs& a, uint32_t nblk, hipStream_t s);
void launch_cat(const WriteArgs& a, uint32_t nbatches, hipStream_t s);
void launch_crc(uint8_t* out, uint64_t off, uint64_t n, uint32_t* acc, hipStream_t s);
// process() of a one-batch input in one launch (k_one)
void launch_one(const OneArgs& o, uint32_t ops, hipStream_t s);
void launch_write_lean(const WriteArgs& a, uint32_t nblocks, hipStream_t s);
// generated integer values (KM_I32 / KM_AGG) staged per batch in LDS (other batches: the wave path)
void launch_write_gen(const WriteArgs& a, uint32_t nblocks, hipStream_t s);
// aggregate-json, in phases separated by host reads of AggjArgs::scal
uint64_t xscan_tiles(uint64_t n);  // u64 scratch slots launch_xscan needs for n items
void launch_aggj_count(const AggjArgs& a, hipStream_t s);
void launch_aggj_keys(const AggjArgs& a, uint64_t* tsum, hipStream_t s);
void launch_aggj_kid(const AggjArgs& a, uint64_t n_ent, hipStream_t s);
void launch_aggj_rows(const AggjArgs& a, hipStream_t s);
void launch_aggj_size(const AggjArgs& a, uint64_t* tsum, hipStream_t s);
void launch_aggj_write(const AggjArgs& a, hipStream_t s);
// the output key order (fsg_keyed.hip): nkr / koff + scal[6] = ord slots, then
// (ord, hrec sized) the hashes and k_aggj_order
void launch_aggj_nk(const AggjArgs& a, uint64_t* tsum, hipStream_t s);
void launch_aggj_hash(const AggjArgs& a, hipStream_t s);
void launch_aggj_order(const AggjArgs& a, hipStream_t s);
void launch_aggj_order_group(const AggjArgs* list, uint32_t n, hipStream_t s);  // one workgroup per chain
void launch_xscan(const uint32_t* in, uint64_t* out, uint64_t* tsum, uint64_t n, unsigned long long* tot,
                  hipStream_t s);
// aggregate-json state kept in HBM (fsg_keyed.hip)
// pass 0: out[0] keys, out[1] records, out[2] arena bytes (sizes the arena); pass 1: the state
void launch_aggj_commit(const AjCommitArgs& c, uint64_t* tsum, int pass, hipStream_t s);
// keyed tables and the union dictionary of the topic-wide merge (fsg_keyed.hip)
void launch_kd_collect(const KdTable& t, const uint64_t* sptr, const uint32_t* slen, const uint32_t* sval, uint32_t n,
                       hipStream_t s);
void launch_kd_rehash(const KdTable& t, uint32_t n, hipStream_t s);
void launch_kd_desc(const KdTable& t, uint32_t n, uint32_t maxn, uint64_t* desc, hipStream_t s);
void launch_kd_union(const KdUnionArgs& u, hipStream_t s);       // tot[0] = K
void launch_kd_ids(const KdUnionArgs& u, hipStream_t s);
void launch_kd_place(const KdUnionArgs& u, uint64_t nkeys, hipStream_t s);  // tot[1] = union bytes
// stateful last stages (SfArgs): filter_look_back / filter_hashset
void launch_sf_lb(const SfArgs& a, hipStream_t s);
void launch_sf_dedup(const SfArgs& a, hipStream_t s);      // decisions assuming no eviction; scal[3] = kept
void launch_sf_dedup_seq(const SfArgs& a, hipStream_t s);  // the sequential BoundedHashSet walk
void launch_sf_compact(const SfArgs& a, hipStream_t s);
void launch_sf_commit(const SfArgs& a, hipStream_t s);     // after k_plan: state through plan.done
// CRC32C check of every stored batch (report only; bad[0] count, bad[1] first index)
void launch_verify_crc(const uint8_t* slice, const uint64_t* bpos, uint32_t nb, unsigned long long* bad,
                       uint32_t* flags, hipStream_t s);
// record-section decompression: pass 0 sizes, 1 writes, 2 record counts
void launch_decompress(const DecArgs& a, int pass, hipStream_t s);
// device framing (FrameArgs)
void launch_frame_cand(const FrameArgs& a, uint32_t nchunks, uint64_t* tsum, hipStream_t s);
void launch_frame_compact(const FrameArgs& a, uint32_t nchunks, hipStream_t s);
void launch_frame_chain(const FrameArgs& a, uint32_t levels, uint64_t* tsum, hipStream_t s);
}  // namespace fsg
