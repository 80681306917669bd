/*
 * vsiq.h — C ABI of the MI355X (gfx950) fake-quantization kernels.
 *
 * The drop-in boundary of this repository: every entry point below replaces
 * one link of VSIQuantization's eager-PyTorch fake-quant chain (reference
 * tranngocduvnvp/VSIQuantization, file:line cited per function).  The
 * reference's own plugin API is Python (CLASS_REGISTRY names, utils/registry.py:
 * 2-27); its Python classes are re-implemented in vsiquantization_amd/ and call
 * these functions through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - All tensor pointers are DEVICE pointers (hipMalloc / torch caching
 *     allocator).  The library never allocates, frees or synchronises.
 *   - `stream` is a hipStream_t passed as void*; NULL = the null stream.
 *   - Return value: 0 on success, a hipError_t (>0) from the launch, or a
 *     negative VSIQ_E* code for invalid arguments (nothing is launched then).
 *   - fp32 element arithmetic is IEEE (true division, rint half-to-even,
 *     NaN-propagating clamp, denormals kept): bit-identical to the reference's
 *     PyTorch CPU path.  Quantization parameters are computed in float64 on
 *     the device exactly as the reference does on the host in Python floats.
 *   - Workspaces: `ws` is a float64 device buffer of at least
 *     vsiq_workspace_doubles(n) entries and `counter` VSIQ_COUNTER_WORDS uint32
 *     device words that are 0 before the first call; every reducing kernel
 *     leaves them 0 when it finishes (stream-ordered reuse is safe, concurrent
 *     reuse on two streams is not).
 *   - Straight-through masks are ONE BIT per element (1 = the rounded value was
 *     inside [qmin, qmax], ClampBackward1 semantics), packed in uint64 words:
 *     a tensor is viewed as `rows` rows of `rowlen` elements (per-tensor: one
 *     row of n); row r owns words [r*W, (r+1)*W) with W = 4*ceil(rowlen/256);
 *     element e of a row lives in word 4*(e/256) + (e%4), bit (e%256)/4.
 *     (That is the wave64 ballot of "element j of each lane's 4-group".)
 *     vsiq_mask_words(rows, rowlen) gives the word count; 8-byte alignment.
 *   - Codes are int8 (symmetric) or uint8 (asymmetric) holding
 *     clamp(round(x/s+zp)); NaN inputs give code 0.
 */
#ifndef VSIQ_H_
#define VSIQ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VSIQ_ABI_VERSION 11

/* uint32 words of a reducing kernel's arrival `counter` (all 0 before the first call) */
#define VSIQ_COUNTER_WORDS 64

#define VSIQ_E_ARG (-1)      /* invalid argument (null pointer, bad size, qmin>qmax) */
#define VSIQ_E_ALIGN (-2)    /* misaligned pointer where alignment is required */
#define VSIQ_E_WS (-3)       /* workspace too small */

/* stats record written by vsiq_observe_f32 (float64 entries) */
#define VSIQ_ST_MIN 0        /* min of this call's non-NaN x (as f64), +inf if none */
#define VSIQ_ST_MAX 1        /* max of this call's non-NaN x, -inf if none */
#define VSIQ_ST_NAN 2        /* count of NaN elements */
#define VSIQ_ST_SUMABS 3     /* sum |x| (f64 accumulation) */
#define VSIQ_ST_SUM 4        /* sum x */
#define VSIQ_ST_SUMSQ 5      /* sum x^2 */
#define VSIQ_ST_N 6          /* element count */
#define VSIQ_ST_MEANABS 7    /* fp32-rounded mean(|x|)        (qm.py:66) */
#define VSIQ_ST_MEAN 8       /* fp32-rounded mean(x)          (qm.py:67) */
#define VSIQ_ST_STD 9        /* fp32-rounded unbiased std(x)  (qm.py:68) */
#define VSIQ_ST_LEN 10

/* qparams record (float64 entries) */
#define VSIQ_QP_SCALE 0      /* scale, Python-float semantics          (minmax.py:70-75) */
#define VSIQ_QP_ZP 1         /* zero point as an integer-valued f64; NaN if Python round() would raise */
#define VSIQ_QP_MIN 2        /* running min_val after this call        (minmax.py:44-45) */
#define VSIQ_QP_MAX 3        /* running max_val after this call        (minmax.py:46-47) */
#define VSIQ_QP_LEN 4

int vsiq_abi_version(void);
const char *vsiq_error_string(int code);

/* float64 workspace entries needed by the reducing kernels for n elements */
int64_t vsiq_workspace_doubles(int64_t n);

/* uint64 words of a 1-bit mask for `rows` rows of `rowlen` elements */
int64_t vsiq_mask_words(int64_t rows, int64_t rowlen);

/* Performance knobs (process-wide; results are identical for every setting). */
/* (keys 1, 5, 8 and 16 -- K3 rows per workgroup / workgroup size, K2 grid, K2 cached-load
   threshold -- were removed in ABI 10: their values are fixed; vsiq_set_tuning rejects them) */
#define VSIQ_TUNE_NONTEMPORAL 2        /* 1 = nontemporal streamed loads/stores (default) */
#define VSIQ_TUNE_OBS_KERNEL 7         /* K2 observer: 0 auto, 1 one-shot, 2 grid-stride */
#define VSIQ_TUNE_LSQ_GROUPS 9         /* K4 groups per lane 2 / 4 / 8 / 16, 0 = by size */
#define VSIQ_TUNE_PC_PACKED 10         /* per-channel fq with given qparams + K6: 1 = packed short
                                          rows / channel columns for K6 on axis 1 (default),
                                          2 = packed rows for K6 too (round-1 form),
                                          0 = one workgroup per row */
#define VSIQ_TUNE_STORE_GATE 11        /* one-round K3 / STE grids: no stores before workgroup
                                          start + N ticks of the 100 MHz wall clock (-1 = auto,
                                          see VSIQ_TUNE_GATE_AUTOTUNE; 0 = off) */
#define VSIQ_TUNE_STORE_DEFER 6        /* one-round grids: hold stores back N x 512 clocks after
                                          the loads (-1 = auto, 0 = off, max 64) */
#define VSIQ_TUNE_GATE_AUTOTUNE 12     /* 1 (default): the automatic store gate is tuned online
                                          per launch site (kernel, grid, bytes, device) from
                                          event-timed launches; 0: fixed 1.05 x the read time
                                          at 7.5 TB/s */
#define VSIQ_TUNE_XCD_ORDER 13         /* where neighbouring workgroups share cache lines (K6
                                          on channel columns of short rows): 2 (default) each
                                          XCD a range of channels, image blocks outermost
                                          (channels % 8 == 0, else 1); 1: XCD-contiguous
                                          block order; 0: hardware order */
#define VSIQ_TUNE_K2O_FORM 14          /* K2o: 0 (default) one-shot, one record per workgroup;
                                          1: grid-stride, vsiq_act_observe_part_f32's records */
#define VSIQ_TUNE_K2O_GROUPS 15        /* K2o one-shot groups per lane 1/2/4/8/16, 0 = default (2) */
#define VSIQ_TUNE_K2O_BLOCK 17         /* K2o one-shot lanes per workgroup 256/512/1024, 0 = default */
int vsiq_set_tuning(int key, int value);

/*
 * Store-gate tuner (VSIQ_TUNE_GATE_AUTOTUNE).  The only state the library keeps
 * between calls besides the knobs: per launch site, a handful of HIP event pairs and
 * the timings they returned (host memory; no device memory, no host sync).
 *   vsiq_gate_tuning_pending: sites launched since the previous call of it that are
 *     still tuning after harvesting finished timings (a caller that wants steady-state
 *     launches runs warm-up steps and calls it after each, until it is 0: sites of other
 *     work that is not running any more do not count);
 *   vsiq_gate_report: one text line per site (label, grid, bytes, chosen ticks, median
 *     launch time per candidate in us) into buf (NUL-terminated, truncated to len);
 *     returns the full length;
 *   vsiq_gate_reset: forget every site and every gate loaded by vsiq_gate_import
 *     (returns 1 and keeps them while timings are still in flight).
 */
int vsiq_gate_tuning_pending(void);
int64_t vsiq_gate_report(char *buf, int64_t len);
int vsiq_gate_reset(void);
/* Re-tune every store-gate launch site from its next launches on (e.g. once a training
 * loop runs under its real load); returns the number of sites.  A tuned site also
 * re-tunes by itself when the median time of its chosen gate drifts by more than 15 %
 * (one launch in 128 is timed).  Results never depend on the gate. */
int vsiq_gate_retune(void);
/* Gate table (ABI 11).  A site's key is "<kernel symbol> <grid> <read bytes>" (stable
 * for one build of the library); a table line is the key and the gate in ticks.
 *   vsiq_gate_export: every tuned site's line (and every loaded line) into buf
 *     (NUL-terminated, truncated to len); returns the full length;
 *   vsiq_gate_import: load lines (e.g. a saved export); a listed site, existing or
 *     first launched later, takes that gate and is never timed; returns the number of
 *     lines, -1 on a malformed line (nothing loaded then);
 *   vsiq_gate_freeze(1): from now on no launch is timed -- sites still tuning, and sites
 *     first launched later without a loaded line, run the fixed default (1.05 x the read
 *     time at 7.5 TB/s); vsiq_gate_retune does nothing while frozen.  Returns the
 *     previous setting.  With a loaded table and freeze, a process's kernel timing no
 *     longer depends on tuner state (no candidate or drift launches). */
int64_t vsiq_gate_export(char *buf, int64_t len);
/* Trace marker (ABI 11): one empty kernel, `vsiq_timed_region_marker`, grid 1 (end 0) or
 * grid 2 (end 1), so a kernel trace can be cut to the region between the two
 * (tools/timed_region_stats.py; bench.py --markers). */
int vsiq_trace_marker(int end, void *stream);

/*
 * K11 (ABI 11): the reference's per-call mean|x| and mean x BIT FOR BIT as torch's CPU
 * kernel computes them on the reference host -- quantization_manager.py:66-67 records
 * torch.mean(torch.abs(x)).cpu().item() and torch.mean(x); qm.py:112 builds the
 * learnable scale from that list.  torch's CPU sum is a cascade whose order depends on
 * the host's thread count (chunks of at::parallel_for) and its vector width (`vec` = 8,
 * the AVX2 Vectorized<float> this torch build dispatches on AVX2 and AVX-512 hosts
 * alike; 16 supported); the activation (VSIQ_ACT_*, SiLU with its own reference layout)
 * is applied first, as the fused layers record act(x).  One extra read of x (opt-in in
 * the Python layer).  out4 (device, nullable): {sum |act(x)|, sum act(x), mean |act(x)|,
 * mean act(x)} as fp32; stats (device, nullable): its VSIQ_ST_MEANABS / VSIQ_ST_MEAN
 * entries overwritten with the two means and VSIQ_ST_STD with torch.std(act(x)) as torch's
 * CPU kernel computes it (qm.py:68: f64 sum of squared deviations from the fp32 mean,
 * rounded to fp32 once; a second read of x).  ws: vsiq_torch_mean_ws_bytes(n, vec,
 * threads) bytes (-1: unsupported arguments -- vec not 8 / 16, threads outside 1..4096,
 * a chunk of 2^30 elements or more).  n = 0 gives NaN means, as torch.mean.
 */
int64_t vsiq_torch_mean_ws_bytes(int64_t n, int vec, int threads);
int vsiq_torch_mean_f32(const float *x, int64_t n, int act, int vec, int threads, float *out4, double *stats,
                        void *ws, int64_t ws_bytes, void *stream);
/* The same on a host (CPU) tensor, out4 in host memory; chunks on the host pool. */
int vsiq_host_torch_mean_f32(const float *x, int64_t n, int act, int vec, int threads, float *out4);
int vsiq_gate_import(const char *text);
int vsiq_gate_freeze(int on);

/*
 * Self-test of the kernels' correctly rounded division x / s (reciprocal +
 * two Newton-Markstein corrections, IEEE fallback outside the proven range):
 * for each of `count` divisors, every one of the 2^32 fp32 dividends is divided
 * both ways and mismatches[k] (uint64, zeroed by the caller) += bitwise differences.
 */
int vsiq_selftest_div(const float *divisors, int count, unsigned long long *mismatches,
                      void *stream);

/*
 * Self-test of the no-check fast paths, over all 2^32 fp32 inputs:
 *   mode 0: the quantizer code clamp(rint(x/s + zp), qmin, qmax) (value, sign of
 *           zero, STE mask bit) of the fast forward element vs the IEEE one, for
 *           every x with |x| <= 2^62, per (scales[k], zero_points[k]);
 *   mode 1: the STE backward quotient RN(RN(g*s)/s) (zero_points unused).
 * counts[2k] += mismatches, counts[2k+1] += inputs checked (uint64, zeroed by the
 * caller); a pair outside the fast domain checks nothing (counts[2k+1] == 0).
 */
int vsiq_selftest_fq(int mode, const float *scales, const float *zero_points, int count,
                     float qmin, float qmax, unsigned long long *counts, void *stream);

/*
 * Per-tensor fake-quant forward (K1).
 * Replaces quantizers/uniform.py:54-55 + :95 (discreate_tensor):
 *   y = (clamp(rint(x/s + zp), qmin, qmax) - zp) * s      (fp32)
 * s = fp32(scale), zp = fp32(zero_point), taken from
 *   - qp_dev[VSIQ_QP_SCALE], qp_dev[VSIQ_QP_ZP]   if qp_dev != NULL (observer output), else
 *   - *scale_dev (f64, a learnable 0-dim Parameter) if scale_dev != NULL, else scale_host;
 *   - *zp_dev (f64) if zp_dev != NULL, else zp_host; zp_round != 0 applies
 *     clamp(rint(zp), qmin, qmax) first (learnable tensor zp, uniform.py:98-102).
 * codes (int8/uint8, nullable) and mask (1-bit words, one row of n, nullable) are
 * optional outputs.
 * discrete != 0 writes the integer-valued fp32 clamp(round(x/s+zp)) into y instead
 * (UniformQuantizer.discreate_tensor, uniform.py:81-96).
 */
int vsiq_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t n,
                    const double *qp_dev, const double *scale_dev, double scale_host,
                    const double *zp_dev, double zp_host, int zp_round, int discrete, int qmin,
                    int qmax, void *stream);

/*
 * Per-tensor observer (K2).
 * Replaces observers/minmax.py:32-88 (observe + get_scale_zero_point, the two
 * `.item()` reductions) and quantizers/quantization_manager.py:66-68 (the
 * mean(|x|)/mean/std statistics) with ONE pass over x and an on-device float64
 * epilogue (last workgroup to finish).
 *   stats_out[VSIQ_ST_LEN]   this call's statistics (nullable)
 *   run_minmax[2]            running (min_val, max_val) fp32 state, in/out (nullable: fresh 0/0)
 *   qp_out[VSIQ_QP_LEN]      qparams from the updated running state (nullable)
 *   qden = 2**(b-1)-1+eps (symmetric) or 2**b-1+eps (asymmetric), computed by the caller in
 *   Python float64 exactly as minmax.py:72/75 writes it.
 */
int vsiq_observe_f32(const float *x, int64_t n, double *stats_out, float *run_minmax,
                     double *qp_out, int symmetric, double qden, double eps,
                     double *ws, int64_t ws_len, uint32_t *counter, void *stream);

/*
 * Observer epilogue alone, from a stats record that was reduced elsewhere (the
 * multi-GPU observer: per-rank vsiq_observe_f32 with run_minmax = qp_out = NULL,
 * RCCL all-reduce MAX over [-min, max] and SUM over the counts/sums, then this).
 * Applies the minmax.py:42-47 running update (NaN count > 0 -> unchanged) and
 * writes qp_out.  One lane, stream-ordered.
 */
int vsiq_observe_finalize(const double *stats, float *run_minmax, double *qp_out, int symmetric,
                          double qden, double eps, void *stream);

/*
 * The same epilogue from `world` per-rank stats records gathered in rank order
 * (gathered[world][VSIQ_ST_LEN], an all_gather of each rank's vsiq_observe_f32 record):
 * folds them (min / max exact, counts and sums in float64 in rank order), writes the
 * whole batch's stats record (stats_out nullable) and applies the running update +
 * qparams.  The per-call multi-GPU observer: one collective and one launch
 * per call.
 */
int vsiq_observe_finalize_ranks(const double *gathered, int world, double *stats_out, float *run_minmax,
                                double *qp_out, int symmetric, double qden, double eps, void *stream);

/*
 * The per-call multi-GPU exchange's fold and the fake quant in ONE launch (K1r):
 * `gathered` = the `world` ranks' stats records of this call (each from
 * vsiq_act_observe_f32 over the rank's shard with run_minmax = qp_out = NULL; one
 * all_gather in rank order).  Every workgroup folds them exactly as
 * vsiq_observe_finalize_ranks does, applies the running update + f64 qparams and
 * fake-quantizes its share of act(c) as vsiq_act_fq_fwd_f32 with those qparams;
 * workgroup 0 writes run_minmax, qp_out and stats_out (nullable).  Bit for bit
 * vsiq_observe_finalize_ranks followed by vsiq_act_fq_fwd_f32(qp_dev = qp_out).
 * Replaces, per rank, minmax.py:42-74 + uniform.py:55,95 of a batch-sharded
 * observe + quantize call (quantization_manager.py:73-90).
 */
int vsiq_act_fq_fwd_ranks_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                              const double *gathered, int world, double *stats_out, float *run_minmax,
                              double *qp_out, int symmetric, double qden, double eps, int qmin, int qmax,
                              void *stream);

/*
 * Per-tensor observe + fake quant of a small tensor in ONE launch (K8): n <=
 * vsiq_observe_fq_max_elems() (65536).  Equal to vsiq_act_observe_f32(c, n, act,
 * stats_out, run_minmax, qp_out, ...) followed by vsiq_act_fq_fwd_f32(c, y, codes, mask,
 * n, act, qp_out, ...): the same running update and f64 qparams record (min/max/qparams
 * exact, stats sums to float64 reordering), y / codes / 1-bit mask bit for bit.  Replaces
 * the reference's per-call observe + quantize (quantization_manager.py:73-90 ->
 * minmax.py:32-74 -> uniform.py:34-56) for one small tensor: BASELINE C1, a calibration
 * call on a weight.  stats_out / run_minmax / qp_out / codes / mask nullable.
 */
int64_t vsiq_observe_fq_max_elems(void);
int vsiq_act_observe_fq_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                            double *stats_out, float *run_minmax, double *qp_out, int symmetric, double qden,
                            double eps, int qmin, int qmax, void *stream);

/*
 * The same per-call observe + fake quant for mid-size tensors (K9): n <=
 * vsiq_observe_fq_parts_max_elems() (262144).  Two launches, no cross-workgroup arrival
 * chain: per-wave K2p records into ws, then every fake-quant workgroup folds them in a
 * fixed order, derives the running update + f64 qparams itself and quantizes its share.
 * Results as vsiq_act_observe_fq_f32: min / max / qparams / running state / y / codes /
 * mask bit for bit equal to vsiq_act_observe_f32 + vsiq_act_fq_fwd_f32, stats sums to
 * float64 reordering (the order of vsiq_observe_fold_parts).  ws: >= 1024 doubles
 * (any vsiq_workspace_doubles(n) buffer), stream-ordered like K2's.  Replaces
 * quantization_manager.py:73-90 -> minmax.py:32-74 -> uniform.py:34-56 for one tensor
 * (BASELINE C1: 256x256).
 */
int64_t vsiq_observe_fq_parts_max_elems(void);
int vsiq_act_observe_fq_parts_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                                  double *stats_out, float *run_minmax, double *qp_out, int symmetric,
                                  double qden, double eps, int qmin, int qmax, double *ws, int64_t ws_len,
                                  void *stream);

/*
 * K9 in ONE launch (K10, ABI 8): the same arguments plus `counter` (the
 * VSIQ_COUNTER_WORDS words of the stream's workspace; it uses words 33-35 and leaves
 * them zero).  The grid is K9's K2p grid (<= 32 workgroups); each workgroup keeps its
 * share of act(c) in registers, stores its K2p records, waits at a grid barrier on the
 * counter, folds every record in K9's order and quantizes from registers.  Results bit
 * for bit equal to vsiq_act_observe_fq_parts_f32, stats included.  A workgroup that
 * waits more than ~42 ms at the barrier (the grid not co-resident) writes NaN and bumps
 * counter word VSIQ_COUNTER_GRID_ERRORS (35) instead of spinning on; the caller reads it
 * (the word is never reset by the library) and treats a non-zero count as an error.  Replaces the same reference call sequence
 * as K9 (quantization_manager.py:73-90 -> minmax.py:32-74 -> uniform.py:34-56).
 * Measured on MI355X no faster than K9 (the barrier's two cross-XCD round trips cost
 * what K9's second launch boundary does), so the manager and BASELINE C1 stay on K9;
 * this is an opt-in (observe_fake_quant(..., parts="k10")).
 */
#define VSIQ_COUNTER_GRID_ERRORS 35
int vsiq_act_observe_fq_grid_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                                 double *stats_out, float *run_minmax, double *qp_out, int symmetric,
                                 double qden, double eps, int qmin, int qmax, double *ws, int64_t ws_len,
                                 uint32_t *counter, void *stream);

/*
 * Deferred-calibration observer (K2p): the K2 pass over act(c) WITHOUT the
 * cross-workgroup fold.  Replaces, like vsiq_act_observe_f32, minmax.py:42-43 +
 * quantization_manager.py:66-68 for an observe-only call (calibrate_qat_model,
 * utils/quantize_manager.py:4-31), whose result nothing reads until calibration ends.
 * Writes vsiq_observe_part_records(n) partial records of VSIQ_PART_LEN doubles
 *   {min, max, nan count, sum|x|, sum x, sum x^2, n, record count}
 * into parts[parts_len] (no workspace, no counter, no running-state update: any
 * number of calls may be in flight on any streams).  vsiq_observe_fold_parts then
 * folds ncalls such slots (call_stride doubles apart, each >= the call's records)
 * into ncalls stats records stats_out[ncalls][VSIQ_ST_LEN] in one launch; the
 * running min/max is replayed from those records (minmax.py:42-47, NaN calls skipped).
 * min/max/nan/n are exact; the sums differ from vsiq_act_observe_f32's only in
 * float64 summation order.
 */
#define VSIQ_PART_LEN 8
#define VSIQ_PART_MAX_RECORDS 4096   /* vsiq_observe_part_records(n) <= this for every n
                                        (one record per wave: at most 1024 workgroups x 4) */
int64_t vsiq_observe_part_records(int64_t n);
int vsiq_act_observe_part_f32(const float *c, int64_t n, int act, double *parts, int64_t parts_len,
                              void *stream);

/*
 * K2o: the deferred observer pass that also writes y = act(c) (n floats): a calibration
 * forward of a fused layer in one pass -- the activation the next layer consumes
 * (modules/fused.py:133) and the deferred observer's records of it, in the
 * vsiq_act_observe_part_f32 record format; vsiq_observe_part_out_records(n) records,
 * one per workgroup (n / 2048 by default; not bounded by VSIQ_PART_MAX_RECORDS).  y
 * bit-identical to
 * vsiq_act_fwd_f32; folded min/max/nan/n equal to K2p's, the sums to float64 summation
 * order (VSIQ_TUNE_K2O_FORM 1: K2p's grid, records bit-identical to it).
 */
int64_t vsiq_observe_part_out_records(int64_t n);
int vsiq_act_observe_part_out_f32(const float *c, float *y, int64_t n, int act, double *parts, int64_t parts_len,
                                  void *stream);
int vsiq_observe_fold_parts(const double *parts, int64_t ncalls, int64_t call_stride,
                            double *stats_out, void *stream);

/*
 * Multi-tensor K2p (K2m): `count` deferred observer calls of one activation `act` in
 * one launch per 32 calls (blocks map to (call, block) through a descriptor table in
 * the kernel arguments).  Each call's records are bit-identical to its own
 * vsiq_act_observe_part_f32 launch.  Replaces, for a calibration forward, the
 * per-layer observer launches of minmax.py:42-43 + quantization_manager.py:66-68
 * (calibrate_qat_model, utils/quantize_manager.py:4-31): the calls of consecutive
 * layers are queued and observed together (QuantizationManager deferred mode).
 */
typedef struct vsiq_part_tensor {
  const float *c;       /* observed tensor (pre-activation when act != NONE), n floats */
  int64_t n;
  double *parts;        /* this call's slot, parts_len >= vsiq_observe_part_records(n) * VSIQ_PART_LEN */
  int64_t parts_len;
} vsiq_part_tensor;
int vsiq_act_observe_part_multi_f32(const vsiq_part_tensor *tensors, int count, int act, void *stream);

/*
 * Per-channel fused observe + qparams + fake-quant forward (K3), axis 0 of a
 * row-major [rows, rowlen] view (OIHW weight: rows = O, rowlen = I*H*W).
 * Build-defined per-channel MinMax: row c is processed as
 *   s_c, z_c = MinMaxObserver(sym).forward(W[c])          (minmax.py:76-88)
 *   Y[c]     = UniformQuantizer(b, sym).quantize(W[c], s_c, z_c, False)  (uniform.py:34-56)
 * run_min/run_max [rows] fp32 running state, in/out (zeros = fresh observers).
 * scale_out/zp_out [rows] f64 (zp NaN where Python round() would raise).
 * row_stats [rows][3] f64 (nullable): sum|x|, sum x, sum x^2 of each row, for the
 * manager's mean(|x|)/mean/std records (quantization_manager.py:66-68).
 * y == NULL observes only (codes/mask must then be NULL too).
 * One read and one write of every element.
 */
int vsiq_pc_observe_fq_f32(const float *x, float *y, void *codes, uint64_t *mask,
                           int64_t rows, int64_t rowlen, float *run_min, float *run_max,
                           double *scale_out, double *zp_out, double *row_stats, int symmetric,
                           int qmin, int qmax, double qden, double eps, void *stream);

/*
 * Per-channel fake-quant forward with given per-row qparams (f64 [rows]).
 * zp_round != 0 applies clamp(rint(zp)) first (learnable zp, uniform.py:98-102).
 */
int vsiq_pc_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t rows,
                       int64_t rowlen, const double *scale, const double *zp, int zp_round,
                       int qmin, int qmax, void *stream);

/*
 * Straight-through backward for fixed (non-learnable) qparams, from the saved mask.
 * Replaces the autograd chain MulBackward0 -> ClampBackward1 -> STE -> DivBackward0 of
 * uniform.py:55,95 with a Python-float scale:
 *   gx = (mask ? g*s : 0) / s      (fp32, bit-exact)
 * s = fp32(scale_dev[i / rowlen]) if scale_dev != NULL (rowlen elements per entry), else
 * fp32(scale_host) and one row of n.  `mask` uses the same rows/rowlen layout.
 */
int vsiq_ste_bwd_f32(const float *g, const uint64_t *mask, float *gx, int64_t n,
                     const double *scale_dev, int64_t rowlen, double scale_host, void *stream);

/*
 * Learnable (LSQ) backward (K4): grad_x plus the scale / zero-point gradients.
 * Replaces autograd over uniform.py:47-56 (ScaleGradient, RoundStraightThrough,
 * clamp, div, mul; uniform.py:242-271):
 *   gx        = (mask ? g*s : 0) / s
 *   grad_s    = gscale * [ sum g*(q-zp) + sum (-(mask?g*s:0)) * ((x/s)/s) ]
 *   grad_zp   = gscale * [ sum (mask?g*s:0) + sum -(g*s) ] * zp_in_range      (zp_learn 1)
 * zp_learn 1: the forward used clamp(rint(zp)) (learned zero point, uniform.py:50-52);
 * zp_learn 2: zp as given with its gradient and no ScaleGradient factor (a symmetric
 *   quantizer handed a gradient-requiring zero point, uniform.py:47-56):
 *   grad_zp = sum (mask?g*s:0) + sum -(g*s);  0: no zero-point gradient.
 * sums of fp32 terms accumulated in float64, fixed reduction order (deterministic).
 * grad_out[0] = grad_s, grad_out[1] = grad_zp (device f64, overwritten).
 */
int vsiq_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t n,
                     const double *scale_dev, double scale_host, const double *zp_dev,
                     double zp_host, int zp_learn, int qmin, int qmax, double gscale,
                     double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
                     void *stream);

/*
 * Multi-tensor ("foreach") learnable fake quant: `count` independent per-tensor
 * LSQ quantizers -- typically the weight quantizer of every fused layer of a model
 * (quantizers/fake_quantize.py:62-63 -> uniform.py:47-56, once per layer and
 * forward in the reference) -- in one forward and one backward launch (up to 32
 * tensors per launch; larger counts are split).  Each tensor's results are
 * bit-identical to vsiq_fq_fwd_f32(x, y, ..., scale_dev, scale_host, zp_dev,
 * zp_host, zp_round = zp_learn) and vsiq_lsq_bwd_f32 on that tensor alone
 * (same element math, blocks and fold order).  The descriptor array is HOST
 * memory; the library copies it into the launch arguments.
 *   forward : y = fq(x), reads x, scale_dev/zp_dev (g, gx, grad_out unused)
 *   backward: gx, grad_out[2] = {grad_scale, grad_zp} from g and x
 * ws / counter as for vsiq_lsq_bwd_f32, ws >= vsiq_lsq_multi_workspace_doubles()
 * doubles; a tensor above 2^19 elements is handed to the single-tensor kernel
 * within the same call.
 */
typedef struct vsiq_lsq_tensor {
  const float *x;           /* quantizer input (e.g. a conv weight), n floats */
  float *y;                 /* forward output */
  const float *g;           /* backward: dL/dy */
  float *gx;                /* backward: dL/dx */
  const double *scale_dev;  /* f64 learnable scale (NULL: scale_host) */
  const double *zp_dev;     /* f64 zero point (NULL: zp_host) */
  double *grad_out;         /* backward: f64[2] {grad_scale, grad_zp}, overwritten */
  int64_t n;
  double scale_host;
  double zp_host;
  double gscale;            /* ScaleGradient factor (uniform.py:48, 58-71) */
  int32_t qmin;
  int32_t qmax;
  int32_t zp_learn;         /* learnable zp: clamp(rint(zp)) in the forward, grad_zp */
  int32_t reserved;
} vsiq_lsq_tensor;
int64_t vsiq_lsq_multi_workspace_doubles(const vsiq_lsq_tensor *tensors, int count);
int vsiq_lsq_fwd_multi_f32(const vsiq_lsq_tensor *tensors, int count, void *stream);
int vsiq_lsq_bwd_multi_f32(const vsiq_lsq_tensor *tensors, int count, double *ws, int64_t ws_len,
                           uint32_t *counter, void *stream);

/*
 * Learnable backward with the scale / zero-point gradient fold deferred (K4d).
 * vsiq_act_lsq_bwd_part_f32 is vsiq_act_lsq_bwd_f32 without the cross-workgroup
 * reduction: grad_x (bit-identical) plus one {sum t, sum z} record per workgroup into
 * records[2 * vsiq_lsq_part_records(n)] -- no workspace drain, no arrival atomics, no
 * last-block fold (3-5 us of every K4 launch at 2-26M elements).  vsiq_lsq_fold_multi
 * then folds `count` such calls (each its own records) into grad_out[2] = {grad_scale,
 * grad_zp} exactly as vsiq_act_lsq_bwd_f32 defines them (to float64 summation order), 64
 * calls per launch pair (chunk folds, then the per-call folds); the fold uses the records
 * as its scratch (their contents are overwritten).  The activation quantizers of a QAT model (quantize_out of every fused
 * layer, fake_quantize.py:49-50 -> uniform.py:47-56) are folded in one launch when
 * autograd has been through all of them (quantizers/deferred.py).
 */
typedef struct vsiq_lsq_fold {
  double *records;         /* the call's records, nrec x {sum t, sum z} (overwritten) */
  int64_t nrec;            /* vsiq_lsq_part_records(n) of the call */
  const double *zp_dev;    /* the zero point the forward used (NULL: zp_host) */
  double zp_host;
  double gscale;           /* ScaleGradient factor */
  double *grad_out;        /* f64[2] {grad_scale, grad_zp}, overwritten */
  int32_t qmin;
  int32_t qmax;
  int32_t zp_learn;
  int32_t reserved;
} vsiq_lsq_fold;
int64_t vsiq_lsq_part_records(int64_t n);
int vsiq_act_lsq_bwd_part_f32(const float *g, const float *c, float *gc, int64_t n, int act,
                              const double *scale_dev, double scale_host, const double *zp_dev, double zp_host,
                              int zp_learn, int qmin, int qmax, double *records, int64_t records_len,
                              void *stream);
int vsiq_lsq_fold_multi(const vsiq_lsq_fold *folds, int count, void *stream);

/*
 * Fused activation + activation fake-quant (K5).  Replaces, in the fused layers,
 * F.relu / F.silu after the conv (modules/fused.py:124-134, :198-206) followed by
 * quantize_out (quantizers/fake_quantize.py:49-50): the conv output c is read
 * once and act(c) is never materialized.  act: VSIQ_ACT_NONE / _RELU / _SILU.
 *   relu(c) = c < 0 ? 0 : c        bwd: c <= 0 ? 0 : g                          (bit-exact)
 *   silu(c) = c / (1 + exp(-c))    bwd: (g*sig) * fma(c, 1 - sig, 1), sig = 1/(1+exp(-c))
 *     bit for bit what torch's CPU silu kernels compute on the reference host: exp is
 *     Sleef_expf_u10 on the vectorized elements and glibc expf on the scalar remainder of
 *     each at::parallel_for chunk.  Which elements those are depends on the host's
 *     vector width and torch thread count; pass them with VSIQ_ACT_SILU_REF(W, threads)
 *     (W = 2 x floats per vector: 32 on AVX-512, 16 on AVX2; plain VSIQ_ACT_SILU = every
 *     element on the vectorized path).  DESIGN.md §2.1.
 * Each entry point is its plain counterpart applied to act(c); the backward ones
 * take c again and return the gradient with respect to c.
 */
#define VSIQ_ACT_NONE 0
#define VSIQ_ACT_RELU 1
#define VSIQ_ACT_SILU 2
/* W in {0, 8, 16, 32, 64}, threads in [0, 32767] (0 and 1: one chunk) */
#define VSIQ_ACT_SILU_REF(W, threads) (VSIQ_ACT_SILU | ((W) << 8) | ((threads) << 16))
int vsiq_act_fq_fwd_f32(const float *c, float *y, void *codes, uint64_t *mask, int64_t n, int act,
                        const double *qp_dev, const double *scale_dev, double scale_host,
                        const double *zp_dev, double zp_host, int zp_round, int discrete, int qmin,
                        int qmax, void *stream);
int vsiq_act_observe_f32(const float *c, int64_t n, int act, double *stats_out, float *run_minmax,
                         double *qp_out, int symmetric, double qden, double eps, double *ws,
                         int64_t ws_len, uint32_t *counter, void *stream);
int vsiq_act_ste_bwd_f32(const float *g, const uint64_t *mask, const float *c, float *gc, int64_t n,
                         int act, const double *scale_dev, int64_t rowlen, double scale_host,
                         void *stream);
int vsiq_act_lsq_bwd_f32(const float *g, const float *c, float *gc, int64_t n, int act,
                         const double *scale_dev, double scale_host, const double *zp_dev,
                         double zp_host, int zp_learn, int qmin, int qmax, double gscale,
                         double *grad_out, double *ws, int64_t ws_len, uint32_t *counter,
                         void *stream);
/*
 * The activation alone (K5's element code, same act argument): y = act(c) and its
 * backward gc = d act(c)/dc * g.  Replaces F.relu / F.silu of the fused layers
 * (modules/fused.py:133, torch.nn.functional.silu's CPU kernel) where the activation's
 * output is not fake-quantized in the same pass (calibration forwards).  act != NONE.
 */
int vsiq_act_fwd_f32(const float *c, float *y, int64_t n, int act, void *stream);
int vsiq_act_bwd_f32(const float *g, const float *c, float *gc, int64_t n, int act, void *stream);
/* Self-test of the two exps SiLU uses (Sleef expf_u10 / glibc expf, op for op): writes
 * both for n inputs; tests compare them bitwise with the oracle (tests/test_gpu_silu.py). */
int vsiq_selftest_exp_f32(const float *x, float *sleef_out, float *glibc_out, int64_t n, void *stream);

/*
 * Per-channel fake quant on a [rows, rowlen] view where row r uses the qparams of
 * channel r % channels (axis 0 of [C, ...]: rows = channels = C; axis 1 of
 * [N, C, ...]: rows = N*C, channels = C).  scale/zp f64 [channels] (zp nullable: 0).
 */
int vsiq_pcm_fq_fwd_f32(const float *x, float *y, void *codes, uint64_t *mask, int64_t rows,
                        int64_t rowlen, int64_t channels, const double *scale, const double *zp,
                        int zp_round, int qmin, int qmax, void *stream);

/*
 * Per-channel learnable (LSQ) backward (K6): LSQFakeQuantize's per-channel path
 * (quantizers/lsq_module.py:134-166: ScaleGradient on scale_param and the rounded
 * zero_point_param_float, per-channel fake quant) and a learnable
 * PerChannelUniformQuantizer.  Same element math as vsiq_lsq_bwd_f32, gradients
 * summed per channel (f64 sums of the fp32 terms, fixed order):
 *   grad_scale_out[c] = gscale * sum_{rows of c} [ g*(q-zp) - (mask?g*s:0)*((x/s)/s) ]
 *   grad_zp_out[c]    = gscale * sum [ (mask?g*s:0) - g*s ] * (rint(zp[c]) in [qmin, qmax])
 * grad_zp_out nullable.  ws: vsiq_pcm_workspace_doubles(rows, rowlen) doubles.
 */
int64_t vsiq_pcm_workspace_doubles(int64_t rows, int64_t rowlen);
int vsiq_pcm_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                         int64_t channels, const double *scale, const double *zp, int zp_learn,
                         int qmin, int qmax, double gscale, double *grad_scale_out,
                         double *grad_zp_out, double *ws, int64_t ws_len, void *stream);
/*
 * The same with per-channel arrival counters (uint32 [>= channels], zero before first
 * use; every call leaves them zero; one set per stream): on the axis-1 channel-column
 * path the last workgroup of each channel folds its records in the launch -- no second
 * launch, the same bits as vsiq_pcm_lsq_bwd_f32.  counters NULL: exactly
 * vsiq_pcm_lsq_bwd_f32.  Other paths ignore the counters.
 */
int vsiq_pcm_lsq_bwd_arrive_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                                int64_t channels, const double *scale, const double *zp, int zp_learn,
                                int qmin, int qmax, double gscale, double *grad_scale_out,
                                double *grad_zp_out, double *ws, int64_t ws_len, uint32_t *counters,
                                int64_t counters_len, void *stream);

/*
 * BatchNorm folding (modules/fused.py:100-108, :294-300), fp32, reference order:
 *   f = gamma / sqrt(running_var + eps);  w_out[r,:] = w[r,:] * f[r]
 *   b_out[r] = beta[r] + (b[r] - running_mean[r]) * f[r]      (b NULL: 0; b_out nullable)
 * rows = out-channels, rowlen = elements per out-channel.  In-place (w_out == w) allowed.
 */
int vsiq_bn_fold_f32(const float *w, const float *b, const float *gamma, const float *beta,
                     const float *running_mean, const float *running_var, float eps, float *w_out,
                     float *b_out, int64_t rows, int64_t rowlen, void *stream);

/*
 * Host path (CPU tensors; the reference's own environment, BASELINE C1): the same
 * element arithmetic on HOST pointers, native C++ loops over fixed 64K-element chunks
 * on up to VSIQ_HOST_THREADS threads (default: the CPUs this process may use, capped by
 * the cgroup CPU quota; a persistent pool for tensors of 4+ chunks); results do not
 * depend on the thread count.  No activation / ReLU run AVX-512 loops where the CPU has
 * them (elementwise bit-identical to the scalar loops; VSIQ_HOST_SIMD=0 forces the
 * scalar ones).  mask: one byte per element.
 *   vsiq_host_observe_f32  = vsiq_act_observe_f32        (minmax.py:42-74, qm.py:66-68)
 *   vsiq_host_fq_fwd_f32   = vsiq_act_fq_fwd_f32         (uniform.py:55,95; qp nullable)
 *   vsiq_host_ste_bwd_f32  = vsiq_act_ste_bwd_f32        (autograd of uniform.py:55,95)
 *   vsiq_host_lsq_bwd_f32  = vsiq_act_lsq_bwd_f32        (autograd of uniform.py:47-56)
 */
int vsiq_host_observe_f32(const float *x, int64_t n, int act, double *stats_out, float *run_minmax, double *qp_out,
                          int symmetric, double qden, double eps);
int vsiq_host_fq_fwd_f32(const float *x, float *y, uint8_t *codes, uint8_t *mask, int64_t n, int act,
                         const double *qp, double scale, double zp, int zp_round, int discrete, int qmin,
                         int qmax);
int vsiq_host_ste_bwd_f32(const float *g, const uint8_t *mask, const float *pre, float *gx, int64_t n, int act,
                          double scale);
int vsiq_host_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t n, int act, double scale, double zp,
                          int zp_learn, int qmin, int qmax, double gscale, double *grad_out);
/* Per-channel (axis 0: rows = out-channels of a [rows, rowlen] view) on the host: each row
 * is the per-tensor host call above on that row alone (SURVEY §0.2's per-channel
 * definition), with one running {min, max} per row (run_min / run_max fp32[rows]) and
 * f64 qparams per row (scale_out / zp_out; zp NaN where Python round() would raise);
 * row_stats (optional) f64[rows][3] = {sum|x|, sum x, sum x^2}; y NULL: observe only.
 * The learnable backward takes one gscale for all rows; grad_*_out are f64[rows]. */
int vsiq_host_pc_observe_fq_f32(const float *x, float *y, uint8_t *mask, int64_t rows, int64_t rowlen,
                                float *run_min, float *run_max, double *scale_out, double *zp_out,
                                double *row_stats, int symmetric, double qden, double eps, int qmin, int qmax);
int vsiq_host_pc_fq_fwd_f32(const float *x, float *y, uint8_t *mask, int64_t rows, int64_t rowlen,
                            const double *scale, const double *zp, int zp_round, int qmin, int qmax);
int vsiq_host_pc_ste_bwd_f32(const float *g, const uint8_t *mask, float *gx, int64_t rows, int64_t rowlen,
                             const double *scale);
int vsiq_host_pc_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                             const double *scale, const double *zp, int zp_learn, int qmin, int qmax, double gscale,
                             double *grad_scale_out, double *grad_zp_out);
/* Per-channel along axis 1 ([N, C, ...] activations, LSQFakeQuantize's broadcast of
 * [1, C, 1, ...] parameters, quantizers/lsq_module.py:141-143) on the host, in the device
 * ABI's vsiq_pcm_* layout: rows = N * channels rows of rowlen elements, row r in channel
 * r % channels; scale / zp f64[channels]; grad_*_out f64[channels], each the f64 sum of
 * the channel's rows in row order times gscale.  channels == rows is the vsiq_host_pc_*
 * call (the same bits). */
int vsiq_host_pcm_fq_fwd_f32(const float *x, float *y, uint8_t *mask, int64_t rows, int64_t rowlen, int64_t channels,
                             const double *scale, const double *zp, int zp_round, int qmin, int qmax);
int vsiq_host_pcm_ste_bwd_f32(const float *g, const uint8_t *mask, float *gx, int64_t rows, int64_t rowlen,
                              int64_t channels, const double *scale);
int vsiq_host_pcm_lsq_bwd_f32(const float *g, const float *x, float *gx, int64_t rows, int64_t rowlen,
                              int64_t channels, const double *scale, const double *zp, int zp_learn, int qmin, int qmax,
                              double gscale, double *grad_scale_out, double *grad_zp_out);
int vsiq_host_threads(void);
int vsiq_host_simd(void);   /* 1: the AVX-512 loops are in use */

#ifdef __cplusplus
}
#endif

#endif /* VSIQ_H_ */
