/*
 * inflow.h — C-ABI of libinflow.so, the MI355X (gfx950) implicit-flow density-evaluation engine.
 *
 * The reference (musikisomorphie/implicit-normalizing-flows) has no FFI: its hot path is the
 * PyTorch op sequence inside lib/layers/implicit_block.py.  Each entry point below replaces one
 * reference call site; the Python drop-in modules (implicit-normalizing-flows_amd/lib/layers)
 * bind them with ctypes.  Conventions:
 *   - every pointer is a DEVICE pointer unless documented otherwise; tensors use the reference's
 *     layout: conv nets NCHW (B, C, H, W) contiguous fp32, fc nets (B, d) row-major fp32;
 *   - `stream` is a hipStream_t (the caller's current stream); nothing synchronises the device
 *     except inf_root_find / inf_imblock_forward, which read one residual norm per Broyden
 *     iteration back to the host exactly where the reference calls .item() (broyden.py:145,157);
 *   - workspace is caller-allocated (inf_workspace_bytes) so the torch caching allocator owns it;
 *   - return value 0 = success, otherwise an InfStatus code (inf_status_string()).
 *   - no process-wide mutable state: every tuning / semantics switch is a per-net option
 *     (inf_net_set_option), the launch profiler is per host thread, and the host readback buffers and the
 *     side stream of inf_imblock_eval are per host thread.  Calls are re-entrant across threads for
 *     distinct nets and workspaces.  A net handle itself (its packed weights, its option values and its cached
 *     f(0) for the first Broyden residual) belongs to one thread at a time, like the nn.Module it mirrors.
 */
#ifndef INFLOW_H
#define INFLOW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum InfStatus {
  INF_OK = 0,
  INF_ERR_INVALID = 1,     /* bad argument / unsupported net shape */
  INF_ERR_HIP = 2,         /* a HIP runtime call failed (see inf_last_hip_error) */
  INF_ERR_WORKSPACE = 3,   /* workspace too small */
  INF_ERR_UNSUPPORTED = 4  /* layer pattern the engine does not implement */
} InfStatus;

typedef enum InfLayerKind {
  INF_LAYER_CONV = 1,    /* InducedNormConv2d  (mixed_lipschitz.py:149-391), stride 1, pad k//2 */
  INF_LAYER_LINEAR = 2,  /* InducedNormLinear  (mixed_lipschitz.py:12-136) */
  INF_ACT_SWISH = 3,     /* Swish              (activations.py:64-71) */
  INF_ACT_SIN = 4        /* Sin                (activations.py:7-12) */
} InfLayerKind;

typedef struct InfLayerDesc {
  int kind;                 /* InfLayerKind */
  int cin, cout, ksize;     /* conv: (cout, cin, k, k) weight; linear: k = 1 */
  const float* weight;      /* raw (un-normalised) weight, device */
  const float* bias;        /* (cout) device, or NULL */
  const float* u;           /* spectral-norm vectors u (codomain) / v (domain), device */
  const float* v;
  float coeff;              /* Lipschitz cap: W_eff = W / max(1, u.(W v) / coeff) */
  const float* beta;        /* Swish beta (1 float) device */
} InfLayerDesc;

typedef struct InfNetDesc {
  int n_layers;
  const InfLayerDesc* layers;   /* host array, nn.Sequential order */
  int channels, height, width;  /* per-sample input shape; fc nets: channels = d, height = width = 1 */
} InfNetDesc;

typedef struct InfNet InfNet;   /* opaque: packed, Lipschitz-normalised weights + launch plan */

typedef struct InfBroydenStats {  /* mirrors the dict returned by broyden() (broyden.py:184-193) */
  int nstep;              /* per-sample mode: the largest per-sample nstep */
  int lowest_step;        /* per-sample mode: the largest per-sample lowest_step */
  int prot_break;         /* 1 => fell back to the Banach fixed point (implicit_block.py:74-75); per-sample: any */
  int n_trace;
  double trace[64];       /* ||g||_F over the batch per iteration; trace[0] is the initial objective */
  double diff;            /* ||g(result)||_F */
  double eps;             /* eps * sqrt(B*d) (broyden.py:131); per-sample mode: eps * sqrt(d) */
  int fixed_point_iters;  /* iterations of the fallback, 0 if unused */
  int convergence;        /* InfConvergence the solve ran with */
  /* per-sample mode only: optional HOST arrays of `batch` ints set by the CALLER before the call (NULL: not
   * written) that receive each sample's nstep, lowest_step and prot_break */
  int* sample_nstep;
  int* sample_lowest_step;
  int* sample_prot_break;
  /* nstep + the extra iterations of accepted line searches (broyden.py:156; == nstep without INF_OPT_LINE_SEARCH) */
  int tnstep;
} InfBroydenStats;

/* ---- library ------------------------------------------------------------------------------ */
int inf_version(void);
/* Releases the calling thread's engine-held host resources (pinned readback slots, events, side streams, profiling
 * events) after waiting for the device.  Call before process exit: lib/_hip registers it with atexit, so it runs before
 * the HIP runtime's own teardown.  Idempotent; nets stay valid and later calls re-create what they need. */
int inf_shutdown(void);
const char* inf_status_string(int status);
int inf_last_hip_error(void);

/* ---- nets: the nnet_x / nnet_z nn.Sequential of InducedNorm layers + activations ------------ */
/* Replaces the per-call module walk of nnet(x) (implicit_flow.py:362-399, train_tabular.py:292-311). */
int inf_net_create(const InfNetDesc* desc, InfNet** out);
int inf_net_destroy(InfNet* net);
/* compute_weight(update=False) for every layer (mixed_lipschitz.py:126-132,320-326,378-386):
 * sigma = u.(W v) on device, W_eff = W / max(1, sigma/coeff), repacked for the MFMA kernels.
 * Call after any parameter change (the Python side tracks tensor versions). */
int inf_net_refresh(InfNet* net, void* stream);
/* Re-points the net at other tensors of the same layout (same layer kinds, shapes and activations as at create), e.g. a
 * DataParallel replica's copies of the parameters (train_img.py:203-204 nn.DataParallel): weight / bias / u / v / beta
 * pointers only, nothing repacked -- call inf_net_refresh when the values differ from the last refresh's.
 * INF_ERR_INVALID when the layout differs (the net is left unchanged). */
int inf_net_set_tensors(InfNet* net, const InfNetDesc* desc);
/* Arithmetic of the fused 3-1-3 conv kernel's three contractions (fused313.hip phases A, B, C).
 *   INF_MFMA_F32    v_mfma_f32_32x32x2_f32: exact fp32 products, k-ordered fp32 accumulation.
 *   INF_MFMA_BF16X6 both operands split exactly into three bf16 pieces (x = hi + mid + lo, truncation),
 *                   the six products down to 2^-16 relative on v_mfma_f32_32x32x16_bf16, fp32 accumulation:
 *                   dropped terms <= 2^-23 relative, i.e. fp32-level error at 16x the per-clock MFMA rate.
 *   INF_MFMA_F16X3  all three contractions with both operands split into two fp16 pieces after a power-of-two
 *                   scale S (weights: per matrix; activations: per pixel column in phases B and C, per tile in
 *                   phase A, from that set's max m, so m*S is in [2^14, 2^15)): x*S = h + l with h = rne16(x*S),
 *                   l = rne16(x*S - h): |x*S - h - l| <= 2^-23 |x*S| while l is a normal fp16
 *                   (|x*S - h| >= 2^-14), <= 2^-25 absolute below that; relative to the set, <= 2^-23 m*S
 *                   for every element (small entries get an absolute, not a relative, bound).  Three products (lh, hl, hh) on
 *                   v_mfma_f32_32x32x16_f16, fp32 accumulation, unscaled exactly (ldexp): fp32-level error of
 *                   each dot product at twice the BF16X6 product rate, 4 instead of 6 operand bytes per weight.
 * Fused fc nets (fcnet.hip / fcnet_h3.hip: the tabular / toy nets' whole forward or forward-mode Jacobian per launch):
 *   INF_MFMA_F16X3 the same two-piece scaled split (weights per matrix, activations per sample column) on
 *                  v_mfma_f32_16x16x32_f16; INF_MFMA_F32 (and BF16X6, which has no fc kernel) exact fp32 MFMA.
 * Default: INFLOW_MFMA=f32 (or fp32) / bf16x6 / f16x3 in the environment at inf_net_create, otherwise F16X3; any
 * other value makes inf_net_create fail with INF_ERR_INVALID.
 * No effect on nets outside the fused paths. */
typedef enum InfMfmaMode { INF_MFMA_F32 = 0, INF_MFMA_BF16X6 = 1, INF_MFMA_F16X3 = 2 } InfMfmaMode;
int inf_net_set_mfma(InfNet* net, int mode);
int inf_net_get_mfma(const InfNet* net);
/* Per-net options (no process-wide switches: two threads driving different nets never share one).  Returns the
 * previous value, or -INF_ERR_INVALID for an unknown option or a value out of range.
 *   INF_OPT_FUSED_K128    which kernel runs the fused VJP, forward (EVAL) and derivative-saving forwards (SAVE,
 *                         EVALSAVE) of 512-wide nets in INF_MFMA_F16X3:
 *                         0 the 64-pixel kernel only; 1 the 128-pixel K-chunked kernel where its grid still covers
 *                         all 256 CUs (default, or INFLOW_FUSED_K128 at inf_net_create); 2 wherever its tile fits;
 *                         3 as 1, with the VJP launches on the two-per-CU 64-pixel kernel (fused313p.hip).
 *                         A paired launch (both branches of an imBlock) follows the first net's value.
 *   INF_OPT_EVAL_OVERLAP  read on net_x of inf_imblock_eval: 1 (default; INFLOW_EVAL_OVERLAP=0 at create for 0) runs
 *                         the x-branch series on a side stream beside the root solve and the z-branch series (the
 *                         streams join before the call returns; needs workspace for a third region); 0 runs both
 *                         series in lockstep on the caller's stream.  Results agree to fp32 roundoff.
 *   INF_OPT_CONVERGENCE   read on the net whose root is solved (nnet_z forward, nnet_x inverse): INF_CONV_GLOBAL
 *                         (default) is the reference's rule, one Frobenius norm over the batch against
 *                         eps sqrt(B d) and one lowest iterate for the batch (broyden.py:131,153-163); with
 *                         INF_CONV_PER_SAMPLE each sample stops on its own norm against eps sqrt(d) with its own
 *                         lowest iterate, stall and protective breaks and Banach fallback -- the reference's result
 *                         for a batch of one, so a sharded batch gives the single-process result row for row.
 *                         INFLOW_CONVERGENCE=per_sample at create selects it.
 *   INF_OPT_K128_EXACT_SCALE  0 (default) / 1: the 128-pixel kernel puts chunk 1's phase-A values at chunk 0's column
 *                         scales and falls back to exact per-chunk scales only for a tile where a value would not fit
 *                         fp16; 1 takes the exact-scale path on every tile (tests: both paths give the same results).
 *   INF_OPT_FC_BLOCK      read on net_z of inf_imblock_eval_exact: where a block kernel exists (fcblock.hip: f16x3
 *                         nets, d = 6 with 3 hidden layers or d = 2 with 1, threshold <= 30; the global rule also needs
 *                         the grid co-resident: batch <= 48 x the co-resident workgroups) the whole block runs in one
 *                         launch, the Broyden state in LDS, the global rule's norm exchanged between workgroups inside
 *                         the launch, the host reading the statistics once.  0 never; 1 (default; INFLOW_FC_BLOCK at
 *                         create) for the per-sample rule only, where it is the faster path; 2 for both rules.
 *                         Otherwise every net evaluation is a launch and the host reads each iteration's norm.
 *   INF_OPT_FC_SERIES     read on the first net of inf_logdet_series / inf_logdet_series_pair: 1 (default;
 *                         INFLOW_FC_SERIES at create) runs the power series of fused f16x3 fc nets (d = 6 with 3 hidden
 *                         layers or d = 2 with 1) as one launch for both nets: one forward pass keeping act' in registers,
 *                         then every term's VJP through the transposed weights' planes, dotted with the probe in the same
 *                         launch; 0 runs one GEMM launch per layer and term.
 *   INF_OPT_LINE_SEARCH   read on the net whose root is solved: 0 (default, the reference's call sites: broyden(...)
 *                         without ls) / 1: broyden(..., ls=True) -- each step's size from line_search(on=True) and
 *                         scalar_search_armijo (broyden.py:24-99; quadratic then cubic backtracking, c1 1e-4, amin 1e-2),
 *                         every trial point's norm read back; stats.tnstep counts the accepted searches' iterations
 *                         (:156).  The global rule only (INF_ERR_UNSUPPORTED with INF_CONV_PER_SAMPLE); the fc block
 *                         kernel is not used with it.
 *   INF_OPT_FUSED_PRESPLIT  1 (default) / 0: the 32-pixel wide-net VJP / forward kernel (net313_kernel_w: CIFAR-10's
 *                         8x8 scale) splits each phase's B operand into its fp16 (h, l) planes once, in LDS, where it is
 *                         produced (phase A's im2col after the halo staging, phases B and C in the epilogues before
 *                         them); 0 splits it per consuming wave, as before round 6.  Bitwise the same results.
 * Unknown values of INFLOW_FUSED_K128 (0-3), INFLOW_FC_BLOCK (0/1/2), INFLOW_EVAL_OVERLAP / INFLOW_FC_SERIES (0/1) and INFLOW_CONVERGENCE (global/per_sample)
 * make inf_net_create fail with INF_ERR_INVALID.
 * FUSED_K128, EVAL_OVERLAP and K128_EXACT_SCALE are performance / test knobs without a reference counterpart (the reference
 * runs the VJP as autograd, implicit_block.py:418-426, and the two series one after the other, :300-322); results
 * agree to fp32 roundoff across their values. */
typedef enum InfNetOption {
  INF_OPT_FUSED_K128 = 1, INF_OPT_EVAL_OVERLAP = 2, INF_OPT_CONVERGENCE = 3, INF_OPT_K128_EXACT_SCALE = 4,
  INF_OPT_FC_BLOCK = 5, INF_OPT_FC_SERIES = 6, INF_OPT_LINE_SEARCH = 7, INF_OPT_FUSED_PRESPLIT = 8
} InfNetOption;
typedef enum InfConvergence { INF_CONV_GLOBAL = 0, INF_CONV_PER_SAMPLE = 1 } InfConvergence;
int inf_net_set_option(InfNet* net, int option, int value);
int inf_net_get_option(const InfNet* net, int option);
/* Workspace for any call below on a net of this shape at this batch size. */
size_t inf_workspace_bytes(const InfNet* net, int batch, int threshold);
/* y = nnet(x). */
int inf_net_forward(InfNet* net, const float* x, float* y, int batch, void* ws, size_t ws_bytes, void* stream);
/* out = v^T J_nnet(x)   (one torch.autograd.grad(g, x, v) of implicit_block.py:422). */
int inf_net_vjp(InfNet* net, const float* x, const float* v, float* out, int batch, void* ws, size_t ws_bytes,
                void* stream);

/* ---- root finding: RootFind (implicit_block.py:51-100) with broyden (broyden.py:123-193) ------ */
/* Solve out + f(out) = y + e(y) from out = 0 with Broyden (ls=False); on prot_break fall back to the
 * Banach iteration from out = y (implicit_block.py:57-65,17-28).  Forward uses (f, e) = (nnet_z, nnet_x);
 * imBlock.inverse uses (nnet_x, nnet_z) (implicit_block.py:236-243).  diff_detail (device, B floats,
 * may be NULL) receives the per-sample residual norms of the returned iterate. */
int inf_root_find(InfNet* net_f, InfNet* net_e, const float* y, float* out, int batch, int threshold, double eps,
                  InfBroydenStats* stats, float* diff_detail, void* ws, size_t ws_bytes, void* stream);
/* RootFind with method 'banach' (implicit_block.py:57-65, 83-87): x_embed = e(y) + y, then find_fixed_point
 * (:17-28) of out <- x_embed - f(out) from out = y: stop once (out - out_prev)^2 / (eps + eps |y|) < 1 everywhere
 * (INF_CONV_PER_SAMPLE on net_f: per sample), or after more than `threshold` iterations.  iters (HOST, may be
 * NULL) receives the iteration count.  ws >= inf_workspace_bytes(net_f, batch, 1). */
int inf_banach_find_root(InfNet* net_f, InfNet* net_e, const float* y, float* out, int batch, int threshold,
                         double eps, int* iters, void* ws, size_t ws_bytes, void* stream);
/* One limited-memory Broyden update for a caller-driven loop (generic broyden(g, x0, ...), broyden.py:
 * 174-181 + the next line_search step :94-99).  Tensors are (B, d) row-major; U/VT are (T, B, d).
 * nstep = iterations done so far (>= 1).  Writes update = -H gx, x_next = x + update and
 * dx_next = x_next - x.  ws >= inf_broyden_workspace_bytes(batch, d, threshold). */
size_t inf_broyden_workspace_bytes(int batch, int d, int threshold);
int inf_broyden_update(float* U, float* VT, const float* dx, const float* dg, const float* gx, const float* x,
                       float* update, float* x_next, float* dx_next, int batch, int d, int threshold, int nstep,
                       void* ws, size_t ws_bytes, void* stream);
/* The trial point of a caller-driven line search (broyden(..., ls=True), broyden.py:79,94,99): x_est = x0 + step * update
 * and dx = x_est - x0 over n floats, the product and the sum rounded separately as the reference's tensor ops do. */
int inf_broyden_line_step(const float* x0, const float* update, float step, float* x_est, float* dx, size_t n,
                          void* stream);
/* imBlock forward value: z* = RootFind(nnet_z, nnet_x, x); z = (nnet_x(x) - nnet_z(z*)) + x
 * (implicit_block.py:226-227). */
int inf_imblock_forward(InfNet* net_x, InfNet* net_z, const float* x, float* z, int batch, int threshold,
                        double eps, InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream);

/* ---- log-det estimators (implicit_block.py:245-350,418-438) --------------------------------- */
/* out[b] = sum_k coeff[k] * <(J^T)^k vareps_b, vareps_b>,  k = 1..n_terms, coeff[k-1] = (-1)^(k+1)/k * c_k
 * (coeff is a HOST array, rounded to fp32 as the reference's scalar*tensor product does). */
int inf_logdet_series(InfNet* net, const float* x, const float* vareps, const float* coeff, int n_terms,
                      float* out, int batch, void* ws, size_t ws_bytes, void* stream);
/* Both series of an imBlock (nnet_x at x, nnet_z at z; implicit_block.py:318-322) in lockstep, one
 * fused launch per term for both nets when the nets take the fused 3-1-3 path.
 * ws >= 2 * inf_workspace_bytes(net, batch, 1). */
int inf_logdet_series_pair(InfNet* net_a, const float* x_a, const float* vareps_a, InfNet* net_b, const float* x_b,
                           const float* vareps_b, const float* coeff, int n_terms, float* out_a, float* out_b,
                           int batch, void* ws, size_t ws_bytes, void* stream);
/* The whole eval pass of an imBlock whose two nets take the fused path (implicit_block.py:220-234 and the
 * eval branch of 245-322): root solve, z = (f_x(x) - f_z(z*)) + x, and both power series with probes
 * eps_x / eps_z and coeff[k-1] = (-1)^(k+1)/k coeff_fn(k); logdet_x[b], logdet_z[b] receive the two
 * series (the block's log-det is their difference).  The x_embed pass also saves f_x's derivatives, so
 * only the z-net needs its own.  INF_ERR_UNSUPPORTED when a net is not fused (use the separate calls).
 * ws >= inf_workspace_bytes(net_x, batch, threshold) + inf_workspace_bytes(net_z, batch, 1).  With a further
 * inf_workspace_bytes(net_x, batch, 1) the x-branch series runs on an internal side stream concurrently with
 * the root solve and the z-branch series (joined into `stream` before return) when net_x's INF_OPT_EVAL_OVERLAP is 1
 * (the default). */
int inf_imblock_eval(InfNet* net_x, InfNet* net_z, const float* x, float* z, const float* eps_x, const float* eps_z,
                     const float* coeff, int n_terms, float* logdet_x, float* logdet_z, int batch, int threshold,
                     double eps, InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream);
/* The whole eval pass of an imBlock on fc nets with d <= 10 (the tabular / toy configs; implicit_block.py:220-234
 * with the exact branch of 245-260, 358-362): log|det(I + J_fx(x))| into logdet_x, the root solve,
 * z = (f_x(x) - f_z(z*)) + x, and log|det(I + J_fz(z))| into logdet_z (the block's log-det is their difference).
 * x, z are (batch, d).  Every net evaluation and both Jacobian log-dets are single launches of the fused fc
 * kernel (fcnet.hip); the x-branch log-det is enqueued ahead of the root solve, so the GPU works on it while the
 * host waits for the solver's residual norms.  INF_ERR_UNSUPPORTED when a net is not on the fused fc path (use the
 * separate calls).  ws >= inf_workspace_bytes(net_z, batch, threshold). */
int inf_imblock_eval_exact(InfNet* net_x, InfNet* net_z, const float* x, float* z, float* logdet_x, float* logdet_z,
                           int batch, int threshold, double eps, InfBroydenStats* stats, void* ws, size_t ws_bytes,
                           void* stream);
/* A SequentialFlow of such fc imBlocks in eval (train_tabular.py:314-336, container.py:12-20) in one call: block i runs
 * inf_imblock_eval_exact on block i-1's z (block 0 on x) and the log-density step logp <- logp - (logdet_x - logdet_z)
 * on the device (implicit_block.py:234; logp_in NULL: 0), writing the last block's z and the final logp (batch).  No
 * host round trip between blocks beyond a block's own.  thresholds / eps: per block; stats: n_blocks entries or NULL.
 * With f16x3 nets on the launch path, block i's z-branch log-det launch also evaluates block i+1's x-branch (log-det
 * and x_embed at the same z): one grid for the two Jacobians; results identical to the blocks called one by one.
 * INF_ERR_UNSUPPORTED (before any launch) when a block is not on the fused fc path; INF_ERR_INVALID when x == z or
 * logp_in == logp_out (the step is not in place here: a re-queued z-branch launch would apply it twice).
 * ws >= inf_flow_chain_workspace_bytes(net_z, n_blocks, batch, thresholds). */
size_t inf_flow_chain_workspace_bytes(InfNet* const* net_z, int n_blocks, int batch, const int* thresholds);
int inf_flow_eval_exact_chain(InfNet* const* net_x, InfNet* const* net_z, int n_blocks, const float* x, float* z,
                              const float* logp_in, float* logp_out, int batch, const int* thresholds,
                              const double* eps, InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream);
/* Neumann gradient surrogate value (implicit_block.py:429-438): w = sum_{k=0}^{n} ncoeff[k] (J^T)^k eps,
 * out[b] = <J^T w, eps>.  ncoeff is a HOST array of n_terms+1 values ((-1)^k c_k, ncoeff[0] = 1). */
int inf_logdet_neumann(InfNet* net, const float* x, const float* vareps, const float* ncoeff, int n_terms,
                       float* out, int batch, void* ws, size_t ws_bytes, void* stream);
/* The Neumann vector itself, w = vareps + sum_{k=1..n} ncoeff[k] vareps^T J^k (neumann_vjp,
 * implicit_block.py:430-436), for the training surrogate's gradient. */
int inf_neumann_vector(InfNet* net, const float* x, const float* vareps, const float* ncoeff, int n_terms, float* w,
                       int batch, void* ws, size_t ws_bytes, void* stream);
/* Both Neumann vectors of an imBlock (x-branch at x with eps_a, z-branch at z with eps_b) in lockstep: one
 * fused VJP launch per term for both nets.  ws >= 2 x inf_workspace_bytes(net, batch, 1). */
int inf_neumann_vector_pair(InfNet* net_a, const float* x_a, const float* vareps_a, InfNet* net_b, const float* x_b,
                            const float* vareps_b, const float* ncoeff, int n_terms, float* w_a, float* w_b,
                            int batch, void* ws, size_t ws_bytes, void* stream);
/* Exact log|det(I + J_nnet(x))| for fc nets with d <= 16 (implicit_block.py:249-260,358-362). */
int inf_logdet_exact(InfNet* net, const float* x, float* out, int batch, void* ws, size_t ws_bytes, void* stream);
/* Implicit backward of an imBlock (imBlock.Backward, implicit_block.py:165-217): given dL/dz = grad, solve
 * dl_dh (I + J_fz(z)) = grad by Broyden from 0 (eps = eps_backward, threshold; lowest iterate), then
 * dl_dx = dl_dh (I + J_fx(x)).  dl_dh is the gradient into z's recompute graph, dl_dx into x.
 * ws >= max(inf_workspace_bytes(net_z, batch, threshold), inf_workspace_bytes(net_x, batch, 1)). */
int inf_imblock_backward(InfNet* net_x, InfNet* net_z, const float* z, const float* x, const float* grad,
                         float* dl_dh, float* dl_dx, int batch, int threshold, double eps, InfBroydenStats* stats,
                         void* ws, size_t ws_bytes, void* stream);
/* Power series with the exact trace, exact_trace=True (implicit_block.py:323-343, iresblock.py:150-157):
 * J = d nnet / dx by forward mode, out[b] = tr(J) + sum_{k=2..n} coeff[k-1] tr(J^k).  fc nets, d <= 16.
 * coeff is a HOST array of n_terms values ((-1)^(k+1)/k coeff_fn(k); coeff[0] is ignored). */
int inf_logdet_exact_trace(InfNet* net, const float* x, const float* coeff, int n_terms, float* out, int batch,
                           void* ws, size_t ws_bytes, void* stream);

/* ---- flow glue (elemwise.py:112-128, act_norm.py:153-193, squeeze.py:242-255,
 *      train_img.py:135-137,543-549) ---------------------------------------------------------- */
/* y = logit(alpha + (1-2alpha) x); logp_out[b] = logp_in[b] - sum(-log(s - s^2) + log(1-2alpha)). */
int inf_logit_forward(const float* x, float* y, const float* logp_in, float* logp_out, int batch, int per_sample,
                      float alpha, void* stream);
/* y = (x + bias_c) * exp(weight_c); logp_out = logp_in - hw * sum_c weight_c. */
int inf_actnorm_forward(const float* x, float* y, const float* weight, const float* bias, const float* logp_in,
                        float* logp_out, int batch, int channels, int hw, void* stream);
/* space-to-depth by 2: (B,C,H,W) -> (B,4C,H/2,W/2), the reference's permute(0,1,3,5,2,4). */
int inf_squeeze2(const float* x, float* y, int batch, int channels, int height, int width, void* stream);
/* out[b] = sum_i (-0.5 log(2 pi) - z_i^2 / 2)  (standard_normal_logprob(z).sum(1)). */
int inf_normal_logprob(const float* z, float* out, int batch, int per_sample, void* stream);
/* Rademacher +-1 probes from a counter-based generator (device RNG mode; the reference-replay mode
 * draws probes on the host, implicit_block.py:297-298). */
int inf_rademacher(float* out, size_t n, uint64_t seed, uint64_t offset, void* stream);

/* ---- measurement: opt-in per-launch timing with HIP events (off by default).  A session is per host thread:
 * it records the launches made by the thread that called inf_profile_begin. ---- */
typedef struct InfKernelStat {
  int tag;          /* kernel instantiation id ("Kernel tags") */
  int launches;
  double total_ms;  /* sum of event-measured launch durations */
  double flops;     /* algorithmic FLOPs of those launches */
  double bytes;     /* algorithmic bytes of those launches */
  double peak_ms;   /* time those launches' MFMA instructions take at the dense matrix peak of their type
                       (f32 157.3 TF; bf16 / f16 2516.6 TF, MI355X_MICROARCH.md): peak_ms / total_ms is the
                       MFMA-pipe fraction, flops / peak_ms the fp32-equivalent peak of the arithmetic used */
} InfKernelStat;
int inf_profile_begin(int max_launches);
int inf_profile_end(InfKernelStat* out, int max_out, int* n_out);

/* ---- Lipschitz power iteration: compute_weight(update=True) of InducedNormConv2d / InducedNormLinear,
 *      spectral (2 -> 2) case (mixed_lipschitz.py:85-124 linear, :276-326 1x1 conv, :328-386 k x k conv;
 *      called by update_lipschitz, train_img.py:786-792) -------------------------------------------- */
typedef struct InfPowerIterDesc {
  int kind;              /* INF_LAYER_CONV or INF_LAYER_LINEAR */
  int cin, cout, ksize;  /* conv: stride 1, padding ksize/2; linear: ksize ignored */
  int height, width;     /* k x k conv: spatial_dims, the (H, W) that u (cout*H*W) and v (cin*H*W) live on */
  const float* weight;   /* raw weight (cout, cin, k, k) / (cout, cin) */
  float* u;              /* module buffers, updated in place (u <- W v / |W v|, v <- W^T u / |W^T u|) */
  float* v;
  float* scale;          /* receives sigma = u . (W v) (the module's `scale` buffer); may be NULL */
} InfPowerIterDesc;
size_t inf_power_iteration_workspace_bytes(const InfPowerIterDesc* desc);
/* Up to max_iters iterations; with use_tol, stop once |du|/sqrt(n_u) < atol + rtol max(u) and the same for
 * v.  iters_used (may be NULL) receives the count. */
int inf_power_iteration(const InfPowerIterDesc* desc, int max_iters, int use_tol, float atol, float rtol,
                        int* iters_used, void* ws, size_t ws_bytes, void* stream);
/* The same for n layers in one call (update_lipschitz over a model, train_img.py:786-792): per-layer
 * iterations and stopping rule unchanged; all unfinished layers advance one speculative chunk between
 * the host's flag reads.  iters_used (may be NULL) receives n counts. */
size_t inf_power_iteration_batch_workspace_bytes(const InfPowerIterDesc* descs, int n);
int inf_power_iteration_batch(const InfPowerIterDesc* descs, int n, int max_iters, int use_tol, float atol,
                              float rtol, int* iters_used, void* ws, size_t ws_bytes, void* stream);

/* ---- parameter gradients (training path; conv nets with swish activations) ------------------------
 * Device buffers per weight layer l (in order; NULL entries / arrays are skipped): dW[l] the gradient of
 * the RAW weight (through W / max(1, u.(W v) / coeff), mixed_lipschitz.py:378-385), db[l] the bias,
 * dbeta[l] the beta of the swish applied after layer l (NULL for the last layer); dpre_beta the
 * preact swish.  Buffers are overwritten. */
typedef struct InfNetGrads {
  float** dW;
  float** db;
  float** dbeta;
  float* dpre_beta;
} InfNetGrads;
size_t inf_grad_workspace_bytes(InfNet* net, int batch);
/* d/dtheta sum(gout * nnet(x)) and d/dx (gx may be NULL): the recompute graph's backward
 * (z = f_x(x0) - f_z(z*) + x0, implicit_block.py:226-227).  Conv nets with Swish; fc nets with Swish / Sin (x, gout,
 * gx in the (B, d) boundary layout). */
int inf_net_param_grad(InfNet* net, const float* x, const float* gout, float* gx, const InfNetGrads* grads,
                       int batch, void* ws, size_t ws_bytes, void* stream);
/* s_b = w_b^T J(x_b) eps_b (w fixed): value[b] (may be NULL) and d/dx, d/dtheta of sum_b s_b -- the
 * memory-efficient Neumann estimator's surrogate and its gradients (implicit_block.py:388-394,437-438).  fc nets:
 * (B, d) boundary layout, value must be NULL. */
int inf_net_surrogate_grad(InfNet* net, const float* x, const float* w, const float* eps, float* value, float* gx,
                           const InfNetGrads* grads, int batch, void* ws, size_t ws_bytes, void* stream);

/* ---- test support: fill the LDS of every CU with NaN (queued on `stream`), so a kernel that reads
 * LDS it never wrote fails deterministically instead of depending on what earlier kernels left. ---- */
int inf_debug_poison_lds(void* stream);
/* ---- test support: the readback contract.  The engine's host-read events (Broyden norm slots, the fc block kernel's
 * statistics) are created without the system-scope fence (hipEventDisableSystemFence: a fenced event idles the GPU and
 * cold-starts L2 after every readback); what the host reads behind them lives in coherent pinned memory that
 * a kernel writes directly (the launch completing the event) or a D2H copy fills.  This runs `iters` rounds of both
 * forms on `stream` with fresh values of n doubles each round, the host waiting exactly as the Broyden loop does, and
 * returns the number of stale values the host saw (0 when the contract holds), or a negative status. ---- */
int inf_debug_readback_check(int iters, int n, void* stream);

/* Gradients of the log-det estimators of an fc net (the training path of train_tabular.py / train_toy.py: the basic
 * power series with create_graph, implicit_block.py:418-426; the brute-force log|det(I + J)|, :249-260; the exact-trace
 * series, :323-343): sum_b gout[b] S_b(x_b) differentiated into every parameter (grads, as inf_net_param_grad) and x
 * (gx, (B, d), nullable); value (B, nullable) receives S_b.  mode:
 *   INF_LOGDET_SERIES  S_b = sum_k coeff[k-1] eps_b^T J^k eps_b, k = 1..n_terms (coeff[k-1] = (-1)^(k+1)/k coeff_fn(k));
 *   INF_LOGDET_EXACT   S_b = log|det(I + J(x_b))| (eps, coeff, n_terms unused);
 *   INF_LOGDET_TRACE   S_b = sum_k coeff[k-1] tr(J^k) (coeff[0] = 1: the bare trace).
 * x, eps (B, d) boundary layout; coeff a host array.  fc nets with Swish / Sin, d <= 16.
 * ws >= inf_logdet_grad_workspace_bytes(net, batch, mode, n_terms). */
typedef enum InfLogdetMode { INF_LOGDET_SERIES = 0, INF_LOGDET_EXACT = 1, INF_LOGDET_TRACE = 2 } InfLogdetMode;
size_t inf_logdet_grad_workspace_bytes(InfNet* net, int batch, int mode, int n_terms);
int inf_logdet_grad(InfNet* net, const float* x, int mode, const float* eps, const float* coeff, int n_terms,
                    const float* gout, float* value, float* gx, const InfNetGrads* grads, int batch, void* ws,
                    size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* INFLOW_H */
