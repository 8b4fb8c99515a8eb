// Internal kernel launch interfaces (host side) for libinflow.
#pragma once
#include "common.h"

namespace inf {

// ------------------------------------------------------------------------------------------
// GEMM:  out[b][m][p] = epi( sum_k A[m][k] * Bop[k][n] ),  n = b * P + p
//   A: (Mpad, Kpad) row-major, zero padded (Mpad multiple of 128, Kpad multiple of 16)
//   Bop from X by one of the loaders below.  f32 in / f32 accumulate (v_mfma_f32_32x32x2_f32).
// ------------------------------------------------------------------------------------------
enum BLoad { BL_DIRECT = 0, BL_IM2COL3 = 1 };
enum Epi { EP_STORE = 0, EP_BIAS = 1, EP_BIAS_ACT = 2, EP_MUL_DERIV = 3, EP_BIAS_PRIMAL = 4,
           // compile-time activation variants of EP_BIAS_ACT (selected by launch_gemm from GemmArgs::act)
           EP_ACT_SWISH = 5, EP_ACT_SIN = 6, EP_ACT_NONE = 7 };

struct GemmArgs {
  const float* A;
  int M, Kpad, Ktot;
  const float* X;         // B-operand source (NCHW; DIRECT: (B, K, P); IM2COL3: (B, Cin, H, W))
  long x_sample;          // sample stride of X in elements
  int P;                  // pixels (columns) per sample
  int N;                  // total columns
  int H, W;               // IM2COL3 geometry (P = H * W)
  const float* pre_beta;  // loader applies swish(., softplus(*pre_beta)) to X when non-null
  float* out;
  long o_sample;          // output sample stride (channel stride is P)
  const float* bias;
  int act;                // Act for EP_BIAS_ACT
  const float* act_beta;  // swish beta
  float* deriv_out;       // EP_BIAS_ACT: act'(a) saved here when non-null
  int write_out;          // EP_BIAS_ACT: write act(a)
  const float* deriv_in;  // EP_MUL_DERIV multiplier (same indexing as out)
  int n_primal;           // EP_BIAS_PRIMAL: columns n < n_primal get the bias
  int x6;                 // 1: split-bf16 MFMA (both operands split exactly into 3 bf16 pieces, common.h)
};
int launch_gemm(const GemmArgs& g, int bload, int epi, hipStream_t s);

// ------------------------------------------------------------------------------------------
// Output stage of a conv net whose last layer produced packed taps Y[b][c*9+t][p] (ks = 3) or
// plain rows Y[b][c][p] (ks = 1): s = sum_t Y[..][shift_t(p)], then a fused epilogue.
// ------------------------------------------------------------------------------------------
enum OutMode { OM_PLAIN = 0, OM_EMBED = 1, OM_RESID = 2, OM_RECOMP = 3, OM_VJP = 4 };
struct OutArgs {
  const float* Y;
  long y_sample;
  int C, H, W, ks;
  int mode;
  const float* bias;
  const float* in0;
  const float* in1;
  const float* in2;
  float* out0;
  float* out1;
  float* out2;            // OM_RESID (optional): the net output f(z) itself
  const float* pre_beta;  // OM_VJP: multiply by swish'(in1) (preact input derivative)
  double* partial;        // (B, nchunk) per-sample partial sums (OM_RESID: g^2, OM_VJP: v.eps)
  int nchunk;
  int sample_sums;        // OM_RESID, conv nets: one block per sample writes the sample's total to partial[b] (the chunk
                          // partials summed in chunk order, as launch_reduce_partials does: the same bits)
  // host side (not read by the kernels): an event for the launch itself to complete (hipExtLaunchKernel's stop event:
  // no marker packet after it), and the flag the launcher sets when it bound it (fc readbacks, engine.hip enqueue_sumsq)
  hipEvent_t stop_ev = nullptr;
  bool* stop_bound = nullptr;
};
int out_nchunk(int per_sample);
int launch_conv_out(const OutArgs& a, int batch, hipStream_t s);

// fc nets: feature-major (d, B) tensors, one thread per sample for the per-sample reductions.
int launch_fc_out(const OutArgs& a, int batch, hipStream_t s);

// ------------------------------------------------------------------------------------------
// misc elementwise / layout
// ------------------------------------------------------------------------------------------
int launch_transpose(const float* x, float* y, int rows, int cols, hipStream_t s);  // y[c][r] = x[r][c]
int launch_axpy_step(const float* x, const float* upd, float* xnew, float* dx, long n, hipStream_t s);
int launch_neg(const float* x, float* y, long n, hipStream_t s);
// x_est = x0 + sc * upd, dx = x_est - x0 (the line search's trial point; product and sum rounded separately)
int launch_line_step(const float* x, const float* upd, float sc, float* xnew, float* dx, long n, hipStream_t s);
// stop_ev (optional): an event the launch itself completes (hipExtLaunchKernel; not while profiling), *stop_bound set
int launch_reduce_partials(const double* partial, int batch, int nchunk, double* out, hipStream_t s,
                           hipEvent_t stop_ev = nullptr, bool* stop_bound = nullptr);

// ------------------------------------------------------------------------------------------
// Broyden low-rank algebra (broyden.py:101-120,174-181), per-sample, layout-generic:
//   element i of sample b lives at b * sb + i * si;  U/VT column j of sample b at
//   j * cs + b * sb + i * si  (cs = column stride).
// ------------------------------------------------------------------------------------------
struct BroydenArgs {
  int batch, d, T;
  long sb, si, cs;
  float* U;
  float* VT;
  const float* dx;
  const float* dg;
  const float* gx;
  const float* x;
  float* xnew;
  float* dxnew;
  float* upd;
  double* part;   // scratch partials
  int m;          // existing columns (nstep - 1) % T
  int ncols;      // columns used by the update (min(nstep, T))
  const int* active;   // per-sample mode (nullable): stopped samples keep x (xnew = x) and their U / VT columns
};
int launch_broyden_update(const BroydenArgs& a, hipStream_t s);

// per-sample convergence (INF_CONV_PER_SAMPLE, pointwise.hip): the stopping rules of broyden.py:153-172 per sample
constexpr int PS_HEAD = 8;   // doubles of per-sample state before the objective ring
// ss: B per-sample sums of squares (+1: receives the number of samples still iterating); k = step (0: initial)
int launch_ps_decide(double* ss, double* state, int* active, int* improved, int B, int k, int T, double eps,
                     hipStream_t s);
int launch_ps_copy(const int* improved, const float* x, const float* f, float* lowx, float* lowf, int B, int d, long sb,
                   long si, hipStream_t s);
int launch_ps_fixed_point(const float* x, const float* xp, const float* y, float* result, int* todo, int B, int d,
                          long sb, long si, float eps, int force, hipStream_t s);

// Spectral scale: sigma = u . (W v) for conv (pad k//2) or matrix; factor = max(1, sigma / coeff)
constexpr int SIGMA_MAX_PARTS = 4096;   // launch_sigma's partial count bound when it splits channels
int launch_sigma(const float* W, const float* u, const float* v, int cout, int cin, int ks, int H, int Wd,
                 float coeff, float* factor_out, float* scratch, hipStream_t s);
// Packed operand:  dst[(mrow)][kcol] built from W / factor with the given pack mode.
enum PackMode { PK_ROWMAJOR = 0, PK_TRANSPOSE = 1, PK_IM2COL_FWD = 2, PK_IM2COL_BWD = 3, PK_TAPS_FWD = 4,
                PK_TAPS_BWD = 5 };
// frag = 1 writes the fragment-major layout of fused313.hip (Mpad multiple of 32, Kpad of 16).
int launch_pack(const float* W, const float* factor, float* dst, int cout, int cin, int ks, int Mpad, int Kpad,
                int mode, hipStream_t s, int frag = 0);
// Split a fragment-major fp32 operand (n = Mpad * Kpad floats) into three bf16 planes per 512-float
// fragment tile: dst[(tile * 3 + plane) * 512 + w] (fused313.hip split phase B).
int launch_split3(const float* src, uint16_t* dst, long n, hipStream_t s);
// Scale exponent of a whole operand (*exp_out = h3_scale_exp(max |src|), common.h) and its two scaled fp16
// planes per 512-float fragment tile: dst[(tile * 2 + plane) * 512 + w] (fused313.hip phase B, F16X3).
int launch_split2h(const float* src, uint16_t* dst, long n, int* exp_out, hipStream_t s);
// Copy of fragment-major fp16 planes (launch_split2h layout, ntiles fragment tiles of 2 x 512 halves) with the k index
// of every 32x16 fragment tile permuted: slot (lane (i, h), 4a + q) <- slot (lane (i, a), 4h + q), i.e. k bits 2, 3 swapped
int launch_permute_k23(const uint16_t* src, uint16_t* dst, long ntiles, hipStream_t s);

// exact small log-det per sample: J[b] = I + T[b] with T stored tangents (d, d, B) feature-major
int launch_logdet_small(const float* tang, float* out, int d, int batch, long stride_j, hipStream_t s);
// the log-det estimators' gradients as stacked (A, b) pairs at x (pointwise.hip logdet_pairs_kernel; fc nets, d <= 16)
enum { LOGDET_SERIES = 0, LOGDET_EXACT = 1, LOGDET_TRACE = 2 };
int launch_logdet_pairs(int mode, const float* tang, const float* eps, const float* x, const float* gout,
                        const float* coeff_host, int n_terms, int d, int batch, float* A, float* bv, float* xr,
                        float* value, float* a_scr, hipStream_t s);
int launch_sum_pairs(const float* gs, int T, int d, int batch, float* gx, hipStream_t s);
// sample_sums: one block per sample, partial[b] = the sample's total (conv_out's OutArgs::sample_sums); stop_ev: the
// launch completes it (hipExtLaunchKernel, not while profiling), *stop_bound set
int launch_resid_bcast(const float* f0, const float* xemb, const float* z, float* g, float* fcur, double* partial,
                       int batch, int per, int nchunk, hipStream_t s, int sample_sums = 0, hipEvent_t stop_ev = nullptr,
                       bool* stop_bound = nullptr);
// conv layout, per-sample sums (d <= 4 OUT_CH chunks): x0 = 0, the residual at it, update = -g0, x1 = x0 + update,
// dx = x1 - x0 in one launch, one block per sample, partial[b] the sample's sum of squares
int launch_broyden_start_sample(const float* f0, const float* xemb, float* x0, float* g, float* fcur, double* partial,
                                hipEvent_t stop_ev, bool* stop_bound, float* upd, float* x1, float* dx, int batch,
                                int per, hipStream_t s);
// fc layout (d, B): f0 holds d values
int launch_resid_bcast_fc(const float* f0, const float* xemb, const float* z, float* g, float* fcur, double* partial,
                          int batch, int d, hipStream_t s);
// x0 = 0, the residual at it, update = -g0, x1 = x0 + update, dx = x1 - x0 in one launch (fc layout)
int launch_broyden_start_fc(const float* f0, const float* xemb, float* x0, float* g, float* fcur, double* partial,
                            hipEvent_t stop_ev, bool* stop_bound, float* upd, float* x1, float* dx, int batch, int d, hipStream_t s);
int launch_vjp_resid(const float* v, const float* y, const float* grad, const float* gprev, float* g, float* dg,
                     double* partial, int batch, int d, int nchunk, int fc, hipStream_t s);
int launch_trace_series(const float* tang, const float* coeff, int n_terms, float* out, int d, int batch,
                        long stride_j, hipStream_t s);
int launch_fwdmode_act(float* a, float* deriv, int d_out, int batch, int ntang, int act, const float* beta,
                       hipStream_t s);

int launch_series_combine(const double* partials, const float* coeff_dev, int n_terms, int batch, int nchunk,
                          float* out, hipStream_t s);

// ------------------------------------------------------------------------------------------
// fused 3-1-3 conv net (fused313.hip): one launch per forward / derivative-saving forward / VJP
// ------------------------------------------------------------------------------------------
enum Net313Mode { MODE_EVAL = 0, MODE_SAVE = 1, MODE_VJP = 2, MODE_EVALSAVE = 3 };
struct Net313Args {
  const float* in;        // (B, C, H, W): x (forward) or v (VJP)
  const float* pre_beta;  // forward: swish preact on `in` (nullptr: none)
  const float* A1;        // phase A operand, fragment-major (HID x K1pad)
  int K1pad;
  const float* A2;        // phase B operand, fragment-major (HID x HID)
  const float* A3;        // phase C operand, fragment-major (M3pad x HID)
  // A1s / A2s / A3s: the same operands split into three bf16 planes (hi, mid, lo; exact: hi + mid + lo
  // equals the fp32 value), fragment-major per (row block, K tile, plane); non-null selects the
  // split-bf16 ("x6") MFMA path of fused313.hip for all three phases
  const void* A1s;
  const void* A2s;
  const void* A3s;
  // A1h / A2h / A3h: the operands as two scaled fp16 planes (h, l) per fragment tile, scales 2^Ah_exp[0..2]
  // (common.h split2h); non-null (with A1s..A3s) selects INF_MFMA_F16X3 (h3 in phase B, and in A / C with H3_AC)
  const void* A1h;
  const void* A2h;
  const void* A3h;
  const int* Ah_exp;
  const void* A3p;        // A3h with the k index's bits 2 and 3 swapped inside every 16-k tile (launch_permute_k23):
                          // phase C of the 128-pixel kernel takes its B operand straight from the phase-B accumulators
  int M3, M3pad;          // 9C taps rows
  const float* b1;
  const float* beta1;
  const float* b2;
  const float* beta2;
  float* d1;              // swish'(a1), B*HID*H*W floats in MFMA-fragment order (fused313.hip dfrag)
  float* d2;              // swish'(a2), same layout
  float* Y;               // (B, M3, H, W) packed taps
  int B, C, H, W, seg;
  // VJP series chaining (conv_out folded into the next term's halo staging):
  const float* in_taps;   // non-null: the input v is the previous term's packed taps (B, M3, H, W),
                          // v = sum of the 9 shifted taps (zero padded), replaces `in`
  const float* vmul_x;    // with in_taps on preact nets: v *= swish'(vmul_x) (beta vmul_beta)
  const float* vmul_beta;
  const float* dot_eps;   // with in_taps: dot_part[img * dot_nchunk + tile] = sum over the tile's own
  double* dot_part;       //   pixels of v * dot_eps (fp64), the previous term's trace partial
  int dot_nchunk;
  float* acc_w;           // with in_taps: acc_w[img, own pixels] += acc_coef * v (Neumann vector accumulation,
  float acc_coef;         //   implicit_block.py:430-436), v the previous term's VJP after the tap sum
  int k128;               // tile policy of the net (INF_OPT_FUSED_K128): 0 64-px only, 1 128-px where the grid
                          //   covers every CU, 2 128-px wherever it fits; a pair launch follows args[0]
  int tile_order;         // 1: the 128-pixel kernel walks the tiles backwards (series terms alternate; args[0])
  int presplit;           // INF_OPT_FUSED_PRESPLIT: the wide 32-pixel kernel's B operands split once in LDS (args[0])
  int exact_scale;        // INF_OPT_K128_EXACT_SCALE: chunk 1's exact-scale path on every tile (args[0]; tests)
};
struct Net313Pair {
  Net313Args a[2];
  int nb0;                // workgroups of net 0; blocks >= nb0 run net 1
  int max_ksplit;         // cap on phase C's K split (8)
  unsigned long long* tbuf;   // INFLOW_PHASE_STAMPS builds only: per-workgroup s_memtime stamps at phase boundaries
  int dbg;                // bit 16: the 128-pixel kernel's chunk-1 exact-scale path on every tile (results unchanged);
                          // bit 32: the wide 32-pixel kernel splits its B operands per consuming wave (no pre-split)
  int reverse;            // 128-pixel kernel: workgroup i runs tile nb - 1 - i (alternating series terms)
  int xcd;                // two nets, 8 | grid: blocks b with (b & 7) < 4 run net 0, the others net 1 (blocks b and
                          // b + 8 share an XCD, MI355X_MICROARCH.md), so each XCD's L2 holds one net's weight planes
};
// (net, tile) of a pair launch's workgroup `bx` (after any reversal); speed-only placement, results do not depend on it
__device__ __forceinline__ int pair_tile(const Net313Pair& pr, int bx, int& sel) {
  if (pr.xcd) {
    sel = (bx & 7) >> 2;
    return (bx >> 3) * 4 + (bx & 3);
  }
  sel = bx >= pr.nb0 ? 1 : 0;
  return bx - (sel ? pr.nb0 : 0);
}
int net313_supported(int hid, int C, int H, int W);
// 128-pixel K-chunked variant (fused313k.hip, INF_MFMA_F16X3 only): MODE_VJP and MODE_EVAL
int net313k_fits(int hid, int C, int H, int W);
int launch_net313k(const Net313Pair& pr, int mode, unsigned nb, hipStream_t s);
// two-per-CU 64-pixel VJP (fused313p.hip, INF_MFMA_F16X3, MODE_VJP)
int net313p_fits(int hid, int C, int H, int W);
int launch_net313p(const Net313Pair& pr, unsigned nb, hipStream_t s);
int launch_net313(const Net313Args& a, int hid, int mode, hipStream_t s);
// layout_nets (> 0) picks the tile variant as if that many nets shared the grid: launches that write
// derivatives for a paired series must use the pair's variant (the d1/d2 layout depends on it)
int launch_net313_multi(const Net313Args* args, int nnets, int hid, int mode, hipStream_t s, int layout_nets = 0);

// ------------------------------------------------------------------------------------------
// fused fc net (fcnet.hip): the tabular / toy nets, one launch per evaluation
// ------------------------------------------------------------------------------------------
constexpr int FC_MAXL = 8;
struct FcLayer {
  const float* A;         // the layer's forward operand, row-major (Mpad, Kpad) (Lipschitz-normalised W)
  const uint16_t* Ah;     // the same as scaled fp16 (h, l) fragment planes (launch_fc_split_h3), or null: exact fp32
  const int* Aexp;        // their scale exponent
  int Kpad;
  const float* b;         // bias
  const float* beta;      // swish beta (hidden layers of Swish nets)
};
struct FcArgs {
  int nl, d, B, act;      // layers, features, batch, Act of the hidden layers
  FcLayer L[FC_MAXL];
  const float* x;         // (d, B) feature-major input
  OutArgs o;              // FWD: fc_out's epilogue (o.Y unused: the net output stays in LDS); JAC: o.out0 set -> the
                          // primal column's OM_EMBED outputs (out0 = f(x), out1 = f(x) + in0)
  float* logdet;          // JAC (optional): log|det(I + J_f(x))| per sample
  float* tang;            // JAC (optional): (d, (d + 1) B) = [f(x) | df/dx_1 | ...], fc_jacobian's layout
  // FWD with br_on: the Broyden update br (broyden_small_kernel's algebra, feature-major sb = 1, si = B) runs first
  // for the workgroup's samples and its x_new is the net input (x unused); OM_RESID's in1 (= x_new) and in2 (= br.gx)
  // then come from registers
  int br_on;
  BroydenArgs br;
  // JAC with rc_fx set: the input is z = (rc_fx - rc_fz) + rc_x (glue.hip recomp_kernel, (d, B) layout), also written to
  // rc_out in the boundary layout (B, d)
  const float* rc_fx;
  const float* rc_fz;
  const float* rc_x;
  float* rc_out;
  // JAC with x_bnd set: the input is read in the boundary layout (B, d) and also written to x_int in the internal
  // layout (d, B) (the transpose launch folded into the staging)
  const float* x_bnd;
  float* x_int;
  // JAC with logdet and lp_out set (the z-branch log-det of a chained block): also the block's log-density step
  // lp_out = lp_in - (lp_ldx - logdet) (glue.hip logp_step_kernel's expression; lp_in null: 0), implicit_block.py:234
  const float* lp_in;
  const float* lp_ldx;
  float* lp_out;
  // JAC of Sin nets on the f16x3 kernels: every layer's Lipschitz cap coeff <= 1, so the tangent columns stay in [-1, 1]
  // and take one fixed scale (fcnet_h3.hip); else per-column maxima
  int tan_fixed;
};
int fcnet_supported(const FcArgs& a, bool jac);
int launch_fcnet(const FcArgs& a, bool jac, hipStream_t s);
// two JAC launches in one grid (f16x3 nets of one shape and activation, e.g. block k's z-branch log-det and block k + 1's
// x-branch log-det + x_embed at the same input): INF_ERR_UNSUPPORTED unless both have f16x3 planes and kernels
struct FcPair {
  FcArgs a[2];
  int nb0;                // workgroups of a[0]
};
int launch_fcnet_jac_pair(const FcArgs& a0, const FcArgs& a1, hipStream_t s);
// the f16x3 kernels (fcnet_h3.hip; launch_fcnet dispatches there when a.L[0].Ah is set)
int launch_fcnet_h3(const FcArgs& a, bool jac, hipStream_t s);
int launch_fcnet_h3_jac_pair(const FcArgs& a0, const FcArgs& a1, hipStream_t s);
// fc weight planes for the f16x3 kernels: the packed (M rows used, Kpad) fp32 operand -> nrt x nks fragment tiles of
// 16 rows x 32 k, two scaled fp16 planes each, *exp_out = h3_scale_exp(max |A|)
int launch_fc_split_h3(const float* A, int M, int Kpad, int nrt, int nks, uint16_t* dst, int* exp_out, hipStream_t s);
// *exp_out = h3_scale_exp(max |src|) (pointwise.hip)
int launch_amax_exp(const float* src, long n, int* exp_out, hipStream_t s);

// one launch per fused fc imBlock evaluation (fcblock.hip): x-branch log-det and x_embed, the Broyden root solve with its
// state in LDS (global rule: one tagged fp64 partial per workgroup and iteration; per-sample rule: no exchange), the z
// recompute and the z-branch log-det
struct FcBlockStats {     // global rule (written by workgroup 0)
  int nstep, lowest_step, prot_break, n_trace;
  double lowest;
  double trace[64];
};
struct FcBlockArgs {
  FcArgs nx, nz;          // the two nets (f16x3 planes); their x / o / br fields are unused
  int B, T, per_sample;
  double eps, eps_ps;     // eps sqrt(B d) (global rule), eps sqrt(d) (per sample)
  const float* x;         // (B, d) boundary layout
  float* z;               // (B, d)
  float* logdet_x;        // (B)
  float* logdet_z;        // (B)
  // internal (d, B) copies for the host's Banach fallback: x, f_x(x), x_embed, the lowest iterate and its f
  float *xin_g, *fx_g, *xemb_g, *lowx_g, *lowf_g;
  unsigned long long* gran;   // 4 sets x grid x 2 granules, zeroed before the launch (with the error word and counter)
  unsigned tag0;              // tag of iteration 0 (> 0); iteration k uses tag0 + k
  FcBlockStats* stats;
  int *s_nstep, *s_lstep, *s_prot;   // per-sample rule: per sample (B)
  double* s_lowest;
  unsigned* error;            // [0] set when a spin timed out, [1] the exchange's arrival counter
  unsigned long long* tbuf;   // phase stamps (INFLOW_PHASE_STAMPS builds), else null
};
int fcblock_supported(const FcBlockArgs& a);
int fcblock_grid(int B);
size_t fcblock_lds_bytes(int d, int T);
// INF_ERR_UNSUPPORTED when the configuration has no kernel or (global rule) the grid cannot be co-resident
int launch_fcblock(const FcBlockArgs& a, hipStream_t s);

// the power-series log-det of fused fc nets in one launch (fcblock.hip fcseries_kernel; basic_logdet_estimator,
// implicit_block.py:418-426): per workgroup of 48 samples, one forward pass keeping act' in registers, then the n_terms
// VJPs v <- v^T J through the transposed net's planes, each dotted with the probe and combined like
// launch_series_combine (fl(c_k * (float) dot) accumulated in fp32 in k order)
struct FcPlanes {
  FcLayer L[FC_MAXL];
};
struct FcSeriesArgs {
  FcPlanes f[2];          // the nets' forward layers (f16x3 planes, exponents, biases, Swish beta)
  FcPlanes t[2];          // their transposed layers: t.L[j] = W_{nl-1-j}^T planes and exponents
  const float* x[2];      // (B, d) boundary layout
  const float* eps[2];    // (B, d) probes
  float* out[2];          // (B)
  float coeff[128];       // c_k, k < n_terms
  int nn, nl, d, act, B, n_terms;
};
int fcseries_supported(const FcSeriesArgs& a);
int launch_fcseries(const FcSeriesArgs& a, hipStream_t s);

// ------------------------------------------------------------------------------------------
// parameter gradients (grad.hip)
// ------------------------------------------------------------------------------------------
struct WgradArgs {
  const float* G;         // (B, M, P) output gradient
  long g_sample;
  const float* X;         // (B, Cin, P) layer input (or a pre-activation with x_beta)
  long x_sample;
  const float* x_beta;    // non-null: X <- swish(X) on load (stored pre-activation of the previous layer)
  int B, P, H, W, ks;     // ks = 1 or 3 (pad ks/2)
  int M, N;               // M = cout, N = cin * ks * ks
  float* slab;            // nsplit * M * N floats
  float* out;             // M * N
  int nsplit, max_split;
};
int launch_wgrad(const WgradArgs& a, hipStream_t s);
// activation algebra of the gradient chains (act: ACT_SWISH with beta, or ACT_SIN)
int launch_act_bwd1(const float* ga, const float* h, int act, const float* beta, float* gprev, double* bpart, long n,
                    int nblocks, hipStream_t s);
int launch_act_tangent(float* hdot, const float* h, int act, const float* beta, long n, hipStream_t s);
int launch_act_apply(const float* h, int act, const float* beta, float* out, long n, hipStream_t s);
int launch_act_bwd2(const float* gbar_adot, const float* gbar_a, const float* h, const float* hdot, int act,
                    const float* beta, float* gbar_hdot, float* gbar_h, double* bpart, long n, int nblocks,
                    hipStream_t s);
int launch_channel_sum(const float* g, int B, int C, int P, float* out, hipStream_t s);
int launch_beta_reduce(const double* bpart, int n, float* out, int accumulate, hipStream_t s);
int launch_sigma_chain(const float* dWe, const float* W, const float* dsig, const float* factor, float coeff,
                       double* dot, float* dW, long n, hipStream_t s);

// ------------------------------------------------------------------------------------------
// opt-in launch timing (inf_profile_begin/end): hipEvents around every engine kernel launch,
// tagged with the kernel instantiation and its algorithmic FLOPs / bytes.  Off by default; a
// debug/measurement facility, not re-entrant.
// ------------------------------------------------------------------------------------------
bool prof_enabled();
void prof_begin_launch(hipStream_t s);
// peak_ms: the launch's MFMA instruction FLOPs at the dense peak of their type (0: not an MFMA kernel)
void prof_end_launch(hipStream_t s, int tag, double flops, double bytes, double peak_ms = 0.0);
constexpr double PEAK_F32_FLOPS_PER_MS = 157.3e9;      // MI355X_MICROARCH.md dense fp32 matrix peak
constexpr double PEAK_BF16_FLOPS_PER_MS = 2516.6e9;    // dense bf16 / f16 MFMA peak

}  // namespace inf
