// Host side of libinflow: net plans, the forward / VJP launch chains, the Broyden driver,
// the log-det estimators and the C-ABI of include/inflow.h.
//
// Reference mapping (all implicit_block.py unless noted):
//   inf_net_refresh       <- InducedNorm*.compute_weight(update=False) (mixed_lipschitz.py:126-132,267-386)
//   inf_net_forward       <- nnet(x)                      (nn.Sequential of InducedNorm + Swish/Sin)
//   inf_net_vjp           <- torch.autograd.grad(g, x, v)                                   (:422)
//   inf_root_find         <- RootFind.apply -> broyden_find_root -> broyden              (:51-100)
//   inf_imblock_forward   <- imBlock.forward value path                                  (:220-230)
//   inf_logdet_series     <- basic_logdet_estimator                                      (:418-426)
//   inf_logdet_neumann    <- neumann_logdet_estimator                                    (:429-438)
//   inf_logdet_exact      <- brute-force batch_jacobian + torch.logdet                   (:249-260)
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <new>
#include <chrono>
#include <functional>
#include <thread>
#include <vector>

#include "glue.h"
#include "kernels.h"

// Events the engine records between its own launches (the host's Broyden readbacks, the side-stream fork / join, the
// profiling brackets) skip the system-scope fence: a system-scope release writes back and invalidates the caches, so the
// next kernel starts with a cold L2 and the CP idles ≈ 5 µs per event (kernel trace).  What the host
// reads through these events lives in coherent pinned memory written by the kernels / copies themselves.
#ifndef INF_EV_SYSFENCE
#define INF_EV_SYSFENCE 0
#endif
constexpr unsigned INF_EV_SYNC = hipEventDisableTiming | (INF_EV_SYSFENCE ? 0u : (unsigned)hipEventDisableSystemFence);
constexpr unsigned INF_EV_TIMING = INF_EV_SYSFENCE ? 0u : (unsigned)hipEventDisableSystemFence;

namespace inf {
static thread_local int g_last_hip = 0;
void set_hip_error(hipError_t e) { g_last_hip = (int)e; }

// ---- opt-in launch timing (per host thread: a profile session records the launches its own thread makes) ----
struct ProfSlot {
  hipEvent_t a, b;
  int tag;
  double flops, bytes, peak_ms;
};
static thread_local std::vector<ProfSlot> g_prof;
static thread_local size_t g_prof_used = 0;
static thread_local bool g_prof_on = false;
bool prof_enabled() { return g_prof_on && g_prof_used < g_prof.size(); }
void prof_begin_launch(hipStream_t s) { (void)hipEventRecord(g_prof[g_prof_used].a, s); }
void prof_end_launch(hipStream_t s, int tag, double flops, double bytes, double peak_ms) {
  ProfSlot& p = g_prof[g_prof_used++];
  (void)hipEventRecord(p.b, s);
  p.tag = tag;
  p.flops = flops;
  p.bytes = bytes;
  p.peak_ms = peak_ms;
}
}  // namespace inf

using namespace inf;

namespace {

constexpr int TAPS_MAX_CH = 64;   // 3x3 convs with fewer output channels than this use packed taps
constexpr int SERIES_MAX = 128;

int round_up(int x, int m) { return (x + m - 1) / m * m; }

struct Operand {
  int load = BL_DIRECT;  // B-operand loader
  int taps = 0;          // output is packed taps (3x3, small M) -> conv_out sums 9 shifts
  int M = 0, Mpad = 0, K = 0, Kpad = 0;
  int pack = PK_ROWMAJOR;
  float* A = nullptr;
};

struct WLayer {
  int kind = 0, cin = 0, cout = 0, ks = 1;
  const float *W = nullptr, *b = nullptr, *u = nullptr, *v = nullptr;
  float coeff = 1.f;
  int act = ACT_NONE;             // activation applied to this layer's output
  const float* act_beta = nullptr;
  Operand f, g;                   // forward, vjp
  float* factor = nullptr;        // device [factor, sigma]
};

}  // namespace

struct InfNet {
  int C = 0, H = 1, W = 1, P = 1, d = 0;
  bool fc = false;
  int pre_act = ACT_NONE;
  const float* pre_beta = nullptr;
  std::vector<WLayer> L;
  int hidden_max = 0;      // channels of the widest intermediate activation
  int rows_max = 0;        // rows of the widest output-stage buffer Y
  float* dev = nullptr;    // packed operands + factors (owned)
  double* scratch = nullptr;
  size_t scratch_doubles = 0;
  int device = 0;
  // fused 3-1-3 path (fused313.hip): fragment-major operands for forward (f) and VJP (b)
  bool fused = false;
  int fhid = 0, K1pad = 0, M3 = 0, M3pad = 0;
  float *F1f = nullptr, *F1b = nullptr, *F2f = nullptr, *F2b = nullptr, *F3f = nullptr, *F3b = nullptr;
  // F1f..F3b split into three bf16 planes each (launch_split3), same order as F1f..F3b
  uint16_t* Fs[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // F1f..F3b as two scaled fp16 planes each (launch_split2h, INF_MFMA_F16X3), same order as Fs; their scale
  // exponents per direction: Fexp[3 * vjp + phase]
  uint16_t* Fh[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  int* Fexp = nullptr;
  // Fh[4], Fh[5] (phase C, forward / VJP) with the k index's bits 2 and 3 swapped per 16-k tile (launch_permute_k23)
  uint16_t* Fhp[2] = {nullptr, nullptr};
  int mfma_mode = INF_MFMA_F32;                 // InfMfmaMode of the fused kernel's phase B
  // f(0) of a conv net (the same image for every sample: zero input, zero padding), cached for the first
  // Broyden residual; computed by a launch of the same batch size (same tile variant -> same bits)
  float* f0 = nullptr;
  int f0_batch = -1;
  // per-net options (inf_net_set_option; defaults from the environment at inf_net_create)
  int k128 = 1;            // INF_OPT_FUSED_K128
  int eval_overlap = 1;    // INF_OPT_EVAL_OVERLAP (read on net_x of inf_imblock_eval)
  int convergence = INF_CONV_GLOBAL;   // INF_OPT_CONVERGENCE (read on the solved net)
  int line_search = 0;                 // INF_OPT_LINE_SEARCH (read on the solved net)
  int exact_scale = 0;     // INF_OPT_K128_EXACT_SCALE
  int presplit = 1;        // INF_OPT_FUSED_PRESPLIT
  int fc_block = 1;        // INF_OPT_FC_BLOCK (read on net_z of inf_imblock_eval_exact)
  int fc_series = 1;       // INF_OPT_FC_SERIES (read on the first net of inf_logdet_series[_pair])
  // fused fc path (fcnet.hip): the whole net in one launch per evaluation (forward and forward-mode Jacobian)
  bool fcfused = false;
  // f16x3 planes of the fused fc layers (fcnet_h3.hip, filled at refresh): layer l at fch + fch_off[l], exponent fchexp[l]
  uint16_t* fch = nullptr;
  int* fchexp = nullptr;
  std::vector<size_t> fch_off;
  // the transposed layers' planes (fcseries_kernel): position j = W_{L-1-j}^T (w.g.A), the same tile shapes as fch's
  // layer j, at fch_off[j], exponent fchtexp[j]
  uint16_t* fcht = nullptr;
  int* fchtexp = nullptr;
};

namespace {

// ---------------------------------------------------------------------------------------------
// workspace carving
// ---------------------------------------------------------------------------------------------
struct WS {
  char* base;
  size_t cap, off;
  bool ok = true;
  template <typename T>
  T* take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    if (off > cap) ok = false;
    return p;
  }
};

struct Bufs {
  float *h0, *h1, *Y;
  std::vector<float*> D;   // saved activation derivatives, one per hidden layer
  float *xin, *xemb, *fx, *xa, *xb, *ga, *gb, *upd, *dx, *dg, *lowest, *va, *vb, *eps_t, *zero, *tmp;
  float *fcur, *flow;      // root solve: f(z) of the latest residual evaluation / of the lowest iterate
  float* fspec;            // root solve: f(z) of the speculative iteration in flight (broyden_core)
  float *U, *VT;
  float *ext0, *ext1;
  double *part, *bpart, *sumsq;   // sumsq: B per-sample sums of squares + 1 (per-sample mode: samples iterating)
  // per-sample convergence (INF_CONV_PER_SAMPLE): state machine, flags, lowest iterate and its f
  double* ps_state;
  int *ps_active, *ps_improved;
  float *ps_lowx, *ps_lowf;
  unsigned int* counter;
  int nchunk;              // per-sample partial chunks of conv_out (residual norms, unfused series)
  float* Y2;               // fused nets: second taps buffer (series terms alternate Y / Y2)
  int snchunk;             // per-sample partial stride of the series slabs (>= tiles per image)
  // fc nets: the device-resident block kernel's (fcblock.hip) exchange words and results: [error word, granules]
  // (zeroed per launch) and [stats, per-sample nstep, lowest_step, prot_break, lowest objective]
  unsigned* bk_sync;
  size_t bk_sync_bytes;
  char* bk_out;
  size_t bk_out_bytes;
  // fc root solve, global rule (broyden_core zero-copy readback): the slot's event, bound by the residual launch itself
  // (OutArgs::stop_ev) when its launcher can, which sets stop_bound; enqueue_sumsq then records no marker after it
  hipEvent_t stop_ev = nullptr;
  bool stop_bound = false;
  bool sample_sums = false;   // conv residuals write each sample's total into bf.part (the readback slot; broyden_core)
};

size_t per_sample_hidden(const InfNet* n) { return (size_t)n->hidden_max * (n->fc ? 1 : n->P); }

// layout-aware sizes: E = B * d elements per vector
// Carves the workspace; returns the bytes required (fits iff result <= cap).  With ws == nullptr it
// only measures.
size_t carve(const InfNet* n, int B, int T, void* ws, size_t cap, Bufs& b) {
  WS w{reinterpret_cast<char*>(ws), cap, 0};
  const size_t E = (size_t)B * n->d;
  const size_t Hs = (size_t)B * per_sample_hidden(n);
  const size_t Ys = (size_t)B * n->rows_max * (n->fc ? 1 : n->P);
  const int nchunk = n->fc ? 1 : out_nchunk(n->d);
  b.nchunk = nchunk;
  b.snchunk = n->fused ? std::max(nchunk, n->P / 32) : nchunk;
  b.h0 = w.take<float>(Hs);
  b.h1 = w.take<float>(Hs);
  b.Y = w.take<float>(Ys);
  b.Y2 = n->fused ? w.take<float>(Ys) : nullptr;
  b.D.resize(n->L.size() > 0 ? n->L.size() - 1 : 0);
  for (auto& p : b.D) p = w.take<float>(Hs);
  float** vecs[] = {&b.xin, &b.xemb, &b.fx, &b.xa, &b.xb, &b.ga, &b.gb, &b.upd,
                    &b.dx, &b.dg, &b.lowest, &b.va, &b.vb, &b.eps_t, &b.zero, &b.tmp, &b.fcur, &b.flow,
                    &b.fspec, &b.ps_lowx, &b.ps_lowf};
  for (float** v : vecs) *v = w.take<float>(E);
  b.U = w.take<float>((size_t)T * E);
  b.VT = w.take<float>((size_t)T * E);
  if (n->fc) {
    const size_t ext = (size_t)(n->d + 1) * B * std::max(n->hidden_max, n->d);
    b.ext0 = w.take<float>(ext);
    b.ext1 = w.take<float>(ext);
  } else {
    b.ext0 = b.ext1 = nullptr;
  }
  b.part = w.take<double>((size_t)B * std::max(nchunk, b.snchunk) * SERIES_MAX);
  const int bch = (n->d + 1023) / 1024;
  b.bpart = w.take<double>((size_t)B * bch * (3 * (size_t)T + 2) + 64);
  b.sumsq = w.take<double>((size_t)B + 1);
  b.counter = w.take<unsigned int>(64);
  b.ps_state = w.take<double>((size_t)B * (PS_HEAD + T));
  b.ps_active = w.take<int>((size_t)B);
  b.ps_improved = w.take<int>((size_t)B);
  if (n->fc) {
    b.bk_sync_bytes = 16 + sizeof(unsigned long long) * 8 * (size_t)fcblock_grid(B);   // 4 sets x 2 granules
    b.bk_sync = reinterpret_cast<unsigned*>(w.take<char>(b.bk_sync_bytes));
    b.bk_out_bytes = sizeof(FcBlockStats) + (sizeof(int) * 3 + sizeof(double)) * (size_t)B + 64;
    b.bk_out = w.take<char>(b.bk_out_bytes);
  } else {
    b.bk_sync = nullptr;
    b.bk_out = nullptr;
    b.bk_sync_bytes = b.bk_out_bytes = 0;
  }
  return w.off + 256;
}

size_t ws_need(const InfNet* n, int B, int T) {
  Bufs b;
  return carve(n, B, T, nullptr, 0, b);
}

// ---------------------------------------------------------------------------------------------
// GEMM argument builders
// ---------------------------------------------------------------------------------------------
GemmArgs gemm_base(const InfNet* n, const Operand& op, const float* X, int in_ch, int B) {
  GemmArgs g;
  memset(&g, 0, sizeof(g));
  g.x6 = n->mfma_mode != INF_MFMA_F32;
  g.A = op.A;
  g.M = op.M;
  g.Kpad = op.Kpad;
  g.Ktot = op.K;
  g.X = X;
  if (n->fc) {        // feature-major (ch, B): one "image" with B pixels
    g.P = B;
    g.N = B;
    g.x_sample = 0;
    g.H = 1;
    g.W = B;
  } else {
    g.P = n->P;
    g.N = B * n->P;
    g.x_sample = (long)in_ch * n->P;
    g.H = n->H;
    g.W = n->W;
  }
  return g;
}

void set_out(const InfNet* n, GemmArgs& g, float* out, int out_rows) {
  g.out = out;
  g.o_sample = n->fc ? 0 : (long)out_rows * n->P;
}

// Forward chain.  mode = OM_* for the output stage, or -1 for "save derivatives only" (log-det prep:
// the last layer is skipped, D[l] = act'(a_l) are kept).  x is in internal layout.
Net313Args net313_args(const InfNet* n, const float* in, int B, Bufs& bf, bool vjp) {
  Net313Args f;
  memset(&f, 0, sizeof(f));
  f.in = in;
  f.pre_beta = vjp ? nullptr : n->pre_beta;
  f.A1 = vjp ? n->F1b : n->F1f;
  f.K1pad = n->K1pad;
  f.A2 = vjp ? n->F2b : n->F2f;
  f.A3 = vjp ? n->F3b : n->F3f;
  const bool spl = n->mfma_mode != INF_MFMA_F32;
  const bool h3 = n->mfma_mode == INF_MFMA_F16X3;
  f.A1s = spl ? (const void*)n->Fs[vjp ? 1 : 0] : nullptr;
  f.A2s = spl ? (const void*)n->Fs[vjp ? 3 : 2] : nullptr;
  f.A3s = spl ? (const void*)n->Fs[vjp ? 5 : 4] : nullptr;
  f.A1h = h3 ? (const void*)n->Fh[vjp ? 1 : 0] : nullptr;
  f.A2h = h3 ? (const void*)n->Fh[vjp ? 3 : 2] : nullptr;
  f.A3h = h3 ? (const void*)n->Fh[vjp ? 5 : 4] : nullptr;
  f.Ah_exp = h3 ? n->Fexp + (vjp ? 3 : 0) : nullptr;
  f.A3p = h3 ? (const void*)n->Fhp[vjp ? 1 : 0] : nullptr;
  f.M3 = n->M3;
  f.M3pad = n->M3pad;
  f.b1 = n->L[0].b;
  f.beta1 = n->L[0].act_beta;
  f.b2 = n->L[1].b;
  f.beta2 = n->L[1].act_beta;
  f.d1 = bf.D[0];
  f.d2 = bf.D[1];
  f.Y = bf.Y;
  f.B = B;
  f.C = n->C;
  f.H = n->H;
  f.W = n->W;
  f.seg = n->W < 64 ? n->W : 64;
  f.k128 = n->k128;
  f.exact_scale = n->exact_scale;
  f.presplit = n->presplit;
  return f;
}

FcArgs fc_args(const InfNet* n, const float* x, int B) {
  FcArgs f;
  memset(&f, 0, sizeof(f));
  f.nl = (int)n->L.size();
  f.d = n->d;
  f.B = B;
  f.act = n->L[0].act;
  const bool h3 = n->mfma_mode == INF_MFMA_F16X3 && n->fch;
  f.tan_fixed = 1;
  for (const WLayer& w : n->L) f.tan_fixed &= w.coeff <= 1.f;
  for (int l = 0; l < f.nl && l < FC_MAXL; ++l) {
    f.L[l].A = n->L[l].f.A;
    f.L[l].Ah = h3 ? n->fch + n->fch_off[l] : nullptr;
    f.L[l].Aexp = h3 ? n->fchexp + l : nullptr;
    f.L[l].Kpad = n->L[l].f.Kpad;
    f.L[l].b = n->L[l].b;
    f.L[l].beta = n->L[l].act_beta;
  }
  f.x = x;
  return f;
}

int run_forward(InfNet* n, const float* x, int B, Bufs& bf, int mode, const OutArgs* oa, hipStream_t s) {
  const int L = (int)n->L.size();
  if (n->fcfused && mode >= OM_PLAIN && mode <= OM_RECOMP) {   // the whole net and fc_out's epilogue in one launch
    FcArgs f = fc_args(n, x, B);
    f.o = *oa;
    f.o.mode = mode;
    f.o.bias = n->L[L - 1].b;
    return launch_fcnet(f, false, s);
  }
  if (n->fused) {
    Net313Args f = net313_args(n, x, B, bf, false);
    INF_TRY(launch_net313(f, n->fhid, mode < 0 ? MODE_SAVE : MODE_EVAL, s));
    if (mode < 0) return INF_OK;
    OutArgs a = *oa;
    a.Y = bf.Y;
    a.y_sample = (long)n->M3 * n->P;
    a.C = n->C;
    a.H = n->H;
    a.W = n->W;
    a.ks = 3;
    a.mode = mode;
    a.bias = n->L[2].b;
    a.pre_beta = nullptr;
    return launch_conv_out(a, B, s);
  }
  const float* cur = x;
  int cur_ch = n->C;
  for (int l = 0; l < L - 1; ++l) {
    const WLayer& w = n->L[l];
    float* out = (l % 2 == 0) ? bf.h0 : bf.h1;
    GemmArgs g = gemm_base(n, w.f, cur, cur_ch, B);
    g.pre_beta = (l == 0) ? n->pre_beta : nullptr;
    set_out(n, g, out, w.cout);
    g.bias = w.b;
    g.act = w.act;
    g.act_beta = w.act_beta;
    g.deriv_out = (mode < 0) ? bf.D[l] : nullptr;
    g.write_out = (mode < 0 && l == L - 2) ? 0 : 1;
    INF_TRY(launch_gemm(g, w.f.load, EP_BIAS_ACT, s));
    cur = out;
    cur_ch = w.cout;
  }
  if (mode < 0) return INF_OK;
  const WLayer& w = n->L[L - 1];
  GemmArgs g = gemm_base(n, w.f, cur, cur_ch, B);
  g.pre_beta = (L == 1) ? n->pre_beta : nullptr;
  set_out(n, g, bf.Y, w.f.M);
  INF_TRY(launch_gemm(g, w.f.load, EP_STORE, s));
  OutArgs a = *oa;
  a.Y = bf.Y;
  a.y_sample = n->fc ? 0 : (long)w.f.M * n->P;
  a.C = n->C;
  a.H = n->H;
  a.W = n->W;
  a.ks = w.f.taps ? 3 : 1;
  a.mode = mode;
  a.bias = w.b;
  a.pre_beta = nullptr;
  return n->fc ? launch_fc_out(a, B, s) : launch_conv_out(a, B, s);
}

// One VJP: vout = v^T J(x), using D saved by run_forward(mode=-1) on x.  partial (B x nchunk doubles,
// may be null) receives the per-sample partial sums of vout . eps.
int run_vjp(InfNet* n, const float* v, float* vout, const float* xin, const float* eps, double* partial, int B,
            Bufs& bf, hipStream_t s) {
  const int L = (int)n->L.size();
  if (n->fused) {
    Net313Args f = net313_args(n, v, B, bf, true);
    INF_TRY(launch_net313(f, n->fhid, MODE_VJP, s));
    OutArgs a;
    memset(&a, 0, sizeof(a));
    a.Y = bf.Y;
    a.y_sample = (long)n->M3 * n->P;
    a.C = n->C;
    a.H = n->H;
    a.W = n->W;
    a.ks = 3;
    a.mode = OM_VJP;
    a.in0 = eps;
    a.in1 = xin;
    a.out0 = vout;
    a.pre_beta = n->pre_beta;
    a.partial = partial;
    a.nchunk = out_nchunk(n->d);
    return launch_conv_out(a, B, s);
  }
  const float* cur = v;
  int cur_ch = n->C;
  for (int l = L - 1; l >= 1; --l) {
    const WLayer& w = n->L[l];
    float* out = ((L - 1 - l) % 2 == 0) ? bf.h0 : bf.h1;
    GemmArgs g = gemm_base(n, w.g, cur, cur_ch, B);
    set_out(n, g, out, w.cin);
    g.deriv_in = bf.D[l - 1];
    INF_TRY(launch_gemm(g, w.g.load, EP_MUL_DERIV, s));
    cur = out;
    cur_ch = w.cin;
  }
  const WLayer& w = n->L[0];
  GemmArgs g = gemm_base(n, w.g, cur, cur_ch, B);
  set_out(n, g, bf.Y, w.g.M);
  INF_TRY(launch_gemm(g, w.g.load, EP_STORE, s));
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.Y = bf.Y;
  a.y_sample = n->fc ? 0 : (long)w.g.M * n->P;
  a.C = n->C;
  a.H = n->H;
  a.W = n->W;
  a.ks = w.g.taps ? 3 : 1;
  a.mode = OM_VJP;
  a.in0 = eps;
  a.in1 = xin;
  a.out0 = vout;
  a.pre_beta = n->pre_beta;
  a.partial = partial;
  a.nchunk = n->fc ? 1 : out_nchunk(n->d);
  return n->fc ? launch_fc_out(a, B, s) : launch_conv_out(a, B, s);
}

// per-sample sums of squares (partials in bf.part) -> host (the reference's .item() per iteration).
// Asynchronous form: the reduction and a D2H copy into pinned host memory are enqueued and an event marks
// them; wait_sumsq blocks on that event.  Two slots per host thread let the Broyden loop keep one
// speculative iteration in flight (broyden_core).  Slots are per thread, so concurrent callers on different
// threads never share one.
struct SumsSlot {
  double* host = nullptr;
  hipEvent_t ev = nullptr;
  int cap = 0;
};
static thread_local SumsSlot g_sums_slots[2];
static int sums_slot(int i, int B, SumsSlot** out) {
  SumsSlot& sl = g_sums_slots[i & 1];
  if (sl.cap < B + 1) {
    if (sl.host) (void)hipHostFree(sl.host);
    sl.host = nullptr;
    const int cap = std::max(B + 1, 1024);
    // coherent: the fc residual launches write their per-sample sums straight into it (broyden_core, zero-copy)
    if (hipHostMalloc(reinterpret_cast<void**>(&sl.host), sizeof(double) * cap, hipHostMallocCoherent) != hipSuccess)
      return INF_ERR_HIP;
    sl.cap = cap;
  }
  if (!sl.ev && hipEventCreateWithFlags(&sl.ev, INF_EV_SYNC) != hipSuccess) return INF_ERR_HIP;
  *out = &sl;
  return INF_OK;
}
// The per-sample stopping decision of step k (INF_CONV_PER_SAMPLE), queued between the reduction and the
// readback: the device state machine (pointwise.hip ps_decide_kernel) and the copy of the improved samples'
// iterate (and f) into the lowest-iterate buffers.  The readback then carries the count of samples iterating.
struct PsStep {
  bool on = false;
  int k = 0, T = 0;
  double eps = 0.0;          // eps * sqrt(d)
  const float* x = nullptr;  // the iterate of this residual
  const float* f = nullptr;  // its f (nullable)
  long sb = 0, si = 0;
};
int enqueue_sumsq(InfNet* f, int B, Bufs& bf, SumsSlot* sl, hipStream_t s, const PsStep* ps = nullptr) {
  // fc nets write one partial per sample: with the global rule those are the sums already (0 + x == x for the
  // non-negative or NaN sums), so the readback takes them directly and the reduction launch is skipped
  const bool ps_on = ps && ps->on;
  const bool direct = (f->fc || bf.sample_sums) && !ps_on;
  if (direct && bf.part == sl->host) {               // the residual launch wrote the sums into the slot itself
    const bool bound = bf.stop_bound && bf.stop_ev == sl->ev;
    bf.stop_bound = false;
    if (bound) return INF_OK;                        // ... and its launch completes the event (no marker packet: the
                                                     // marker after a launch idles the GPU ~4.4 us)
    INF_HIP(hipEventRecord(sl->ev, s));
    return INF_OK;
  }
  if (!direct && !ps_on) {                            // global rule: the reduction writes the sums into the slot
    bool bound = false;                              // (and completes the slot's event itself: no marker packet)
    INF_TRY(launch_reduce_partials(bf.part, B, f->fc ? 1 : bf.nchunk, sl->host, s, sl->ev, &bound));
    if (!bound) INF_HIP(hipEventRecord(sl->ev, s));
    return INF_OK;
  }
  if (!direct) INF_TRY(launch_reduce_partials(bf.part, B, f->fc ? 1 : bf.nchunk, bf.sumsq, s));
  int n = B;
  if (ps_on) {
    INF_TRY(launch_ps_decide(bf.sumsq, bf.ps_state, bf.ps_active, bf.ps_improved, B, ps->k, ps->T, ps->eps, s));
    INF_TRY(launch_ps_copy(bf.ps_improved, ps->x, ps->f, bf.ps_lowx, bf.ps_lowf, B, f->d, ps->sb, ps->si, s));
    n = B + 1;
  }
  INF_HIP(hipMemcpyAsync(sl->host, direct ? bf.part : bf.sumsq, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  INF_HIP(hipEventRecord(sl->ev, s));
  return INF_OK;
}
// Host wait on a readback event.  A blocking hipEventSynchronize that has to wait long (e.g. behind a whole
// log-det series) lets the runtime put the thread to sleep, and its wake-up comes late, with the GPU idle
// and nothing else queued; polling hipEventQuery keeps the host turnaround at the copy's latency.  The poll
// spins for at most 100 us, then yields the core between polls (other host threads, e.g. data loaders, run),
// and after 5 ms sleeps 20 us per poll.  INFLOW_BLOCKING_WAIT=1 restores the blocking wait.
int host_wait(hipEvent_t ev) {
  static const bool blocking = [] {
    const char* e = getenv("INFLOW_BLOCKING_WAIT");
    return e && e[0] == '1';
  }();
  if (blocking) {
    INF_HIP(hipEventSynchronize(ev));
    return INF_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return INF_OK;
    if (q != hipErrorNotReady) {
      set_hip_error(q);
      return INF_ERR_HIP;
    }
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
    if (us > 5000) std::this_thread::sleep_for(std::chrono::microseconds(20));
    else if (us > 100) std::this_thread::yield();
  }
}
// n_active (may be null): the per-sample mode's count of samples still iterating after this step
int wait_sumsq(SumsSlot* sl, int B, std::vector<double>& host_sumsq, int* n_active = nullptr) {
  INF_TRY(host_wait(sl->ev));
  memcpy(host_sumsq.data(), sl->host, sizeof(double) * B);
  if (n_active) *n_active = (int)sl->host[B];
  return INF_OK;
}
int read_sumsq(InfNet* f, int B, Bufs& bf, std::vector<double>& host_sumsq, hipStream_t s) {
  SumsSlot* sl = nullptr;
  INF_TRY(sums_slot(0, B, &sl));
  INF_TRY(enqueue_sumsq(f, B, bf, sl, s));
  return wait_sumsq(sl, B, host_sumsq);
}

// residual evaluation g = x_embed - f(z) - z (+ dg = g - g_prev), f(z) kept in bf.fcur, per-sample partial sums of
// squares in bf.part.  zsub is the subtracted "- z" term: z itself for Broyden, zeros for the Banach map.
int eval_resid_part(InfNet* f, const float* z, const float* zsub, const float* xemb, float* gout, float* dg,
                    const float* gprev, int B, Bufs& bf, hipStream_t s) {
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.in0 = xemb;
  a.in1 = zsub;
  a.in2 = gprev;
  a.out0 = gout;
  a.out1 = dg;
  a.out2 = bf.fcur;
  a.partial = bf.part;
  a.nchunk = bf.nchunk;
  a.sample_sums = bf.sample_sums;
  a.stop_ev = bf.stop_ev;
  a.stop_bound = &bf.stop_bound;
  return run_forward(f, z, B, bf, OM_RESID, &a, s);
}
// the same, synchronously, with the per-sample sums of squares on the host
int eval_resid(InfNet* f, const float* z, const float* zsub, const float* xemb, float* gout, float* dg,
               const float* gprev, int B, Bufs& bf, std::vector<double>& host_sumsq, hipStream_t s) {
  INF_TRY(eval_resid_part(f, z, zsub, xemb, gout, dg, gprev, B, bf, s));
  return read_sumsq(f, B, bf, host_sumsq, s);
}

// vjp residual of the implicit backward (implicit_block.py:186-190): g = (y + y^T J) - grad
int vjp_resid_part(InfNet* f, const float* y, const float* zi, const float* gradi, float* gout, float* dg,
                   const float* gprev, int B, Bufs& bf, hipStream_t s) {
  INF_TRY(run_vjp(f, y, bf.tmp, zi, nullptr, nullptr, B, bf, s));
  return launch_vjp_resid(bf.tmp, y, gradi, gprev, gout, dg, bf.part, B, f->d, f->fc ? 1 : bf.nchunk, f->fc, s);
}

double total(const std::vector<double>& v) {
  double t = 0.0;
  for (double x : v) t += x;
  return t;
}

// x (boundary layout) -> internal layout buffer
const float* to_internal(InfNet* n, const float* x, float* buf, int B, hipStream_t s, int* st) {
  if (!n->fc) return x;
  *st = launch_transpose(x, buf, B, n->d, s);
  return buf;
}
int to_boundary(InfNet* n, const float* xi, float* out, int B, hipStream_t s) {
  if (!n->fc) {
    if (xi != out) INF_HIP(hipMemcpyAsync(out, xi, sizeof(float) * (size_t)B * n->d, hipMemcpyDeviceToDevice, s));
    return INF_OK;
  }
  return launch_transpose(xi, out, n->d, B, s);
}

bool same_shape(const InfNet* a, const InfNet* b) {
  return a->C == b->C && a->H == b->H && a->W == b->W && a->fc == b->fc && a->d == b->d;
}

// Broyden root find on internal-layout buffers.  Solves z with g(z) = xemb - f(z) - z = 0.
// Result (lowest iterate) in bf.lowest.  y (internal) is the Banach fallback start.
// resid(x, gout, dg, gprev): residual g(x) -> gout (+ dg = g - gprev when gprev), per-sample partial sums of
// squares -> bf.part, and (root solves) f(x) -> bf.fcur.  broyden_core reduces and reads them back.
using ResidFn = std::function<int(const float* x, float* gout, float* dg, const float* gprev)>;
// update + residual in one launch (fused fc nets): the update ba computes ba.xnew, then the residual at it, as resid
using StepFn = std::function<int(const BroydenArgs& ba, float* gout, float* dg, const float* gprev)>;
// Broyden's start in one launch: x0 = 0, g0 = g(x0) (+ f(x0) in bf.fcur, partials in bf.part), update = -g0,
// x1 = x0 + update, dx = x1 - x0
using StartFn = std::function<int(float* x0, float* g0, float* upd, float* x1, float* dx)>;
// Work that follows the solve, queued speculatively when the loop queues no further iteration (the pending one is predicted
// to be the last, or the threshold ends the loop): fn(x, f) runs on the pending iterate and its f; x / f record what it
// was queued for, so the caller can tell whether the solve's result (bf.lowest, bf.flow) is that iterate
struct SpecTail {
  std::function<int(const float* x, const float* f)> fn;
  const float* x = nullptr;
  const float* f = nullptr;
};

// Copies the per-sample results (INF_CONV_PER_SAMPLE) into the stats and the caller's optional host arrays.
static int ps_collect(Bufs& bf, int B, int T, InfBroydenStats& stats, std::vector<double>& lowest_ss,
                      hipStream_t s) {
  const int stride = PS_HEAD + T;
  std::vector<double> st((size_t)B * stride);
  INF_HIP(hipMemcpyAsync(st.data(), bf.ps_state, sizeof(double) * st.size(), hipMemcpyDeviceToHost, s));
  INF_HIP(hipStreamSynchronize(s));
  int nmax = 0, lmax = 0, prot = 0;
  double d2 = 0.0;
  lowest_ss.assign(B, 0.0);
  for (int b = 0; b < B; ++b) {
    const double* p = st.data() + (size_t)b * stride;
    const int ns = (int)p[3], ls = (int)p[4], pb = (int)p[5];
    nmax = std::max(nmax, ns);
    lmax = std::max(lmax, ls);
    prot |= pb;
    lowest_ss[b] = p[1] * p[1];
    d2 += lowest_ss[b];
    if (stats.sample_nstep) stats.sample_nstep[b] = ns;
    if (stats.sample_lowest_step) stats.sample_lowest_step[b] = ls;
    if (stats.sample_prot_break) stats.sample_prot_break[b] = pb;
  }
  stats.nstep = nmax;
  stats.tnstep = nmax;
  stats.lowest_step = lmax;
  stats.prot_break = prot;
  stats.diff = sqrt(d2);
  return INF_OK;
}

// broyden.py:123-193 with the residual as a callback; the result (lowest iterate) is in bf.lowest.
// f->convergence selects the stopping rule: INF_CONV_GLOBAL is the reference's (one Frobenius norm over the
// batch against eps sqrt(B d), one lowest iterate for the batch); INF_CONV_PER_SAMPLE runs the same rules per
// sample against eps sqrt(d) (the reference's result for a batch of one, i.e. independent of how the batch is
// sharded), with the decisions taken on the device (ps_decide_kernel) and stopped samples frozen.
// stats.sample_* (host arrays, nullable) receive the per-sample outcome in that mode.
#ifndef SAMPLE_SUMS
#define SAMPLE_SUMS 1   // 0: conv residuals write chunk partials and a reduction launch sums them (A/B builds)
#endif

int broyden_core(InfNet* f, const ResidFn& resid, int B, int T, double eps_in, InfBroydenStats& stats,
                 std::vector<double>& lowest_ss, Bufs& bf, hipStream_t s, bool keep_f = false,
                 const StepFn* step_fn = nullptr, const StartFn* start_fn = nullptr, SpecTail* tail = nullptr,
                 bool resid_sample_sums = false) {
  const size_t E = (size_t)B * f->d;
  const long cs = (long)E;
  const long sb = f->fc ? 1 : f->d, si = f->fc ? B : 1;
  const bool per_sample = f->convergence == INF_CONV_PER_SAMPLE;
  std::vector<double> ss(B);
  lowest_ss.assign(B, 0.0);
  const double eps = eps_in * sqrt((double)E);                       // broyden.py:131
  const double eps_ps = eps_in * sqrt((double)f->d);                 // the same rule for a batch of one
  {
    int *a = stats.sample_nstep, *b = stats.sample_lowest_step, *c = stats.sample_prot_break;
    memset(&stats, 0, sizeof(stats));
    stats.sample_nstep = a;
    stats.sample_lowest_step = b;
    stats.sample_prot_break = c;
  }
  stats.eps = per_sample ? eps_ps : eps;
  stats.convergence = f->convergence;

  // One iteration of lookahead: while the host waits for iteration k's residual norm (the reference's
  // .item(), broyden.py:157), iteration k+1's low-rank update and residual are already queued behind it, so
  // the GPU does not idle through the host round trip.  If k stops the loop, k+1's work is discarded: it
  // only wrote scratch (per-sample mode: the device decisions of step k already froze every sample it
  // stopped).  Iterates rotate through {xa, xb, lowest} and f(z) through {fcur, flow, fspec}: the decided
  // lowest, the pending and the speculative one are always distinct buffers; the lowest iterate
  // (broyden.py:159-162) is tracked by pointer (per-sample mode: copied per sample into ps_lowx / ps_lowf) and
  // the Bufs pointers are permuted at the end so that bf.lowest / bf.flow name the result.
  float* xpool[3] = {bf.xa, bf.xb, bf.lowest};
  float* fpool[3] = {bf.fcur, bf.flow, bf.fspec};
  auto pick = [](float* const* pool, const float* a, const float* b) {
    for (int i = 0; i < 3; ++i)
      if (pool[i] != a && pool[i] != b) return pool[i];
    return pool[0];
  };
  SumsSlot* slot[2];
  INF_TRY(sums_slot(0, B, &slot[0]));
  INF_TRY(sums_slot(1, B, &slot[1]));
  PsStep ps;
  ps.on = per_sample;
  ps.T = T;
  ps.eps = eps_ps;
  ps.sb = sb;
  ps.si = si;
  auto sums = [&](int k, const float* xk, const float* fk, SumsSlot* sl) {
    ps.k = k;
    ps.x = xk;
    ps.f = keep_f ? fk : nullptr;
    return enqueue_sumsq(f, B, bf, sl, s, &ps);
  };
  float *gx = bf.ga, *gn = bf.gb;
  float* x = xpool[0];
  float *low = per_sample ? bf.ps_lowx : x, *flow = nullptr;
  // (U / VT need no zeroing: every update reads only the columns j < m, j < ncols that earlier steps of this solve
  // wrote, as broyden.py:174-181 reads Us[..., :nstep - 1])
  // the one-launch start (fc nets, global rule: nothing is queued between the residual and the first step)
  const bool fused_start = start_fn && !per_sample && T > 0;
  if (!fused_start) INF_HIP(hipMemsetAsync(x, 0, sizeof(float) * E, s));
  bf.fcur = fpool[0];
  // zero-copy readback (fc nets, global rule): each residual launch writes its per-sample sums straight into the
  // pinned slot its norm is read from (bf.part points there while it is enqueued), so no copy launch sits between
  // the residual and the event the host waits on; bf.part is restored on every return path
  // conv nets whose residual launches can write per-sample totals (resid_sample_sums: the root solve's
  // eval_resid_part / resid_bcast, d <= 4 residual chunks per sample): the residual launch itself sums each sample
  // over its chunks (one block per sample, conv_out_resid_sample_kernel) into the slot, so no reduction launch sits
  // between it and the readback either.  (The implicit backward's residual writes chunk partials: not here.)
  const bool zc = (f->fc || (resid_sample_sums && SAMPLE_SUMS && out_nchunk(f->d) <= 4)) && !per_sample;
  struct PartRestore {
    Bufs& b;
    double* p;
    hipEvent_t e;
    ~PartRestore() {
      b.part = p;
      b.stop_ev = e;
      b.stop_bound = false;
      b.sample_sums = false;
    }
  } part_restore{bf, bf.part, bf.stop_ev};
  auto target = [&](SumsSlot* sl) {
    if (zc) {
      bf.part = sl->host;
      bf.stop_ev = sl->ev;
      bf.sample_sums = !f->fc;
    }
  };
  target(slot[0]);
  float* xp = nullptr;
  float* fp = nullptr;
  if (fused_start) {
    xp = pick(xpool, low, x);
    INF_TRY((*start_fn)(x, gx, bf.upd, xp, bf.dx));
  } else {
    INF_TRY(resid(x, gx, nullptr, nullptr));
  }
  INF_TRY(sums(0, x, bf.fcur, slot[0]));
  if (keep_f) flow = per_sample ? bf.ps_lowf : bf.fcur;
  // iteration 1 is queued before the initial norm is read (update = -g0, x1 = x0 + update, :144)
  if (T > 0) {
    if (!fused_start) {
      xp = pick(xpool, low, x);
      INF_TRY(launch_neg(gx, bf.upd, (long)E, s));
      INF_TRY(launch_axpy_step(x, bf.upd, xp, bf.dx, (long)E, s));
    }
    fp = pick(fpool, flow, bf.fcur);
    bf.fcur = fp;
    target(slot[1]);
    INF_TRY(resid(xp, gn, bf.dg, gx));
    INF_TRY(sums(1, xp, fp, slot[1]));
  }
  int n_active = B;
  INF_TRY(wait_sumsq(slot[0], B, ss, per_sample ? &n_active : nullptr));
  const double init = sqrt(total(ss));
  double obj = init, lowest = init;
  lowest_ss = ss;
  int nstep = 0, lowest_step = 0;
  std::vector<double> trace{init};
  // low-rank update from iterate `step` (x = xfrom, g = gfrom) to xto (broyden.py:174-181)
  auto update_args = [&](int step, float* xfrom, float* gfrom, float* xto) {
    BroydenArgs ba;
    memset(&ba, 0, sizeof(ba));
    ba.batch = B;
    ba.d = f->d;
    ba.T = T;
    ba.sb = sb;
    ba.si = si;
    ba.cs = cs;
    ba.U = bf.U;
    ba.VT = bf.VT;
    ba.dx = bf.dx;
    ba.dg = bf.dg;
    ba.gx = gfrom;
    ba.x = xfrom;
    ba.xnew = xto;
    ba.dxnew = bf.dx;
    ba.upd = bf.upd;
    ba.part = bf.bpart;
    ba.m = (step - 1) % T;
    ba.ncols = std::min(step, T);
    ba.active = per_sample ? bf.ps_active : nullptr;
    return ba;
  };
  auto update = [&](int step, float* xfrom, float* gfrom, float* xto) {
    return launch_broyden_update(update_args(step, xfrom, gfrom, xto), s);
  };
  const bool go = per_sample ? (n_active > 0 && T > 0) : (obj >= eps && nstep < T);   // broyden.py:153
  if (go) {
    int ps_ = 1;
    double prev_obj = -1.0;
    for (;;) {
      // pending = iteration nstep + 1 (iterate xp, residual in gn, f in fp, norms in slot[ps_]).  The next
      // iteration is queued before the pending norm is read, unless the threshold forbids it or the
      // observed contraction predicts that the pending iteration converges (then it would be wasted work).
      const bool allow = nstep + 1 < T;
      const bool likely_last = !per_sample && prev_obj > 0.0 && obj * (obj / prev_obj) < eps;
      float *xs = nullptr, *fs = nullptr;
      auto enqueue_next = [&](int pending_step) -> int {
        target(slot[1 - ps_]);
        xs = pick(xpool, low, xp);
        fs = pick(fpool, flow, fp);
        if (step_fn) {
          bf.fcur = fs;
          INF_TRY((*step_fn)(update_args(pending_step, xp, gn, xs), gx, bf.dg, gn));
        } else {
          INF_TRY(update(pending_step, xp, gn, xs));
          bf.fcur = fs;
          INF_TRY(resid(xs, gx, bf.dg, gn));
        }
        return sums(pending_step + 1, xs, fs, slot[1 - ps_]);
      };
      const bool spec = allow && !likely_last;
      if (spec) {
        INF_TRY(enqueue_next(nstep + 1));
      } else if (tail && tail->fn && !per_sample && keep_f) {
        INF_TRY(tail->fn(xp, fp));
        tail->x = xp;
        tail->f = fp;
      }
      INF_TRY(wait_sumsq(slot[ps_], B, ss, per_sample ? &n_active : nullptr));
      nstep += 1;
      x = xp;
      prev_obj = obj;
      obj = sqrt(total(ss));
      trace.push_back(obj);
      if (per_sample) {
        if (n_active == 0 || !allow) break;
      } else {
        if (obj < lowest) {                                             // :159-162
          low = xp;
          if (keep_f) flow = fp;
          lowest = obj;
          lowest_step = nstep;
          lowest_ss = ss;
        }
        if (obj < eps) break;
        if (obj < 3 * eps && nstep == T) {                              // :165-168
          const size_t k0 = trace.size() > (size_t)T ? trace.size() - T : 0;
          double mx = trace[k0], mn = trace[k0];
          for (size_t k = k0; k < trace.size(); ++k) {
            mx = std::max(mx, trace[k]);
            mn = std::min(mn, trace[k]);
          }
          if (mx / mn < 1.3) break;
        }
        if (obj > init * 1e6) {                                         // :169-172
          stats.prot_break = 1;
          break;
        }
        if (!allow) break;                                              // nstep == T
      }
      if (!spec) {
        // the loop goes on past the iterate the tail was queued for: that iterate is no longer the candidate result,
        // and its buffers go back to the pools (a later iterate may reuse them), so the tail no longer names it
        if (tail) tail->x = tail->f = nullptr;
        INF_TRY(enqueue_next(nstep));
      }
      xp = xs;
      fp = fs;
      ps_ = 1 - ps_;
      std::swap(gx, gn);                                                // gn: the new pending residual
    }
  }
  stats.n_trace = (int)std::min<size_t>(trace.size(), 64);
  for (int k = 0; k < stats.n_trace; ++k) stats.trace[k] = trace[k];
  if (per_sample) {
    // the pool buffers are scratch; the result is the per-sample lowest iterate
    bf.lowest = bf.ps_lowx;
    bf.flow = bf.ps_lowf;
    bf.xa = xpool[0];
    bf.xb = xpool[1];
    bf.fcur = fpool[0];
    bf.fspec = fpool[2];
    return ps_collect(bf, B, T, stats, lowest_ss, s);
  }
  // name the result: bf.lowest = the lowest iterate, bf.flow = its f; the other buffers become scratch
  {
    float* rest[2];
    int k = 0;
    for (float* p : xpool)
      if (p != low && k < 2) rest[k++] = p;
    bf.lowest = low;
    bf.xa = rest[0];
    bf.xb = rest[1];
    float* fr[2];
    k = 0;
    const float* fl = flow ? flow : fpool[1];
    for (float* p : fpool)
      if (p != fl && k < 2) fr[k++] = p;
    bf.flow = const_cast<float*>(fl);
    bf.fcur = fr[0];
    bf.fspec = fr[1];
  }
  stats.nstep = nstep;
  stats.tnstep = nstep;
  stats.lowest_step = lowest_step;
  stats.diff = lowest;
  return INF_OK;
}

// _safe_norm(g)**2 (broyden.py:18-21,81) from the per-sample sums of squares: the fp32 norm squared in fp32, inf when
// any entry is not finite
static float ls_phi(const std::vector<double>& ss) {
  const double t = total(ss);
  if (!std::isfinite(t)) return INFINITY;
  const float n = (float)sqrt(t);
  return n * n;
}

// broyden.py:123-193 with line_search(on=True) (:66-99) and scalar_search_armijo (:24-63; c1 = 1e-4, alpha0 = 1,
// amin = 1e-2, derphi0 = -phi0), the global rule.  Each step: the trial point x0 + s update (launch_line_step; s = 1 is
// the update launch's own x + update), its residual and norm read back (one host round trip per evaluation: the step
// size decides the next point, so nothing is speculated), the quadratic then cubic backtracking in fp32 as the
// reference's 0-d fp32 tensors compute it, the last evaluation reused when the accepted step is the stored one (:77-78,
// 95-96).  A failed search takes the full step with ite = 0 and evaluates it again (:90-98).  stats.tnstep counts
// nstep + the accepted searches' extra iterations (:156).  Result (lowest iterate) in bf.lowest, its f in bf.flow.
int broyden_core_ls(InfNet* f, const ResidFn& resid, int B, int T, double eps_in, InfBroydenStats& stats,
                    std::vector<double>& lowest_ss, Bufs& bf, hipStream_t s, bool keep_f) {
#pragma clang fp contract(off)
  const size_t E = (size_t)B * f->d;
  const long cs = (long)E;
  const long sb = f->fc ? 1 : f->d, si = f->fc ? B : 1;
  {
    int *a = stats.sample_nstep, *b = stats.sample_lowest_step, *c = stats.sample_prot_break;
    memset(&stats, 0, sizeof(stats));
    stats.sample_nstep = a;
    stats.sample_lowest_step = b;
    stats.sample_prot_break = c;
  }
  const double eps = eps_in * sqrt((double)E);                       // broyden.py:131
  stats.eps = eps;
  stats.convergence = INF_CONV_GLOBAL;
  float* xpool[3] = {bf.xa, bf.xb, bf.lowest};
  float* fpool[3] = {bf.fcur, bf.flow, bf.fspec};
  auto pick = [](float* const* pool, const float* a, const float* b) {
    for (int i = 0; i < 3; ++i)
      if (pool[i] != a && pool[i] != b) return pool[i];
    return pool[0];
  };
  float* x = xpool[0];
  float* fx = fpool[0];
  float *gx = bf.ga, *gt = bf.gb;
  std::vector<double> ss(B), ss_t(B);
  INF_HIP(hipMemsetAsync(x, 0, sizeof(float) * E, s));
  bf.fcur = fx;
  INF_TRY(resid(x, gx, nullptr, nullptr));
  INF_TRY(read_sumsq(f, B, bf, ss, s));
  const double init = sqrt(total(ss));
  double obj = init, lowest = init;
  lowest_ss = ss;
  float* low = x;
  float* flow = keep_f ? fx : nullptr;
  int nstep = 0, tnstep = 0, lowest_step = 0;
  std::vector<double> trace{init};
  INF_TRY(launch_neg(gx, bf.upd, (long)E, s));                      // update = -gx (:144)
  float* xt = pick(xpool, low, x);
  INF_TRY(launch_axpy_step(x, bf.upd, xt, bf.dx, (long)E, s));       // the s = 1 trial point
  bool xt_full = true;                                               // xt holds x + 1 * update
  auto update_args = [&](int step, float* xfrom, float* gfrom, float* xto) {
    BroydenArgs ba;
    memset(&ba, 0, sizeof(ba));
    ba.batch = B;
    ba.d = f->d;
    ba.T = T;
    ba.sb = sb;
    ba.si = si;
    ba.cs = cs;
    ba.U = bf.U;
    ba.VT = bf.VT;
    ba.dx = bf.dx;
    ba.dg = bf.dg;
    ba.gx = gfrom;
    ba.x = xfrom;
    ba.xnew = xto;
    ba.dxnew = bf.dx;
    ba.upd = bf.upd;
    ba.part = bf.bpart;
    ba.m = (step - 1) % T;
    ba.ncols = std::min(step, T);
    return ba;
  };
  while (obj >= eps && nstep < T) {                                  // :153
    // ---- line_search(update, x, gx, g, on=True): the stored evaluation starts as (s = 0, phi0, g0)
    const float phi0 = ls_phi(ss), der = -phi0;
    float st_s = 0.f, st_phi = phi0;
    bool st_init = true;                                             // the stored evaluation is (x, gx) itself
    float* ft = nullptr;
    auto phi = [&](float sv, float& out) -> int {                   // :76-86
      if (sv == st_s) {
        out = st_phi;
        return INF_OK;
      }
      if (!(sv == 1.f && xt_full)) INF_TRY(launch_line_step(x, bf.upd, sv, xt, bf.dx, (long)E, s));
      xt_full = sv == 1.f;
      ft = pick(fpool, flow, fx);
      bf.fcur = ft;
      INF_TRY(resid(xt, gt, bf.dg, gx));                             // g, f and dg = g - g0 of the trial point
      INF_TRY(read_sumsq(f, B, bf, ss_t, s));
      out = ls_phi(ss_t);
      st_s = sv;
      st_phi = out;
      st_init = false;
      return INF_OK;
    };
    const float c1 = 1e-4f, amin = 1e-2f;
    float acc = 1.f;
    bool found = false;
    int ite = 0;
    float pa0;
    INF_TRY(phi(1.f, pa0));                                          // scalar_search_armijo (:24-63)
    if (pa0 <= phi0 + c1 * der) {
      found = true;
    } else {
      float a0 = 1.f;
      float a1 = -der * 1.f / 2.f / (pa0 - phi0 - der * a0);
      float pa1;
      INF_TRY(phi(a1, pa1));
      while (a1 > amin) {
        const float fac = a0 * a0 * (a1 * a1) * (a1 - a0);
        const float r1 = pa1 - phi0 - der * a1, r0 = pa0 - phi0 - der * a0;
        float a = a0 * a0 * r1 - a1 * a1 * r0;
        a = a / fac;
        float b = -(a0 * a0 * a0) * r1 + a1 * a1 * a1 * r0;
        b = b / fac;
        float a2 = (-b + sqrtf(fabsf(b * b - 3.f * a * der))) / (3.f * a);
        float pa2;
        INF_TRY(phi(a2, pa2));
        ite += 1;
        if (pa2 <= phi0 + c1 * a2 * der) {
          acc = a2;
          found = true;
          break;
        }
        if ((a1 - a2) > a1 / 2.f || (1.f - a2 / a1) < 0.96f) a2 = a1 / 2.f;
        a0 = a1;
        a1 = a2;
        pa0 = pa1;
        pa1 = pa2;
      }
    }
    if (!found) {                                                    // :90-92
      acc = 1.f;
      ite = 0;
    }
    if (acc != st_s) {                                               // :94-98 (a fresh evaluation at the step)
      st_s = acc + 1.f;                                              // (anything else: phi evaluates)
      float unused;
      INF_TRY(phi(acc, unused));
    } else if (st_init) {                                            // the accepted step is 0: x0 and g0 themselves
      INF_TRY(launch_line_step(x, bf.upd, 0.f, xt, bf.dx, (long)E, s));
      ft = pick(fpool, flow, fx);
      INF_HIP(hipMemcpyAsync(gt, gx, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
      INF_HIP(hipMemsetAsync(bf.dg, 0, sizeof(float) * E, s));
      if (keep_f) INF_HIP(hipMemcpyAsync(ft, fx, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
      ss_t = ss;
      xt_full = false;
    }
    // ---- the step is taken: x_est, g(x_est), delta_x (bf.dx), delta_g (bf.dg)
    x = xt;
    std::swap(gx, gt);
    fx = ft;
    ss = ss_t;
    nstep += 1;
    tnstep += ite + 1;                                               // :155-156
    obj = sqrt(total(ss));
    trace.push_back(obj);
    if (obj < lowest) {                                              // :159-162
      low = x;
      if (keep_f) flow = fx;
      lowest = obj;
      lowest_step = nstep;
      lowest_ss = ss;
    }
    if (obj < eps) break;                                            // :163-164
    if (obj < 3 * eps && nstep == T) {                               // :165-168
      const size_t k0 = trace.size() > (size_t)T ? trace.size() - T : 0;
      double mx = trace[k0], mn = trace[k0];
      for (size_t k = k0; k < trace.size(); ++k) {
        mx = std::max(mx, trace[k]);
        mn = std::min(mn, trace[k]);
      }
      if (mx / mn < 1.3) break;
    }
    if (obj > init * 1e6) {                                          // :169-172
      stats.prot_break = 1;
      break;
    }
    // the rank-1 update and update = -matvec(...) (:174-181); its x + update is the next search's s = 1 point
    xt = pick(xpool, low, x);
    INF_TRY(launch_broyden_update(update_args(nstep, x, gx, xt), s));
    xt_full = true;
  }
  stats.n_trace = (int)std::min<size_t>(trace.size(), 64);
  for (int k = 0; k < stats.n_trace; ++k) stats.trace[k] = trace[k];
  {
    float* rest[2];
    int k = 0;
    for (float* p : xpool)
      if (p != low && k < 2) rest[k++] = p;
    bf.lowest = low;
    bf.xa = rest[0];
    bf.xb = rest[1];
    float* fr[2];
    k = 0;
    const float* fl = flow ? flow : fpool[1];
    for (float* p : fpool)
      if (p != fl && k < 2) fr[k++] = p;
    bf.flow = const_cast<float*>(fl);
    bf.fcur = fr[0];
    bf.fspec = fr[1];
  }
  stats.nstep = nstep;
  stats.tnstep = tnstep;
  stats.lowest_step = lowest_step;
  stats.diff = lowest;
  return INF_OK;
}

// f(0) for sample 0 of a conv net, computed once per (weights, batch size) with a B-sized launch
static int ensure_f0(InfNet* f, int B, Bufs& bf, hipStream_t s) {
  if (f->f0_batch == B) return INF_OK;
  const size_t per = (size_t)f->d;
  if (!f->f0 && hipMalloc(&f->f0, per * sizeof(float)) != hipSuccess) return INF_ERR_HIP;
  INF_HIP(hipMemsetAsync(bf.zero, 0, sizeof(float) * per * B, s));
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.out0 = bf.fcur;
  INF_TRY(run_forward(f, bf.zero, B, bf, OM_PLAIN, &a, s));
  // sample 0's f(0): conv layout (B, d) row 0; fc layout (d, B) column 0
  if (f->fc)
    INF_HIP(hipMemcpy2DAsync(f->f0, sizeof(float), bf.fcur, sizeof(float) * (size_t)B, sizeof(float), per,
                             hipMemcpyDeviceToDevice, s));
  else
    INF_HIP(hipMemcpyAsync(f->f0, bf.fcur, per * sizeof(float), hipMemcpyDeviceToDevice, s));
  f->f0_batch = B;
  return INF_OK;
}

// find_fixed_point (implicit_block.py:17-28) of z <- x_embed - f(z) from z0 = y (internal layout):
//   x, x_prev = g(y), y; while not all((x - x_prev)^2 / (eps + eps |y|) < 1): x, x_prev = g(x), x; i += 1;
//   break once i > threshold.
// todo == nullptr: the reference's batch-wide test (torch.all over the batch), result for every sample in
// bf.lowest.  todo (host, B flags): the same loop per sample (a batch of one each, in lockstep launches); only
// the flagged samples' rows of bf.lowest are replaced.  *iters = the loop's i.
static int banach_solve(InfNet* f, const float* y, int B, double eps_in, int threshold, const int* todo, Bufs& bf,
                        hipStream_t s, int* iters) {
  const size_t E = (size_t)B * f->d;
  const long sb = f->fc ? 1 : f->d, si = f->fc ? B : 1;
  float *zc = bf.xa, *zn = bf.xb;
  INF_HIP(hipMemsetAsync(bf.zero, 0, sizeof(float) * E, s));
  std::vector<double> dummy(B);
  int it = 0;
  // x = g(y), x_prev = y
  INF_TRY(eval_resid(f, y, bf.zero, bf.xemb, zc, nullptr, nullptr, B, bf, dummy, s));
  INF_HIP(hipMemcpyAsync(zn, y, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
  if (!todo) {
    for (;;) {
      unsigned int bad = 0;
      INF_HIP(hipMemsetAsync(bf.counter, 0, sizeof(unsigned int), s));
      INF_TRY(glue_fixed_point_check(zc, zn, y, (long)E, (float)eps_in, bf.counter, s));
      INF_HIP(hipMemcpyAsync(&bad, bf.counter, sizeof(unsigned int), hipMemcpyDeviceToHost, s));
      INF_HIP(hipStreamSynchronize(s));
      if (bad == 0) break;
      INF_TRY(eval_resid(f, zc, bf.zero, bf.xemb, zn, nullptr, nullptr, B, bf, dummy, s));
      std::swap(zc, zn);
      it += 1;
      if (it > threshold) break;
    }
    INF_HIP(hipMemcpyAsync(bf.lowest, zc, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
    *iters = it;
    return INF_OK;
  }
  std::vector<int> flags(todo, todo + B);
  INF_HIP(hipMemcpyAsync(bf.ps_improved, flags.data(), sizeof(int) * B, hipMemcpyHostToDevice, s));
  for (;;) {
    INF_TRY(launch_ps_fixed_point(zc, zn, y, bf.lowest, bf.ps_improved, B, f->d, sb, si, (float)eps_in, 0, s));
    INF_HIP(hipMemcpyAsync(flags.data(), bf.ps_improved, sizeof(int) * B, hipMemcpyDeviceToHost, s));
    INF_HIP(hipStreamSynchronize(s));
    bool any = false;
    for (int b = 0; b < B; ++b) any = any || flags[b];
    if (!any) break;
    INF_TRY(eval_resid(f, zc, bf.zero, bf.xemb, zn, nullptr, nullptr, B, bf, dummy, s));
    std::swap(zc, zn);
    it += 1;
    if (it > threshold) {      // the remaining samples take the latest iterate
      INF_TRY(launch_ps_fixed_point(zc, zn, y, bf.lowest, bf.ps_improved, B, f->d, sb, si, (float)eps_in, 1, s));
      break;
    }
  }
  *iters = it;
  return INF_OK;
}

// A zeroed stats struct carrying the caller's optional per-sample host arrays.
static InfBroydenStats stats_for(const InfBroydenStats* caller) {
  InfBroydenStats st;
  memset(&st, 0, sizeof(st));
  if (caller) {
    st.sample_nstep = caller->sample_nstep;
    st.sample_lowest_step = caller->sample_lowest_step;
    st.sample_prot_break = caller->sample_prot_break;
  }
  return st;
}

int broyden_solve(InfNet* f, const float* y, int B, int T, double eps_in, InfBroydenStats* st, float* diff_detail,
                  Bufs& bf, hipStream_t s, SpecTail* tail = nullptr) {
  InfBroydenStats stats = stats_for(st);
  std::vector<double> lowest_ss;
  INF_TRY(ensure_f0(f, B, bf, s));
  bool first = true;             // Broyden starts at z = 0 (broyden.py:136-144): f(0) is cached (per batch size, so
                                 // that it has the bits of the batch's own kernels)
  const ResidFn resid = [&](const float* x, float* gout, float* dg, const float* gprev) {
    if (first) {
      first = false;
      if (f->fc) return launch_resid_bcast_fc(f->f0, bf.xemb, x, gout, bf.fcur, bf.part, B, f->d, s);
      return launch_resid_bcast(f->f0, bf.xemb, x, gout, bf.fcur, bf.part, B, f->d, bf.nchunk, s, bf.sample_sums,
                                bf.stop_ev, &bf.stop_bound);
    }
    return eval_resid_part(f, x, x, bf.xemb, gout, dg, gprev, B, bf, s);
  };
  // fused fc nets: each later iteration's update and residual are one launch (fcnet.hip br_on)
  const StepFn step = [&](const BroydenArgs& ba, float* gout, float* dg, const float* gprev) {
    OutArgs a;
    memset(&a, 0, sizeof(a));
    a.in0 = bf.xemb;
    a.in1 = ba.xnew;
    a.in2 = gprev;
    a.out0 = gout;
    a.out1 = dg;
    a.out2 = bf.fcur;
    a.partial = bf.part;
    a.nchunk = bf.nchunk;
    a.stop_ev = bf.stop_ev;
    a.stop_bound = &bf.stop_bound;
    a.mode = OM_RESID;
    a.bias = f->L.back().b;
    FcArgs fa = fc_args(f, ba.xnew, B);
    fa.o = a;
    fa.br_on = 1;
    fa.br = ba;
    return launch_fcnet(fa, false, s);
  };
  const StartFn start = [&](float* x0, float* g0, float* upd, float* x1, float* dx) {
    first = false;
    if (!f->fc)          // (conv: broyden_core's zero-copy per-sample sums are on whenever this start is passed)
      return launch_broyden_start_sample(f->f0, bf.xemb, x0, g0, bf.fcur, bf.part, bf.stop_ev, &bf.stop_bound, upd,
                                         x1, dx, B, f->d, s);
    return launch_broyden_start_fc(f->f0, bf.xemb, x0, g0, bf.fcur, bf.part, bf.stop_ev, &bf.stop_bound, upd, x1, dx,
                                   B, f->d, s);
  };
  // conv nets: the one-launch start where the residual sums go straight into the readback slot (broyden_core zc)
  const bool conv_start = !f->fc && SAMPLE_SUMS && out_nchunk(f->d) <= 4;
  if (f->line_search) {
    // line_search(on=True) (broyden.py:66-99): the global rule only (a per-sample step size is not the reference's)
    if (f->convergence != INF_CONV_GLOBAL) return INF_ERR_UNSUPPORTED;
    INF_TRY(broyden_core_ls(f, resid, B, T, eps_in, stats, lowest_ss, bf, s, /*keep_f=*/true));
  } else {
    INF_TRY(broyden_core(f, resid, B, T, eps_in, stats, lowest_ss, bf, s, /*keep_f=*/true, f->fcfused ? &step : nullptr,
                         (f->fc || conv_start) ? &start : nullptr, tail, /*resid_sample_sums=*/true));
  }
  if (diff_detail) {
    std::vector<float> dd(B);
    for (int b = 0; b < B; ++b) dd[b] = (float)sqrt(lowest_ss[b]);
    INF_HIP(hipMemcpyAsync(diff_detail, dd.data(), sizeof(float) * B, hipMemcpyHostToDevice, s));
    INF_HIP(hipStreamSynchronize(s));
  }
  if (stats.prot_break) {
    // banach_find_root (implicit_block.py:57-65,74-75): z <- x_embed - f(z) from z0 = y, <= 1000 iterations;
    // per-sample mode: only the samples whose own solve broke, each with its own stopping test
    std::vector<int> todo;
    if (f->convergence == INF_CONV_PER_SAMPLE) {
      const int stride = PS_HEAD + T;
      std::vector<double> pst((size_t)B * stride);
      INF_HIP(hipMemcpyAsync(pst.data(), bf.ps_state, sizeof(double) * pst.size(), hipMemcpyDeviceToHost, s));
      INF_HIP(hipStreamSynchronize(s));
      todo.resize(B);
      for (int b = 0; b < B; ++b) todo[b] = (int)pst[(size_t)b * stride + 5];
    }
    int it = 0;
    INF_TRY(banach_solve(f, y, B, eps_in, 1000, todo.empty() ? nullptr : todo.data(), bf, s, &it));
    stats.fixed_point_iters = it;
  }
  if (st) *st = stats;
  return INF_OK;
}

// inf_imblock_eval_exact on the device-resident block kernel (fcblock.hip): one launch, one readback of its
// statistics; a protective break runs the Banach fallback and the recompute on the host path (as below).
static thread_local char* g_bk_host = nullptr;
static thread_local size_t g_bk_host_cap = 0;
static thread_local hipEvent_t g_bk_ev = nullptr;
int fc_block_eval(InfNet* nx, InfNet* nz, const float* x, float* z, float* logdet_x, float* logdet_z, int B, int T,
                  double eps_in, InfBroydenStats* stats, Bufs& bf, hipStream_t s) {
  if (nx->mfma_mode != INF_MFMA_F16X3 || nz->mfma_mode != INF_MFMA_F16X3 || !bf.bk_sync || nz->line_search)
    return INF_ERR_UNSUPPORTED;
  FcBlockArgs a;
  memset(&a, 0, sizeof(a));
  a.nx = fc_args(nx, nullptr, B);
  a.nz = fc_args(nz, nullptr, B);
  a.B = B;
  a.T = T;
  a.per_sample = nz->convergence == INF_CONV_PER_SAMPLE;
  if (!fcblock_supported(a)) return INF_ERR_UNSUPPORTED;
  const int d = nz->d;
  a.eps = eps_in * sqrt((double)B * d);                              // broyden.py:131
  a.eps_ps = eps_in * sqrt((double)d);
  a.x = x;
  a.z = z;
  a.logdet_x = logdet_x;
  a.logdet_z = logdet_z;
  a.xin_g = bf.xin;
  a.fx_g = bf.fx;
  a.xemb_g = bf.xemb;
  a.lowx_g = bf.lowest;
  a.lowf_g = bf.flow;
  a.error = bf.bk_sync;
  a.gran = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(bf.bk_sync) + 16);
  a.tag0 = 1;
  FcBlockStats* dst = reinterpret_cast<FcBlockStats*>(bf.bk_out);
  a.stats = dst;
  a.s_nstep = reinterpret_cast<int*>(bf.bk_out + sizeof(FcBlockStats));
  a.s_lstep = a.s_nstep + B;
  a.s_prot = a.s_lstep + B;
  a.s_lowest = reinterpret_cast<double*>(bf.bk_out + ((sizeof(FcBlockStats) + sizeof(int) * 3 * (size_t)B + 7) & ~(size_t)7));
  INF_HIP(hipMemsetAsync(bf.bk_sync, 0, bf.bk_sync_bytes, s));
  {
    const int st = launch_fcblock(a, s);
    if (st != INF_OK) return st;
  }
  // one readback: the error word and the statistics (per-sample rule: the per-sample arrays too)
  const size_t nbytes = a.per_sample ? bf.bk_out_bytes : sizeof(FcBlockStats);
  if (g_bk_host_cap < nbytes + 16) {
    if (g_bk_host) (void)hipHostFree(g_bk_host);
    g_bk_host = nullptr;
    g_bk_host_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&g_bk_host), nbytes + 16, hipHostMallocCoherent) != hipSuccess)
      return INF_ERR_HIP;
    g_bk_host_cap = nbytes + 16;
  }
  INF_HIP(hipMemcpyAsync(g_bk_host, bf.bk_sync, 16, hipMemcpyDeviceToHost, s));
  INF_HIP(hipMemcpyAsync(g_bk_host + 16, bf.bk_out, nbytes, hipMemcpyDeviceToHost, s));
  if (!g_bk_ev && hipEventCreateWithFlags(&g_bk_ev, INF_EV_SYNC) != hipSuccess) return INF_ERR_HIP;
  hipEvent_t ev = g_bk_ev;
  INF_HIP(hipEventRecord(ev, s));
  INF_TRY(host_wait(ev));
  if (*reinterpret_cast<unsigned*>(g_bk_host) != 0) {
    set_hip_error(hipErrorLaunchTimeOut);
    return INF_ERR_HIP;
  }
  const FcBlockStats* hs = reinterpret_cast<const FcBlockStats*>(g_bk_host + 16);
  InfBroydenStats st = stats_for(stats);
  st.convergence = nz->convergence;
  if (!a.per_sample) {
    st.nstep = hs->nstep;
    st.lowest_step = hs->lowest_step;
    st.prot_break = hs->prot_break;
    st.n_trace = std::min(hs->n_trace, 64);
    for (int k = 0; k < st.n_trace; ++k) st.trace[k] = hs->trace[k];
    st.diff = hs->lowest;
    st.eps = a.eps;
  } else {
    const char* base = g_bk_host + 16;
    const int* sn = reinterpret_cast<const int*>(base + sizeof(FcBlockStats));
    const int* sl = sn + B;
    const int* sp = sl + B;
    const double* slo = reinterpret_cast<const double*>(
        base + ((sizeof(FcBlockStats) + sizeof(int) * 3 * (size_t)B + 7) & ~(size_t)7));
    double d2 = 0.0;
    for (int b = 0; b < B; ++b) {
      st.nstep = std::max(st.nstep, sn[b]);
      st.lowest_step = std::max(st.lowest_step, sl[b]);
      st.prot_break |= sp[b];
      d2 += slo[b] * slo[b];
      if (st.sample_nstep) st.sample_nstep[b] = sn[b];
      if (st.sample_lowest_step) st.sample_lowest_step[b] = sl[b];
      if (st.sample_prot_break) st.sample_prot_break[b] = sp[b];
    }
    st.diff = sqrt(d2);
    st.eps = a.eps_ps;
  }
  st.tnstep = st.nstep;
  if (st.prot_break) {
    // banach_find_root (implicit_block.py:57-65,74-75) from z0 = x, as broyden_solve does, on the buffers the kernel
    // left: x_embed, f_x(x), x and the lowest iterates (per-sample rule: only the samples whose own solve broke)
    std::vector<int> todo;
    if (a.per_sample) {
      const int* sp = reinterpret_cast<const int*>(g_bk_host + 16 + sizeof(FcBlockStats)) + 2 * B;
      todo.assign(sp, sp + B);
    }
    int it = 0;
    INF_TRY(banach_solve(nz, bf.xin, B, eps_in, 1000, todo.empty() ? nullptr : todo.data(), bf, s, &it));
    st.fixed_point_iters = it;
    OutArgs o;
    memset(&o, 0, sizeof(o));
    o.in0 = bf.fx;
    o.in1 = bf.xin;
    o.out0 = bf.tmp;
    INF_TRY(run_forward(nz, bf.lowest, B, bf, OM_RECOMP, &o, s));
    FcArgs fjz = fc_args(nz, bf.tmp, B);
    fjz.logdet = logdet_z;
    INF_TRY(launch_fcnet(fjz, true, s));
    INF_TRY(to_boundary(nx, bf.tmp, z, B, s));
  }
  if (stats) *stats = st;
  return INF_OK;
}

// ---------------------------------------------------------------------------------------------
// Parameter gradients (training path) on the generic GEMM operands (W_eff packed at refresh).
// Nets whose intermediate activations are Swish or Sin: layer l computes h_l = W_l * in_l + b_l,
// in_0 = preact(x), in_l = act(h_{l-1}) (applied once from the stored pre-activation).  Conv nets in their (B, C, H, W)
// layout; fc nets feature-major (d, N), N columns as one image of N pixels (gemm_base) -- the C-ABI entries transpose
// the (B, d) boundary tensors in and out.
// ---------------------------------------------------------------------------------------------
struct GradBufs {
  std::vector<float*> H, Hd, Ad;     // pre-activations, their tangents, activation tangents (Ad[0]: input)
  std::vector<float*> A;             // layer inputs after their activation (A[0] = preact(x)), computed once per call
  float *gA, *gB, *hA, *hB, *gad, *ga, *Y, *slab, *dWe, *dWe2, *dsig, *xin, *tmp_in, *act;
  float *x_t, *w_t, *e_t, *gx_t;     // fc nets: the internal-layout (d, N) copies of the boundary inputs / x-gradient
  double *bpart, *dot;
  int max_split;
};
constexpr int GRAD_SPLIT = 32;
constexpr int GRAD_BLOCKS = 512;

size_t carve_grad(const InfNet* n, int B, void* ws, size_t cap, GradBufs& g) {
  WS w{reinterpret_cast<char*>(ws), cap, 0};
  const size_t hid = (size_t)B * n->hidden_max * n->P, in = (size_t)B * n->d;
  const int L = (int)n->L.size();
  size_t mn = 1;
  for (const auto& l : n->L) mn = std::max(mn, (size_t)l.cout * l.cin * l.ks * l.ks);
  g.H.resize(L > 0 ? L - 1 : 0);
  g.Hd.resize(L > 0 ? L - 1 : 0);
  g.Ad.resize(L > 0 ? L : 0);
  for (auto& p : g.H) p = w.take<float>(hid);
  for (auto& p : g.Hd) p = w.take<float>(hid);
  for (int l = 0; l < L; ++l) g.Ad[l] = w.take<float>(l == 0 ? in : hid);
  g.A.resize(L > 0 ? L : 0);
  for (int l = 0; l < L; ++l) g.A[l] = w.take<float>(l == 0 ? in : hid);
  for (float** p : {&g.gA, &g.gB, &g.hA, &g.hB, &g.gad, &g.ga}) *p = w.take<float>(std::max(hid, in));
  g.Y = w.take<float>((size_t)B * n->rows_max * n->P);
  g.slab = w.take<float>((size_t)GRAD_SPLIT * mn);
  g.dWe = w.take<float>(mn);
  g.dWe2 = w.take<float>(mn);
  g.dsig = w.take<float>(mn);
  g.xin = w.take<float>(in);
  g.tmp_in = w.take<float>(in);
  for (float** p : {&g.x_t, &g.w_t, &g.e_t, &g.gx_t}) *p = n->fc ? w.take<float>(in) : nullptr;
  g.act = w.take<float>(std::max(hid, in));   // swish of a stored pre-activation (weight-gradient operand)
  g.bpart = w.take<double>(std::max<size_t>(GRAD_BLOCKS + 64, glue_batched_dot_scratch(B, (long)n->hidden_max * n->P) + 64));
  g.dot = w.take<double>(128);      // [0] the dot, [1..64] its block partials
  g.max_split = GRAD_SPLIT;
  return w.off + 256;
}

// Input of layer l as the GEMMs consume it: x (l = 0) or H[l-1], with its swish (preact / activation)
// applied once into gb.A[l] instead of in every output tile's loader.  Returns the operand, no beta left.
static int layer_input(InfNet* n, int l, const float* x, GradBufs& gb, int B, hipStream_t s, const float** out) {
  const float* in = l == 0 ? x : gb.H[l - 1];
  const int act = l == 0 ? n->pre_act : n->L[l - 1].act;
  const float* pb = l == 0 ? n->pre_beta : n->L[l - 1].act_beta;
  if (act == ACT_NONE) {
    *out = in;
    return INF_OK;
  }
  const long ne = (long)B * n->L[l].cin * n->P;
  INF_TRY(launch_act_apply(in, act, pb, gb.A[l], ne, s));
  *out = gb.A[l];
  return INF_OK;
}

// h_l = W_l * in (+ b_l); in gets swish(., pre_beta) on load when pre_beta is set.  l < L-1 (no taps).
static int layer_fwd(InfNet* n, int l, const float* in, const float* pre_beta, bool bias, float* out, int B,
                     hipStream_t s) {
  const WLayer& w = n->L[l];
  GemmArgs g = gemm_base(n, w.f, in, w.cin, B);
  g.pre_beta = pre_beta;
  set_out(n, g, out, w.cout);
  g.bias = bias ? w.b : nullptr;
  return launch_gemm(g, w.f.load, bias ? EP_BIAS : EP_STORE, s);
}

// out = W_l^T gout  (input-side gradient of layer l, no activation factor)
static int layer_vjp(InfNet* n, int l, const float* gout, float* out, int B, GradBufs& gb, hipStream_t s) {
  const WLayer& w = n->L[l];
  GemmArgs g = gemm_base(n, w.g, gout, w.cout, B);
  if (w.g.taps) {
    set_out(n, g, gb.Y, w.g.M);
    INF_TRY(launch_gemm(g, w.g.load, EP_STORE, s));
    OutArgs a;
    memset(&a, 0, sizeof(a));
    a.Y = gb.Y;
    a.y_sample = (long)w.g.M * n->P;
    a.C = w.cin;
    a.H = n->H;
    a.W = n->W;
    a.ks = 3;
    a.mode = OM_VJP;
    a.out0 = out;
    return launch_conv_out(a, B, s);
  }
  set_out(n, g, out, w.cin);
  return launch_gemm(g, w.g.load, EP_STORE, s);
}

// dW_eff of layer l = sum_{b,p} G (x) X~ (accumulate: add into gb.dWe), X = in_l
static int layer_wgrad(InfNet* n, int l, const float* G, const float* X, const float* x_beta, float* out, int B,
                       GradBufs& gb, hipStream_t s) {
  const WLayer& w = n->L[l];
  WgradArgs a;
  memset(&a, 0, sizeof(a));
  a.G = G;
  a.X = X;
  a.x_beta = x_beta;
  a.B = n->fc ? 1 : B;               // fc: one image of B columns
  a.P = n->fc ? B : n->P;
  a.H = n->fc ? 1 : n->H;
  a.W = n->fc ? B : n->W;
  a.g_sample = (long)w.cout * a.P;
  a.x_sample = (long)w.cin * a.P;
  a.ks = w.ks;
  a.M = w.cout;
  a.N = w.cin * w.ks * w.ks;
  a.slab = gb.slab;
  a.out = out;
  a.max_split = gb.max_split;
  return launch_wgrad(a, s);
}

// dW (raw weight) from dW_eff through W_eff = W / max(1, sigma / coeff), sigma = u . (W v)
static int layer_sigma_chain(InfNet* n, int l, const float* dWe, float* dW, GradBufs& gb, hipStream_t s) {
  const WLayer& w = n->L[l];
  const bool spatial = w.ks > 1;
  WgradArgs a;                                  // dsigma/dW = u (x) v~ (one "sample")
  memset(&a, 0, sizeof(a));
  a.G = w.u;
  a.X = w.v;
  a.B = 1;
  a.P = spatial ? n->P : 1;
  a.H = spatial ? n->H : 1;
  a.W = spatial ? n->W : 1;
  a.g_sample = (long)w.cout * a.P;
  a.x_sample = (long)w.cin * a.P;
  a.ks = w.ks;
  a.M = w.cout;
  a.N = w.cin * w.ks * w.ks;
  a.slab = gb.slab;
  a.out = gb.dsig;
  a.max_split = gb.max_split;
  INF_TRY(launch_wgrad(a, s));
  return launch_sigma_chain(dWe, w.W, gb.dsig, w.factor, w.coeff, gb.dot, dW, (long)w.cout * w.cin * w.ks * w.ks, s);
}

static bool grad_supported(const InfNet* n) {
  if (n->L.empty()) return false;
  for (size_t l = 0; l + 1 < n->L.size(); ++l)
    if (n->L[l].act != ACT_SWISH && n->L[l].act != ACT_SIN) return false;
  if (n->L.back().act != ACT_NONE) return false;
  if (n->fc && n->pre_act != ACT_NONE) return false;
  return n->pre_act == ACT_NONE || n->pre_act == ACT_SWISH;
}

static float* grad_out(float* const* arr, int l) { return arr ? arr[l] : nullptr; }

// layer l's gradients from G_hd (against the tangent input) and G_h (against the primal input, may be null)
static int layer_param_grads(InfNet* n, int l, const float* G_tan, const float* X_tan, const float* G_pri,
                             const float* X_pri, const float* X_pri_beta, const InfNetGrads* gr, int B, GradBufs& gb,
                             hipStream_t s) {
  const WLayer& w = n->L[l];
  float* dW = grad_out(gr->dW, l);
  if (dW) {
    const long mn = (long)w.cout * w.cin * w.ks * w.ks;
    // the primal operand's swish once per element, not inside every output tile's loader
    if (G_pri && X_pri_beta) {
      INF_TRY(launch_act_apply(X_pri, ACT_SWISH, X_pri_beta, gb.act, (long)B * w.cin * n->P, s));
      X_pri = gb.act;
      X_pri_beta = nullptr;
    }
    if (G_tan) {
      INF_TRY(layer_wgrad(n, l, G_tan, X_tan, nullptr, gb.dWe, B, gb, s));
      if (G_pri) {
        INF_TRY(layer_wgrad(n, l, G_pri, X_pri, X_pri_beta, gb.dWe2, B, gb, s));
        INF_TRY(glue_add(gb.dWe2, gb.dWe, gb.dWe, mn, s));
      }
    } else {
      INF_TRY(layer_wgrad(n, l, G_pri, X_pri, X_pri_beta, gb.dWe, B, gb, s));
    }
    INF_TRY(layer_sigma_chain(n, l, gb.dWe, dW, gb, s));
  }
  float* db = grad_out(gr->db, l);
  if (db) {
    if (G_pri) INF_TRY(n->fc ? launch_channel_sum(G_pri, 1, w.cout, B, db, s) : launch_channel_sum(G_pri, B, w.cout, n->P, db, s));
    else INF_HIP(hipMemsetAsync(db, 0, sizeof(float) * w.cout, s));
  }
  return INF_OK;
}

}  // namespace

// ==============================================================================================
// C-ABI
// ==============================================================================================
extern "C" {

int inf_version(void) { return 1; }

const char* inf_status_string(int s) {
  switch (s) {
    case INF_OK: return "ok";
    case INF_ERR_INVALID: return "invalid argument";
    case INF_ERR_HIP: return "HIP runtime error";
    case INF_ERR_WORKSPACE: return "workspace too small";
    case INF_ERR_UNSUPPORTED: return "unsupported net layout";
    default: return "unknown status";
  }
}

int inf_last_hip_error(void) { return inf::g_last_hip; }

// Re-points a net at other tensors of the same layout (a DataParallel replica's copies of the parameters on another
// device, lib/_hip native_net): the pointers the refresh and the launches read change, nothing is repacked -- the caller
// refreshes only when the values differ from the last refresh's.
int inf_net_set_tensors(InfNet* n, const InfNetDesc* desc) {
  if (!n || !desc || desc->n_layers <= 0 || !desc->layers) return INF_ERR_INVALID;
  int i = 0;
  const bool pre = desc->layers[0].kind == INF_ACT_SWISH || desc->layers[0].kind == INF_ACT_SIN;
  if (pre != (n->pre_act != ACT_NONE)) return INF_ERR_INVALID;
  if (pre) i = 1;
  size_t l = 0;
  std::vector<WLayer> L = n->L;
  const float* pre_beta = pre ? desc->layers[0].beta : n->pre_beta;
  for (; i < desc->n_layers; ++i) {
    const InfLayerDesc& d = desc->layers[i];
    if (d.kind == INF_LAYER_CONV || d.kind == INF_LAYER_LINEAR) {
      if (l >= L.size()) return INF_ERR_INVALID;
      WLayer& w = L[l++];
      const int ks = d.kind == INF_LAYER_LINEAR ? 1 : d.ksize;
      if (w.kind != d.kind || w.cin != d.cin || w.cout != d.cout || w.ks != ks || !d.weight || !d.bias || !d.u || !d.v)
        return INF_ERR_INVALID;
      w.W = d.weight;
      w.b = d.bias;
      w.u = d.u;
      w.v = d.v;
    } else if (d.kind == INF_ACT_SWISH || d.kind == INF_ACT_SIN) {
      if (l == 0 || L[l - 1].act != (d.kind == INF_ACT_SWISH ? ACT_SWISH : ACT_SIN)) return INF_ERR_INVALID;
      L[l - 1].act_beta = d.beta;
    } else {
      return INF_ERR_INVALID;
    }
  }
  if (l != L.size()) return INF_ERR_INVALID;
  n->L = L;
  n->pre_beta = pre_beta;
  return INF_OK;
}

int inf_net_create(const InfNetDesc* desc, InfNet** out) {
  if (!desc || !out || desc->n_layers <= 0 || !desc->layers) return INF_ERR_INVALID;
  InfNet* n = new (std::nothrow) InfNet();
  if (!n) return INF_ERR_INVALID;
  n->C = desc->channels;
  n->H = desc->height;
  n->W = desc->width;
  n->P = n->H * n->W;
  n->d = n->C * n->P;
  int i = 0;
  // leading activation (preact, implicit_flow.py:371-373)
  if (desc->layers[0].kind == INF_ACT_SWISH || desc->layers[0].kind == INF_ACT_SIN) {
    n->pre_act = desc->layers[0].kind == INF_ACT_SWISH ? ACT_SWISH : ACT_SIN;
    n->pre_beta = desc->layers[0].beta;
    if (n->pre_act != ACT_SWISH) { delete n; return INF_ERR_UNSUPPORTED; }
    i = 1;
  }
  for (; i < desc->n_layers; ++i) {
    const InfLayerDesc& d = desc->layers[i];
    if (d.kind == INF_LAYER_CONV || d.kind == INF_LAYER_LINEAR) {
      WLayer w;
      w.kind = d.kind;
      w.cin = d.cin;
      w.cout = d.cout;
      w.ks = d.kind == INF_LAYER_LINEAR ? 1 : d.ksize;
      w.W = d.weight;
      w.b = d.bias;
      w.u = d.u;
      w.v = d.v;
      w.coeff = d.coeff;
      if (w.ks != 1 && w.ks != 3) { delete n; return INF_ERR_UNSUPPORTED; }
      if (!w.b) { delete n; return INF_ERR_UNSUPPORTED; }
      n->L.push_back(w);
    } else if (d.kind == INF_ACT_SWISH || d.kind == INF_ACT_SIN) {
      if (n->L.empty() || n->L.back().act != ACT_NONE) { delete n; return INF_ERR_UNSUPPORTED; }
      n->L.back().act = d.kind == INF_ACT_SWISH ? ACT_SWISH : ACT_SIN;
      n->L.back().act_beta = d.beta;
    } else {
      delete n;
      return INF_ERR_INVALID;
    }
  }
  const int L = (int)n->L.size();
  if (L == 0 || n->L.back().act != ACT_NONE) { delete n; return INF_ERR_UNSUPPORTED; }
  n->fc = n->L[0].kind == INF_LAYER_LINEAR;
  if (n->fc) {
    n->d = n->C;
    n->P = 1;
  }
  // channel chain: C -> ... -> C
  int ch = n->C;
  for (auto& w : n->L) {
    if (w.cin != ch || (n->fc && w.kind != INF_LAYER_LINEAR) || (!n->fc && w.kind != INF_LAYER_CONV)) {
      delete n;
      return INF_ERR_UNSUPPORTED;
    }
    ch = w.cout;
  }
  if (ch != n->C) { delete n; return INF_ERR_UNSUPPORTED; }
  if (n->fc && n->C > 32) { delete n; return INF_ERR_UNSUPPORTED; }
  // plans
  size_t floats = 0;
  for (int l = 0; l < L; ++l) {
    WLayer& w = n->L[l];
    const bool last = l == L - 1, first = l == 0;
    if (l < L - 1) n->hidden_max = std::max(n->hidden_max, w.cout);
    // forward operand
    if (w.ks == 1) {
      w.f = Operand{BL_DIRECT, 0, w.cout, 0, w.cin, 0, PK_ROWMAJOR, nullptr};
    } else if (last && w.cout < TAPS_MAX_CH) {
      w.f = Operand{BL_DIRECT, 1, 9 * w.cout, 0, w.cin, 0, PK_TAPS_FWD, nullptr};
    } else {
      w.f = Operand{BL_IM2COL3, 0, w.cout, 0, 9 * w.cin, 0, PK_IM2COL_FWD, nullptr};
    }
    if (!last && w.f.taps) { delete n; return INF_ERR_UNSUPPORTED; }
    // vjp operand (maps grad wrt output -> grad wrt input)
    if (w.ks == 1) {
      w.g = Operand{BL_DIRECT, 0, w.cin, 0, w.cout, 0, PK_TRANSPOSE, nullptr};
    } else if (first && w.cin < TAPS_MAX_CH) {
      w.g = Operand{BL_DIRECT, 1, 9 * w.cin, 0, w.cout, 0, PK_TAPS_BWD, nullptr};
    } else {
      w.g = Operand{BL_IM2COL3, 0, w.cin, 0, 9 * w.cout, 0, PK_IM2COL_BWD, nullptr};
    }
    for (Operand* op : {&w.f, &w.g}) {
      op->Mpad = round_up(op->M, 128);
      op->Kpad = round_up(op->K, 16);
      floats += (size_t)op->Mpad * op->Kpad + 64;
    }
    floats += 64;   // factor
    if (last) n->rows_max = std::max(n->rows_max, w.f.M);
    if (first) n->rows_max = std::max(n->rows_max, w.g.M);
  }
  if (L == 1) n->hidden_max = std::max(n->hidden_max, 1);
  // fused fc net (fcnet.hip): 128-wide hidden layers with one activation kind, no input pre-activation
  {
    const char* off = getenv("INFLOW_NO_FUSED");
    bool ok = n->fc && n->pre_act == ACT_NONE && L >= 2 && L <= FC_MAXL && !(off && off[0] == '1');
    for (int l = 0; ok && l < L; ++l) {
      const WLayer& w = n->L[l];
      if (l < L - 1 && (w.cout != 128 || w.act != n->L[0].act)) ok = false;
    }
    if (ok) {
      FcArgs f;
      memset(&f, 0, sizeof(f));
      f.nl = L;
      f.d = n->d;
      f.act = n->L[0].act;
      for (int l = 0; l < L; ++l) f.L[l].Kpad = n->L[l].f.Kpad;
      n->fcfused = fcnet_supported(f, false) != 0;
    }
    if (n->fcfused) {
      // f16x3 planes (fcnet_h3.hip): the input layer 8 row tiles x 1 k step, hidden 8 x 4, output 1 x 4; fragment tiles
      // of 2 x 512 halves.  The fused fc kernels default to f16x3 (INFLOW_MFMA=f32 / fp32: exact fp32 MFMA; the fc
      // kernels have no bf16x6 variant, bf16x6 selects exact fp32 for them)
      size_t halves = 0;
      for (int l = 0; l < L; ++l) {
        n->fch_off.push_back(halves);
        const int nrt = l == L - 1 ? 1 : 8, nks = l == 0 ? 1 : 4;
        halves += (size_t)nrt * nks * 1024;
      }
      if (hipMalloc(&n->fch, 2 * halves * sizeof(uint16_t)) != hipSuccess ||
          hipMalloc(&n->fchexp, 2 * (size_t)L * sizeof(int)) != hipSuccess) {
        if (n->fch) (void)hipFree(n->fch);
        delete n;
        return INF_ERR_HIP;
      }
      n->fcht = n->fch + halves;            // one allocation each: freed with fch / fchexp
      n->fchtexp = n->fchexp + L;
      n->mfma_mode = INF_MFMA_F16X3;
      const char* mm = getenv("INFLOW_MFMA");
      if (mm && *mm) {
        if (!strcmp(mm, "f32") || !strcmp(mm, "fp32") || !strcmp(mm, "bf16x6")) n->mfma_mode = INF_MFMA_F32;
        else if (strcmp(mm, "f16x3") != 0) {
          fprintf(stderr, "libinflow: INFLOW_MFMA=%s is not one of f32, fp32, bf16x6, f16x3\n", mm);
          (void)hipFree(n->fch);
          (void)hipFree(n->fchexp);
          delete n;
          return INF_ERR_INVALID;
        }
      }
    }
  }
  // fused 3-1-3 conv net (run_cifar10.sh nets): 3x3 C->H, swish, 1x1 H->H, swish, 3x3 H->C
  {
    const char* off = getenv("INFLOW_NO_FUSED");
    const bool shape_ok = !n->fc && L == 3 && n->L[0].ks == 3 && n->L[1].ks == 1 && n->L[2].ks == 3 &&
                          n->L[0].act == ACT_SWISH && n->L[1].act == ACT_SWISH &&
                          n->L[0].cout == n->L[1].cin && n->L[1].cin == n->L[1].cout && n->L[1].cout == n->L[2].cin;
    if (shape_ok && !(off && off[0] == '1') && net313_supported(n->L[1].cout, n->C, n->H, n->W)) {
      n->fused = true;
      n->fhid = n->L[1].cout;
      n->K1pad = round_up(9 * n->C, 16);
      n->M3 = 9 * n->C;
      n->M3pad = round_up(9 * n->C, 32);
      floats += 2 * ((size_t)n->fhid * n->K1pad + (size_t)n->fhid * n->fhid + (size_t)n->M3pad * n->fhid) + 6 * 64;
      // split planes: 3 bf16 (= 1.5 floats) per element of each of the six operands
      floats += 3 * ((size_t)n->fhid * n->K1pad + (size_t)n->fhid * n->fhid + (size_t)n->M3pad * n->fhid) + 6 * 64;
      // F16X3 planes: 2 fp16 (= 1 float) per element of each of the six operands, plus the scale exponents
      floats += 2 * ((size_t)n->fhid * n->K1pad + (size_t)n->fhid * n->fhid + (size_t)n->M3pad * n->fhid) + 6 * 64 + 64;
      floats += 2 * (size_t)n->M3pad * n->fhid + 2 * 64;   // the permuted phase-C planes Fhp
      n->rows_max = std::max(n->rows_max, n->M3);
      const char* mm = getenv("INFLOW_MFMA");             // "f32" / "fp32" / "bf16x6" / "f16x3" (default)
      n->mfma_mode = INF_MFMA_F16X3;
      if (mm && *mm) {
        if (!strcmp(mm, "f32") || !strcmp(mm, "fp32")) n->mfma_mode = INF_MFMA_F32;
        else if (!strcmp(mm, "bf16x6")) n->mfma_mode = INF_MFMA_BF16X6;
        else if (strcmp(mm, "f16x3") != 0) {
          fprintf(stderr, "libinflow: INFLOW_MFMA=%s is not one of f32, fp32, bf16x6, f16x3\n", mm);
          delete n;
          return INF_ERR_INVALID;
        }
      }
    }
  }
  {
    // defaults of the per-net options; an unrecognised value fails inf_net_create (as INFLOW_MFMA does) rather
    // than silently selecting another rule
    struct EnvOpt { const char* name; int* slot; const char* const* values; int n; };
    static const char* const k128_v[] = {"0", "1", "2"};
    static const char* const k128_v4[] = {"0", "1", "2", "3"};
    static const char* const bin_v[] = {"0", "1"};
    static const char* const conv_v[] = {"global", "per_sample"};
    const EnvOpt opts[] = {{"INFLOW_FUSED_K128", &n->k128, k128_v4, 4},
                           {"INFLOW_EVAL_OVERLAP", &n->eval_overlap, bin_v, 2},
                           {"INFLOW_CONVERGENCE", &n->convergence, conv_v, 2},
                           {"INFLOW_FC_BLOCK", &n->fc_block, k128_v, 3},
                           {"INFLOW_FC_SERIES", &n->fc_series, bin_v, 2},
                           {"INFLOW_FUSED_PRESPLIT", &n->presplit, bin_v, 2}};
    for (const EnvOpt& o : opts) {
      const char* e = getenv(o.name);
      if (!e || !*e) continue;
      int v = -1;
      for (int i = 0; i < o.n; ++i)
        if (!strcmp(e, o.values[i])) v = i;
      if (v < 0) {
        fprintf(stderr, "libinflow: %s=%s is not one of", o.name, e);
        for (int i = 0; i < o.n; ++i) fprintf(stderr, " %s", o.values[i]);
        fprintf(stderr, "\n");
        delete n;
        return INF_ERR_INVALID;
      }
      *o.slot = v;
    }
  }
  // sigma scratch: one partial per 256 output elements of the largest conv (or per channel-split block)
  size_t sc = SIGMA_MAX_PARTS + 64;
  for (auto& w : n->L) sc = std::max(sc, (size_t)w.cout * (n->fc ? 1 : n->P) / 256 + 64);
  n->scratch_doubles = sc;
  if (hipGetDevice(&n->device) != hipSuccess) n->device = 0;
  if (hipMalloc(&n->dev, floats * sizeof(float)) != hipSuccess ||
      hipMalloc(&n->scratch, sc * sizeof(double)) != hipSuccess) {
    if (n->dev) (void)hipFree(n->dev);
    delete n;
    return INF_ERR_HIP;
  }
  float* p = n->dev;
  for (auto& w : n->L) {
    for (Operand* op : {&w.f, &w.g}) {
      op->A = p;
      p += (size_t)op->Mpad * op->Kpad + 64;
    }
    w.factor = p;
    p += 64;
  }
  if (n->fused) {
    float** bufs[] = {&n->F1f, &n->F1b, &n->F2f, &n->F2b, &n->F3f, &n->F3b};
    const size_t sz[] = {(size_t)n->fhid * n->K1pad, (size_t)n->fhid * n->K1pad, (size_t)n->fhid * n->fhid,
                         (size_t)n->fhid * n->fhid, (size_t)n->M3pad * n->fhid, (size_t)n->M3pad * n->fhid};
    for (int i = 0; i < 6; ++i) {
      *bufs[i] = p;
      p += sz[i] + 64;
    }
    for (int i = 0; i < 6; ++i) {
      n->Fs[i] = reinterpret_cast<uint16_t*>(p);
      p += (3 * sz[i] + 1) / 2 + 64;
    }
    for (int i = 0; i < 6; ++i) {
      n->Fh[i] = reinterpret_cast<uint16_t*>(p);
      p += sz[i] + 64;
    }
    n->Fexp = reinterpret_cast<int*>(p);
    p += 64;
    for (int i = 0; i < 2; ++i) {
      n->Fhp[i] = reinterpret_cast<uint16_t*>(p);
      p += (size_t)n->M3pad * n->fhid + 64;
    }
  }
  *out = n;
  return INF_OK;
}

int inf_net_set_mfma(InfNet* n, int mode) {
  if (!n || (mode != INF_MFMA_F32 && mode != INF_MFMA_BF16X6 && mode != INF_MFMA_F16X3)) return INF_ERR_INVALID;
  // the cached f(0) (ensure_f0) carries the bits of the arithmetic it was computed with
  if (n->mfma_mode != mode) n->f0_batch = -1;
  n->mfma_mode = mode;
  return INF_OK;
}
int inf_net_get_mfma(const InfNet* n) { return n ? n->mfma_mode : -1; }

int inf_net_destroy(InfNet* n) {
  if (!n) return INF_OK;
  if (n->dev) (void)hipFree(n->dev);
  if (n->scratch) (void)hipFree(n->scratch);
  if (n->f0) (void)hipFree(n->f0);
  if (n->fch) (void)hipFree(n->fch);
  if (n->fchexp) (void)hipFree(n->fchexp);
  delete n;
  return INF_OK;
}

int inf_net_refresh(InfNet* n, void* stream) {
  if (!n) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  n->f0_batch = -1;
  for (auto& w : n->L) {
    const int H = n->fc ? 1 : (w.ks == 1 ? 1 : n->H), Wd = n->fc ? 1 : (w.ks == 1 ? 1 : n->W);
    INF_TRY(launch_sigma(w.W, w.u, w.v, w.cout, w.cin, w.ks, H, Wd, w.coeff, w.factor,
                         reinterpret_cast<float*>(n->scratch), s));
    INF_TRY(launch_pack(w.W, w.factor, w.f.A, w.cout, w.cin, w.ks, w.f.Mpad, w.f.Kpad, w.f.pack, s));
    INF_TRY(launch_pack(w.W, w.factor, w.g.A, w.cout, w.cin, w.ks, w.g.Mpad, w.g.Kpad, w.g.pack, s));
  }
  if (n->fch) {
    const int L = (int)n->L.size();
    for (int l = 0; l < L; ++l) {
      const WLayer& w = n->L[l];
      const int nrt = l == L - 1 ? 1 : 8, nks = l == 0 ? 1 : 4;
      INF_TRY(launch_fc_split_h3(w.f.A, w.cout, w.f.Kpad, nrt, nks, n->fch + n->fch_off[l], n->fchexp + l, s));
      // transposed position j = L-1-l: rows cin, k = cout (w.g.A = W^T, row stride g.Kpad), position j's tile shape
      const int j = L - 1 - l, trt = j == L - 1 ? 1 : 8, tks = j == 0 ? 1 : 4;
      INF_TRY(launch_fc_split_h3(w.g.A, w.cin, w.g.Kpad, trt, tks, n->fcht + n->fch_off[j], n->fchtexp + j, s));
    }
  }
  if (n->fused) {
    const WLayer &l0 = n->L[0], &l1 = n->L[1], &l2 = n->L[2];
    const int H = n->fhid;
    INF_TRY(launch_pack(l0.W, l0.factor, n->F1f, l0.cout, l0.cin, 3, H, n->K1pad, PK_IM2COL_FWD, s, 1));
    INF_TRY(launch_pack(l2.W, l2.factor, n->F1b, l2.cout, l2.cin, 3, H, n->K1pad, PK_IM2COL_BWD, s, 1));
    INF_TRY(launch_pack(l1.W, l1.factor, n->F2f, H, H, 1, H, H, PK_ROWMAJOR, s, 1));
    INF_TRY(launch_pack(l1.W, l1.factor, n->F2b, H, H, 1, H, H, PK_TRANSPOSE, s, 1));
    INF_TRY(launch_pack(l2.W, l2.factor, n->F3f, l2.cout, l2.cin, 3, n->M3pad, H, PK_TAPS_FWD, s, 1));
    INF_TRY(launch_pack(l0.W, l0.factor, n->F3b, l0.cout, l0.cin, 3, n->M3pad, H, PK_TAPS_BWD, s, 1));
    const float* src[6] = {n->F1f, n->F1b, n->F2f, n->F2b, n->F3f, n->F3b};
    const long cnt[6] = {(long)H * n->K1pad, (long)H * n->K1pad, (long)H * H, (long)H * H, (long)n->M3pad * H,
                         (long)n->M3pad * H};
    for (int i = 0; i < 6; ++i) INF_TRY(launch_split3(src[i], n->Fs[i], cnt[i], s));
    for (int i = 0; i < 6; ++i) INF_TRY(launch_split2h(src[i], n->Fh[i], cnt[i], n->Fexp + 3 * (i & 1) + i / 2, s));
    for (int i = 0; i < 2; ++i) INF_TRY(launch_permute_k23(n->Fh[4 + i], n->Fhp[i], cnt[4 + i] / 512, s));
  }
  return INF_OK;
}

size_t inf_workspace_bytes(const InfNet* n, int batch, int threshold) {
  if (!n || batch <= 0) return 0;
  return ws_need(n, batch, std::max(threshold, 1));
}

int inf_net_forward(InfNet* n, const float* x, float* y, int B, void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !y || B <= 0) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  int st = INF_OK;
  const float* xi = to_internal(n, x, bf.xin, B, s, &st);
  INF_TRY(st);
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.out0 = n->fc ? bf.tmp : y;
  INF_TRY(run_forward(n, xi, B, bf, OM_PLAIN, &a, s));
  if (n->fc) INF_TRY(to_boundary(n, bf.tmp, y, B, s));
  return INF_OK;
}

int inf_net_vjp(InfNet* n, const float* x, const float* v, float* out, int B, void* ws, size_t ws_bytes,
                void* stream) {
  if (!n || !x || !v || !out || B <= 0) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  int st = INF_OK;
  const float* xi = to_internal(n, x, bf.xin, B, s, &st);
  INF_TRY(st);
  const float* vi = to_internal(n, v, bf.eps_t, B, s, &st);
  INF_TRY(st);
  INF_TRY(run_forward(n, xi, B, bf, -1, nullptr, s));
  float* o = n->fc ? bf.tmp : out;
  INF_TRY(run_vjp(n, vi, o, xi, nullptr, nullptr, B, bf, s));
  if (n->fc) INF_TRY(to_boundary(n, bf.tmp, out, B, s));
  return INF_OK;
}

static int root_find_common(InfNet* f, InfNet* e, const float* y, int B, int T, double eps, InfBroydenStats* stats,
                            float* diff_detail, Bufs& bf, const float** yi_out, hipStream_t s) {
  int st = INF_OK;
  const float* yi = to_internal(f, y, bf.xin, B, s, &st);
  INF_TRY(st);
  // x_embed = e(y) + y ; fx = e(y)   (implicit_block.py:71)
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.in0 = yi;
  a.out0 = bf.fx;
  a.out1 = bf.xemb;
  INF_TRY(run_forward(e, yi, B, bf, OM_EMBED, &a, s));
  INF_TRY(broyden_solve(f, yi, B, T, eps, stats, diff_detail, bf, s));
  *yi_out = yi;
  return INF_OK;
}

int inf_root_find(InfNet* f, InfNet* e, const float* y, float* out, int B, int T, double eps, InfBroydenStats* stats,
                  float* diff_detail, void* ws, size_t ws_bytes, void* stream) {
  if (!f || !e || !y || !out || B <= 0 || T <= 0 || T > 64 || !same_shape(f, e)) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(f, B, T, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  const float* yi;
  INF_TRY(root_find_common(f, e, y, B, T, eps, stats, diff_detail, bf, &yi, s));
  return to_boundary(f, bf.lowest, out, B, s);
}

int inf_imblock_forward(InfNet* nx, InfNet* nz, const float* x, float* z, int B, int T, double eps,
                        InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream) {
  if (!nx || !nz || !x || !z || B <= 0 || T <= 0 || T > 64 || !same_shape(nx, nz)) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(nx, B, T, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  const float* xi;
  InfBroydenStats st = stats_for(stats);
  INF_TRY(root_find_common(nz, nx, x, B, T, eps, &st, nullptr, bf, &xi, s));
  if (stats) *stats = st;
  // z = (nnet_x(x) - nnet_z(z*)) + x   (implicit_block.py:227).  nnet_z(z*) was evaluated by the residual
  // that produced the lowest iterate (same input, same kernel: the same bits) and kept in bf.flow; only
  // after the Banach fallback (prot_break) is it evaluated again.
  if (!st.prot_break) {
    INF_TRY(glue_recomp(bf.fx, bf.flow, xi, nx->fc ? bf.tmp : z, (long)B * nx->d, s));
    if (nx->fc) INF_TRY(to_boundary(nx, bf.tmp, z, B, s));
    return INF_OK;
  }
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.in0 = bf.fx;
  a.in1 = xi;
  a.out0 = nx->fc ? bf.tmp : z;
  INF_TRY(run_forward(nz, bf.lowest, B, bf, OM_RECOMP, &a, s));
  if (nx->fc) INF_TRY(to_boundary(nx, bf.tmp, z, B, s));
  return INF_OK;
}

// Implicit backward of an imBlock (imBlock.Backward.backward, implicit_block.py:176-217):
//   dl_dh: Broyden root of g(y) = y (I + J_fz(z)) - grad from y = 0 (eps_backward, threshold), lowest iterate;
//   dl_dx = dl_dh (I + J_fx(x)).
int inf_imblock_backward(InfNet* nx, InfNet* nz, const float* z, const float* x, const float* grad, float* dl_dh,
                         float* dl_dx, int B, int T, double eps, InfBroydenStats* stats, void* ws, size_t ws_bytes,
                         void* stream) {
  if (!nx || !nz || !z || !x || !grad || !dl_dh || !dl_dx || B <= 0 || T <= 0 || T > 64 || !same_shape(nx, nz))
    return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  {
    Bufs bf;
    if (!ws || carve(nz, B, T, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
    int st = INF_OK;
    const float* zi = to_internal(nz, z, bf.xin, B, s, &st);
    INF_TRY(st);
    const float* gi = to_internal(nz, grad, bf.xemb, B, s, &st);
    INF_TRY(st);
    INF_TRY(run_forward(nz, zi, B, bf, -1, nullptr, s));      // activation derivatives at z
    InfBroydenStats bs = stats_for(stats);
    std::vector<double> lowest_ss;
    const ResidFn resid = [&](const float* y, float* gout, float* dg, const float* gprev) {
      return vjp_resid_part(nz, y, zi, gi, gout, dg, gprev, B, bf, s);
    };
    INF_TRY(broyden_core(nz, resid, B, T, eps, bs, lowest_ss, bf, s));
    if (stats) *stats = bs;
    INF_TRY(to_boundary(nz, bf.lowest, dl_dh, B, s));
  }
  // dl_dx = dl_dh + dl_dh^T J_fx(x)   (Fx = nnet_x(x) + x; Fx.backward(dl_dh), :210-213)
  Bufs bf;
  if (carve(nx, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  int st = INF_OK;
  const float* xi = to_internal(nx, x, bf.xin, B, s, &st);
  INF_TRY(st);
  const float* hi = to_internal(nx, dl_dh, bf.eps_t, B, s, &st);
  INF_TRY(st);
  INF_TRY(run_forward(nx, xi, B, bf, -1, nullptr, s));
  INF_TRY(run_vjp(nx, hi, bf.va, xi, nullptr, nullptr, B, bf, s));
  INF_TRY(glue_add(bf.va, hi, nx->fc ? bf.tmp : dl_dx, (long)B * nx->d, s));
  if (nx->fc) INF_TRY(to_boundary(nx, bf.tmp, dl_dx, B, s));
  return INF_OK;
}

// Power series of 1 or 2 fused nets of the same shape (the x- and z-branch of an imBlock advance in
// lockstep: one launch per term over both nets' tiles).  Term k's VJP stages term k-1's packed taps
// directly (tap sum, preact swish', trace partial -- conv_out's work), so a term is ONE launch; only
// the last term's taps go through conv_out.  Series slabs: part[k][b][snchunk] (zeroed first: the
// fused kernel fills one entry per tile, conv_out one per 1024-element chunk).
// Neumann mode (wouts != nullptr, ncoeff a host array of n_terms + 1): instead of the trace partials, each
// term's staging accumulates w += ncoeff[k] v_k for its own pixels (w starts as eps, the last term's taps go
// through conv_out), i.e. the Neumann vector of implicit_block.py:430-436 for 1 or 2 nets in lockstep.
int series_fused(InfNet* const* nets, const float* const* xs, const float* const* es, int nn, const float* coeff,
                 int n_terms, float* const* outs, int B, Bufs* bfs, hipStream_t s, unsigned save_mask = 3u,
                 float* const* wouts = nullptr, const float* ncoeff = nullptr) {
  Net313Args args[2];
  for (int i = 0; i < nn; ++i) {
    args[i] = net313_args(nets[i], xs[i], B, bfs[i], false);
    if (!wouts) INF_HIP(hipMemsetAsync(bfs[i].part, 0, sizeof(double) * n_terms * B * bfs[i].snchunk, s));
    else INF_HIP(hipMemcpyAsync(wouts[i], es[i], sizeof(float) * (size_t)B * nets[i]->d, hipMemcpyDeviceToDevice, s));
  }
  // activation derivatives (in the pair's tile layout); a net whose d1/d2 are already saved is skipped
  const unsigned all = (1u << nn) - 1u;
  if ((save_mask & all) == all) {
    INF_TRY(launch_net313_multi(args, nn, nets[0]->fhid, MODE_SAVE, s));
  } else {
    for (int i = 0; i < nn; ++i)
      if (save_mask & (1u << i)) INF_TRY(launch_net313_multi(&args[i], 1, nets[0]->fhid, MODE_SAVE, s, nn));
  }
  for (int k = 0; k < n_terms; ++k) {
    for (int i = 0; i < nn; ++i) {
      InfNet* n = nets[i];
      Bufs& bf = bfs[i];
      Net313Args& v = args[i];
      v = net313_args(n, es[i], B, bf, true);
      v.Y = (k % 2 == 0) ? bf.Y : bf.Y2;
      // serpentine: odd terms walk the tiles backwards, so a term starts on the derivative tiles the previous
      // one read last (still in the memory-side cache: s0 pair 349 -> 338 us per term)
      v.tile_order = k & 1;
      if (k > 0) {
        v.in = nullptr;
        v.in_taps = (k % 2 == 1) ? bf.Y : bf.Y2;
        v.vmul_x = n->pre_beta ? xs[i] : nullptr;
        v.vmul_beta = n->pre_beta;
        if (wouts) {
          v.acc_w = wouts[i];
          v.acc_coef = ncoeff[k];
        } else {
          v.dot_eps = es[i];
          v.dot_part = bf.part + (size_t)(k - 1) * B * bf.snchunk;
          v.dot_nchunk = bf.snchunk;
        }
      }
    }
    INF_TRY(launch_net313_multi(args, nn, nets[0]->fhid, MODE_VJP, s));
  }
  if (wouts) {
    for (int i = 0; i < nn; ++i) {
      InfNet* n = nets[i];
      Bufs& bf = bfs[i];
      OutArgs a;
      memset(&a, 0, sizeof(a));
      a.Y = ((n_terms - 1) % 2 == 0) ? bf.Y : bf.Y2;
      a.y_sample = (long)n->M3 * n->P;
      a.C = n->C;
      a.H = n->H;
      a.W = n->W;
      a.ks = 3;
      a.mode = OM_VJP;
      a.in1 = xs[i];
      a.out0 = bf.va;
      a.pre_beta = n->pre_beta;
      a.nchunk = bf.snchunk;
      INF_TRY(launch_conv_out(a, B, s));
      INF_TRY(glue_axpy_scaled(wouts[i], bf.va, ncoeff[n_terms], (long)B * n->d, s));
    }
    return INF_OK;
  }
  for (int i = 0; i < nn; ++i) {
    InfNet* n = nets[i];
    Bufs& bf = bfs[i];
    OutArgs a;
    memset(&a, 0, sizeof(a));
    a.Y = ((n_terms - 1) % 2 == 0) ? bf.Y : bf.Y2;
    a.y_sample = (long)n->M3 * n->P;
    a.C = n->C;
    a.H = n->H;
    a.W = n->W;
    a.ks = 3;
    a.mode = OM_VJP;
    a.in0 = es[i];
    a.in1 = xs[i];
    a.out0 = bf.va;
    a.pre_beta = n->pre_beta;
    a.partial = bf.part + (size_t)(n_terms - 1) * B * bf.snchunk;
    a.nchunk = bf.snchunk;
    INF_TRY(launch_conv_out(a, B, s));
  }
  for (int i = 0; i < nn; ++i)
    INF_TRY(launch_series_combine(bfs[i].part, coeff, n_terms, B, bfs[i].snchunk, outs[i], s));
  return INF_OK;
}

// One non-blocking side stream (+ fork / join events) per host thread and device, created on first use
// and kept for the process lifetime (calls on one thread are serial, so it is never shared concurrently).
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
static thread_local SideStream g_side[16];
static SideStream* side_stream() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  SideStream& ss = g_side[dev];
  if (!ss.s) {
    if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    if (hipEventCreateWithFlags(&ss.fork, INF_EV_SYNC) != hipSuccess ||
        hipEventCreateWithFlags(&ss.join, INF_EV_SYNC) != hipSuccess)
      return nullptr;
  }
  return &ss;
}

// Joins the side stream into the caller's stream when the eval pass returns, on every path after the fork
// (an error return included): the caller's next call may reuse the workspace the side stream still uses.
struct SideJoin {
  SideStream* side = nullptr;
  hipStream_t s = nullptr;
  ~SideJoin() {
    if (!side) return;
    (void)hipEventRecord(side->join, side->s);
    (void)hipStreamWaitEvent(s, side->join, 0);
  }
};

// Whole eval pass of an imBlock on fused nets (implicit_block.py:220-234 + 245-322 in eval): the x-net's
// x_embed launch also saves its activation derivatives at x (MODE_EVALSAVE), Broyden solves for z*,
// z = (f_x(x) - f_z(z*)) + x, then the paired power series of both branches with only the z-net's SAVE.
int inf_imblock_eval(InfNet* nx, InfNet* nz, const float* x, float* z, const float* eps_x, const float* eps_z,
                     const float* coeff, int n_terms, float* logdet_x, float* logdet_z, int B, int T, double eps,
                     InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream) {
  if (!nx || !nz || !x || !z || !eps_x || !eps_z || !coeff || !logdet_x || !logdet_z || B <= 0 || T <= 0 || T > 64 ||
      n_terms < 1 || n_terms > SERIES_MAX || !same_shape(nx, nz))
    return INF_ERR_INVALID;
  if (!(nx->fused && nz->fused && nx->fhid == nz->fhid)) return INF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const size_t half = ws_need(nx, B, T), zneed = ws_need(nz, B, 1), xneed = ws_need(nx, B, 1);
  if (!ws || ws_bytes < half + zneed) return INF_ERR_WORKSPACE;
  char* w0 = reinterpret_cast<char*>(ws);
  Bufs bfa, bfb, bfc;
  carve(nx, B, T, w0, half, bfa);
  carve(nz, B, 1, w0 + half, zneed, bfb);
  // Overlapped schedule (default; inf_net_set_option(INF_OPT_EVAL_OVERLAP, 0) or INFLOW_EVAL_OVERLAP=0 at create turn it off; needs workspace for a
  // third region): the x-branch series depends only on x, so it runs on a side stream while this stream does the
  // root solve (sync-bound, and short of work at the 8x8 scale) and then the z-branch series; the two streams join
  // before returning.  Concurrent series launches also desynchronise the CUs' d1/d2 bursts (every 1-WG/CU tile
  // of one launch reads its derivatives in the same phase): 2268 -> 2432 samples/s at B=64 with the 128-pixel VJP.
  const bool overlap = nx->eval_overlap && ws_bytes >= half + zneed + xneed;
  if (overlap) {
    carve(nx, B, 1, w0 + half + zneed, xneed, bfc);
    bfc.D = bfa.D;                              // the x_embed pass saves f_x's derivatives into bfa.D
  }
  const int layout = overlap ? 1 : 2;           // single-net series launches, or the pair's tile layout
  // x_embed = f_x(x) + x, saving f_x's derivatives at x (implicit_block.py:71)
  {
    Net313Args f = net313_args(nx, x, B, bfa, false);
    INF_TRY(launch_net313_multi(&f, 1, nx->fhid, MODE_EVALSAVE, s, layout));
    OutArgs a;
    memset(&a, 0, sizeof(a));
    a.Y = bfa.Y;
    a.y_sample = (long)nx->M3 * nx->P;
    a.C = nx->C;
    a.H = nx->H;
    a.W = nx->W;
    a.ks = 3;
    a.mode = OM_EMBED;
    a.bias = nx->L[2].b;
    a.in0 = x;
    a.out0 = bfa.fx;
    a.out1 = bfa.xemb;
    INF_TRY(launch_conv_out(a, B, s));
  }
  SideJoin join;
  if (overlap) {
    SideStream* side = side_stream();
    if (!side) return INF_ERR_HIP;
    INF_HIP(hipEventRecord(side->fork, s));
    INF_HIP(hipStreamWaitEvent(side->s, side->fork, 0));
    join.side = side;
    join.s = s;
    InfNet* nets1[1] = {nx};
    const float* xs1[1] = {x};
    const float* es1[1] = {eps_x};
    float* outs1[1] = {logdet_x};
    INF_TRY(series_fused(nets1, xs1, es1, 1, coeff, n_terms, outs1, B, &bfc, side->s, /*save_mask=*/0u));
  }
  InfBroydenStats st = stats_for(stats);
  INF_TRY(broyden_solve(nz, x, B, T, eps, &st, nullptr, bfa, s));
  if (stats) *stats = st;
  if (!st.prot_break) {
    INF_TRY(glue_recomp(bfa.fx, bfa.flow, x, z, (long)B * nx->d, s));
  } else {
    OutArgs a;
    memset(&a, 0, sizeof(a));
    a.in0 = bfa.fx;
    a.in1 = x;
    a.out0 = z;
    INF_TRY(run_forward(nz, bfa.lowest, B, bfa, OM_RECOMP, &a, s));
  }
  if (overlap) {
    InfNet* nets1[1] = {nz};
    const float* xs1[1] = {z};
    const float* es1[1] = {eps_z};
    float* outs1[1] = {logdet_z};
    return series_fused(nets1, xs1, es1, 1, coeff, n_terms, outs1, B, &bfb, s, /*save_mask=*/1u);   // join: ~SideJoin
  }
  InfNet* nets[2] = {nx, nz};
  const float* xs[2] = {x, z};
  const float* es[2] = {eps_x, eps_z};
  float* outs[2] = {logdet_x, logdet_z};
  Bufs bfs[2] = {bfa, bfb};
  return series_fused(nets, xs, es, 2, coeff, n_terms, outs, B, bfs, s, /*save_mask=*/2u);
}

// The next block's x-branch folded into this block's z-branch Jacobian launch (the chain call): both evaluate their net
// at this block's z, so one grid holds the two (launch_fcnet_jac_pair: 2 x 625 workgroups at B = 10 000 take 85 us
// against 2 x 56 us as two launches).  bf: the next block's buffers (its xin / fx / xemb), logdet: its
// logdet_x; done: the last launch this block queued was the pair (else the next block runs its own x-branch launch).
struct FcNextX {
  InfNet* nx = nullptr;
  Bufs* bf = nullptr;
  float* logdet = nullptr;
  bool done = false;
};
// The block's log-density step lout = lin - (logdet_x - logdet_z) folded into its z-branch Jacobian launch (the chain
// call); done: the last launch this block queued wrote it (else the caller runs glue_logp_step)
struct FcLogpStep {
  const float* lin = nullptr;
  float* lout = nullptr;
  bool done = false;
};
// whether inf_imblock_eval_exact takes the block kernel (fcblock.hip) for this solved net
static bool fc_block_first(const InfNet* nz) {
  return nz->fc_block == 2 || (nz->fc_block == 1 && nz->convergence == INF_CONV_PER_SAMPLE);
}
// f16x3 planes on both nets of a pair launch, same shape
static bool fc_pair_ok(const InfNet* a, const InfNet* b) {
  return a->fcfused && b->fcfused && a->mfma_mode == INF_MFMA_F16X3 && b->mfma_mode == INF_MFMA_F16X3 &&
         same_shape(a, b) && !a->L.empty() && !b->L.empty() && a->L[0].act == b->L[0].act;
}

// inf_imblock_eval_exact on carved buffers.  x_done: bf's xin / fx / xemb and logdet_x hold this block's x-branch
// already (the previous block's pair launch); next (nullable): fold the next block's x-branch into the z-branch launch.
static int eval_exact_fc(InfNet* nx, InfNet* nz, const float* x, float* z, float* logdet_x, float* logdet_z, int B,
                         int T, double eps, InfBroydenStats* stats, Bufs& bf, hipStream_t s, bool x_done,
                         FcNextX* next, FcLogpStep* lp = nullptr) {
  if (next) next->done = false;
  if (lp) lp->done = false;
  // x in the internal layout: written by the x-branch JAC launch's staging (it reads x in the boundary layout)
  const float* xi = bf.xin;
  if (fc_block_first(nz)) {
    // the whole block in one launch (fcblock.hip); falls through to the launch-per-iteration path below when the
    // configuration has no block kernel or (global rule) its grid cannot be co-resident.  The default (1) takes it for
    // the per-sample rule only: under the global rule the launch path is faster
    const int st = fc_block_eval(nx, nz, x, z, logdet_x, logdet_z, B, T, eps, stats, bf, s);
    if (st != INF_ERR_UNSUPPORTED) return st;
  }
  // log|det(I + J_fx(x))| (implicit_block.py:358-362) and x_embed = f_x(x) + x (:71) in one launch: the JAC kernel's primal
  // column is f_x(x) with the FWD kernel's bits (the same 16-column tiles, k slices and partial order), so the x_embed
  // launch is folded into it.  (Run beside the root solve on the side stream instead, the JAC launch took every CU
  // first and the x_embed launch waited behind it anyway)  Then the root solve and
  // z = (f_x(x) - f_z(z*)) + x   (implicit_block.py:74-80, 227)
  OutArgs a;
  memset(&a, 0, sizeof(a));
  if (!x_done) {
    FcArgs fjx = fc_args(nx, nullptr, B);
    fjx.x_bnd = x;
    fjx.x_int = bf.xin;
    fjx.logdet = logdet_x;
    fjx.o.in0 = xi;
    fjx.o.out0 = bf.fx;
    fjx.o.out1 = bf.xemb;
    INF_TRY(launch_fcnet(fjx, true, s));
  }
  // z = (f_x(x) - f_z(z*)) + x computed in the staging of the log|det(I + J_fz(z))| launch, which also writes z in the
  // boundary layout (the recompute and transpose launches of the path below, in one).  The solve queues it on its
  // predicted last iterate before it reads that iterate's norm (SpecTail), so the GPU does not wait for the host's
  // stop decision; if the solve's result is another iterate (or it breaks), it is queued again on the result.  With
  // next, the same launch evaluates the next block's x-branch at that z (its input recomputed in its own staging).
  auto jac_z = [&](const float* flow) {
    FcArgs fjz = fc_args(nz, nullptr, B);
    fjz.logdet = logdet_z;
    fjz.rc_fx = bf.fx;
    fjz.rc_fz = flow;
    fjz.rc_x = xi;
    fjz.rc_out = z;
    if (lp) {
      fjz.lp_in = lp->lin;
      fjz.lp_ldx = logdet_x;
      fjz.lp_out = lp->lout;
      lp->done = true;
    }
    if (next) {
      FcArgs fjn = fc_args(next->nx, nullptr, B);
      fjn.rc_fx = bf.fx;
      fjn.rc_fz = flow;
      fjn.rc_x = xi;
      fjn.x_int = next->bf->xin;
      fjn.logdet = next->logdet;
      fjn.o.out0 = next->bf->fx;
      fjn.o.out1 = next->bf->xemb;
      const int st = launch_fcnet_jac_pair(fjz, fjn, s);
      next->done = st == INF_OK;
      if (st != INF_ERR_UNSUPPORTED) return st;
    }
    return launch_fcnet(fjz, true, s);
  };
  SpecTail tail;
  tail.fn = [&](const float*, const float* f) { return jac_z(f); };
  InfBroydenStats sst = stats_for(stats);
  INF_TRY(broyden_solve(nz, xi, B, T, eps, &sst, nullptr, bf, s, nz->convergence == INF_CONV_GLOBAL ? &tail : nullptr));
  if (stats) *stats = sst;
  if (!sst.prot_break) {
    if (tail.x && tail.x == bf.lowest && tail.f == bf.flow) return INF_OK;   // the speculative launch has the result
    return jac_z(bf.flow);
  }
  if (next) next->done = false;
  if (lp) lp->done = false;
  memset(&a, 0, sizeof(a));
  a.in0 = bf.fx;
  a.in1 = xi;
  a.out0 = bf.tmp;
  INF_TRY(run_forward(nz, bf.lowest, B, bf, OM_RECOMP, &a, s));
  // log|det(I + J_fz(z))| at the recomputed z
  FcArgs fjz = fc_args(nz, bf.tmp, B);
  fjz.logdet = logdet_z;
  INF_TRY(launch_fcnet(fjz, true, s));
  return to_boundary(nx, bf.tmp, z, B, s);
}

static int eval_exact_check(InfNet* nx, InfNet* nz, const float* x, int B) {
  if (!nx->fcfused || !nz->fcfused || nx->d > 10) return INF_ERR_UNSUPPORTED;
  FcArgs probe = fc_args(nx, x, B);
  FcArgs probe_z = fc_args(nz, x, B);
  if (!fcnet_supported(probe, true) || !fcnet_supported(probe_z, true)) return INF_ERR_UNSUPPORTED;
  return INF_OK;
}

int inf_imblock_eval_exact(InfNet* nx, InfNet* nz, const float* x, float* z, float* logdet_x, float* logdet_z, int B,
                           int T, double eps, InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream) {
  if (!nx || !nz || !x || !z || !logdet_x || !logdet_z || B <= 0 || T <= 0 || T > 64 || !same_shape(nx, nz))
    return INF_ERR_INVALID;
  INF_TRY(eval_exact_check(nx, nz, x, B));
  Bufs bf;
  if (!ws || carve(nz, B, T, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  return eval_exact_fc(nx, nz, x, z, logdet_x, logdet_z, B, T, eps, stats, bf, (hipStream_t)stream, false, nullptr);
}

size_t inf_flow_chain_workspace_bytes(InfNet* const* net_z, int n_blocks, int batch, const int* thresholds) {
  if (!net_z || n_blocks <= 0 || batch <= 0 || !thresholds) return 0;
  size_t blk = 0;
  for (int i = 0; i < n_blocks; ++i)
    if (net_z[i]) blk = std::max(blk, inf_workspace_bytes(net_z[i], batch, thresholds[i]));
  const size_t d = net_z[0] ? (size_t)net_z[0]->d : 0;
  // two block workspaces (consecutive blocks alternate: the pair launch writes the next block's buffers while this
  // block's are live), two z and logp buffers, two logdet_x / logdet_z pairs
  return 2 * ((blk + 255) & ~(size_t)255) + 256 * 8 + sizeof(float) * ((size_t)2 * batch * d + (size_t)6 * batch);
}

// SequentialFlow of fc imBlocks in eval (train_tabular.py:314-336; container.py:12-20): block i is
// inf_imblock_eval_exact on the previous block's z, its log-density step logp <- logp - (logdet_x - logdet_z) on the device
// (implicit_block.py:234), the blocks back to back on the stream with no host round trip between them beyond the ones a
// block itself makes.  On the launch path (global rule, f16x3 nets) block i's z-branch Jacobian launch also evaluates
// block i + 1's x-branch (FcNextX): consecutive blocks alternate between two workspaces and logdet buffers.
int inf_flow_eval_exact_chain(InfNet* const* net_x, InfNet* const* net_z, int n_blocks, const float* x, float* z,
                              const float* logp_in, float* logp_out, int B, const int* thresholds, const double* eps,
                              InfBroydenStats* stats, void* ws, size_t ws_bytes, void* stream) {
  // logp_in == logp_out is refused: a block's log-density step is folded into its z-branch launch, which runs again
  // when the predicted last iterate was not the result, and would then read the already-updated log p
  if (!net_x || !net_z || n_blocks <= 0 || !x || !z || !logp_out || B <= 0 || !thresholds || !eps || x == z ||
      logp_in == logp_out)
    return INF_ERR_INVALID;
  for (int i = 0; i < n_blocks; ++i) {
    InfNet *nx = net_x[i], *nz = net_z[i];
    if (!nx || !nz || !same_shape(nx, nz) || !same_shape(nz, net_z[0]) || thresholds[i] <= 0 || thresholds[i] > 64)
      return INF_ERR_INVALID;
    INF_TRY(eval_exact_check(nx, nz, x, B));
  }
  if (!ws || ws_bytes < inf_flow_chain_workspace_bytes(net_z, n_blocks, B, thresholds)) return INF_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const size_t E = (size_t)B * net_z[0]->d;
  size_t blk = 0;
  for (int i = 0; i < n_blocks; ++i) blk = std::max(blk, inf_workspace_bytes(net_z[i], B, thresholds[i]));
  blk = (blk + 255) & ~(size_t)255;
  char* base = reinterpret_cast<char*>(ws);
  size_t off = 2 * blk;
  auto take = [&](size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    char* p = base + off;
    off += bytes;
    return reinterpret_cast<float*>(p);
  };
  float* zb[2] = {take(sizeof(float) * E), take(sizeof(float) * E)};
  float* ldx[2] = {take(sizeof(float) * B), take(sizeof(float) * B)};
  float* ldz[2] = {take(sizeof(float) * B), take(sizeof(float) * B)};
  float* lp[2] = {take(sizeof(float) * B), take(sizeof(float) * B)};
  Bufs bfs[2];
  auto carve_block = [&](int i) {
    return carve(net_z[i], B, thresholds[i], base + (size_t)(i & 1) * blk, blk, bfs[i & 1]) <= blk ? INF_OK
                                                                                                   : INF_ERR_WORKSPACE;
  };
  INF_TRY(carve_block(0));
  const float* in = x;
  const float* lin = logp_in;
  bool x_done = false;
  for (int i = 0; i < n_blocks; ++i) {
    const bool last = i == n_blocks - 1;
    float* out = last ? z : zb[i & 1];
    float* lout = last ? logp_out : lp[i & 1];
    FcNextX nxt;
    FcNextX* np = nullptr;
    if (!last) {
      INF_TRY(carve_block(i + 1));
      if (!fc_block_first(net_z[i]) && !fc_block_first(net_z[i + 1]) && fc_pair_ok(net_z[i], net_x[i + 1])) {
        nxt.nx = net_x[i + 1];
        nxt.bf = &bfs[(i + 1) & 1];
        nxt.logdet = ldx[(i + 1) & 1];
        np = &nxt;
      }
    }
    FcLogpStep lps;
    lps.lin = lin;
    lps.lout = lout;
    INF_TRY(eval_exact_fc(net_x[i], net_z[i], in, out, ldx[i & 1], ldz[i & 1], B, thresholds[i], eps[i],
                          stats ? &stats[i] : nullptr, bfs[i & 1], s, x_done, np, &lps));
    if (!lps.done) INF_TRY(glue_logp_step(lin, ldx[i & 1], ldz[i & 1], lout, B, s));
    x_done = np && nxt.done;
    in = out;
    lin = lout;
  }
  return INF_OK;
}

// The power series of fused f16x3 fc nets in one launch for the pair (fcblock.hip fcseries_kernel; inputs in the
// boundary layout), when the first net's INF_OPT_FC_SERIES is 1 and a kernel exists for the shape; else
// INF_ERR_UNSUPPORTED and the caller takes the per-layer path
static int fc_series(InfNet* const* nets, const float* const* xs, const float* const* es, const float* coeff,
                     int n_terms, float* const* outs, int nn, int B, hipStream_t s) {
  if (!nets[0]->fc_series || n_terms < 1) return INF_ERR_UNSUPPORTED;
  for (int i = 0; i < nn; ++i)
    if (!nets[i]->fcfused || !nets[i]->fcht || nets[i]->mfma_mode != INF_MFMA_F16X3) return INF_ERR_UNSUPPORTED;
  FcSeriesArgs a;
  memset(&a, 0, sizeof(a));
  a.nn = nn;
  a.nl = (int)nets[0]->L.size();
  a.d = nets[0]->d;
  a.act = nets[0]->L[0].act;
  a.B = B;
  a.n_terms = n_terms;
  for (int k = 0; k < n_terms; ++k) a.coeff[k] = coeff[k];
  for (int i = 0; i < nn; ++i) {
    const InfNet* n = nets[i];
    if ((int)n->L.size() != a.nl || n->d != a.d || n->L[0].act != a.act || a.nl > FC_MAXL) return INF_ERR_UNSUPPORTED;
    for (int l = 0; l < a.nl; ++l) {
      FcLayer& f = a.f[i].L[l];
      f.A = n->L[l].f.A;
      f.Ah = n->fch + n->fch_off[l];
      f.Aexp = n->fchexp + l;
      f.Kpad = n->L[l].f.Kpad;
      f.b = n->L[l].b;
      f.beta = n->L[l].act_beta;
      FcLayer& t = a.t[i].L[l];
      t.A = n->L[a.nl - 1 - l].g.A;                 // W_{nl-1-l}^T fp32 (the input layer's exact contraction)
      t.Kpad = n->L[a.nl - 1 - l].g.Kpad;
      t.Ah = n->fcht + n->fch_off[l];
      t.Aexp = n->fchtexp + l;
    }
    a.x[i] = xs[i];
    a.eps[i] = es[i];
    a.out[i] = outs[i];
  }
  return launch_fcseries(a, s);
}

// try_fc: the one-launch fc series first (inf_logdet_series); the pair's per-net fallback has already asked the first net
static int series_single(InfNet* n, const float* x, const float* vareps, const float* coeff, int n_terms, float* out,
                         int B, void* ws, size_t ws_bytes, hipStream_t s, bool try_fc) {
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  if (n_terms == 0) {
    INF_HIP(hipMemsetAsync(out, 0, sizeof(float) * B, s));
    return INF_OK;
  }
  if (try_fc) {
    InfNet* nets1[1] = {n};
    const int st = fc_series(nets1, &x, &vareps, coeff, n_terms, &out, 1, B, s);
    if (st != INF_ERR_UNSUPPORTED) return st;
  }
  int st = INF_OK;
  const float* xi = to_internal(n, x, bf.xin, B, s, &st);
  INF_TRY(st);
  const float* ei = to_internal(n, vareps, bf.eps_t, B, s, &st);
  INF_TRY(st);
  if (n->fused) return series_fused(&n, &xi, &ei, 1, coeff, n_terms, &out, B, &bf, s);
  INF_TRY(run_forward(n, xi, B, bf, -1, nullptr, s));
  const float* v = ei;
  for (int k = 0; k < n_terms; ++k) {
    float* vo = (k % 2 == 0) ? bf.va : bf.vb;
    INF_TRY(run_vjp(n, v, vo, xi, ei, bf.part + (size_t)k * B * bf.nchunk, B, bf, s));
    v = vo;
  }
  return launch_series_combine(bf.part, coeff, n_terms, B, bf.nchunk, out, s);
}

int inf_logdet_series(InfNet* n, const float* x, const float* vareps, const float* coeff, int n_terms, float* out,
                      int B, void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !vareps || !coeff || !out || B <= 0 || n_terms < 0 || n_terms > SERIES_MAX) return INF_ERR_INVALID;
  return series_single(n, x, vareps, coeff, n_terms, out, B, ws, ws_bytes, (hipStream_t)stream, true);
}

// Both log-det series of an imBlock (x-branch and z-branch, implicit_block.py:318-322) advanced in
// lockstep: when both nets take the fused path, every term is ONE launch over both nets' tiles.
// ws must hold 2 x inf_workspace_bytes(net, batch, 1).
int inf_logdet_series_pair(InfNet* na, const float* xa, const float* ea, InfNet* nb, const float* xb, const float* eb,
                           const float* coeff, int n_terms, float* out_a, float* out_b, int B, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!na || !nb || !xa || !xb || !ea || !eb || !coeff || !out_a || !out_b || B <= 0 || n_terms < 0 ||
      n_terms > SERIES_MAX || !same_shape(na, nb))
    return INF_ERR_INVALID;
  const size_t half = ws_need(na, B, 1);
  if (!ws || ws_bytes < 2 * half) return INF_ERR_WORKSPACE;
  char* w0 = reinterpret_cast<char*>(ws);
  if (n_terms > 0) {
    InfNet* nets2[2] = {na, nb};
    const float* xs2[2] = {xa, xb};
    const float* es2[2] = {ea, eb};
    float* outs2[2] = {out_a, out_b};
    const int st = fc_series(nets2, xs2, es2, coeff, n_terms, outs2, 2, B, (hipStream_t)stream);
    if (st != INF_ERR_UNSUPPORTED) return st;
  }
  if (!(na->fused && nb->fused && na->fhid == nb->fhid)) {
    INF_TRY(series_single(na, xa, ea, coeff, n_terms, out_a, B, w0, half, (hipStream_t)stream, false));
    return series_single(nb, xb, eb, coeff, n_terms, out_b, B, w0 + half, half, (hipStream_t)stream, false);
  }
  hipStream_t s = (hipStream_t)stream;
  Bufs bfa, bfb;
  carve(na, B, 1, w0, half, bfa);
  carve(nb, B, 1, w0 + half, half, bfb);
  if (n_terms == 0) {
    INF_HIP(hipMemsetAsync(out_a, 0, sizeof(float) * B, s));
    INF_HIP(hipMemsetAsync(out_b, 0, sizeof(float) * B, s));
    return INF_OK;
  }
  InfNet* nets[2] = {na, nb};
  const float* xs[2] = {xa, xb};
  const float* es[2] = {ea, eb};
  float* outs[2] = {out_a, out_b};
  Bufs bfs[2] = {bfa, bfb};
  return series_fused(nets, xs, es, 2, coeff, n_terms, outs, B, bfs, s);
}

// neumann_vjp of neumann_logdet_estimator (implicit_block.py:429-436): w = eps + sum_k ncoeff[k] eps^T J^k,
// accumulated in k order into bf.tmp (internal layout).  Leaves the activation derivatives of x saved.
static int neumann_w(InfNet* n, const float* xi, const float* ei, const float* ncoeff, int n_terms, int B, Bufs& bf,
                     hipStream_t s) {
  const size_t E = (size_t)B * n->d;
  INF_TRY(run_forward(n, xi, B, bf, -1, nullptr, s));
  INF_HIP(hipMemcpyAsync(bf.tmp, ei, sizeof(float) * E, hipMemcpyDeviceToDevice, s));
  const float* v = ei;
  for (int k = 1; k <= n_terms; ++k) {
    float* vo = (k % 2 == 1) ? bf.va : bf.vb;
    INF_TRY(run_vjp(n, v, vo, xi, nullptr, nullptr, B, bf, s));
    INF_TRY(glue_axpy_scaled(bf.tmp, vo, ncoeff[k], (long)E, s));
    v = vo;
  }
  return INF_OK;
}

int inf_neumann_vector(InfNet* n, const float* x, const float* vareps, const float* ncoeff, int n_terms, float* w,
                       int B, void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !vareps || !ncoeff || !w || B <= 0 || n_terms < 0) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  int st = INF_OK;
  const float* xi = to_internal(n, x, bf.xin, B, s, &st);
  INF_TRY(st);
  const float* ei = to_internal(n, vareps, bf.eps_t, B, s, &st);
  INF_TRY(st);
  INF_TRY(neumann_w(n, xi, ei, ncoeff, n_terms, B, bf, s));
  return to_boundary(n, bf.tmp, w, B, s);
}

// Both nets' Neumann vectors (x- and z-branch of an imBlock's training log-det) in lockstep: one fused VJP
// launch per term for both nets with the accumulation folded into the next term's staging.  Nets off the
// fused path (or n_terms == 0) fall back to two inf_neumann_vector computations.
int inf_neumann_vector_pair(InfNet* na, const float* xa, const float* ea, InfNet* nb, const float* xb,
                            const float* eb, const float* ncoeff, int n_terms, float* wa, float* wb, int B, void* ws,
                            size_t ws_bytes, void* stream) {
  if (!na || !nb || !xa || !xb || !ea || !eb || !ncoeff || !wa || !wb || B <= 0 || n_terms < 0 || !same_shape(na, nb))
    return INF_ERR_INVALID;
  const size_t half = ws_bytes / 2;
  if (!(na->fused && nb->fused && na->fhid == nb->fhid) || n_terms == 0) {
    INF_TRY(inf_neumann_vector(na, xa, ea, ncoeff, n_terms, wa, B, ws, half, stream));
    return inf_neumann_vector(nb, xb, eb, ncoeff, n_terms, wb, B, reinterpret_cast<char*>(ws) + half, half, stream);
  }
  hipStream_t s = (hipStream_t)stream;
  Bufs bfs[2];
  if (!ws || carve(na, B, 1, ws, half, bfs[0]) > half ||
      carve(nb, B, 1, reinterpret_cast<char*>(ws) + half, half, bfs[1]) > half)
    return INF_ERR_WORKSPACE;
  InfNet* nets[2] = {na, nb};
  const float* xs[2] = {xa, xb};
  const float* es[2] = {ea, eb};
  float* wouts[2] = {wa, wb};
  float* outs[2] = {nullptr, nullptr};
  return series_fused(nets, xs, es, 2, nullptr, n_terms, outs, B, bfs, s, 3u, wouts, ncoeff);
}

int inf_logdet_neumann(InfNet* n, const float* x, const float* vareps, const float* ncoeff, int n_terms, float* out,
                       int B, void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !vareps || !ncoeff || !out || B <= 0 || n_terms < 0) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  int st = INF_OK;
  const float* xi = to_internal(n, x, bf.xin, B, s, &st);
  INF_TRY(st);
  const float* ei = to_internal(n, vareps, bf.eps_t, B, s, &st);
  INF_TRY(st);
  INF_TRY(neumann_w(n, xi, ei, ncoeff, n_terms, B, bf, s));
  INF_TRY(run_vjp(n, bf.tmp, bf.va, xi, ei, bf.part, B, bf, s));
  const float one = 1.f;
  return launch_series_combine(bf.part, &one, 1, B, bf.nchunk, out, s);
}

// Forward-mode Jacobian of a small fc net: [primal | d tangents] pushed through every layer; returns
// the tangent block (J[i][j] of sample b at t[i*(d+1)*B + (j+1)*B + b]) in *tang.
static int fc_jacobian(InfNet* n, const float* x, int B, Bufs& bf, const float** tang, hipStream_t s) {
  const int d = n->d;
  int st = INF_OK;
  const float* xi = to_internal(n, x, bf.xin, B, s, &st);
  INF_TRY(st);
  if (n->fcfused) {
    FcArgs f = fc_args(n, xi, B);
    f.tang = bf.ext1;
    if (fcnet_supported(f, true)) {
      INF_TRY(launch_fcnet(f, true, s));
      *tang = bf.ext1;
      return INF_OK;
    }
  }
  INF_TRY(glue_init_tangents(xi, bf.ext0, d, B, s));
  const int cols = (d + 1) * B;
  const float* cur = bf.ext0;
  for (size_t l = 0; l < n->L.size(); ++l) {
    const WLayer& w = n->L[l];
    float* o = (l % 2 == 0) ? bf.ext1 : bf.ext0;
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = w.f.A;
    g.M = w.f.M;
    g.Kpad = w.f.Kpad;
    g.Ktot = w.f.K;
    g.X = cur;
    g.x_sample = 0;
    g.P = cols;
    g.N = cols;
    g.H = 1;
    g.W = cols;
    g.out = o;
    g.o_sample = 0;
    g.bias = w.b;
    g.n_primal = B;
    INF_TRY(launch_gemm(g, BL_DIRECT, EP_BIAS_PRIMAL, s));
    if (w.act != ACT_NONE) INF_TRY(launch_fwdmode_act(o, nullptr, w.cout, B, d, w.act, w.act_beta, s));
    cur = o;
  }
  *tang = cur;
  return INF_OK;
}

int inf_logdet_exact(InfNet* n, const float* x, float* out, int B, void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !out || B <= 0) return INF_ERR_INVALID;
  if (!n->fc || n->d > 16 || n->pre_act != ACT_NONE) return INF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  if (n->fcfused) {                   // forward-mode Jacobian and the LU in one launch
    int st = INF_OK;
    const float* xi = to_internal(n, x, bf.xin, B, s, &st);
    INF_TRY(st);
    FcArgs f = fc_args(n, xi, B);
    f.logdet = out;
    if (fcnet_supported(f, true)) return launch_fcnet(f, true, s);
  }
  const float* tang = nullptr;
  INF_TRY(fc_jacobian(n, x, B, bf, &tang, s));
  return launch_logdet_small(tang, out, n->d, B, B, s);
}

int inf_logdet_exact_trace(InfNet* n, const float* x, const float* coeff, int n_terms, float* out, int B, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!n || !x || !coeff || !out || B <= 0 || n_terms < 1 || n_terms > SERIES_MAX) return INF_ERR_INVALID;
  if (!n->fc || n->d > 16 || n->pre_act != ACT_NONE) return INF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(n, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  const float* tang = nullptr;
  INF_TRY(fc_jacobian(n, x, B, bf, &tang, s));
  return launch_trace_series(tang, coeff, n_terms, out, n->d, B, B, s);
}

size_t inf_broyden_workspace_bytes(int batch, int d, int threshold) {
  const size_t nchunk = (size_t)(d + 1023) / 1024;
  return sizeof(double) * ((size_t)batch * nchunk * (3 * (size_t)threshold + 2) + 64);
}

int inf_broyden_update(float* U, float* VT, const float* dx, const float* dg, const float* gx, const float* x,
                       float* update, float* x_next, float* dx_next, int B, int d, int T, int nstep, void* ws,
                       size_t ws_bytes, void* stream) {
  if (!U || !VT || !dx || !dg || !gx || !x || !update || !x_next || !dx_next || B <= 0 || d <= 0 || T <= 0 ||
      T > 64 || nstep < 1 || nstep > T)
    return INF_ERR_INVALID;
  if (!ws || ws_bytes < inf_broyden_workspace_bytes(B, d, T)) return INF_ERR_WORKSPACE;
  BroydenArgs ba;
  memset(&ba, 0, sizeof(ba));
  ba.batch = B;
  ba.d = d;
  ba.T = T;
  ba.sb = d;
  ba.si = 1;
  ba.cs = (long)B * d;
  ba.U = U;
  ba.VT = VT;
  ba.dx = dx;
  ba.dg = dg;
  ba.gx = gx;
  ba.x = x;
  ba.xnew = x_next;
  ba.dxnew = dx_next;
  ba.upd = update;
  ba.part = reinterpret_cast<double*>(ws);
  ba.m = (nstep - 1) % T;
  ba.ncols = std::min(nstep, T);
  return launch_broyden_update(ba, (hipStream_t)stream);
}

int inf_broyden_line_step(const float* x0, const float* update, float step, float* x_est, float* dx, size_t n,
                          void* stream) {
  if (!x0 || !update || !x_est || !dx || n == 0) return INF_ERR_INVALID;
  return launch_line_step(x0, update, step, x_est, dx, (long)n, (hipStream_t)stream);
}

// ---- teardown ---------------------------------------------------------------------------------
// The calling thread's engine-held host resources: the pinned readback slots and their events, the block kernel's
// statistics buffer and event, the side streams and their fork / join events, the profiling events.  They were kept
// for the process lifetime and left to the HIP runtime's own exit-time teardown; releasing them before it (lib/_hip
// registers this with atexit) leaves that teardown nothing of ours.  Waits for the device first.  Idempotent; nets stay
// valid and the next call re-creates what it needs.
int inf_shutdown(void) {
  int rc = INF_OK;
  if (hipDeviceSynchronize() != hipSuccess) rc = INF_ERR_HIP;
  for (SumsSlot& sl : g_sums_slots) {
    if (sl.host) (void)hipHostFree(sl.host);
    if (sl.ev) (void)hipEventDestroy(sl.ev);
    sl = SumsSlot{};
  }
  if (g_bk_host) (void)hipHostFree(g_bk_host);
  g_bk_host = nullptr;
  g_bk_host_cap = 0;
  if (g_bk_ev) (void)hipEventDestroy(g_bk_ev);
  g_bk_ev = nullptr;
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (int dev = 0; dev < 16; ++dev) {
    SideStream& ss = g_side[dev];
    if (!ss.s) continue;
    (void)hipSetDevice(dev);
    (void)hipStreamSynchronize(ss.s);
    if (ss.fork) (void)hipEventDestroy(ss.fork);
    if (ss.join) (void)hipEventDestroy(ss.join);
    (void)hipStreamDestroy(ss.s);
    ss = SideStream{};
  }
  (void)hipSetDevice(cur);
  for (auto& p : g_prof) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  g_prof.clear();
  g_prof_used = 0;
  g_prof_on = false;
  return rc;
}

// ---- launch timing --------------------------------------------------------------------------
int inf_profile_begin(int max_launches) {
  if (max_launches <= 0) return INF_ERR_INVALID;
  for (auto& p : g_prof) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  g_prof.assign((size_t)max_launches, ProfSlot{});
  for (auto& p : g_prof) {
    INF_HIP(hipEventCreateWithFlags(&p.a, INF_EV_TIMING));
    INF_HIP(hipEventCreateWithFlags(&p.b, INF_EV_TIMING));
  }
  g_prof_used = 0;
  g_prof_on = true;
  return INF_OK;
}

int inf_profile_end(InfKernelStat* out, int max_out, int* n_out) {
  g_prof_on = false;
  std::vector<InfKernelStat> agg;
  for (size_t i = 0; i < g_prof_used; ++i) {
    ProfSlot& p = g_prof[i];
    INF_HIP(hipEventSynchronize(p.b));
    float ms = 0.f;
    INF_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    InfKernelStat* st = nullptr;
    for (auto& s : agg)
      if (s.tag == p.tag) st = &s;
    if (!st) {
      InfKernelStat z;
      memset(&z, 0, sizeof(z));
      z.tag = p.tag;
      agg.push_back(z);
      st = &agg.back();
    }
    st->launches += 1;
    st->total_ms += ms;
    st->flops += p.flops;
    st->bytes += p.bytes;
    st->peak_ms += p.peak_ms;
  }
  const int n = (int)std::min<size_t>(agg.size(), (size_t)std::max(max_out, 0));
  for (int i = 0; i < n; ++i) out[i] = agg[i];
  if (n_out) *n_out = (int)agg.size();
  g_prof_used = 0;
  return INF_OK;
}

// ---- flow glue ------------------------------------------------------------------------------
int inf_logit_forward(const float* x, float* y, const float* logp_in, float* logp_out, int B, int per, float alpha,
                      void* stream) {
  if (!x || !y || !logp_out || B <= 0 || per <= 0) return INF_ERR_INVALID;
  return glue_logit(x, y, logp_in, logp_out, B, per, alpha, (hipStream_t)stream);
}
int inf_actnorm_forward(const float* x, float* y, const float* w, const float* b, const float* logp_in,
                        float* logp_out, int B, int C, int hw, void* stream) {
  if (!x || !y || !w || !b || B <= 0) return INF_ERR_INVALID;
  return glue_actnorm(x, y, w, b, logp_in, logp_out, B, C, hw, (hipStream_t)stream);
}
int inf_squeeze2(const float* x, float* y, int B, int C, int H, int W, void* stream) {
  if (!x || !y || B <= 0 || (H & 1) || (W & 1)) return INF_ERR_INVALID;
  return glue_squeeze2(x, y, B, C, H, W, (hipStream_t)stream);
}
int inf_normal_logprob(const float* z, float* out, int B, int per, void* stream) {
  if (!z || !out || B <= 0) return INF_ERR_INVALID;
  return glue_normal_logprob(z, out, B, per, (hipStream_t)stream);
}
int inf_rademacher(float* out, size_t n, uint64_t seed, uint64_t offset, void* stream) {
  if (!out && n) return INF_ERR_INVALID;
  return glue_rademacher(out, n, seed, offset, (hipStream_t)stream);
}
}  // extern "C"

namespace {
// sum(gout * f(x)) differentiated into every parameter (and x, into gx when given) on internal-layout tensors: conv
// (B, C, H, W), fc (d, B)
int param_grad_core(InfNet* n, const float* x, const float* gout, float* gx, const InfNetGrads* gr, int B, GradBufs& gb,
                    hipStream_t s) {
  const int L = (int)n->L.size();
  const long hidP = (long)n->P;
  // forward: pre-activations (each layer's input activated once, gb.A)
  std::vector<const float*> Ain(L, nullptr);
  for (int l = 0; l < L; ++l) {
    INF_TRY(layer_input(n, l, x, gb, B, s, &Ain[l]));
    if (l + 1 < L) INF_TRY(layer_fwd(n, l, Ain[l], nullptr, true, gb.H[l], B, s));
  }
  // backward
  const float* g = gout;
  float* bufs[2] = {gb.gA, gb.gB};
  for (int l = L - 1; l >= 0; --l) {
    INF_TRY(layer_param_grads(n, l, nullptr, nullptr, g, Ain[l], nullptr, gr, B, gb, s));
    if (l > 0) {
      const WLayer& prev = n->L[l - 1];
      const long ne = (long)B * prev.cout * hidP;
      INF_TRY(layer_vjp(n, l, g, gb.ga, B, gb, s));
      float* gp = bufs[l & 1];
      INF_TRY(launch_act_bwd1(gb.ga, gb.H[l - 1], prev.act, prev.act_beta, gp, gb.bpart, ne, GRAD_BLOCKS, s));
      float* dbeta = grad_out(gr->dbeta, l - 1);
      if (dbeta && prev.act == ACT_SWISH) INF_TRY(launch_beta_reduce(gb.bpart, GRAD_BLOCKS, dbeta, 0, s));
      g = gp;
    } else if (gx || (n->pre_beta && gr->dpre_beta)) {
      const long ne = (long)B * n->d;
      float* gin = gx ? gx : gb.tmp_in;
      if (n->pre_beta) {
        INF_TRY(layer_vjp(n, 0, g, gb.ga, B, gb, s));
        INF_TRY(launch_act_bwd1(gb.ga, x, ACT_SWISH, n->pre_beta, gin, gb.bpart, ne, GRAD_BLOCKS, s));
        if (gr->dpre_beta) INF_TRY(launch_beta_reduce(gb.bpart, GRAD_BLOCKS, gr->dpre_beta, 0, s));
      } else {
        INF_TRY(layer_vjp(n, 0, g, gin, B, gb, s));
      }
    }
  }
  return INF_OK;
}
}  // namespace

extern "C" {
// Gradient of sum(gout * f(x)) with respect to every parameter of the net (and x): the recompute graph of the training
// forward (implicit_block.py:226-227) and the first-order terms of any caller.  Conv nets (Swish) and fc nets (Swish /
// Sin; x, gout, gx in the (B, d) boundary layout).
int inf_net_param_grad(InfNet* n, const float* x, const float* gout, float* gx, const InfNetGrads* gr, int B,
                       void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !gout || !gr || B <= 0) return INF_ERR_INVALID;
  if (!grad_supported(n)) return INF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  GradBufs gb;
  if (!ws || carve_grad(n, B, ws, ws_bytes, gb) > ws_bytes) return INF_ERR_WORKSPACE;
  if (!n->fc) return param_grad_core(n, x, gout, gx, gr, B, gb, s);
  INF_TRY(launch_transpose(x, gb.x_t, B, n->d, s));
  INF_TRY(launch_transpose(gout, gb.w_t, B, n->d, s));
  INF_TRY(param_grad_core(n, gb.x_t, gb.w_t, gx ? gb.gx_t : nullptr, gr, B, gb, s));
  if (gx) INF_TRY(launch_transpose(gb.gx_t, gx, n->d, B, s));
  return INF_OK;
}

}  // extern "C"

namespace {
// s = sum_b w_b^T J(x_b) eps_b (w, eps fixed) differentiated into x (gx) and every parameter, forward-over-reverse, on
// internal-layout tensors; the per-sample value s_b (conv nets only: value non-null)
int surrogate_core(InfNet* n, const float* x, const float* w, const float* eps, float* value, float* gx,
                   const InfNetGrads* gr, int B, GradBufs& gb, hipStream_t s) {
  const int L = (int)n->L.size();
  const long nin = (long)B * n->d;
  // input tangent: eps * preact'(x) (or eps)
  const float* in_tan = eps;
  if (n->pre_beta) {
    INF_HIP(hipMemcpyAsync(gb.Ad[0], eps, sizeof(float) * nin, hipMemcpyDeviceToDevice, s));
    INF_TRY(launch_act_tangent(gb.Ad[0], x, ACT_SWISH, n->pre_beta, nin, s));
    in_tan = gb.Ad[0];
  }
  // forward: primal pre-activations H, tangents Hd, activation tangents Ad
  std::vector<const float*> Ain(L, nullptr);     // each layer's input activated once (gb.A)
  for (int l = 0; l + 1 < L; ++l) {
    INF_TRY(layer_input(n, l, x, gb, B, s, &Ain[l]));
    INF_TRY(layer_fwd(n, l, Ain[l], nullptr, true, gb.H[l], B, s));
    const float* tin = l == 0 ? in_tan : gb.Ad[l];
    INF_TRY(layer_fwd(n, l, tin, nullptr, false, gb.Hd[l], B, s));
    const long ne = (long)B * n->L[l].cout * n->P;
    INF_HIP(hipMemcpyAsync(gb.Ad[l + 1], gb.Hd[l], sizeof(float) * ne, hipMemcpyDeviceToDevice, s));
    INF_TRY(launch_act_tangent(gb.Ad[l + 1], gb.H[l], n->L[l].act, n->L[l].act_beta, ne, s));
  }
  // reverse: G_tan = gbar of the layer's tangent output, G_pri = gbar of its primal output
  const float* G_tan = w;
  const float* G_pri = nullptr;
  float* tb[2] = {gb.gA, gb.gB};
  float* pb2[2] = {gb.hA, gb.hB};
  for (int l = L - 1; l >= 0; --l) {
    const float* X_tan = l == 0 ? in_tan : gb.Ad[l];
    if (!Ain[l]) INF_TRY(layer_input(n, l, x, gb, B, s, &Ain[l]));   // (the last layer's input)
    const float* X_pri = Ain[l];
    const float* xb = nullptr;
    INF_TRY(layer_param_grads(n, l, G_tan, X_tan, G_pri, X_pri, xb, gr, B, gb, s));
    INF_TRY(layer_vjp(n, l, G_tan, gb.gad, B, gb, s));
    if (G_pri) INF_TRY(layer_vjp(n, l, G_pri, gb.ga, B, gb, s));
    if (l == L - 1 && value) {
      // s_b = sum w . (W_{L-1} * adot_{L-2}) = sum (W_{L-1}^T w) . adot_{L-2}
      const long per = (long)n->L[l].cin * n->P;
      INF_TRY(glue_batched_dot(gb.gad, X_tan, value, B, per, gb.bpart, s));
    }
    if (l > 0) {
      const WLayer& prev = n->L[l - 1];
      const long ne = (long)B * prev.cout * n->P;
      float* nt = tb[l & 1];
      float* np = pb2[l & 1];
      INF_TRY(launch_act_bwd2(gb.gad, G_pri ? gb.ga : nullptr, gb.H[l - 1], gb.Hd[l - 1], prev.act, prev.act_beta, nt,
                              np, gb.bpart, ne, GRAD_BLOCKS, s));
      float* dbeta = grad_out(gr->dbeta, l - 1);
      if (dbeta && prev.act == ACT_SWISH) INF_TRY(launch_beta_reduce(gb.bpart, GRAD_BLOCKS, dbeta, 0, s));
      G_tan = nt;
      G_pri = np;
    } else {
      float* gin = gx ? gx : gb.tmp_in;
      if (n->pre_beta) {
        // x-gradient: gbar_adot eps s''(x) + gbar_a s'(x); beta: ... (act_bwd2 with h = x, hdot = eps)
        INF_TRY(launch_act_bwd2(gb.gad, G_pri ? gb.ga : nullptr, x, eps, ACT_SWISH, n->pre_beta, gb.xin, gin, gb.bpart,
                                nin, GRAD_BLOCKS, s));
        if (gr->dpre_beta) INF_TRY(launch_beta_reduce(gb.bpart, GRAD_BLOCKS, gr->dpre_beta, 0, s));
      } else if (gx) {
        if (G_pri) INF_HIP(hipMemcpyAsync(gx, gb.ga, sizeof(float) * nin, hipMemcpyDeviceToDevice, s));
        else INF_HIP(hipMemsetAsync(gx, 0, sizeof(float) * nin, s));
      }
    }
  }
  return INF_OK;
}
}  // namespace

extern "C" {
// Gradient of s = sum_b w_b^T J(x_b) eps_b (w fixed) with respect to x and every parameter, and the value s_b per
// sample (conv nets): the memory-efficient Neumann estimator's surrogate (implicit_block.py:388-394,437-438),
// forward-over-reverse on the engine.  fc nets: x, w, eps, gx in the (B, d) boundary layout, value NULL.
int inf_net_surrogate_grad(InfNet* n, const float* x, const float* w, const float* eps, float* value, float* gx,
                           const InfNetGrads* gr, int B, void* ws, size_t ws_bytes, void* stream) {
  if (!n || !x || !w || !eps || !gr || B <= 0) return INF_ERR_INVALID;
  if (!grad_supported(n) || (n->fc && value)) return INF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  GradBufs gb;
  if (!ws || carve_grad(n, B, ws, ws_bytes, gb) > ws_bytes) return INF_ERR_WORKSPACE;
  if (!n->fc) return surrogate_core(n, x, w, eps, value, gx, gr, B, gb, s);
  INF_TRY(launch_transpose(x, gb.x_t, B, n->d, s));
  INF_TRY(launch_transpose(w, gb.w_t, B, n->d, s));
  INF_TRY(launch_transpose(eps, gb.e_t, B, n->d, s));
  INF_TRY(surrogate_core(n, gb.x_t, gb.w_t, gb.e_t, nullptr, gx ? gb.gx_t : nullptr, gr, B, gb, s));
  if (gx) INF_TRY(launch_transpose(gb.gx_t, gx, n->d, B, s));
  return INF_OK;
}

// ---- the log-det estimators' gradients for fc nets (the training path of train_tabular.py / train_toy.py) -----------
static size_t logdet_grad_layout(InfNet* n, int B, int mode, int n_terms, char* ws, size_t cap, Bufs* bf, GradBufs* gb,
                                 float** A, float** bv, float** xr, float** gxs, float** eps_t, float** a_scr) {
  const int T = mode == LOGDET_SERIES ? n_terms : n->d;
  const long N = (long)T * B;
  Bufs bf0;
  GradBufs gb0;
  const size_t s1 = (carve(n, B, 1, ws, ws ? cap : 0, bf ? *bf : bf0) + 255) & ~(size_t)255;
  char* w2 = ws ? ws + s1 : nullptr;
  const size_t s2 = (carve_grad(n, (int)N, w2, ws ? (cap > s1 ? cap - s1 : 0) : 0, gb ? *gb : gb0) + 255) & ~(size_t)255;
  WS w{ws ? ws + s1 + s2 : nullptr, ws ? (cap > s1 + s2 ? cap - s1 - s2 : 0) : 0, 0};
  float* p[6];
  const size_t cnt[6] = {(size_t)n->d * N, (size_t)n->d * N, (size_t)n->d * N, (size_t)n->d * N, (size_t)n->d * B,
                         mode == LOGDET_SERIES ? (size_t)n_terms * n->d * B : 1};
  for (int i = 0; i < 6; ++i) p[i] = w.take<float>(cnt[i]);
  if (A) {
    *A = p[0];
    *bv = p[1];
    *xr = p[2];
    *gxs = p[3];
    *eps_t = p[4];
    *a_scr = p[5];
  }
  return s1 + s2 + w.off + 256;
}

size_t inf_logdet_grad_workspace_bytes(InfNet* n, int B, int mode, int n_terms) {
  if (!n || B <= 0 || mode < LOGDET_SERIES || mode > LOGDET_TRACE || (mode != LOGDET_EXACT && n_terms < 1)) return 0;
  return logdet_grad_layout(n, B, mode, n_terms, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                            nullptr, nullptr);
}

// g . S(x) differentiated into every parameter of an fc net and into x, S_b one of the log-det estimators of a sample
// (mode INF_LOGDET_SERIES / EXACT / TRACE, pointwise.hip logdet_pairs_kernel): the Jacobian per sample (fc_jacobian),
// the estimator's bilinear pairs at x, then one forward-over-reverse pass over the T B stacked pairs (surrogate_core:
// the GEMM chains of the generic path, N = T B columns), the x-gradient summed over each sample's pairs.
int inf_logdet_grad(InfNet* n, const float* x, int mode, const float* eps, const float* coeff, int n_terms,
                    const float* gout, float* value, float* gx, const InfNetGrads* gr, int B, void* ws, size_t ws_bytes,
                    void* stream) {
  if (!n || !x || !gr || B <= 0 || mode < LOGDET_SERIES || mode > LOGDET_TRACE) return INF_ERR_INVALID;
  if (mode == LOGDET_SERIES && (!eps || !coeff || n_terms < 1 || n_terms > 128)) return INF_ERR_INVALID;
  if (mode == LOGDET_TRACE && (!coeff || n_terms < 1 || n_terms > 128)) return INF_ERR_INVALID;
  if (!n->fc || n->d > 16 || !grad_supported(n)) return INF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  GradBufs gb;
  float *A, *bv, *xr, *gxs, *eps_t, *a_scr;
  const int nt = mode == LOGDET_EXACT ? 1 : n_terms;
  if (!ws || logdet_grad_layout(n, B, mode, nt, reinterpret_cast<char*>(ws), ws_bytes, &bf, &gb, &A, &bv, &xr, &gxs,
                                &eps_t, &a_scr) > ws_bytes)
    return INF_ERR_WORKSPACE;
  const int T = mode == LOGDET_SERIES ? n_terms : n->d;
  const float* tang = nullptr;
  INF_TRY(fc_jacobian(n, x, B, bf, &tang, s));                     // also leaves x internal in bf.xin
  if (mode == LOGDET_SERIES) INF_TRY(launch_transpose(eps, eps_t, B, n->d, s));
  const float one = 1.f;
  INF_TRY(launch_logdet_pairs(mode, tang, eps_t, bf.xin, gout, mode == LOGDET_EXACT ? &one : coeff, nt, n->d, B, A, bv,
                              xr, value, a_scr, s));
  INF_TRY(surrogate_core(n, xr, A, bv, nullptr, gx ? gxs : nullptr, gr, T * B, gb, s));
  if (gx) INF_TRY(launch_sum_pairs(gxs, T, n->d, B, gx, s));
  return INF_OK;
}

size_t inf_grad_workspace_bytes(InfNet* n, int B) {
  if (!n || B <= 0) return 0;
  GradBufs gb;
  return carve_grad(n, B, nullptr, 0, gb);
}

int inf_debug_poison_lds(void* stream) { return glue_poison_lds((hipStream_t)stream); }

// readback contract check (inflow.h): round r writes base_r + i (i < n) into a pinned coherent slot, once from a kernel
// whose launch completes the slot's event (the zero-copy Broyden sums) and once through a device buffer and a D2H copy
// followed by a recorded event (the reduction + copy form); the host waits with host_wait and compares every value
__global__ void readback_pattern_kernel(double* out, int n, double base) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = base + (double)i;
}
int inf_debug_readback_check(int iters, int n, void* stream) {
  if (iters < 0 || n <= 0 || n > (1 << 20)) return -INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  double* host = nullptr;
  double* dev = nullptr;
  hipEvent_t ev = nullptr;
  int bad = 0, rc = INF_OK;
  if (hipHostMalloc(reinterpret_cast<void**>(&host), sizeof(double) * n, hipHostMallocCoherent) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&dev), sizeof(double) * n) != hipSuccess ||
      hipEventCreateWithFlags(&ev, INF_EV_SYNC) != hipSuccess) {
    rc = INF_ERR_HIP;
  }
  const dim3 grid((n + 255) / 256), blk(256);
  for (int r = 0; r < iters && rc == INF_OK; ++r) {
    for (int form = 0; form < 2 && rc == INF_OK; ++form) {
      const double base = 1e6 * (2 * r + form + 1);
      if (form == 0) {
        hipExtLaunchKernelGGL(readback_pattern_kernel, grid, blk, 0, s, nullptr, ev, 0, host, n, base);
      } else {
        hipLaunchKernelGGL(readback_pattern_kernel, grid, blk, 0, s, dev, n, base);
        if (hipMemcpyAsync(host, dev, sizeof(double) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipEventRecord(ev, s) != hipSuccess) rc = INF_ERR_HIP;
      }
      if (hipGetLastError() != hipSuccess) rc = INF_ERR_HIP;
      if (rc == INF_OK) rc = host_wait(ev);
      for (int i = 0; i < n && rc == INF_OK; ++i) bad += host[i] != base + (double)i;
    }
  }
  (void)hipStreamSynchronize(s);
  if (ev) (void)hipEventDestroy(ev);
  if (dev) (void)hipFree(dev);
  if (host) (void)hipHostFree(host);
  return rc == INF_OK ? bad : -rc;
}

int inf_net_set_option(InfNet* n, int option, int value) {
  if (!n) return -INF_ERR_INVALID;
  int* slot = nullptr;
  int lo = 0, hi = 0;
  switch (option) {
    case INF_OPT_FUSED_K128: slot = &n->k128; hi = 3; break;
    case INF_OPT_EVAL_OVERLAP: slot = &n->eval_overlap; hi = 1; break;
    case INF_OPT_CONVERGENCE: slot = &n->convergence; hi = 1; break;
    case INF_OPT_LINE_SEARCH: slot = &n->line_search; hi = 1; break;
    case INF_OPT_K128_EXACT_SCALE: slot = &n->exact_scale; hi = 1; break;
    case INF_OPT_FC_BLOCK: slot = &n->fc_block; hi = 2; break;
    case INF_OPT_FC_SERIES: slot = &n->fc_series; hi = 1; break;
    case INF_OPT_FUSED_PRESPLIT: slot = &n->presplit; hi = 1; break;
    default: return -INF_ERR_INVALID;
  }
  if (value < lo || value > hi) return -INF_ERR_INVALID;
  const int prev = *slot;
  *slot = value;
  // the kernel-variant options change the bits of f(0): the cached value is recomputed on next use
  if (prev != value && (option == INF_OPT_FUSED_K128 || option == INF_OPT_K128_EXACT_SCALE)) n->f0_batch = -1;
  return prev;
}

int inf_net_get_option(const InfNet* n, int option) {
  if (!n) return -INF_ERR_INVALID;
  switch (option) {
    case INF_OPT_FUSED_K128: return n->k128;
    case INF_OPT_EVAL_OVERLAP: return n->eval_overlap;
    case INF_OPT_CONVERGENCE: return n->convergence;
    case INF_OPT_LINE_SEARCH: return n->line_search;
    case INF_OPT_K128_EXACT_SCALE: return n->exact_scale;
    case INF_OPT_FC_BLOCK: return n->fc_block;
    case INF_OPT_FC_SERIES: return n->fc_series;
    case INF_OPT_FUSED_PRESPLIT: return n->presplit;
    default: return -INF_ERR_INVALID;
  }
}

int inf_banach_find_root(InfNet* f, InfNet* e, const float* y, float* out, int B, int threshold, double eps,
                         int* iters, void* ws, size_t ws_bytes, void* stream) {
  if (!f || !e || !y || !out || B <= 0 || threshold < 0 || !same_shape(f, e)) return INF_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  Bufs bf;
  if (!ws || carve(f, B, 1, ws, ws_bytes, bf) > ws_bytes) return INF_ERR_WORKSPACE;
  int st = INF_OK;
  const float* yi = to_internal(f, y, bf.xin, B, s, &st);
  INF_TRY(st);
  // x_embed = e(y) + y  (implicit_block.py:60)
  OutArgs a;
  memset(&a, 0, sizeof(a));
  a.in0 = yi;
  a.out0 = bf.fx;
  a.out1 = bf.xemb;
  INF_TRY(run_forward(e, yi, B, bf, OM_EMBED, &a, s));
  std::vector<int> todo;
  if (f->convergence == INF_CONV_PER_SAMPLE) todo.assign(B, 1);
  int it = 0;
  INF_TRY(banach_solve(f, yi, B, eps, threshold, todo.empty() ? nullptr : todo.data(), bf, s, &it));
  if (iters) *iters = it;
  return to_boundary(f, bf.lowest, out, B, s);
}

}  // extern "C"
