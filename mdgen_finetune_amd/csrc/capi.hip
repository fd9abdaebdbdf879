// extern "C" entry points of libmdgen_hip.so (declared in include/mdgen_hip.h).
// Argument validation happens here, on the host, before any launch: a kernel is never
// started on shapes it does not support.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <cmath>

#include <string>
#include <vector>

#include "../../include/mdgen_hip.h"
#include "common.h"

namespace mdg {
struct GemmPlan {
  int cfg;
  size_t smem;
  int bm, bn;
};
GemmPlan gemm_plan(const mdg_gemm_desc& p);
hipError_t gemm_launch(const mdg_gemm_desc& p, const GemmPlan& g, hipStream_t s);
bool mlp_fused_supported(const mdg_gemm_desc& f1, const mdg_gemm_desc& f2);
hipError_t mlp_fused_launch(const mdg_gemm_desc& f1, const mdg_gemm_desc& f2, hipStream_t s, float* part,
                            const mdg_gemm_desc* pre = nullptr);
bool mlp_pre_supported(const mdg_gemm_desc& r, const mdg_gemm_desc& f1, const mdg_gemm_desc& f2);
int mlp_split_factor(int M, int F);
hipError_t train_pack_launch(const mdg_train_pack& p, hipStream_t s);
hipError_t train_unpack_launch(const mdg_train_unpack& u, hipStream_t s);
bool ipa_core_supported(int L, int c, int Pq, int Pv);
hipError_t ipa_core_fwd_launch(int B, int L, int H, const float* q, const float* kv, const float* qp, const float* kvp,
                               const float* mask, const float* rots, const float* trans, const float* hw, float wc,
                               float* out, int flags, hipStream_t s);
hipError_t ipa_core_bwd_launch(int B, int L, int H, const float* q, const float* kv, const float* qp, const float* kvp,
                               const float* mask, const float* rots, const float* trans, const float* hw, float wc,
                               const float* dout, float* dq, float* dkv, float* dqp, float* dkvp, float* dhw_part,
                               int flags, hipStream_t s);
bool rowln_splitk_supported(const mdg_gemm_desc& r, int S);
bool rowln_bm32_supported(const mdg_gemm_desc& r);
hipError_t rowln_bm32_launch(const mdg_gemm_desc& p, hipStream_t s);
hipError_t rowln_splitk_launch(const mdg_gemm_desc& r, hipStream_t s, float* part, int S);
bool final_euler_supported(const mdg_gemm_desc& p);
hipError_t final_euler_launch(const mdg_gemm_desc& p, hipStream_t s);
bool rowln_qkv_supported(const mdg_gemm_desc& r, const mdg_gemm_desc& q);
hipError_t rowln_qkv_launch(const mdg_gemm_desc& r, const mdg_gemm_desc& q, hipStream_t s);
hipError_t attn_temporal_launch(int dtype, int B, int T, int L, int H, int D, const void* qkv_t,
                                const float* kbias, const float* kvb, void* out, hipStream_t s,
                                float* lse = nullptr, bool packed = false, void* out_lo = nullptr);
hipError_t attn_spatial_launch(int dtype, int nf, int L, int H, int D, const void* qkv,
                               const float* kvb, const float* mask, void* out, hipStream_t s);
hipError_t embed_launch(int N, int T, int L, int C, int K, const float* x, const float* W,
                        const float* bias, const float* base, const float* pos, const float* emb,
                        const int64_t* idx, const float* ipa, float* out, hipStream_t s);
hipError_t mask_bias_launch(int B, int T, int L, const float* mask, float* kbias, float* kbias_s, hipStream_t s);
hipError_t ln_mod_launch(int dtype, int M, int C, const float* h, const float* mods, int mod_stride,
                         int rows_per_mod, int shift_off, int scale_off, float eps, void* xn,
                         hipStream_t s, float* stats = nullptr);
hipError_t set_vpad_launch(int dtype, void* v, size_t rows, int D, hipStream_t s);
hipError_t embed_ln_launch(int N, int TL, int L, int C, int K, const float* x, const float* Wt, const float* base,
                           const float* ipa, const float* mods, int mod_stride, int shift_off, int scale_off,
                           float eps, float* h, void* xn, hipStream_t s);
hipError_t prep_latents_launch(int B, int T, int L, int lat, int tps, int no_offsets, int cond_mode,
                               int cond_interval, const float* rots, const float* trans, const float* torsions,
                               float* latents, float* x_cond, int64_t* cond_mask, hipStream_t s);
hipError_t latents_to_atom14_launch(int B, int T, int L, int lat, int tors_off, int renorm, const float* samples,
                                    const float* ref_rots, const float* ref_trans, const int64_t* aatype,
                                    const float* default_frames, const int* group_idx, const float* atom_mask,
                                    const float* lit, float* atom14, float* out_rots, float* out_trans,
                                    hipStream_t s);
// train.hip
int ln_gate_bwd_blocks(int TL);
hipError_t ln_gate_bwd_launch(int dtype, int M, int C, int TL, const void* dxn, const float* hln, const float* stats,
                              const float* mods, int mod_stride, int shift_off, int scale_off, const float* dh_res,
                              float* dh_out, const void* y, int gate_off, void* dy, float* part, hipStream_t s);
int attn_bwd_parts(int dtype, int B, int T, int L, int generic);
hipError_t attn_temporal_bwd_launch(int dtype, int B, int T, int L, int H, int D, const void* qkv_t,
                                    const float* kbias, const float* kvb, const void* o, const void* o_lo,
                                    const void* dout,
                                    const float* lse, const float* rope, int rope_rows, void* dop, float* delta,
                                    void* dqkv, int ldq, float* bpart, float qscale, float kscale, int generic,
                                    float* dqacc, hipStream_t s);
int attn_spatial_bwd_parts(int nf, int L, int H, int D);
hipError_t attn_spatial_bwd_launch(int dtype, int nf, int L, int H, int D, const void* qkv, const float* kvb,
                                   const float* mask, const void* dout, const float* rope, int rope_rows, void* dqkv,
                                   float* bpart, float qscale, hipStream_t s);
// cond.hip
hipError_t temb_freq_launch(int R, int half, float mult, const float* t, const float* freqs, float* out,
                            hipStream_t s);
hipError_t cond_scatter_launch(int S, int B, int nl, int C, int W, int lanes, const float* all, float* mods,
                               float* mods_final, hipStream_t s);
hipError_t ipa_init_launch(int R, int B, int L, int C, int mstride, const int64_t* aatype, const float* aa_emb, const float* rel7,
                           const float* w, const float* bias, const float* mask, float* x, float* mask_rep,
                           hipStream_t s);
hipError_t add_inplace_launch(size_t n, float* y, const float* x, hipStream_t s);
bool ipa_attn_supported(int c, int pq, int pv);
hipError_t ipa_attn_launch(int R, int B, int L, int H, int c, int pq, int pv, const float* proj, int ldp,
                           const float* rots, const float* trans, const float* mask, const float* head_weights,
                           float* out, int ldc, hipStream_t s);
hipError_t tps_rel7_launch(int B, int L, const float* rots, const float* trans, const float* erots,
                           const float* etrans, float* out, hipStream_t s);
// train_glue.hip
size_t embed_bwd_ws_bytes(int B, int T, int L, int C, int K1, int K2, int E);
hipError_t embed_bwd_launch(int B, int T, int L, int C, int K1, const float* x1, int K2, const float* x2,
                            const int64_t* idx, int E, const float* dh, float* dw1, float* dw2, float* db, float* demb,
                            float* dipa, float* ws, hipStream_t s);
hipError_t final_fwd_train_launch(int N, int rows_per_b, int lat, const float* h, const float* mods, const float* w,
                                  const float* bias, float* v, float* stats, hipStream_t s);
size_t final_bwd_ws_bytes(int N, int rows_per_b, int lat);
hipError_t final_bwd_train_launch(int N, int rows_per_b, int lat, const float* h, const float* stats, const float* mods,
                                  const float* w, const float* dv, float* dh, float* dw, float* dbias, float* dmods,
                                  float* ws, hipStream_t s);
// wgrad.hip
size_t wgrad_ws_bytes(int dtype, int N, int M, int K, bool need_w, bool need_b);
hipError_t wgrad_launch(int dtype, int N, int M, int K, const void* dy, int ldy, const void* x, int ldx, float* dw,
                        int lddw, float* db, float* ws, hipStream_t s);
// train_glue.hip: the flow-matching plan and loss
hipError_t gvp_plan_launch(int B, long long npb, int path, const float* t, const float* x0, const float* x1, float* xt,
                           float* ut, hipStream_t s);
size_t gvp_loss_ws_bytes(int B, long long npb);
hipError_t gvp_loss_fwd_launch(int B, int T, int L, int K, const float* out, const float* ut, const float* mask,
                               const int64_t* ms, float* loss, float* den, float* ws, hipStream_t s);
hipError_t gvp_loss_bwd_launch(int B, int T, int L, int K, const float* out, const float* ut, const float* mask,
                               const int64_t* ms, const float* g, const float* den, float* dout, hipStream_t s);
// optim.hip
int adam_chunks(int nt, const mdg_adam_tensor* t);
size_t adam_table_bytes(int nt, int nc);
void adam_table_build(int nt, int nc, const mdg_adam_tensor* t, void* table);
size_t adam_ws_bytes(int nc);
hipError_t adam_step_launch(int nt, int nc, const void* table, double lr, double b1, double b2, double eps, double wd,
                            int decoupled, double max_norm, float* gnorm, float* ws, hipStream_t s);
// linear_small.hip
int seg_total(const mdg_seg_linear* s);
bool seg_linear_shape_ok(int M, int K);
size_t seg_linear_ws_bytes(int M, int K, int total);
hipError_t seg_linear_fwd_launch(int M, int K, const float* x, int ldx, int act, const mdg_seg_linear* s, hipStream_t st);
hipError_t seg_linear_bwd_launch(int M, int K, const float* x, int ldx, int act, const mdg_seg_linear* s, float* dx,
                                 int lddx, float* ws, hipStream_t st);
}  // namespace mdg

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#ifdef MDG_DIAGNOSTICS
// Diagnostic builds only (make DIAG=1; tools/lane_snap.py, tools/lane_hist.py): the product
// library has none of this state, so its calls stay reentrant (include/mdgen_hip.h).
// Diagnostic (MDG_DEBUG_COHERENCE, tools/lane_hist.py): inside a denoise step every checked
// launch is followed by a small kernel on the same stream.  =1: each of its waves performs an
// agent-scope release + acquire (L2 write-back + invalidate on the XCD it runs on, L1 invalidate
// on its CU); =2: the same launch with an empty body (timing control).
__global__ void coherence_kernel(int fence) {
  if (fence) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

thread_local hipStream_t g_dbg_stream = nullptr;  // the denoise step's stream (may be the null stream)
thread_local bool g_dbg_in_step = false;

// Diagnostic (tools/lane_snap.py): with a snapshot buffer set (mdg_debug_snapshots), every
// checked launch inside a denoise step is followed by device copies of the step's workspace,
// residual h and latents x into the next free slot of the buffer, on the launch's stream (so a
// captured graph replays them).  Slots are labelled with the launch and the workspace pointer.
struct DbgRegion {
  const void* p;
  size_t n;
};
thread_local DbgRegion g_dbg_regions[3];
struct DbgSnap {
  char* dst = nullptr;
  size_t cap = 0, used = 0;
  std::vector<std::string> label;
  std::vector<size_t> off;
  std::vector<const void*> ws;
};
DbgSnap g_snap;

void debug_snapshot(const char* what) {
  size_t need = 0;
  for (const DbgRegion& r : g_dbg_regions) need += (r.n + 255) & ~(size_t)255;
  if (!g_snap.dst || g_snap.used + need > g_snap.cap) return;
  g_snap.label.push_back(what);
  g_snap.off.push_back(g_snap.used);
  g_snap.ws.push_back(g_dbg_regions[0].p);
  for (const DbgRegion& r : g_dbg_regions) {
    if (r.n) (void)hipMemcpyAsync(g_snap.dst + g_snap.used, r.p, r.n, hipMemcpyDeviceToDevice, g_dbg_stream);
    g_snap.used += (r.n + 255) & ~(size_t)255;
  }
}

int debug_coherence() {
  static const int v = [] {
    const char* e = getenv("MDG_DEBUG_COHERENCE");
    return e ? atoi(e) : 0;
  }();
  return v;
}

#endif  // MDG_DIAGNOSTICS

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) {
#ifdef MDG_DIAGNOSTICS
    if (g_dbg_in_step && debug_coherence())
      hipLaunchKernelGGL(coherence_kernel, dim3(1024), dim3(64), 0, g_dbg_stream, debug_coherence() == 1 ? 1 : 0);
    if (g_dbg_in_step && g_snap.dst) debug_snapshot(what);
#endif
    return MDG_OK;
  }
  return fail((int)e, "%s: %s", what, hipGetErrorString(e));
}

size_t ct_size(int dtype) { return dtype == MDG_BF16 ? 2 : 4; }
size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// residue counts from which the spatial attention runs on the MFMA (temporal) kernel
constexpr int kSpatialMfmaMinL = 16;

// bf16 tetrapeptide path: spatial q|k|v projection + attention as one launch
// (MDG_EPI_ATTN_SPATIAL); MDG_FUSE_SPATIAL=0 selects the two-launch path (A/B knob)
bool fuse_spatial_attn(const mdg_dims& d) {
  static const bool on = [] {
    const char* e = getenv("MDG_FUSE_SPATIAL");
    return !(e && e[0] == '0');
  }();
  return on && d.dtype == MDG_BF16 && d.L == 4 && d.D == 24 && d.H % 2 == 0;
}

// bf16, head_dim % 8 == 0: temporal attention planes stored packed (row stride D);
// MDG_PACKED_PLANES=0 keeps the padded planes (A/B knob)
bool packed_planes(const mdg_dims& d) {
  static const bool on = [] {
    const char* e = getenv("MDG_PACKED_PLANES");
    return !(e && e[0] == '0');
  }();
  return on && d.dtype == MDG_BF16 && d.D % 8 == 0 && d.D < MDG_DP;
}

// bf16, C = 384: the block's MLP as one kernel (hidden activation on chip); MDG_FUSED_MLP=0
// keeps fc1 + fc2 (A/B knob)
bool fused_mlp_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_FUSED_MLP");
    return !(e && e[0] == '0');
  }();
  return on;
}

// fewer than 64 row tiles of 128: a one-block-per-tile kernel would leave most CUs idle even
// with a second lane beside it (the engine runs 2 lanes from B = 8; a B = 8 lane has 125 tiles)
bool small_m(long long N) { return (N + 127) / 128 < 64; }

// bf16, C = 384, packed planes: the spatial out_proj row-LN and the temporal q|k|v projection
// as one kernel (LN_t(h) stays on chip); MDG_FUSED_QKV=0 keeps the two launches (A/B knob).
// Small M takes the two launches (the q|k|v GEMM then runs on 9x the blocks).
bool fused_qkv_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_FUSED_QKV");
    return !(e && e[0] == '0');
  }();
  return on;
}

// MDG_ROWLN_BM32=0: a lone chain's small-M out_proj row-LN GEMMs split over K (round 3) instead of
// on 32-row tiles (A/B knob)
bool rowln_bm32_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_ROWLN_BM32");
    return !(e && e[0] == '0');
  }();
  return on;
}

// MDG_MLP_PRE=1: the temporal out_proj row-LN GEMM as the fused MLP's prologue (one launch;
// gemm.hip mlp_rowln_kernel PRE).  Off by default: bit-identical, but measured neutral (round 5,
// same box, 2 x 2 alternating runs: 4.698 / 4.698 M frames/s fused vs 4.712 / 4.709 M two launches)
// -- the step is the sum of the kernels' chip time (two lanes already fill the launch gaps and
// tails), and the prologue costs what the launch did: its 12 K-steps plus an HBM-bound epilogue.
bool mlp_pre_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_MLP_PRE");
    return e && e[0] == '1';
  }();
  return on;
}

// bf16, latent <= 32: the FinalLayer + Euler update as its own one-pass kernel;
// MDG_FAST_FINAL=0 keeps the generic EULER GEMM (A/B knob)
bool fast_final_on() {
  static const bool on = [] {
    const char* e = getenv("MDG_FAST_FINAL");
    return !(e && e[0] == '0');
  }();
  return on;
}

struct WsLayout {
  size_t qkv_s, qkv_t, o, hid, xn, kbias, kbias_s, mlp_part, total;
  int mlp_split;  // > 1: [mlp_split][N][C] fp32 partials at mlp_part (small-M MLP / out_proj)
};

WsLayout ws_layout(const mdg_dims& d) {
  const size_t cs = ct_size(d.dtype);
  const size_t N = (size_t)d.B * d.T * d.L;
  WsLayout w;
  size_t off = 0;
  w.qkv_s = off; off += align256(N * 3 * d.H * d.D * cs);
  w.qkv_t = off; off += align256(3ull * d.B * d.L * d.H * d.T * dp_of(d.D) * cs);
  w.o = off;     off += align256(N * d.C * cs);
  w.hid = off;   off += align256(N * d.F * cs);
  w.xn = off;    off += align256(N * d.C * cs);
  w.kbias = off; off += align256((size_t)d.B * d.L * d.T * sizeof(float));
  w.kbias_s = off; off += align256(N * sizeof(float));
  // the small-M fused MLP's fc2 partials ([split][N][C] fp32; bf16 C = 384 only, else empty)
  const int split = (d.dtype == MDG_BF16 && d.C == 384 && d.F % 128 == 0) ? mdg::mlp_split_factor((int)N, d.F) : 1;
  w.mlp_part = off; off += split > 1 ? align256((size_t)split * N * d.C * sizeof(float)) : 0;
  w.mlp_split = split;
  w.total = off;
  return w;
}

int check_dims(const mdg_dims* d) {
  if (!d) return fail(MDG_E_ARG, "null dims");
  if (d->dtype != MDG_F32 && d->dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", d->dtype);
  if (d->B <= 0 || d->T <= 0 || d->L <= 0 || d->H <= 0)
    return fail(MDG_E_SHAPE, "B,T,L,H must be positive (%d,%d,%d,%d)", d->B, d->T, d->L, d->H);
  if (d->C != d->H * d->D) return fail(MDG_E_SHAPE, "C (%d) != H*D (%d*%d)", d->C, d->H, d->D);
  if (d->D % 4 || d->D >= MDG_DP_WIDE)
    return fail(MDG_E_SHAPE, "head_dim %d unsupported (multiple of 4, < %d)", d->D, MDG_DP_WIDE);
  if (d->C % 64 || d->C > 512) return fail(MDG_E_SHAPE, "embed_dim %d unsupported (64k, <= 512)", d->C);
  if (d->F % 64) return fail(MDG_E_SHAPE, "ffn dim %d not a multiple of 64", d->F);
  if (d->latent <= 0 || d->latent > 64) return fail(MDG_E_SHAPE, "latent %d unsupported", d->latent);
  if (d->num_layers < 0 || d->num_layers > MDG_MAX_LAYERS) return fail(MDG_E_SHAPE, "num_layers %d", d->num_layers);
  if ((long long)d->B * d->T * d->L >= (1ll << 31) / d->F) return fail(MDG_E_SHAPE, "problem too large");
  if (d->dtype == MDG_F32 && d->C > 384)
    return fail(MDG_E_SHAPE, "f32 path: embed_dim %d > 384 exceeds the LDS-resident LN block", d->C);
  return MDG_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

__global__ void stamp_kernel(unsigned long long* dst, int slot) {
  if (threadIdx.x == 0) dst[slot + threadIdx.x] = wall_clock64();
}

extern "C" {

int mdg_abi_version(void) { return MDG_ABI_VERSION; }

int mdg_stamp(uint64_t* dst, int32_t slot, void* stream) {
  if (!dst || slot < 0) return fail(MDG_E_ARG, "mdg_stamp: null buffer or negative slot");
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long*)dst, slot);
  return hip_check(hipGetLastError(), "mdg_stamp");
}

int mdg_wall_clock_khz(int32_t* khz) {
  int dev = 0, v = 0;
  if (!khz) return fail(MDG_E_ARG, "mdg_wall_clock_khz: null output");
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess) return hip_check(e, "mdg_wall_clock_khz");
  *khz = v;
  return MDG_OK;
}

const char* mdg_last_error_string(void) { return g_err.c_str(); }

size_t mdg_workspace_bytes(const mdg_dims* d) {
  if (check_dims(d)) return 0;
  return ws_layout(*d).total;
}

int mdg_workspace_offsets(const mdg_dims* d, size_t offsets[6]) {
  if (int e = check_dims(d)) return e;
  if (!offsets) return fail(MDG_E_ARG, "null offsets");
  const WsLayout w = ws_layout(*d);
  offsets[0] = w.qkv_s; offsets[1] = w.qkv_t; offsets[2] = w.o;
  offsets[3] = w.hid; offsets[4] = w.xn; offsets[5] = w.kbias;
  return 0;
}

int mdg_workspace_init(const mdg_dims* d, void* ws, void* stream) {
  if (int e = check_dims(d)) return e;
  if (!ws) return fail(MDG_E_ARG, "null workspace");
  const WsLayout w = ws_layout(*d);
  hipStream_t s = (hipStream_t)stream;
  if (int e = hip_check(hipMemsetAsync(ws, 0, w.total, s), "workspace memset")) return e;
  // 1.0 in pad column D of every temporal K row (softmax offset) and V row (row sum)
  const size_t vrows = (size_t)d->B * d->L * d->H * d->T;
  char* k = (char*)ws + w.qkv_t + vrows * dp_of(d->D) * ct_size(d->dtype);
  return hip_check(mdg::set_vpad_launch(d->dtype, k, 2 * vrows, d->D, s), "set_vpad");
}

int mdg_prepare_mask(const mdg_dims* d, const float* mask, void* ws, void* stream) {
  if (int e = check_dims(d)) return e;
  if (!mask || !ws) return fail(MDG_E_ARG, "null mask/workspace");
  const WsLayout w = ws_layout(*d);
  return hip_check(mdg::mask_bias_launch(d->B, d->T, d->L, mask, (float*)((char*)ws + w.kbias),
                                         (float*)((char*)ws + w.kbias_s), (hipStream_t)stream),
                   "mask_bias");
}

int mdg_gemm(const mdg_gemm_desc* g, void* stream) {
  if (!g) return fail(MDG_E_ARG, "null gemm desc");
  if (g->dtype != MDG_F32 && g->dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", g->dtype);
  if (!g->A || !g->W) return fail(MDG_E_ARG, "gemm: null A or W");
  if (g->M <= 0 || g->N <= 0 || g->K <= 0 || g->K % 64)
    return fail(MDG_E_SHAPE, "gemm: M,N,K = %d,%d,%d (K must be a multiple of 64)", g->M, g->N, g->K);
  const size_t cs = ct_size(g->dtype);
  if (g->ldw < g->K || (g->ldw * cs) % 16 || !aligned16(g->W))
    return fail(MDG_E_SHAPE, "gemm: W must be 16-B aligned with ldw >= K and ldw*size %% 16 == 0");
  if (g->a_mode == MDG_A_LNMOD) {
    if (g->K > 512 || g->lda < g->K) return fail(MDG_E_SHAPE, "gemm LNMOD: K=%d lda=%d", g->K, g->lda);
    if (g->mods && g->rows_per_mod <= 0) return fail(MDG_E_ARG, "gemm: rows_per_mod");
    if ((g->ln_w == nullptr) != (g->ln_b == nullptr)) return fail(MDG_E_ARG, "gemm: ln_w/ln_b");
  } else if (g->a_mode == MDG_A_PLAIN) {
    if (g->lda < g->K || (g->lda * cs) % 16 || !aligned16(g->A))
      return fail(MDG_E_SHAPE, "gemm PLAIN: A must be 16-B aligned, lda >= K");
  } else {
    return fail(MDG_E_ARG, "gemm: a_mode %d", g->a_mode);
  }
  switch (g->epi) {
    case MDG_EPI_STORE:
      if (!g->out || g->ldo < g->N || g->ldo % 4) return fail(MDG_E_ARG, "gemm STORE: out/ldo");
      break;
    case MDG_EPI_GATE_RES:
      if (!g->resid || g->ldr < g->N || g->ldr % 4) return fail(MDG_E_ARG, "gemm GATE_RES: resid/ldr");
      if (g->gate && g->rows_per_mod <= 0) return fail(MDG_E_ARG, "gemm: rows_per_mod");
      if (g->xn_out) {
        if (g->dtype != MDG_BF16 || g->a_mode != MDG_A_PLAIN || !g->xn_mods || g->rows_per_mod <= 0 ||
            !(g->N == 128 || g->N == 256 || g->N == 384 || g->N == 512) || g->ldr % 2)
          return fail(MDG_E_SHAPE, "gemm GATE_RES+LN: bf16 PLAIN, N in {128,256,384,512}, xn_mods, rows_per_mod");
      }
      break;
    case MDG_EPI_QKV:
      if (g->qkv_layout == MDG_QKV_TEMPORAL_PACKED && (g->D % 8 || g->D >= MDG_DP))
        return fail(MDG_E_SHAPE, "gemm QKV packed: D=%d (multiple of 8, < %d)", g->D, MDG_DP);
      if (g->qkv_layout < MDG_QKV_SPATIAL || g->qkv_layout > MDG_QKV_TEMPORAL_PACKED)
        return fail(MDG_E_ARG, "gemm QKV: layout %d", g->qkv_layout);
      if (!g->qkv_out || g->D <= 0 || g->D % 4 || g->D >= MDG_DP_WIDE || g->N != 3 * g->H * g->D)
        return fail(MDG_E_SHAPE, "gemm QKV: N=%d H=%d D=%d", g->N, g->H, g->D);
      if (g->T <= 0 || g->L <= 0 || g->M % (g->T * g->L))
        return fail(MDG_E_SHAPE, "gemm QKV: M=%d not a multiple of T*L", g->M);
      if (g->rope && g->rope_rows < (g->qkv_layout == MDG_QKV_SPATIAL ? g->L : g->T))
        return fail(MDG_E_SHAPE, "gemm QKV: rope table too short");
      break;
    case MDG_EPI_ATTN_SPATIAL:
      if (g->dtype != MDG_BF16 || g->a_mode != MDG_A_PLAIN || g->L != 4 || g->D != 24 || g->H <= 0 || g->H % 2 ||
          g->N != 3 * g->H * g->D || g->M % 4 || g->K % 32 || g->lda % 8 || g->ldw % 8)
        return fail(MDG_E_SHAPE, "gemm ATTN_SPATIAL: bf16 PLAIN, L=4, D=24, even H, N=3HD, M%%4==0 (M=%d N=%d H=%d D=%d L=%d)",
                    g->M, g->N, g->H, g->D, g->L);
      if (!g->out || g->ldo < g->H * g->D || g->ldo % 4 || !g->kvb) return fail(MDG_E_ARG, "gemm ATTN_SPATIAL: out/ldo/kvb");
      if (g->rope && g->rope_rows < g->L) return fail(MDG_E_SHAPE, "gemm ATTN_SPATIAL: rope table too short");
      break;
    case MDG_EPI_EULER:
      if (g->n_valid <= 0 || g->n_valid > g->N || g->ldo < g->n_valid)
        return fail(MDG_E_SHAPE, "gemm EULER: n_valid=%d N=%d ldo=%d", g->n_valid, g->N, g->ldo);
      if (g->out && !g->x_in) return fail(MDG_E_ARG, "gemm EULER: x_out without x_in");
      break;
    default:
      return fail(MDG_E_ARG, "gemm: epi %d", g->epi);
  }
  if (g->epi == MDG_EPI_EULER && fast_final_on() && mdg::final_euler_supported(*g))
    return hip_check(mdg::final_euler_launch(*g, (hipStream_t)stream), "final euler launch");
  const mdg::GemmPlan plan = mdg::gemm_plan(*g);
  if (plan.cfg < 0) return fail(MDG_E_SHAPE, "gemm: no tile fits N=%d", g->N);
  if (plan.smem > 160 * 1024)
    return fail(MDG_E_SHAPE, "gemm: K=%d needs %zu B of LDS (> 160 KiB)", g->K, plan.smem);
  return hip_check(mdg::gemm_launch(*g, plan, (hipStream_t)stream), "gemm launch");
}

int mdg_attn_spatial(int32_t dtype, int32_t n_frames, int32_t L, int32_t H, int32_t D,
                     const void* qkv, const float* kvb, const float* mask, void* out,
                     void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", dtype);
  if (!qkv || !kvb || !out) return fail(MDG_E_ARG, "attn_spatial: null pointer");
  if (n_frames <= 0 || L <= 0 || H <= 0 || D <= 0 || D % 4 || D >= MDG_DP_WIDE)
    return fail(MDG_E_SHAPE, "attn_spatial: nf=%d L=%d H=%d D=%d", n_frames, L, H, D);
  return hip_check(mdg::attn_spatial_launch(dtype, n_frames, L, H, D, qkv, kvb, mask, out,
                                            (hipStream_t)stream),
                   "attn_spatial");
}

int mdg_attn_temporal(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D,
                      const void* qkv_t, const float* kbias, const float* kvb, void* out,
                      void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", dtype);
  if (!qkv_t || !kbias || !kvb || !out) return fail(MDG_E_ARG, "attn_temporal: null pointer");
  if (B <= 0 || T <= 0 || L <= 0 || H <= 0 || D <= 0 || D % 4 || D >= MDG_DP_WIDE)
    return fail(MDG_E_SHAPE, "attn_temporal: B=%d T=%d L=%d H=%d D=%d", B, T, L, H, D);
  if (H > 65535 || B * L > 65535) return fail(MDG_E_SHAPE, "attn_temporal: grid too large");
  return hip_check(mdg::attn_temporal_launch(dtype, B, T, L, H, D, qkv_t, kbias, kvb, out,
                                             (hipStream_t)stream),
                   "attn_temporal");
}

int mdg_attn_temporal_packed(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D,
                             const void* qkv_t, const float* kbias, const float* kvb, void* out, void* stream) {
  if (dtype != MDG_BF16) return fail(MDG_E_DTYPE, "attn_temporal_packed: bf16 only (dtype %d)", dtype);
  if (!qkv_t || !kbias || !kvb || !out) return fail(MDG_E_ARG, "attn_temporal_packed: null pointer");
  if (B <= 0 || T <= 0 || L <= 0 || H <= 0 || D <= 0 || D % 8 || D >= MDG_DP)
    return fail(MDG_E_SHAPE, "attn_temporal_packed: B=%d T=%d L=%d H=%d D=%d (D multiple of 8, < %d)", B, T, L, H, D,
                MDG_DP);
  if (H > 65535 || B * L > 65535) return fail(MDG_E_SHAPE, "attn_temporal_packed: grid too large");
  return hip_check(mdg::attn_temporal_launch(dtype, B, T, L, H, D, qkv_t, kbias, kvb, out, (hipStream_t)stream,
                                             nullptr, true),
                   "attn_temporal_packed");
}

int mdg_attn_temporal_lse(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D,
                          const void* qkv_t, const float* kbias, const float* kvb, void* out, void* out_lo,
                          float* lse, void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", dtype);
  if (!qkv_t || !kbias || !kvb || !out || !lse) return fail(MDG_E_ARG, "attn_temporal_lse: null pointer");
  if (out_lo && dtype != MDG_BF16) return fail(MDG_E_ARG, "attn_temporal_lse: out_lo is for bf16 (f32 O is exact)");
  if (B <= 0 || T <= 0 || L <= 0 || H <= 0 || D <= 0 || D % 4 || D >= MDG_DP_WIDE)
    return fail(MDG_E_SHAPE, "attn_temporal_lse: B=%d T=%d L=%d H=%d D=%d (head_dim < %d)", B, T, L, H, D,
                MDG_DP_WIDE);
  if (H > 65535 || B * L > 65535) return fail(MDG_E_SHAPE, "attn_temporal_lse: grid too large");
  return hip_check(mdg::attn_temporal_launch(dtype, B, T, L, H, D, qkv_t, kbias, kvb, out, (hipStream_t)stream, lse,
                                             false, out_lo),
                   "attn_temporal_lse");
}

int mdg_embed(int32_t N, int32_t T, int32_t L, int32_t C, int32_t K, const float* x,
              const float* Wt, const float* bias, const float* base, const float* pos,
              const float* emb, const int64_t* idx, const float* ipa, float* out, void* stream) {
  if (!x || !Wt || !out) return fail(MDG_E_ARG, "embed: null x/Wt/out");
  if (N <= 0 || T <= 0 || L <= 0 || C <= 0 || C % 4 || C > 512 || K <= 0 || K > 32 || N % (T * L))
    return fail(MDG_E_SHAPE, "embed: N=%d T=%d L=%d C=%d K=%d", N, T, L, C, K);
  if ((emb == nullptr) != (idx == nullptr)) return fail(MDG_E_ARG, "embed: emb/idx");
  return hip_check(mdg::embed_launch(N, T, L, C, K, x, Wt, bias, base, pos, emb, idx, ipa, out,
                                     (hipStream_t)stream),
                   "embed");
}

int mdg_final_euler(int32_t dtype, int32_t N, int32_t rows_per_b, int32_t C, int32_t latent,
                    const void* w_final, const float* b_final, const float* mods_final,
                    const float* h, const float* x_in, float dt, float* x_out, float* v_out,
                    void* stream) {
  if (!w_final || !b_final || !mods_final || !h) return fail(MDG_E_ARG, "final_euler: null pointer");
  if (N <= 0 || rows_per_b <= 0 || latent <= 0 || latent > 64)
    return fail(MDG_E_SHAPE, "final_euler: N=%d latent=%d", N, latent);
  mdg_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.dtype = dtype;
  g.a_mode = MDG_A_LNMOD;
  g.epi = MDG_EPI_EULER;
  g.M = N; g.N = (latent + 31) / 32 * 32; g.K = C;
  g.A = h; g.lda = C; g.W = w_final; g.ldw = C; g.bias = b_final;
  g.mods = mods_final; g.mod_stride = 2 * C; g.rows_per_mod = rows_per_b; g.shift_off = 0; g.scale_off = C;
  g.ln_eps = 1e-6f;
  g.out = x_out; g.ldo = latent; g.x_in = x_in; g.v_out = v_out; g.dt = dt; g.n_valid = latent;
  return mdg_gemm(&g, stream);
}

// Where the layer's LayerNorm+modulate inputs come from.  `xn_ready`: the caller already put
// LN_spatial(h) in the xn workspace (the previous layer's fused fc2 epilogue).  `next_mods`:
// the fc2 epilogue also produces the NEXT consumer's LN input (next layer's spatial LN, or the
// FinalLayer's) with shift/scale at next_shift/next_scale of rows of stride next_stride.
struct LnHandoff {
  bool xn_ready;
  const float* next_mods;
  int next_stride, next_shift, next_scale;
  bool alone = false;  // mdg_step_io.chain_alone: the small-M split-K out_proj route may run
};

static int layer_fwd_impl(const mdg_dims* d, const mdg_layer_weights* w, const float* rope_l, const float* rope_t,
                          const float* mods, const float* mask, float* h, void* ws, void* stream,
                          const LnHandoff& ho) {
  const WsLayout lay = ws_layout(*d);
  char* wsb = (char*)ws;
  const int B = d->B, T = d->T, L = d->L, C = d->C, H = d->H, D = d->D, F = d->F;
  const int N = B * T * L;
  const float qs = 1.0f / sqrtf((float)D);
  void* qkv_s = wsb + lay.qkv_s;
  void* qkv_t = wsb + lay.qkv_t;
  void* o = wsb + lay.o;
  void* hid = wsb + lay.hid;
  const float* kbias = (const float*)(wsb + lay.kbias);

  void* xn = wsb + lay.xn;
  hipStream_t s = (hipStream_t)stream;
  const int TL = T * L, ms = 9 * C;
  // out_proj row-LN GEMMs: split-K over the workspace's partials when M is small
  auto rowln_gemm = [&](const mdg_gemm_desc& g) -> int {
    // at most MDG_ROWLN_SPLITK K pieces of the 12 K-steps (default 1 = off).  Measured: a B = 1
    // window (one chain, 32 tiles) +7 % at 2-4 pieces, but a TPS B = 16 window (two lanes of 25
    // tiles sharing the chip) -9 % at 2 and -26 % at 12: the fp32 partials' write + re-read cost
    // more than the CUs the other lane leaves idle.  Keying it on the launch's B (< 4: a chain
    // alone on the chip) broke the lanes' bit-identity to one chain (a 2-lane window of B = 4
    // would split, the single chain would not), so it stays an explicit choice.
    static const int smax_env = [] {
      const char* e = getenv("MDG_ROWLN_SPLITK");
      return e ? atoi(e) : 1;
    }();
    // a chain alone on the chip (mdg_step_io.chain_alone): up to 4 pieces (round 3, B = 1
    // window +8 %: 1.51 -> 1.64 M frames/s in round 2's measurement)
    const int smax = smax_env > 1 ? smax_env : (ho.alone ? 4 : 1);
    int S = 1;
    for (int d2 = 2; d2 <= smax && d2 <= lay.mlp_split; ++d2)
      if (12 % d2 == 0 && ((N + 127) / 128) * d2 <= 320) S = d2;
    // a lone chain: 32-row tiles (4x the blocks, full K, no partials) before split-K (round 5)
    if (small_m(N) && ho.alone && rowln_bm32_on() && mdg::rowln_bm32_supported(g))
      return hip_check(mdg::rowln_bm32_launch(g, s), "rowln 32-row launch");
    if (small_m(N) && mdg::rowln_splitk_supported(g, S))
      return hip_check(mdg::rowln_splitk_launch(g, s, (float*)(wsb + lay.mlp_part), S), "rowln split-K launch");
    return mdg_gemm(&g, stream);
  };
  // LN + adaLN modulate into the CT activation buffer (latent_model.py:467/475/489)
  // fused hand-off: the bf16 path with C in {128..512} produces each LN input inside the
  // preceding gated-residual GEMM (gemm_rowln_kernel); otherwise a stand-alone ln_mod pass
  const bool fuse = d->dtype == MDG_BF16 && (C == 128 || C == 256 || C == 384 || C == 512);
  auto ln = [&](int shift_off, int scale_off) -> int {
    return hip_check(mdg::ln_mod_launch(d->dtype, N, C, h, mods, ms, TL, shift_off, scale_off, 1e-6f, xn, s),
                     "ln_mod");
  };

  mdg_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.dtype = d->dtype;
  g.M = N;
  g.a_mode = MDG_A_PLAIN;
  g.mods = mods;
  g.mod_stride = ms;
  g.rows_per_mod = TL;
  g.H = H; g.D = D; g.T = T; g.L = L;

  // ---- spatial attention: x += gate_l * mha_l(mod(LN x))      (latent_model.py:466-472)
  if (!(fuse && ho.xn_ready))
    if (int e = ln(0, C)) return e;
  mdg_gemm_desc q = g;
  q.epi = MDG_EPI_QKV;
  q.N = 3 * C; q.K = C; q.A = xn; q.lda = C; q.W = w->wqkv[0]; q.ldw = C; q.bias = w->bqkv[0];
  q.rope = rope_l; q.rope_rows = L + 1;
  // bf16 with D % 8 == 0: the attention planes are stored packed (row stride D, 24 of the padded
  // 32 columns); the attention kernel synthesises the pad column while staging
  const bool packed = packed_planes(*d);
  auto attn_t = [&](int Bq, int Tq, int Lq, const float* kb, const float* kvb) -> int {
    return packed ? mdg_attn_temporal_packed(d->dtype, Bq, Tq, Lq, H, D, qkv_t, kb, kvb, o, stream)
                  : mdg_attn_temporal(d->dtype, Bq, Tq, Lq, H, D, qkv_t, kb, kvb, o, stream);
  };
  const int tlayout = packed ? MDG_QKV_TEMPORAL_PACKED : MDG_QKV_TEMPORAL;
  if (L >= kSpatialMfmaMinL && (size_t)B * T <= 65535) {
    // long residue axis (ATLAS crop 256): every frame is one attention sequence of L tokens;
    // the temporal MFMA kernel runs it with (B', T', L') = (B*T, L, 1) — same token order
    q.qkv_layout = tlayout; q.qkv_out = qkv_t; q.qscale = qs * 1.4426950408889634f;
    q.T = L; q.L = 1;
    if (int e = mdg_gemm(&q, stream)) return e;
    q.T = T; q.L = L;
    const float* kbias_s = (const float*)(wsb + lay.kbias_s);
    if (int e = attn_t(B * T, L, 1, kbias_s, w->kvb[0])) return e;
  } else if (fuse_spatial_attn(*d)) {
    // q|k|v of the 4 residues stay on chip: projection + attention -> o in one launch
    q.epi = MDG_EPI_ATTN_SPATIAL; q.qscale = qs;
    q.out = o; q.ldo = C; q.kvb = w->kvb[0]; q.key_mask = mask;
    q.qkv_out = qkv_s;  // unused by the product kernel (a diagnostic build dumps its q|k|v tile there)
    if (int e = mdg_gemm(&q, stream)) return e;
  } else {
    q.qkv_layout = MDG_QKV_SPATIAL; q.qkv_out = qkv_s; q.qscale = qs;
    if (int e = mdg_gemm(&q, stream)) return e;
    if (int e = mdg_attn_spatial(d->dtype, B * T, L, H, D, qkv_s, w->kvb[0], mask, o, stream)) return e;
  }
  mdg_gemm_desc r = g;
  r.epi = MDG_EPI_GATE_RES;
  r.N = C; r.K = C; r.A = o; r.lda = C; r.W = w->wo[0]; r.ldw = C; r.bias = w->bo[0];
  r.resid = h; r.ldr = C; r.gate = mods; r.gate_off = 2 * C;
  if (fuse) {  // + LN_temporal(h) -> xn
    r.xn_out = xn; r.xn_mods = mods; r.xn_mod_stride = ms; r.xn_shift_off = 3 * C; r.xn_scale_off = 4 * C;
    r.ln_eps = 1e-6f;
  }

  // ---- temporal attention: x += gate_t * mha_t(mod(LN x))     (latent_model.py:474-486)
  q.epi = MDG_EPI_QKV;  // (the spatial launch above may have been the fused ATTN_SPATIAL form)
  q.W = w->wqkv[1]; q.bias = w->bqkv[1];
  q.qkv_layout = tlayout; q.qkv_out = qkv_t; q.qscale = qs * 1.4426950408889634f;
  q.rope = rope_t; q.rope_rows = T + 1;
  if (fuse && fused_qkv_on() && !small_m(N) && mdg::rowln_qkv_supported(r, q)) {
    // out_proj + gated residual + LN_t + q|k|v in one launch (xn is not written)
    if (int e = hip_check(mdg::rowln_qkv_launch(r, q, s), "rowln_qkv launch")) return e;
  } else {
    if (int e = rowln_gemm(r)) return e;
    if (!fuse)
      if (int e = ln(3 * C, 4 * C)) return e;
    if (int e = mdg_gemm(&q, stream)) return e;
  }
  if (int e = attn_t(B, T, L, kbias, w->kvb[1])) return e;
  r.W = w->wo[1]; r.bias = w->bo[1]; r.gate_off = 5 * C;
  if (fuse) {  // + LN_mlp(h) -> xn
    r.xn_shift_off = 6 * C; r.xn_scale_off = 7 * C;
  }

  // ---- MLP: x += gate_m * fc2(gelu(fc1(mod(LN x))))           (latent_model.py:488-491)
  mdg_gemm_desc f1 = g;
  f1.epi = MDG_EPI_STORE; f1.act = MDG_ACT_GELU;
  f1.N = F; f1.K = C; f1.A = xn; f1.lda = C; f1.W = w->w1; f1.ldw = C; f1.bias = w->b1;
  f1.out = hid; f1.ldo = F;
  mdg_gemm_desc f2 = g;
  f2.epi = MDG_EPI_GATE_RES;
  f2.N = C; f2.K = F; f2.A = hid; f2.lda = F; f2.W = w->w2; f2.ldw = F; f2.bias = w->b2;
  f2.resid = h; f2.ldr = C; f2.gate = mods; f2.gate_off = 8 * C;
  if (fuse && ho.next_mods) {  // + the next consumer's LN(h) -> xn
    f2.xn_out = xn; f2.xn_mods = ho.next_mods; f2.xn_mod_stride = ho.next_stride;
    f2.xn_shift_off = ho.next_shift; f2.xn_scale_off = ho.next_scale; f2.ln_eps = 1e-6f;
  }
  const bool mlp1 = fuse && fused_mlp_on() && mdg::mlp_fused_supported(f1, f2);
  if (mlp1 && mlp_pre_on() && mdg::mlp_pre_supported(r, f1, f2))  // out_proj + MLP: one launch
    return hip_check(mdg::mlp_fused_launch(f1, f2, (hipStream_t)stream, nullptr, &r), "out_proj + mlp fused launch");
  if (int e = rowln_gemm(r)) return e;
  if (!fuse)
    if (int e = ln(6 * C, 7 * C)) return e;
  if (mlp1)
    return hip_check(mdg::mlp_fused_launch(f1, f2, (hipStream_t)stream, (float*)(wsb + lay.mlp_part)),
                     "mlp fused launch");
  if (int e = mdg_gemm(&f1, stream)) return e;
  return mdg_gemm(&f2, stream);
}

int mdg_mlp_fused(const mdg_gemm_desc* f1, const mdg_gemm_desc* f2, void* stream) {
  if (!f1 || !f2) return fail(MDG_E_ARG, "mlp_fused: null descriptor");
  if (!f1->A || !f1->W || !f2->W || !f2->resid) return fail(MDG_E_ARG, "mlp_fused: null pointer");
  if (!mdg::mlp_fused_supported(*f1, *f2))
    return fail(MDG_E_SHAPE, "mlp_fused: outside the envelope (bf16, K=N=384, F %% 128, rows_per_mod >= 128) "
                "M=%d C=%d F=%d", f1->M, f1->K, f1->N);
  return hip_check(mdg::mlp_fused_launch(*f1, *f2, (hipStream_t)stream, nullptr), "mlp fused launch");
}

int mdg_rowln_mlp(const mdg_gemm_desc* r, const mdg_gemm_desc* f1, const mdg_gemm_desc* f2, void* stream) {
  if (!r || !f1 || !f2) return fail(MDG_E_ARG, "rowln_mlp: null descriptor");
  if (!r->A || !r->W || !r->resid || !f1->W || !f2->W || !f2->resid) return fail(MDG_E_ARG, "rowln_mlp: null pointer");
  if (!mdg::mlp_pre_supported(*r, *f1, *f2))
    return fail(MDG_E_SHAPE, "rowln_mlp: outside the envelope (bf16, K=N=384, one-pass MLP (>= 64 row tiles), "
                "out_proj.xn_out == fc1.A, out_proj.resid == fc2.resid, rows_per_mod >= 128) M=%d", r->M);
  return hip_check(mdg::mlp_fused_launch(*f1, *f2, (hipStream_t)stream, nullptr, r), "rowln_mlp launch");
}

int mdg_rowln_qkv(const mdg_gemm_desc* r, const mdg_gemm_desc* q, void* stream) {
  if (!r || !q) return fail(MDG_E_ARG, "rowln_qkv: null descriptor");
  if (!r->A || !r->W || !r->resid || !q->W || !q->qkv_out) return fail(MDG_E_ARG, "rowln_qkv: null pointer");
  if (!mdg::rowln_qkv_supported(*r, *q))
    return fail(MDG_E_SHAPE, "rowln_qkv: outside the envelope (bf16, C=384, LN output, packed temporal planes, "
                "head_dim %% 8 == 0 and <= 48, rows_per_mod >= 128) M=%d D=%d", r->M, q->D);
  return hip_check(mdg::rowln_qkv_launch(*r, *q, (hipStream_t)stream), "rowln_qkv launch");
}

int mdg_layer_fwd(const mdg_dims* d, const mdg_layer_weights* w, const float* rope_l,
                  const float* rope_t, const float* mods, const float* mask, float* h, void* ws,
                  void* stream) {
  if (int e = check_dims(d)) return e;
  if (!w || !mods || !h || !ws) return fail(MDG_E_ARG, "layer_fwd: null pointer");
  return layer_fwd_impl(d, w, rope_l, rope_t, mods, mask, h, ws, stream, LnHandoff{false, nullptr, 0, 0, 0});
}

// Layers [first, last) of one denoising step; `first == 0` also runs the embedding (+ layer
// 0's LN input), `last == num_layers` also the FinalLayer + Euler update.
static int denoise_range(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws, int first, int last,
                         void* stream) {
  if (!m || !io) return fail(MDG_E_ARG, "denoise_step: null model/io");
  const mdg_dims* d = &m->dims;
  if (int e = check_dims(d)) return e;
  if (!io->x_in || !io->base || !io->mods || !io->mods_final || !io->h)
    return fail(MDG_E_ARG, "denoise_step: null io pointer");
  const int N = d->B * d->T * d->L;
  const size_t mstride = (size_t)d->B * 9 * d->C;
  const WsLayout lay = ws_layout(*d);
  void* xn = (char*)ws + lay.xn;
  const int C = d->C;
  const bool fuse = d->dtype == MDG_BF16 && (C == 128 || C == 256 || C == 384 || C == 512);
  if (first < 0 || last > d->num_layers || first > last) return fail(MDG_E_ARG, "denoise_step: layer range");
  if (first > 0) {
    // resumes a step whose layers [0, first) already ran: h and (fused path) xn are in place
  } else if (fuse) {  // embedding + layer 0's spatial LN input in one pass; later LN inputs
                      // come out of the fused fc2 epilogues
    if (int e = hip_check(mdg::embed_ln_launch(N, d->T * d->L, d->L, C, d->latent, io->x_in, m->w_l2e_t, io->base,
                                               io->ipa, io->mods, 9 * C, 0, C, 1e-6f, io->h, xn,
                                               (hipStream_t)stream), "embed_ln"))
      return e;
  } else if (int e = mdg_embed(N, d->T, d->L, d->C, d->latent, io->x_in, m->w_l2e_t, nullptr, io->base,
                               nullptr, nullptr, nullptr, io->ipa, io->h, stream)) {
    return e;
  }
  for (int i = first; i < last; ++i) {
    const bool final_next = i + 1 == d->num_layers;  // the next LN input is the FinalLayer's
    const LnHandoff ho{fuse, final_next ? io->mods_final : io->mods + (i + 1) * mstride, final_next ? 2 * C : 9 * C,
                       0, C, io->chain_alone != 0};
    if (!m->layers[i].wqkv[0]) return fail(MDG_E_ARG, "denoise_step: layer %d weights missing", i);
    if (int e = layer_fwd_impl(d, &m->layers[i], m->rope_l, m->rope_t, io->mods + i * mstride, mask, io->h, ws,
                               stream, ho))
      return e;
  }
  if (last < d->num_layers) return 0;
  // FinalLayer: LN + modulate (layers.py:73) into xn (already there on the fused path), then
  // the EULER-epilogue GEMM
  if (!fuse)
    if (int e = hip_check(mdg::ln_mod_launch(d->dtype, N, C, io->h, io->mods_final, 2 * C, d->T * d->L, 0, C, 1e-6f,
                                             xn, (hipStream_t)stream), "ln_mod(final)"))
      return e;
  mdg_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.dtype = d->dtype;
  g.a_mode = MDG_A_PLAIN;
  g.epi = MDG_EPI_EULER;
  g.M = N; g.N = (d->latent + 31) / 32 * 32; g.K = d->C;
  g.A = xn; g.lda = d->C; g.W = m->w_final; g.ldw = d->C; g.bias = m->b_final;
  g.out = io->x_out; g.ldo = d->latent; g.x_in = io->x_in; g.v_out = io->v_out; g.dt = io->dt;
  g.n_valid = d->latent;
  return mdg_gemm(&g, stream);  // bf16: the one-pass final_euler_kernel
}

#ifdef MDG_DIAGNOSTICS
static int denoise_range_dbg(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws, int first,
                             int last, void* stream) {
  g_dbg_stream = (hipStream_t)stream;
  g_dbg_in_step = true;
  if (m && io && g_snap.dst) {
    const mdg_dims& d = m->dims;
    const size_t N = (size_t)d.B * d.T * d.L;
    g_dbg_regions[0] = {ws, ws_layout(d).total};
    g_dbg_regions[1] = {io->h, N * d.C * sizeof(float)};
    g_dbg_regions[2] = {io->x_out ? io->x_out : io->x_in, N * d.latent * sizeof(float)};
  }
  const int e = denoise_range(m, io, mask, ws, first, last, stream);
  g_dbg_stream = nullptr;
  g_dbg_in_step = false;
  return e;
}

#else
static int denoise_range_dbg(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws, int first,
                             int last, void* stream) {
  return denoise_range(m, io, mask, ws, first, last, stream);
}
#endif

int mdg_denoise_step(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws, void* stream) {
  if (!m) return fail(MDG_E_ARG, "denoise_step: null model/io");
  return denoise_range_dbg(m, io, mask, ws, 0, m->dims.num_layers, stream);
}

int mdg_denoise_step_layers(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws,
                            int32_t first_layer, int32_t last_layer, void* stream) {
  return denoise_range_dbg(m, io, mask, ws, first_layer, last_layer, stream);
}

int mdg_describe_plan(const mdg_dims* d, char* buf, size_t n) {
  if (int e = check_dims(d)) return e;
  if (!buf || n == 0) return fail(MDG_E_ARG, "describe_plan: null buffer");
  const int C = d->C;
  const bool fuse = d->dtype == MDG_BF16 && (C == 128 || C == 256 || C == 384 || C == 512);
  const char* spatial;
  if (d->L >= kSpatialMfmaMinL && (size_t)d->B * d->T <= 65535)
    spatial = "qkv_gemm(temporal layout)+attn_temporal_mfma(one sequence per frame)";
  else if (fuse_spatial_attn(*d))
    spatial = "gemm_qkv_attn_spatial(fused projection+attention)";
  else
    spatial = "qkv_gemm(spatial layout)+attn_spatial(valu)";
  snprintf(buf, n,
           "{\"dtype\": \"%s\", \"spatial\": \"%s\", \"ln_handoff\": \"%s\", "
           "\"temporal\": \"%s+%s\", \"planes\": \"%s\", \"mlp\": \"%s\", "
           "\"final\": \"%s\"}",
           d->dtype == MDG_BF16 ? "bf16" : "f32", spatial,
           fuse ? "fused into gated-residual row-LN GEMM epilogues" : "stand-alone ln_mod pass",
           (fuse && fused_qkv_on() && C == 384 && packed_planes(*d) && d->D <= 48 && d->T * d->L >= 128 &&
            !small_m((long long)d->B * d->T * d->L))
               ? "rowln_qkv(spatial out_proj+gated residual+LN_t+q|k|v in one kernel, LN_t on chip)"
               : "qkv_gemm",
           d->D >= MDG_DP ? (d->dtype == MDG_BF16 ? "attn_temporal(wide heads: bf16 16x16x32 mfma, 64-col rows)"
                                                  : "attn_temporal(wide heads: f32 16x16x4 mfma, 64-col rows)")
           : d->dtype == MDG_BF16 ? "attn_temporal_bf16(32x32x16 mfma)" : "attn_temporal(f32 16x16x4 mfma)",
           packed_planes(*d) ? "packed (row stride = head_dim)" : "padded (row stride MDG_HEAD_STRIDE)",
           (fuse && fused_mlp_on() && d->dtype == MDG_BF16 && d->C == 384 && d->T * d->L >= 128)
               ? (mdg::mlp_split_factor(d->B * d->T * d->L, d->F) > 1
                      ? "mlp_fused(small M: hidden chunks split over blocks, fp32 partials + row-LN pass)"
                      : "mlp_fused(fc1+gelu+fc2+gated residual+LN in one kernel, hidden on chip)")
           : fuse ? "fc1_gemm(gelu)+fc2_rowln_gemm"
                  : "fc1_gemm(gelu)+fc2_gate_res_gemm",
           (d->dtype == MDG_BF16 && fast_final_on() && d->latent <= 32 && (C == 128 || C == 256 || C == 384 || C == 512))
               ? "final_euler_kernel(one pass, W in LDS)"
               : "euler_epilogue_gemm");
  return MDG_OK;
}

int mdg_prep_latents(int32_t B, int32_t T, int32_t L, int32_t latent, int32_t flags, int32_t cond_interval,
                     const float* rots, const float* trans, const float* torsions, float* latents,
                     float* x_cond, int64_t* cond_mask, void* stream) {
  if (!rots || !trans || !latents) return fail(MDG_E_ARG, "prep_latents: null rots/trans/latents");
  if (B <= 0 || T <= 0 || L <= 0) return fail(MDG_E_SHAPE, "prep_latents: B,T,L = %d,%d,%d", B, T, L);
  const int tps = (flags & MDG_PREP_TPS) ? 1 : 0;
  if (latent != (tps ? 28 : 21))
    return fail(MDG_E_SHAPE, "prep_latents: latent %d != %d (offsets + 14 torsion channels)", latent, tps ? 28 : 21);
  if (flags & ~(MDG_PREP_TPS | MDG_PREP_NO_OFFSETS | MDG_PREP_COND_FIRST | MDG_PREP_COND_LAST) || cond_interval < 0)
    return fail(MDG_E_ARG, "prep_latents: flags 0x%x / cond_interval %d", flags, cond_interval);
  return hip_check(mdg::prep_latents_launch(B, T, L, latent, tps, (flags & MDG_PREP_NO_OFFSETS) ? 1 : 0, flags,
                                            cond_interval, rots, trans, torsions, latents, x_cond, cond_mask,
                                            (hipStream_t)stream),
                   "prep_latents");
}

int mdg_latents_to_atom14(int32_t B, int32_t T, int32_t L, int32_t latent, int32_t tors_off, int32_t renorm,
                          const float* samples, const float* ref_rots, const float* ref_trans,
                          const int64_t* aatype, const float* default_frames, const int32_t* group_idx,
                          const float* atom_mask, const float* lit, float* atom14, float* out_rots,
                          float* out_trans, void* stream) {
  if (!samples || !ref_rots || !ref_trans || !aatype || !default_frames || !group_idx || !atom_mask || !lit || !atom14)
    return fail(MDG_E_ARG, "latents_to_atom14: null pointer");
  if ((out_rots == nullptr) != (out_trans == nullptr)) return fail(MDG_E_ARG, "latents_to_atom14: out_rots/out_trans");
  if (B <= 0 || T <= 0 || L <= 0 || tors_off < 7 || latent < tors_off + 14)
    return fail(MDG_E_SHAPE, "latents_to_atom14: B,T,L=%d,%d,%d latent=%d tors_off=%d", B, T, L, latent, tors_off);
  return hip_check(mdg::latents_to_atom14_launch(B, T, L, latent, tors_off, renorm ? 1 : 0, samples, ref_rots,
                                                 ref_trans, aatype, default_frames, group_idx, atom_mask, lit,
                                                 atom14, out_rots, out_trans, (hipStream_t)stream),
                   "latents_to_atom14");
}

// ------------------------------------------------------------------------------------------
// Training entry points (train.hip kernels + the GEMM's training epilogues).
int mdg_mask_bias(int32_t B, int32_t T, int32_t L, const float* mask, float* kbias_t, float* kbias_s, void* stream) {
  if (!mask || !kbias_t || !kbias_s) return fail(MDG_E_ARG, "mask_bias: null pointer");
  if (B <= 0 || T <= 0 || L <= 0) return fail(MDG_E_SHAPE, "mask_bias: B,T,L = %d,%d,%d", B, T, L);
  return hip_check(mdg::mask_bias_launch(B, T, L, mask, kbias_t, kbias_s, (hipStream_t)stream), "mask_bias");
}

static int init_planes(const mdg_dims* d, void* planes, int B, int T, int L, hipStream_t s) {
  const size_t cs = ct_size(d->dtype);
  const size_t rows = (size_t)B * L * d->H * T;
  const size_t dp = dp_of(d->D);
  if (int e = hip_check(hipMemsetAsync(planes, 0, 3 * rows * dp * cs, s), "planes memset")) return e;
  return hip_check(mdg::set_vpad_launch(d->dtype, (char*)planes + rows * dp * cs, 2 * rows, d->D, s), "set_vpad");
}

// the row-LN route of the training forward (gemm.hip kCfgRowTrain); MDG_TRAIN_ROWLN=0: the GEMM +
// mdg_ln_mod pair (A/B)
static constexpr int kCfgRowTrainId = 105;
static bool train_rowln_on() {
  static const bool v = [] {
    const char* e = getenv("MDG_TRAIN_ROWLN");
    return !(e && e[0] == '0');
  }();
  return v;
}

int mdg_layer_fwd_train(const mdg_dims* d, const mdg_layer_weights* w, const float* rope_l, const float* rope_t,
                        const float* mods, const float* mask, const float* kbias_t, const float* kbias_s,
                        const float* h_in, float* h_out, const mdg_layer_saved* sv, void* stream) {
  if (int e = check_dims(d)) return e;
  if (!w || !mods || !kbias_t || !h_in || !h_out || !sv || h_in == h_out)
    return fail(MDG_E_ARG, "layer_fwd_train: null pointer or h_in == h_out");
  for (int i = 0; i < 3; ++i)
    if (!sv->xn[i] || !sv->stats[i] || !sv->y[i]) return fail(MDG_E_ARG, "layer_fwd_train: saved xn/stats/y %d", i);
  if (!sv->qkv_s || !sv->qkv_t || !sv->lse_t || !sv->o[0] || !sv->o[1] || !sv->h1 || !sv->h2 || !sv->u || !sv->act)
    return fail(MDG_E_ARG, "layer_fwd_train: null saved buffer");
  const int B = d->B, T = d->T, L = d->L, C = d->C, H = d->H, D = d->D, F = d->F;
  const int N = B * T * L, TL = T * L, ms = 9 * C;
  const bool long_l = L >= kSpatialMfmaMinL && (size_t)B * T <= 65535;
  if (long_l && (!sv->lse_s || !kbias_s)) return fail(MDG_E_ARG, "layer_fwd_train: L >= 16 needs lse_s, kbias_s");
  if (!long_l && L >= kSpatialMfmaMinL) return fail(MDG_E_SHAPE, "layer_fwd_train: B*T > 65535 at L >= 16");
  const float qs = 1.0f / sqrtf((float)D), log2e = 1.4426950408889634f;
  hipStream_t s = (hipStream_t)stream;
  if (sv->init_planes) {
    if (int e = init_planes(d, sv->qkv_t, B, T, L, s)) return e;
    if (long_l)
      if (int e = init_planes(d, sv->qkv_s, B * T, L, 1, s)) return e;
  }
  auto ln = [&](const float* h, int i, int shift_off, int scale_off) -> int {
    return hip_check(mdg::ln_mod_launch(d->dtype, N, C, h, mods, ms, TL, shift_off, scale_off, 1e-6f, sv->xn[i], s,
                                        sv->stats[i]), "ln_mod(train)");
  };
  mdg_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.dtype = d->dtype; g.M = N; g.a_mode = MDG_A_PLAIN;
  g.mods = mods; g.mod_stride = ms; g.rows_per_mod = TL;
  g.H = H; g.D = D; g.T = T; g.L = L;

  // ---- spatial sublayer (latent_model.py:466-472)
  if (!sv->xn0_given)
    if (int e = ln(h_in, 0, 0, C)) return e;
  mdg_gemm_desc q = g;
  q.epi = MDG_EPI_QKV; q.N = 3 * C; q.K = C; q.A = sv->xn[0]; q.lda = C; q.W = w->wqkv[0]; q.ldw = C;
  q.bias = w->bqkv[0]; q.rope = rope_l; q.rope_rows = L + 1;
  if (long_l) {
    q.qkv_layout = MDG_QKV_TEMPORAL; q.qkv_out = sv->qkv_s; q.qscale = qs * log2e; q.T = L; q.L = 1;
    if (int e = mdg_gemm(&q, stream)) return e;
    if (int e = mdg_attn_temporal_lse(d->dtype, B * T, L, 1, H, D, sv->qkv_s, kbias_s, w->kvb[0], sv->o[0], sv->o_lo[0], sv->lse_s,
                                      stream))
      return e;
    q.T = T; q.L = L;
  } else {
    q.qkv_layout = MDG_QKV_SPATIAL; q.qkv_out = sv->qkv_s; q.qscale = qs;
    if (int e = mdg_gemm(&q, stream)) return e;
    if (int e = mdg_attn_spatial(d->dtype, B * T, L, H, D, sv->qkv_s, w->kvb[0], mask, sv->o[0], stream)) return e;
  }
  mdg_gemm_desc r = g;
  r.epi = MDG_EPI_GATE_RES; r.N = C; r.K = C; r.A = sv->o[0]; r.lda = C; r.W = w->wo[0]; r.ldw = C; r.bias = w->bo[0];
  r.resid_in = h_in; r.resid = sv->h1; r.ldr = C; r.gate = mods; r.gate_off = 2 * C; r.aux = sv->y[0]; r.ldaux = C;
  // the out_proj and the NEXT sublayer's LayerNorm + modulate as one row-LN launch (its xn, the
  // LN row statistics and the pre-gate value saved), where the bf16 row-LN GEMM takes the shape;
  // otherwise the GEMM then mdg_ln_mod.  Returns 1 when the LN was fused.
  auto out_proj_ln = [&](mdg_gemm_desc& rr, int next, int shift_off, int scale_off, bool& fused) -> int {
    fused = false;
    if (train_rowln_on()) {
      mdg_gemm_desc f = rr;
      f.xn_out = sv->xn[next]; f.xn_mods = mods; f.xn_mod_stride = ms; f.xn_shift_off = shift_off;
      f.xn_scale_off = scale_off; f.ln_eps = 1e-6f; f.ln_stats = sv->stats[next];
      if (mdg::gemm_plan(f).cfg == kCfgRowTrainId) {
        fused = true;
        return mdg_gemm(&f, stream);
      }
    }
    return mdg_gemm(&rr, stream);
  };
  bool fused_ln = false;
  if (sv->skip_temporal) {
    if (int e = out_proj_ln(r, 2, 6 * C, 7 * C, fused_ln)) return e;
  } else {
    if (int e = out_proj_ln(r, 1, 3 * C, 4 * C, fused_ln)) return e;
  }

  // ---- temporal sublayer (latent_model.py:474-486); skipped for the IPA layers' tail (gate 0)
  const float* h_mlp = sv->h1;
  bool mlp_ln_done = sv->skip_temporal && fused_ln;
  if (!sv->skip_temporal) {
    if (!fused_ln)
      if (int e = ln(sv->h1, 1, 3 * C, 4 * C)) return e;
    q.epi = MDG_EPI_QKV; q.A = sv->xn[1]; q.W = w->wqkv[1]; q.bias = w->bqkv[1];
    q.qkv_layout = MDG_QKV_TEMPORAL; q.qkv_out = sv->qkv_t; q.qscale = qs * log2e; q.rope = rope_t; q.rope_rows = T + 1;
    if (int e = mdg_gemm(&q, stream)) return e;
    if (int e = mdg_attn_temporal_lse(d->dtype, B, T, L, H, D, sv->qkv_t, kbias_t, w->kvb[1], sv->o[1], sv->o_lo[1], sv->lse_t,
                                      stream))
      return e;
    r.A = sv->o[1]; r.W = w->wo[1]; r.bias = w->bo[1]; r.resid_in = sv->h1; r.resid = sv->h2; r.gate_off = 5 * C;
    r.aux = sv->y[1];
    if (int e = out_proj_ln(r, 2, 6 * C, 7 * C, mlp_ln_done)) return e;
    h_mlp = sv->h2;
  }

  // ---- MLP (latent_model.py:488-491)
  if (!mlp_ln_done)
    if (int e = ln(h_mlp, 2, 6 * C, 7 * C)) return e;
  mdg_gemm_desc f1 = g;
  f1.epi = MDG_EPI_STORE; f1.act = MDG_ACT_GELU; f1.N = F; f1.K = C; f1.A = sv->xn[2]; f1.lda = C; f1.W = w->w1;
  f1.ldw = C; f1.bias = w->b1; f1.out = sv->act; f1.ldo = F; f1.aux = sv->u; f1.ldaux = F;
  if (int e = mdg_gemm(&f1, stream)) return e;
  mdg_gemm_desc f2 = g;
  f2.epi = MDG_EPI_GATE_RES; f2.N = C; f2.K = F; f2.A = sv->act; f2.lda = F; f2.W = w->w2; f2.ldw = F; f2.bias = w->b2;
  f2.resid_in = h_mlp; f2.resid = h_out; f2.ldr = C; f2.gate = mods; f2.gate_off = 8 * C; f2.aux = sv->y[2];
  f2.ldaux = C;
  if (!sv->xn_next) return mdg_gemm(&f2, stream);
  if (!sv->stats_next || !sv->mods_next) return fail(MDG_E_ARG, "layer_fwd_train: xn_next without stats / mods");
  // the next layer's first LayerNorm (LN_s with its adaLN rows) in fc2's row-LN epilogue, or after it
  if (train_rowln_on()) {
    mdg_gemm_desc f = f2;
    f.xn_out = sv->xn_next; f.xn_mods = sv->mods_next; f.xn_mod_stride = ms; f.xn_shift_off = 0;
    f.xn_scale_off = C; f.ln_eps = 1e-6f; f.ln_stats = sv->stats_next;
    if (mdg::gemm_plan(f).cfg == kCfgRowTrainId) return mdg_gemm(&f, stream);
  }
  if (int e = mdg_gemm(&f2, stream)) return e;
  return hip_check(mdg::ln_mod_launch(d->dtype, N, C, h_out, sv->mods_next, ms, TL, 0, C, 1e-6f, sv->xn_next, s,
                                      sv->stats_next), "ln_mod(next)");
}

int32_t mdg_ln_gate_bwd_blocks(int32_t rows_per_b) { return rows_per_b > 0 ? mdg::ln_gate_bwd_blocks(rows_per_b) : 0; }

int mdg_ln_gate_bwd(int32_t dtype, int32_t M, int32_t C, int32_t rows_per_b, const void* dxn, const float* h_ln,
                    const float* stats, const float* mods, int32_t mod_stride, int32_t shift_off, int32_t scale_off,
                    const float* dh_res, float* dh_out, const void* y, int32_t gate_off, void* dy, float* part,
                    void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", dtype);
  if (M <= 0 || C <= 0 || C > 512 || C % 64 || rows_per_b <= 0 || M % rows_per_b)
    return fail(MDG_E_SHAPE, "ln_gate_bwd: M=%d C=%d rows_per_b=%d", M, C, rows_per_b);
  if (!mods || !dh_res || !dh_out || !part) return fail(MDG_E_ARG, "ln_gate_bwd: null mods/dh/part");
  if (dxn && (!h_ln || !stats)) return fail(MDG_E_ARG, "ln_gate_bwd: dxn without h_ln/stats");
  if (y && !dy) return fail(MDG_E_ARG, "ln_gate_bwd: y without dy");
  return hip_check(mdg::ln_gate_bwd_launch(dtype, M, C, rows_per_b, dxn, h_ln, stats, mods, mod_stride, shift_off,
                                           scale_off, dh_res, dh_out, y, gate_off, dy, part, (hipStream_t)stream),
                   "ln_gate_bwd");
}

int32_t mdg_attn_temporal_bwd_parts(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t generic) {
  if (B <= 0 || T <= 0 || L <= 0) return 0;
  return mdg::attn_bwd_parts(dtype, B, T, L, generic);
}

int32_t mdg_attn_spatial_bwd_parts(int32_t n_frames, int32_t L, int32_t H, int32_t D) {
  if (n_frames <= 0 || L <= 0 || H <= 0) return 0;
  return mdg::attn_spatial_bwd_parts(n_frames, L, H, D);
}

size_t mdg_attn_temporal_bwd_scratch(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D) {
  if (D <= 0 || D >= MDG_DP_WIDE) return 0;
  const size_t rows = (size_t)B * L * H * T, dp = dp_of(D);
  // + the fused bf16 kernel's fp32 dQ accumulator when the keys take more than one 256-key pass
  const size_t acc = (dtype == MDG_BF16 && T > 256 && D < MDG_DP) ? align256(rows * MDG_DP * sizeof(float)) : 0;
  return align256(rows * dp * ct_size(dtype)) + align256(rows * sizeof(float)) + acc;
}

int mdg_attn_temporal_bwd(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D, const void* qkv_t,
                          const float* kbias, const float* kvb, const void* o, const void* o_lo, const void* dout,
                          const float* lse,
                          const float* rope, int32_t rope_rows, void* scratch, void* dqkv, int32_t ld_dqkv,
                          float* bpart, float qscale, float kscale, int32_t generic, void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", dtype);
  if (!qkv_t || !kbias || !kvb || !o || !dout || !lse || !scratch || !dqkv || !bpart)
    return fail(MDG_E_ARG, "attn_temporal_bwd: null pointer");
  if (B <= 0 || T <= 0 || L <= 0 || H <= 0 || D <= 0 || D % 4 || D >= MDG_DP_WIDE || ld_dqkv < 3 * H * D ||
      ld_dqkv % 4)
    return fail(MDG_E_SHAPE, "attn_temporal_bwd: B=%d T=%d L=%d H=%d D=%d ld=%d", B, T, L, H, D, ld_dqkv);
  // wide heads (head_dim 32..63) run the scalar kernels only: the caller sizes bpart for them
  if (D >= MDG_DP && dtype == MDG_BF16 && generic != 1)
    return fail(MDG_E_ARG, "attn_temporal_bwd: head_dim %d takes generic = 1 (the scalar kernels)", D);
  if (rope && rope_rows < T) return fail(MDG_E_SHAPE, "attn_temporal_bwd: rope table too short");
  if ((size_t)B * L * H > 65535u * 256u) return fail(MDG_E_SHAPE, "attn_temporal_bwd: grid too large");
  const size_t rows = (size_t)B * L * H * T;
  void* dop = scratch;
  float* delta = (float*)((char*)scratch + align256(rows * dp_of(D) * ct_size(dtype)));
  float* dqacc = (float*)((char*)delta + align256(rows * sizeof(float)));
  if (generic < 0 || generic > 2) return fail(MDG_E_ARG, "attn_temporal_bwd: generic=%d (0, 1, 2)", generic);
  return hip_check(mdg::attn_temporal_bwd_launch(dtype, B, T, L, H, D, qkv_t, kbias, kvb, o, o_lo, dout, lse, rope,
                                                 rope_rows, dop, delta, dqkv, ld_dqkv, bpart, qscale, kscale,
                                                 dtype == MDG_F32 ? 1 : generic, dqacc, (hipStream_t)stream),
                   "attn_temporal_bwd");
}

int mdg_attn_spatial_bwd(int32_t dtype, int32_t n_frames, int32_t L, int32_t H, int32_t D, const void* qkv,
                         const float* kvb, const float* mask, const void* dout, const float* rope, int32_t rope_rows,
                         void* dqkv, float* bpart, float qscale, void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "dtype %d", dtype);
  if (!qkv || !kvb || !dout || !dqkv || !bpart) return fail(MDG_E_ARG, "attn_spatial_bwd: null pointer");
  if (n_frames <= 0 || L <= 0 || L > 16 || H <= 0 || D <= 0 || D % 4 || D >= MDG_DP_WIDE)
    return fail(MDG_E_SHAPE, "attn_spatial_bwd: nf=%d L=%d H=%d D=%d (L <= 16, head_dim < %d)", n_frames, L, H, D,
                MDG_DP_WIDE);
  if (rope && rope_rows < L) return fail(MDG_E_SHAPE, "attn_spatial_bwd: rope table too short");
  return hip_check(mdg::attn_spatial_bwd_launch(dtype, n_frames, L, H, D, qkv, kvb, mask, dout, rope, rope_rows, dqkv,
                                                bpart, qscale, (hipStream_t)stream),
                   "attn_spatial_bwd");
}

int mdg_ipa_core_fwd(int32_t B, int32_t L, int32_t H, int32_t c, int32_t Pq, int32_t Pv, const float* q,
                     const float* kv, const float* qp, const float* kvp, const float* mask, const float* rots,
                     const float* trans, const float* hw, float wc, float* out, int32_t flags, void* stream) {
  if (!q || !kv || !qp || !kvp || !mask || !rots || !trans || !hw || !out) return fail(MDG_E_ARG, "ipa_core_fwd: null");
  if (B <= 0 || H <= 0 || !mdg::ipa_core_supported(L, c, Pq, Pv))
    return fail(MDG_E_SHAPE, "ipa_core_fwd: B=%d L=%d H=%d c=%d Pq=%d Pv=%d (L <= 256, c = 32, 8 + 8 points)", B, L, H,
                c, Pq, Pv);
  if (flags & ~(MDG_IPA_LOCAL_POINTS | MDG_IPA_RAW_HW)) return fail(MDG_E_ARG, "ipa_core_fwd: flags %d", flags);
  return hip_check(mdg::ipa_core_fwd_launch(B, L, H, q, kv, qp, kvp, mask, rots, trans, hw, wc, out, flags,
                                            (hipStream_t)stream),
                   "ipa_core_fwd");
}

int mdg_ipa_core_bwd(int32_t B, int32_t L, int32_t H, int32_t c, int32_t Pq, int32_t Pv, const float* q,
                     const float* kv, const float* qp, const float* kvp, const float* mask, const float* rots,
                     const float* trans, const float* hw, float wc, const float* dout, float* dq, float* dkv,
                     float* dqp, float* dkvp, float* dhw_part, int32_t flags, void* stream) {
  if (!q || !kv || !qp || !kvp || !mask || !rots || !trans || !hw || !dout || !dq || !dkv || !dqp || !dkvp ||
      !dhw_part)
    return fail(MDG_E_ARG, "ipa_core_bwd: null");
  if (B <= 0 || H <= 0 || !mdg::ipa_core_supported(L, c, Pq, Pv))
    return fail(MDG_E_SHAPE, "ipa_core_bwd: B=%d L=%d H=%d c=%d Pq=%d Pv=%d (L <= 256, c = 32, 8 + 8 points)", B, L, H,
                c, Pq, Pv);
  if (flags & ~(MDG_IPA_LOCAL_POINTS | MDG_IPA_RAW_HW)) return fail(MDG_E_ARG, "ipa_core_bwd: flags %d", flags);
  return hip_check(mdg::ipa_core_bwd_launch(B, L, H, q, kv, qp, kvp, mask, rots, trans, hw, wc, dout, dq, dkv, dqp,
                                            dkvp, dhw_part, flags, (hipStream_t)stream),
                   "ipa_core_bwd");
}

int mdg_train_pack_layer(const mdg_train_pack* p, void* stream) {
  if (!p) return fail(MDG_E_ARG, "train_pack: null");
  if (p->dtype != MDG_F32 && p->dtype != MDG_BF16) return fail(MDG_E_DTYPE, "train_pack: dtype %d", p->dtype);
  if (p->C <= 0 || p->H <= 0 || p->D <= 0 || p->C != p->H * p->D || p->D % 2 || p->D >= MDG_DP_WIDE || p->F <= 0)
    return fail(MDG_E_SHAPE, "train_pack: C=%d H=%d D=%d F=%d", p->C, p->H, p->D, p->F);
  for (int i = 0; i < 2; ++i) {
    if (!p->wq[i] || !p->wk[i] || !p->wv[i] || !p->bq[i] || !p->bk[i] || !p->bv[i] || !p->wo[i] || !p->bias_k[i] ||
        !p->bias_v[i] || !p->wqkv[i] || !p->wqkv_t[i] || !p->bqkv[i] || !p->wo_p[i] || !p->wo_t[i] || !p->kvb[i])
      return fail(MDG_E_ARG, "train_pack: null pointer (attention %d)", i);
    if (p->rope && (!p->rope_tab[i] || p->rope_pos[i] < 0 || p->rope_pos[i] >= p->rope_rows[i]))
      return fail(MDG_E_SHAPE, "train_pack: rope table %d (pos %d rows %d)", i, p->rope_pos[i], p->rope_rows[i]);
  }
  if (!p->w1 || !p->w2 || !p->w1_p || !p->w1_t || !p->w2_p || !p->w2_t) return fail(MDG_E_ARG, "train_pack: MLP");
  return hip_check(mdg::train_pack_launch(*p, (hipStream_t)stream), "train_pack");
}

int mdg_train_unpack_layer(const mdg_train_unpack* u, void* stream) {
  if (!u) return fail(MDG_E_ARG, "train_unpack: null");
  if (u->C <= 0 || u->H <= 0 || u->H > 128 || u->D <= 0 || u->C != u->H * u->D || u->D % 2 || u->D >= MDG_DP_WIDE || u->B <= 0 ||
      u->nblk <= 0)
    return fail(MDG_E_SHAPE, "train_unpack: C=%d H=%d D=%d B=%d nblk=%d", u->C, u->H, u->D, u->B, u->nblk);
  for (int i = 0; i < 2; ++i) {
    if (!u->gwqkv[i] || !u->gbqkv[i] || !u->bpart[i] || u->parts[i] <= 0 || !u->gq[i] || !u->gk[i] || !u->gv[i] ||
        !u->gbq[i] || !u->gbk[i] || !u->gbv[i] || !u->gbias_k[i] || !u->gbias_v[i])
      return fail(MDG_E_ARG, "train_unpack: null pointer (attention %d)", i);
    if (u->rope && (!u->rope_tab[i] || u->rope_pos[i] < 0 || u->rope_pos[i] >= u->rope_rows[i]))
      return fail(MDG_E_SHAPE, "train_unpack: rope table %d", i);
  }
  for (int k = 0; k < 4; ++k)
    if (!u->part[k]) return fail(MDG_E_ARG, "train_unpack: part %d", k);
  if (!u->dmods || !u->gbo[0] || !u->gbo[1] || !u->gb2) return fail(MDG_E_ARG, "train_unpack: outputs");
  return hip_check(mdg::train_unpack_launch(*u, (hipStream_t)stream), "train_unpack");
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Conditioning precompute (mdg_precompute_cond): t-embedding, every adaLN modulation and the
// IPA prepend for all S time points of a window, fp32 throughout.
namespace {

struct CondLayout {
  int R, M, W, P, Ppad, Kout, Kpad;
  size_t emb, hmid, sc, all, x2, xn, proj, cat, qkv, o, hid, mrep, kb_t, kb_s, rel7, total;
};

CondLayout cond_layout(const mdg_cond_dims& d) {
  CondLayout c;
  c.R = d.S * d.B;
  c.M = c.R * d.L;
  c.W = d.num_layers * 9 * d.C + 2 * d.C + d.ipa_layers * 6 * d.C;
  const int H = d.ipa_heads;
  c.P = H * d.ipa_c * 3 + 3 * H * d.ipa_qk + 3 * H * (d.ipa_qk + d.ipa_v);
  c.Ppad = (c.P + 31) / 32 * 32;
  c.Kout = H * (d.ipa_c + 4 * d.ipa_v);
  c.Kpad = (c.Kout + 63) / 64 * 64;
  const size_t f = sizeof(float), M = (size_t)c.M, C = d.C;
  const bool ipa = d.ipa_layers > 0;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += align256(bytes); return o; };
  c.emb = take((size_t)c.R * d.freq_dim * f);
  c.hmid = take((size_t)c.R * C * f);
  c.sc = take((size_t)c.R * C * f);
  c.all = take((size_t)c.R * c.W * f);
  const size_t qkv_spatial = M * 3 * C * f;
  const size_t qkv_planes = 3ull * c.R * d.H * d.L * dp_of(d.D) * f;
  c.x2 = take(ipa && d.tps ? M * C * f : 0);
  c.xn = take(ipa ? M * C * f : 0);
  c.proj = take(ipa ? M * c.Ppad * f : 0);
  c.cat = take(ipa ? M * c.Kpad * f : 0);
  c.qkv = take(ipa ? (qkv_spatial > qkv_planes ? qkv_spatial : qkv_planes) : 0);
  c.o = take(ipa ? M * C * f : 0);
  c.hid = take(ipa ? M * 4 * C * f : 0);
  c.mrep = take(ipa ? M * f : 0);
  c.kb_t = take(ipa ? M * f : 0);
  c.kb_s = take(ipa ? M * f : 0);
  c.rel7 = take(ipa && d.tps ? 2ull * d.B * d.L * 7 * f : 0);
  c.total = off;
  return c;
}

int check_cond_dims(const mdg_cond_dims* d) {
  if (!d) return fail(MDG_E_ARG, "null cond dims");
  if (d->S <= 0 || d->B <= 0 || d->L <= 0 || d->C <= 0 || d->num_layers < 0 || d->num_layers > MDG_MAX_LAYERS ||
      d->ipa_layers < 0 || d->ipa_layers > MDG_MAX_LAYERS)
    return fail(MDG_E_SHAPE, "cond: S,B,L,C,layers = %d,%d,%d,%d,%d/%d", d->S, d->B, d->L, d->C, d->num_layers,
                d->ipa_layers);
  if (d->C % 64 || d->C > 384) return fail(MDG_E_SHAPE, "cond: embed_dim %d (64k, <= 384 on the fp32 path)", d->C);
  if (d->freq_dim <= 0 || d->freq_dim % 64) return fail(MDG_E_SHAPE, "cond: freq_dim %d (64k)", d->freq_dim);
  if ((long long)d->S * d->B * d->L * 4 * d->C >= (1ll << 31)) return fail(MDG_E_SHAPE, "cond: problem too large");
  if (d->ipa_layers > 0) {
    if (d->H <= 0 || d->C != d->H * d->D || d->D % 4 || d->D >= MDG_DP_WIDE)
      return fail(MDG_E_SHAPE, "cond: IPA-layer MHA C=%d H=%d D=%d", d->C, d->H, d->D);
    if (d->ipa_heads <= 0 || !mdg::ipa_attn_supported(d->ipa_c, d->ipa_qk, d->ipa_v))
      return fail(MDG_E_SHAPE, "cond: IPA heads=%d c=%d P_q=%d P_v=%d has no kernel instance", d->ipa_heads, d->ipa_c,
                  d->ipa_qk, d->ipa_v);
  }
  return MDG_OK;
}

}  // namespace

extern "C" {

size_t mdg_cond_workspace_bytes(const mdg_cond_dims* d) {
  if (check_cond_dims(d)) return 0;
  return cond_layout(*d).total;
}

int mdg_tps_rel7(int32_t B, int32_t L, const float* rots, const float* trans, const float* end_rots,
                 const float* end_trans, float* out, void* stream) {
  if (!rots || !trans || !end_rots || !end_trans || !out) return fail(MDG_E_ARG, "tps_rel7: null pointer");
  if (B <= 0 || L <= 0) return fail(MDG_E_SHAPE, "tps_rel7: B=%d L=%d", B, L);
  return hip_check(mdg::tps_rel7_launch(B, L, rots, trans, end_rots, end_trans, out, (hipStream_t)stream), "tps_rel7");
}

int mdg_precompute_cond(const mdg_cond_model* m, const mdg_cond_io* io, void* ws, void* stream) {
  if (!m || !io || !ws) return fail(MDG_E_ARG, "precompute_cond: null model/io/workspace");
  const mdg_cond_dims& d = m->dims;
  if (int e = check_cond_dims(&d)) return e;
  if (!io->t || !io->mods || !io->mods_final || !m->t_freqs || !m->t_w0 || !m->t_w2 || !m->ada_w)
    return fail(MDG_E_ARG, "precompute_cond: null t / outputs / t-embedder / adaLN weights");
  const CondLayout c = cond_layout(d);
  char* wb = (char*)ws;
  auto F = [&](size_t off) { return (float*)(wb + off); };
  hipStream_t s = (hipStream_t)stream;
  const int C = d.C;

  mdg_gemm_desc g;
  memset(&g, 0, sizeof(g));
  g.dtype = MDG_F32;
  g.a_mode = MDG_A_PLAIN;
  g.out_f32 = 1;

  // ---- c = TimestepEmbedder(t * mult); only SiLU(c) is consumed (every adaLN Linear, and the
  //      IPA layers', is nn.Sequential(SiLU, Linear)), so mlp.2's epilogue applies the SiLU
  if (int e = hip_check(mdg::temb_freq_launch(c.R, d.freq_dim / 2, m->time_multiplier, io->t, m->t_freqs,
                                              F(c.emb), s), "temb_freq"))
    return e;
  mdg_gemm_desc t0 = g;
  t0.epi = MDG_EPI_STORE; t0.act = MDG_ACT_SILU;
  t0.M = c.R; t0.N = C; t0.K = d.freq_dim; t0.A = F(c.emb); t0.lda = d.freq_dim;
  t0.W = m->t_w0; t0.ldw = d.freq_dim; t0.bias = m->t_b0; t0.out = F(c.hmid); t0.ldo = C;
  if (int e = mdg_gemm(&t0, stream)) return e;
  mdg_gemm_desc t2 = t0;
  t2.K = C; t2.A = F(c.hmid); t2.lda = C; t2.W = m->t_w2; t2.ldw = C; t2.bias = m->t_b2; t2.out = F(c.sc);
  if (int e = mdg_gemm(&t2, stream)) return e;
  // ---- every adaLN modulation in one GEMM, rows scattered to the denoiser's layouts
  mdg_gemm_desc ad = g;
  ad.epi = MDG_EPI_STORE;
  ad.M = c.R; ad.N = c.W; ad.K = C; ad.A = F(c.sc); ad.lda = C; ad.W = m->ada_w; ad.ldw = C; ad.bias = m->ada_b;
  ad.out = F(c.all); ad.ldo = c.W;
  if (int e = mdg_gemm(&ad, stream)) return e;
  const int lanes = io->lanes > 1 ? io->lanes : 1;
  if (d.B % lanes) return fail(MDG_E_SHAPE, "precompute_cond: B=%d not a multiple of lanes=%d", d.B, lanes);
  if (int e = hip_check(mdg::cond_scatter_launch(d.S, d.B, d.num_layers, C, c.W, lanes, F(c.all), io->mods,
                                                 io->mods_final, s), "cond_scatter"))
    return e;
  if (d.ipa_layers == 0) return MDG_OK;

  // ---- IPA prepend (run_ipa, latent_model.py:179-214) on M = S*B*L residue tokens
  if (!io->ipa || !io->mask || !io->rots || !io->trans) return fail(MDG_E_ARG, "precompute_cond: IPA inputs");
  if (io->aatype && !m->aa_emb) return fail(MDG_E_ARG, "precompute_cond: aatype without aa_emb");
  if (d.tps && (!io->end_rots || !io->end_trans || !m->l2e_f_w || !m->l2e_r_w))
    return fail(MDG_E_ARG, "precompute_cond: TPS end frames / latent_to_emb_f/_r");
  const int L = d.L, M = c.M, H = d.H, D = d.D;
  const float* rel7 = io->rel7;
  if (d.tps && !rel7) {
    if (int e = hip_check(mdg::tps_rel7_launch(d.B, L, io->rots, io->trans, io->end_rots, io->end_trans, F(c.rel7), s),
                          "tps_rel7"))
      return e;
    rel7 = F(c.rel7);
  }
  const bool long_l = L >= kSpatialMfmaMinL && c.R <= 65535;
  if (int e = hip_check(hipMemsetAsync(wb + c.cat, 0, (size_t)M * c.Kpad * sizeof(float), s), "cond memset"))
    return e;
  if (long_l) {  // the q|k|v planes of the MFMA route: zero pads, 1.0 in k / v pad column D
    const size_t rows = (size_t)c.R * H * L;
    if (int e = hip_check(hipMemsetAsync(wb + c.qkv, 0, 3 * rows * dp_of(D) * sizeof(float), s), "cond memset"))
      return e;
    if (int e = hip_check(mdg::set_vpad_launch(MDG_F32, F(c.qkv) + rows * dp_of(D), 2 * rows, D, s), "set_vpad"))
      return e;
  }
  const int ipa_mod0 = d.num_layers * 9 * C + 2 * C;
  const float qs = 1.0f / sqrtf((float)D);
  for (int stack = 0; stack < (d.tps ? 2 : 1); ++stack) {
    // stack 0: x (sim) or x_r (TPS, start frames) -> io->ipa; stack 1: x_f (end frames) -> x2
    float* x = stack == 0 ? io->ipa : F(c.x2);
    const float* rots = stack == 0 ? io->rots : io->end_rots;
    const float* trans = stack == 0 ? io->trans : io->end_trans;
    const float* r7 = d.tps ? rel7 + (size_t)(stack == 0 ? 1 : 0) * d.B * L * 7 : nullptr;
    const float* lw = d.tps ? (stack == 0 ? m->l2e_r_w : m->l2e_f_w) : nullptr;
    const float* lb = d.tps ? (stack == 0 ? m->l2e_r_b : m->l2e_f_b) : nullptr;
    if (int e = hip_check(mdg::ipa_init_launch(c.R, d.B, L, C, io->mask_stride > 0 ? io->mask_stride : L, io->aatype, io->aatype ? m->aa_emb : nullptr, r7, lw, lb,
                                               io->mask, x, F(c.mrep), s), "ipa_init"))
      return e;
    if (long_l && stack == 0)
      if (int e = hip_check(mdg::mask_bias_launch(c.R, 1, L, F(c.mrep), F(c.kb_t), F(c.kb_s), s), "mask_bias"))
        return e;
    for (int li = 0; li < d.ipa_layers; ++li) {
      const mdg_ipa_layer_weights& w = m->ipa[li];
      if (!w.w_proj || !w.w_out || !w.wqkv || !w.wo || !w.w1 || !w.w2 || !w.kvb || !w.head_weights)
        return fail(MDG_E_ARG, "precompute_cond: IPA layer %d weights missing", li);
      const float* mods = F(c.all) + ipa_mod0 + li * 6 * C;  // shift_l scale_l gate_l shift_m scale_m gate_m
      // x += linear_out(IPA(ipa_norm(x)))
      mdg_gemm_desc pj = g;
      pj.a_mode = MDG_A_LNMOD; pj.epi = MDG_EPI_STORE;
      pj.M = M; pj.N = c.Ppad; pj.K = C; pj.A = x; pj.lda = C; pj.W = w.w_proj; pj.ldw = C; pj.bias = w.b_proj;
      pj.ln_w = w.ln_w; pj.ln_b = w.ln_b; pj.ln_eps = 1e-5f; pj.out = F(c.proj); pj.ldo = c.Ppad;
      if (int e = mdg_gemm(&pj, stream)) return e;
      if (int e = hip_check(mdg::ipa_attn_launch(c.R, d.B, L, d.ipa_heads, d.ipa_c, d.ipa_qk, d.ipa_v, F(c.proj), c.Ppad,
                                                 rots, trans, F(c.mrep), w.head_weights, F(c.cat), c.Kpad, s),
                            "ipa_attn"))
        return e;
      mdg_gemm_desc po = g;
      po.epi = MDG_EPI_GATE_RES;
      po.M = M; po.N = C; po.K = c.Kpad; po.A = F(c.cat); po.lda = c.Kpad; po.W = w.w_out; po.ldw = c.Kpad;
      po.bias = w.b_out; po.resid = x; po.ldr = C;
      if (int e = mdg_gemm(&po, stream)) return e;
      // x += gate_l * mha_l(modulate(LN x, shift_l, scale_l), mask)
      if (int e = hip_check(mdg::ln_mod_launch(MDG_F32, M, C, x, mods, c.W, L, 0, C, 1e-6f, F(c.xn), s), "ln_mod"))
        return e;
      mdg_gemm_desc q = g;
      q.epi = MDG_EPI_QKV;
      q.M = M; q.N = 3 * C; q.K = C; q.A = F(c.xn); q.lda = C; q.W = w.wqkv; q.ldw = C; q.bias = w.bqkv;
      q.H = H; q.D = D; q.T = 1; q.L = L; q.rope = m->rope_l; q.rope_rows = L + 1;
      if (long_l) {
        q.qkv_layout = MDG_QKV_TEMPORAL; q.qkv_out = F(c.qkv); q.qscale = qs * 1.4426950408889634f;
        q.T = L; q.L = 1;
        if (int e = mdg_gemm(&q, stream)) return e;
        if (int e = mdg_attn_temporal(MDG_F32, c.R, L, 1, H, D, F(c.qkv), F(c.kb_s), w.kvb, F(c.o), stream)) return e;
      } else {
        q.qkv_layout = MDG_QKV_SPATIAL; q.qkv_out = F(c.qkv); q.qscale = qs;
        if (int e = mdg_gemm(&q, stream)) return e;
        if (int e = mdg_attn_spatial(MDG_F32, c.R, L, H, D, F(c.qkv), w.kvb, F(c.mrep), F(c.o), stream)) return e;
      }
      mdg_gemm_desc r = g;
      r.epi = MDG_EPI_GATE_RES;
      r.M = M; r.N = C; r.K = C; r.A = F(c.o); r.lda = C; r.W = w.wo; r.ldw = C; r.bias = w.bo;
      r.resid = x; r.ldr = C; r.gate = mods; r.gate_off = 2 * C; r.mod_stride = c.W; r.rows_per_mod = L;
      if (int e = mdg_gemm(&r, stream)) return e;
      // x += gate_m * fc2(gelu(fc1(modulate(LN x, shift_m, scale_m))))
      if (int e = hip_check(mdg::ln_mod_launch(MDG_F32, M, C, x, mods, c.W, L, 3 * C, 4 * C, 1e-6f, F(c.xn), s),
                            "ln_mod"))
        return e;
      mdg_gemm_desc f1 = g;
      f1.epi = MDG_EPI_STORE; f1.act = MDG_ACT_GELU;
      f1.M = M; f1.N = 4 * C; f1.K = C; f1.A = F(c.xn); f1.lda = C; f1.W = w.w1; f1.ldw = C; f1.bias = w.b1;
      f1.out = F(c.hid); f1.ldo = 4 * C;
      if (int e = mdg_gemm(&f1, stream)) return e;
      mdg_gemm_desc f2 = r;
      f2.K = 4 * C; f2.A = F(c.hid); f2.lda = 4 * C; f2.W = w.w2; f2.ldw = 4 * C; f2.bias = w.b2; f2.gate_off = 5 * C;
      if (int e = mdg_gemm(&f2, stream)) return e;
    }
  }
  if (d.tps)  // x_r + x_f (latent_model.py:211)
    if (int e = hip_check(mdg::add_inplace_launch((size_t)M * C, io->ipa, F(c.x2), s), "ipa add")) return e;
  return MDG_OK;
}

size_t mdg_embed_bwd_workspace_bytes(int32_t B, int32_t T, int32_t L, int32_t C, int32_t K1, int32_t K2, int32_t E) {
  if (B <= 0 || T <= 0 || L <= 0 || C <= 0 || K1 <= 0 || K2 < 0 || E < 0) return 0;
  return mdg::embed_bwd_ws_bytes(B, T, L, C, K1, K2, E);
}

int mdg_embed_bwd(int32_t B, int32_t T, int32_t L, int32_t C, int32_t K1, const float* x1, int32_t K2, const float* x2,
                  const int64_t* idx, int32_t E, const float* dh, float* dw1, float* dw2, float* db, float* demb,
                  float* dipa, void* ws, size_t ws_bytes, void* stream) {
  if (!x1 || !dh || !ws) return fail(MDG_E_ARG, "embed_bwd: null x1 / dh / ws");
  if (B <= 0 || T <= 0 || L <= 0 || L > 8 || C <= 0 || C % 128 || K1 <= 0 || K1 > 32 || (x2 && (K2 <= 0 || K2 > 32)) ||
      (idx && (E <= 0 || E > 4)))
    return fail(MDG_E_SHAPE, "embed_bwd: B=%d T=%d L=%d C=%d K1=%d K2=%d E=%d (L <= 8, C %% 128, K <= 32, E <= 4)", B, T,
                L, C, K1, K2, E);
  const size_t need = mdg::embed_bwd_ws_bytes(B, T, L, C, K1, x2 ? K2 : 0, idx ? E : 0);
  if (ws_bytes < need) return fail(MDG_E_ARG, "embed_bwd: workspace %zu < %zu bytes", ws_bytes, need);
  return hip_check(mdg::embed_bwd_launch(B, T, L, C, K1, x1, x2 ? K2 : 0, x2, idx, idx ? E : 0, dh, dw1, dw2, db, demb,
                                         dipa, (float*)ws, (hipStream_t)stream),
                   "embed_bwd");
}

int mdg_final_fwd_train(int32_t N, int32_t rows_per_b, int32_t C, int32_t latent, const float* h, const float* mods,
                        const float* w, const float* bias, float* v, float* stats, void* stream) {
  if (!h || !mods || !w || !v || !stats) return fail(MDG_E_ARG, "final_fwd_train: null pointer");
  if (C != 384 || (latent != 21 && latent != 28) || N <= 0 || rows_per_b <= 0 || N % rows_per_b)
    return fail(MDG_E_SHAPE, "final_fwd_train: N=%d rows_per_b=%d C=%d latent=%d (C = 384, latent 21 / 28)", N,
                rows_per_b, C, latent);
  return hip_check(mdg::final_fwd_train_launch(N, rows_per_b, latent, h, mods, w, bias, v, stats, (hipStream_t)stream),
                   "final_fwd_train");
}

size_t mdg_final_bwd_workspace_bytes(int32_t N, int32_t rows_per_b, int32_t latent) {
  if (N <= 0 || rows_per_b <= 0 || latent <= 0) return 0;
  return mdg::final_bwd_ws_bytes(N, rows_per_b, latent);
}

int mdg_final_bwd_train(int32_t N, int32_t rows_per_b, int32_t C, int32_t latent, const float* h, const float* stats,
                        const float* mods, const float* w, const float* dv, float* dh, float* dw, float* dbias,
                        float* dmods, void* ws, size_t ws_bytes, void* stream) {
  if (!h || !stats || !mods || !w || !dv || !dh || !dw || !dmods || !ws)
    return fail(MDG_E_ARG, "final_bwd_train: null pointer");
  if (C != 384 || (latent != 21 && latent != 28) || N <= 0 || rows_per_b <= 0 || N % rows_per_b)
    return fail(MDG_E_SHAPE, "final_bwd_train: N=%d rows_per_b=%d C=%d latent=%d (C = 384, latent 21 / 28)", N,
                rows_per_b, C, latent);
  const size_t need = mdg::final_bwd_ws_bytes(N, rows_per_b, latent);
  if (ws_bytes < need) return fail(MDG_E_ARG, "final_bwd_train: workspace %zu < %zu bytes", ws_bytes, need);
  return hip_check(mdg::final_bwd_train_launch(N, rows_per_b, latent, h, stats, mods, w, dv, dh, dw, dbias, dmods,
                                               (float*)ws, (hipStream_t)stream),
                   "final_bwd_train");
}

size_t mdg_wgrad_workspace_bytes(int32_t dtype, int32_t N, int32_t M, int32_t K, int32_t need_dw, int32_t need_db) {
  if ((dtype != MDG_F32 && dtype != MDG_BF16) || N <= 0 || M <= 0 || K <= 0) return 0;
  return mdg::wgrad_ws_bytes(dtype, N, M, K, need_dw != 0, need_db != 0);
}

int mdg_wgrad(int32_t dtype, int32_t N, int32_t M, int32_t K, const void* dy, int32_t ldy, const void* x, int32_t ldx,
              float* dw, int32_t lddw, float* db, void* ws, size_t ws_bytes, void* stream) {
  if (dtype != MDG_F32 && dtype != MDG_BF16) return fail(MDG_E_DTYPE, "wgrad: dtype %d", dtype);
  if (!dy || (dw && !x) || (!dw && !db)) return fail(MDG_E_ARG, "wgrad: null dy / x / outputs");
  if (N <= 0 || M < 8 || K < 8 || M % 8 || K % 8 || ldy < M || ldy % 8 || (dw && (ldx < K || ldx % 8 || lddw < K)))
    return fail(MDG_E_SHAPE, "wgrad: N=%d M=%d K=%d ldy=%d ldx=%d lddw=%d (M, K, ld multiples of 8)", N, M, K, ldy, ldx,
                lddw);
  if (dtype == MDG_BF16 && N % 32) return fail(MDG_E_SHAPE, "wgrad bf16: N=%d not a multiple of 32 (pad with zero rows)", N);
  if (!aligned16(dy) || (dw && (!aligned16(x) || !aligned16(dw) || lddw % 4)))
    return fail(MDG_E_SHAPE, "wgrad: operands and dw must be 16-B aligned, lddw a multiple of 4");
  const size_t need = mdg::wgrad_ws_bytes(dtype, N, M, K, dw != nullptr, db != nullptr);
  if (!ws || ws_bytes < need) return fail(MDG_E_ARG, "wgrad: workspace %zu < %zu bytes", ws_bytes, need);
  return hip_check(mdg::wgrad_launch(dtype, N, M, K, dy, ldy, x, ldx, dw, lddw, db, (float*)ws, (hipStream_t)stream),
                   "wgrad");
}

int mdg_gvp_plan(int32_t B, int64_t n_per_b, int32_t path, const float* t, const float* x0, const float* x1, float* xt,
                 float* ut, void* stream) {
  if (!t || !x0 || !x1 || !xt || !ut) return fail(MDG_E_ARG, "gvp_plan: null pointer");
  if (B <= 0 || n_per_b <= 0 || (path != 0 && path != 1)) return fail(MDG_E_SHAPE, "gvp_plan: B=%d n=%lld path=%d", B, (long long)n_per_b, path);
  return hip_check(mdg::gvp_plan_launch(B, n_per_b, path, t, x0, x1, xt, ut, (hipStream_t)stream), "gvp_plan");
}

size_t mdg_gvp_loss_workspace_bytes(int32_t B, int64_t n_per_b) {
  if (B <= 0 || n_per_b <= 0) return 0;
  return mdg::gvp_loss_ws_bytes(B, n_per_b);
}

int mdg_gvp_loss_fwd(int32_t B, int32_t T, int32_t L, int32_t K, const float* out, const float* ut, const float* mask,
                     const int64_t* mask_strides, float* loss, float* den, void* ws, size_t ws_bytes, void* stream) {
  if (!out || !ut || !mask || !mask_strides || !loss || !den || !ws) return fail(MDG_E_ARG, "gvp_loss_fwd: null pointer");
  if (B <= 0 || T <= 0 || L <= 0 || K <= 0) return fail(MDG_E_SHAPE, "gvp_loss_fwd: B=%d T=%d L=%d K=%d", B, T, L, K);
  const size_t need = mdg::gvp_loss_ws_bytes(B, (long long)T * L * K);
  if (ws_bytes < need) return fail(MDG_E_ARG, "gvp_loss_fwd: workspace %zu < %zu bytes", ws_bytes, need);
  return hip_check(mdg::gvp_loss_fwd_launch(B, T, L, K, out, ut, mask, mask_strides, loss, den, (float*)ws,
                                            (hipStream_t)stream), "gvp_loss_fwd");
}

int mdg_gvp_loss_bwd(int32_t B, int32_t T, int32_t L, int32_t K, const float* out, const float* ut, const float* mask,
                     const int64_t* mask_strides, const float* gloss, const float* den, float* dout, void* stream) {
  if (!out || !ut || !mask || !mask_strides || !gloss || !den || !dout) return fail(MDG_E_ARG, "gvp_loss_bwd: null pointer");
  if (B <= 0 || T <= 0 || L <= 0 || K <= 0) return fail(MDG_E_SHAPE, "gvp_loss_bwd: B=%d T=%d L=%d K=%d", B, T, L, K);
  return hip_check(mdg::gvp_loss_bwd_launch(B, T, L, K, out, ut, mask, mask_strides, gloss, den, dout,
                                            (hipStream_t)stream), "gvp_loss_bwd");
}

int32_t mdg_adam_chunks(int32_t n_tensors, const mdg_adam_tensor* tensors) {
  if (n_tensors <= 0 || !tensors) return -1;
  return mdg::adam_chunks(n_tensors, tensors);
}

size_t mdg_adam_table_bytes(int32_t n_tensors, const mdg_adam_tensor* tensors) {
  const int nc = mdg_adam_chunks(n_tensors, tensors);
  return nc <= 0 ? 0 : mdg::adam_table_bytes(n_tensors, nc);
}

int mdg_adam_table_build(int32_t n_tensors, const mdg_adam_tensor* tensors, void* table, size_t table_bytes) {
  if (n_tensors <= 0 || !tensors || !table) return fail(MDG_E_ARG, "adam_table_build: null pointer or no tensors");
  const int nc = mdg::adam_chunks(n_tensors, tensors);
  if (nc <= 0) return fail(MDG_E_SHAPE, "adam_table_build: a tensor has no elements");
  for (int i = 0; i < n_tensors; ++i) {
    const mdg_adam_tensor& t = tensors[i];
    if (!t.p || !t.g || !t.m || !t.v || !t.step) return fail(MDG_E_ARG, "adam_table_build: tensor %d: null pointer", i);
  }
  const size_t need = mdg::adam_table_bytes(n_tensors, nc);
  if (table_bytes < need) return fail(MDG_E_ARG, "adam_table_build: table %zu < %zu bytes", table_bytes, need);
  mdg::adam_table_build(n_tensors, nc, tensors, table);
  return MDG_OK;
}

size_t mdg_adam_workspace_bytes(int32_t n_chunks) { return n_chunks <= 0 ? 0 : mdg::adam_ws_bytes(n_chunks); }

int mdg_adam_step(int32_t n_tensors, int32_t n_chunks, const void* table, double lr, double beta1, double beta2,
                  double eps, double weight_decay, int32_t decoupled, double max_norm, float* gnorm, void* ws,
                  size_t ws_bytes, void* stream) {
  if (!table || !ws) return fail(MDG_E_ARG, "adam_step: null pointer");
  if (n_tensors <= 0 || n_chunks < n_tensors) return fail(MDG_E_SHAPE, "adam_step: %d tensors, %d chunks", n_tensors, n_chunks);
  if (!(lr >= 0.0) || !(beta1 >= 0.0 && beta1 < 1.0) || !(beta2 >= 0.0 && beta2 < 1.0) || !(eps >= 0.0) ||
      !(weight_decay >= 0.0) || !std::isfinite(max_norm))
    return fail(MDG_E_ARG, "adam_step: lr %g betas (%g, %g) eps %g weight_decay %g max_norm %g", lr, beta1, beta2, eps,
                weight_decay, max_norm);
  const size_t need = mdg::adam_ws_bytes(n_chunks);
  if (ws_bytes < need) return fail(MDG_E_ARG, "adam_step: workspace %zu < %zu bytes", ws_bytes, need);
  return hip_check(mdg::adam_step_launch(n_tensors, n_chunks, table, lr, beta1, beta2, eps, weight_decay, decoupled,
                                         max_norm, gnorm, (float*)ws, (hipStream_t)stream),
                   "adam_step");
}

size_t mdg_seg_linear_bwd_workspace_bytes(int32_t M, int32_t K, const mdg_seg_linear* s) {
  const int tot = mdg::seg_total(s);
  if (M <= 0 || K <= 0 || tot <= 0) return 0;
  return mdg::seg_linear_ws_bytes(M, K, tot);
}

static int seg_check(const char* what, int32_t M, int32_t K, const float* x, int32_t ldx, int32_t in_act,
                     const mdg_seg_linear* s) {
  if (!x || !s) return fail(MDG_E_ARG, "%s: null x / segments", what);
  if (in_act != MDG_ACT_NONE && in_act != MDG_ACT_SILU) return fail(MDG_E_ARG, "%s: in_act %d", what, in_act);
  if (mdg::seg_total(s) <= 0)
    return fail(MDG_E_SHAPE, "%s: nseg %d (1..%d, every n > 0)", what, s->nseg, MDG_SEG_MAX);
  if (!mdg::seg_linear_shape_ok(M, K) || ldx < K || ldx % 4 || ((uintptr_t)x & 15))
    return fail(MDG_E_SHAPE, "%s: M=%d K=%d ldx=%d (K %% 4 == 0, K <= 1024, x 16-B aligned, ldx %% 4 == 0)", what, M,
                K, ldx);
  for (int i = 0; i < s->nseg; ++i)
    if ((uintptr_t)s->w[i] & 15) return fail(MDG_E_SHAPE, "%s: weight %d not 16-B aligned", what, i);
  for (int i = 0; i < s->nseg; ++i)
    if (!s->w[i]) return fail(MDG_E_ARG, "%s: null weight of segment %d", what, i);
  return MDG_OK;
}

int mdg_seg_linear_fwd(int32_t M, int32_t K, const float* x, int32_t ldx, int32_t in_act, const mdg_seg_linear* s,
                       void* stream) {
  if (int e = seg_check("seg_linear_fwd", M, K, x, ldx, in_act, s)) return e;
  for (int i = 0; i < s->nseg; ++i)
    if (!s->y[i] || s->ldy[i] < s->n[i] || (s->resid[i] && s->ldr[i] < s->n[i]))
      return fail(MDG_E_ARG, "seg_linear_fwd: segment %d output null or ld < n", i);
  return hip_check(mdg::seg_linear_fwd_launch(M, K, x, ldx, in_act, s, (hipStream_t)stream), "seg_linear_fwd");
}

int mdg_seg_linear_bwd(int32_t M, int32_t K, const float* x, int32_t ldx, int32_t in_act, const mdg_seg_linear* s,
                       float* dx, int32_t lddx, void* ws, size_t ws_bytes, void* stream) {
  if (int e = seg_check("seg_linear_bwd", M, K, x, ldx, in_act, s)) return e;
  for (int i = 0; i < s->nseg; ++i)
    if (!s->dy[i] || s->lddy[i] < s->n[i]) return fail(MDG_E_ARG, "seg_linear_bwd: segment %d dy null or ld < n", i);
  if (dx && lddx < K) return fail(MDG_E_SHAPE, "seg_linear_bwd: lddx %d < K %d", lddx, K);
  const size_t need = dx ? mdg::seg_linear_ws_bytes(M, K, mdg::seg_total(s)) : 0;
  if (need && (!ws || ws_bytes < need)) return fail(MDG_E_ARG, "seg_linear_bwd: workspace %zu < %zu bytes", ws_bytes, need);
  return hip_check(mdg::seg_linear_bwd_launch(M, K, x, ldx, in_act, s, dx, lddx, (float*)ws, (hipStream_t)stream),
                   "seg_linear_bwd");
}

}  // extern "C"

#ifdef MDG_DIAGNOSTICS
// ---- diagnostics (not part of the ABI in include/mdgen_hip.h; tools/lane_snap.py)
extern "C" int mdg_debug_snapshots(void* dst, size_t cap) {
  g_snap.dst = (char*)dst;
  g_snap.cap = dst ? cap : 0;
  g_snap.used = 0;
  g_snap.label.clear();
  g_snap.off.clear();
  g_snap.ws.clear();
  return 0;
}
// i < 0: the number of snapshots taken; else slot i's byte offset, workspace and label
extern "C" int mdg_debug_snapshot_info(int i, size_t* off, void** ws, char* label, size_t n) {
  if (i < 0) return (int)g_snap.off.size();
  if (i >= (int)g_snap.off.size()) return -1;
  *off = g_snap.off[i];
  *ws = (void*)g_snap.ws[i];
  snprintf(label, n, "%s", g_snap.label[i].c_str());
  return 0;
}
#endif  // MDG_DIAGNOSTICS
