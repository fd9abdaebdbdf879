/*
 * mdgen_hip.h — C ABI of libmdgen_hip.so, the MI355X (gfx950) denoising hot path of MDGen.
 *
 * Replaces, on the device, the reference's eager-PyTorch forward of one flow-matching
 * denoising step and the Euler update around it:
 *   LatentMDGenModel.forward        src/mdgen/model/latent_model.py:216-269
 *   LatentMDGenLayer.forward        src/mdgen/model/latent_model.py:456-493
 *   AttentionWithRoPE / MultiheadAttention (rope + bias_kv path)
 *                                   latent_model.py:329-338, src/mdgen/model/mha.py:161-407
 *   FinalLayer                      src/mdgen/model/layers.py:58-75
 *   torchdiffeq Euler step used by Sampler.sample_ode('euler')
 *                                   src/mdgen/transport/integrators.py:95-114
 * The reference is pure Python, so there is no reference FFI to mirror; the Python-side
 * drop-in (mdgen_finetune_amd.model.latent_model.LatentMDGenModel.forward and
 * mdgen_finetune_amd.transport.Sampler.sample_ode) binds these entry points with ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Contract (every entry point):
 *   - all tensor arguments are CALLER-OWNED DEVICE pointers, contiguous row-major;
 *   - `stream` is a hipStream_t (passed as void*); calls are asynchronous and stream-ordered;
 *   - no allocation, no host synchronisation, no globals: calls are reentrant and
 *     hipGraph-capturable;
 *   - return 0 on success, else an MDG_E_* code or a hipError_t (launch failure);
 *     mdg_last_error_string() (thread-local) describes the last failure.
 * Token order is n = (b*T + t)*L + l (the reference's [B,T,L,C] layout flattened).
 */
#ifndef MDGEN_HIP_H
#define MDGEN_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDG_ABI_VERSION 24
#define MDG_MAX_LAYERS 16
#define MDG_SEG_MAX 16 /* segments of one mdg_seg_linear */
#define MDG_DP 32      /* padded head dim of the attention operand buffers for head_dim <= 31 */
#define MDG_DP_WIDE 64 /* ... and for 32 <= head_dim <= 63 (column head_dim of the padded k / v rows
                          carries the softmax offset / row sum, so it must exist) */
#define MDG_HEAD_STRIDE(D) ((D) < MDG_DP ? MDG_DP : MDG_DP_WIDE)

typedef enum { MDG_F32 = 0, MDG_BF16 = 1 } mdg_dtype;

enum {
  MDG_OK = 0,
  MDG_E_SHAPE = 1001, /* unsupported / inconsistent dimensions */
  MDG_E_DTYPE = 1002, /* unknown dtype enum */
  MDG_E_ARG = 1003,   /* null pointer or bad enum */
};

/* GEMM building block: out = epilogue( prologue(A) . W^T + bias ) */
enum { MDG_A_PLAIN = 0, MDG_A_LNMOD = 1 };
enum { MDG_EPI_STORE = 0, MDG_EPI_GATE_RES = 1, MDG_EPI_QKV = 2, MDG_EPI_EULER = 3, MDG_EPI_ATTN_SPATIAL = 4 };
enum { MDG_ACT_NONE = 0, MDG_ACT_GELU = 1, MDG_ACT_SILU = 2, MDG_ACT_DGELU = 3 };
enum { MDG_QKV_SPATIAL = 0, MDG_QKV_TEMPORAL = 1, MDG_QKV_TEMPORAL_PACKED = 2 };

typedef struct {
  int32_t B, T, L;    /* batch, frames (num_frames), residues (crop) */
  int32_t C, H, D, F; /* embed_dim, mha_heads, head_dim = C/H, ffn dim (4C) */
  int32_t latent;     /* latent channels: 21 (sim), 28 (tps) */
  int32_t num_layers;
  int32_t dtype;      /* mdg_dtype of the packed GEMM / attention operands */
} mdg_dims;

typedef struct {
  const void* wqkv[2];  /* CT [3C][C], rows q|k|v (nn.Linear layout); [0]=mha_l, [1]=mha_t.
                           With RoPE, each q and k head's D rows are PAIR-INTERLEAVED:
                           row 2i = dim i, row 2i+1 = dim i + D/2 (v rows natural). */
  const float* bqkv[2]; /* [3C], same row order */
  const void* wo[2];    /* CT [C][C] out_proj */
  const float* bo[2];   /* [C] */
  const float* kvb[2];  /* [H][2][MDG_HEAD_STRIDE(D)]: bias_k RoPE-rotated at position S (=L or T) in the
                           interleaved order, bias_v natural order with bias_v[D] = 1 (the
                           softmax row sum rides in the pad column) */
  const void* w1;       /* CT [F][C] fc1 */
  const float* b1;      /* [F] */
  const void* w2;       /* CT [C][F] fc2 */
  const float* b2;      /* [C] */
} mdg_layer_weights;

typedef struct {
  mdg_dims dims;
  const float* w_l2e_t; /* latent_to_emb.weight TRANSPOSED: [latent][C] fp32 */
  const void* w_final;  /* emb_to_latent.linear.weight, CT [round_up(latent,32)][C], pad rows 0 */
  const float* b_final; /* [round_up(latent,32)], pad 0 */
  const float* rope_l;  /* [L+1][D/2] cos, then [L+1][D/2] sin (spatial) */
  const float* rope_t;  /* [T+1][D/2] cos, then [T+1][D/2] sin (temporal) */
  mdg_layer_weights layers[MDG_MAX_LAYERS];
} mdg_model;

typedef struct {
  const float* x_in;       /* [N][latent] noisy latents x_t */
  float* x_out;            /* [N][latent] x_t + dt * v (may alias x_in); null = skip */
  float* v_out;            /* [N][latent] velocity v; null = skip */
  const float* base;       /* [N][C] step-invariant embedding (cond_to_emb + mask_to_emb +
                              pos_embed + biases), from mdg_embed once per window */
  const float* ipa;        /* [B][L][C] IPA prepend for this step's t (null = none) */
  const float* mods;       /* [num_layers][B][9C] adaLN chunks for this step's t */
  const float* mods_final; /* [B][2C] FinalLayer adaLN (shift, scale) */
  float dt;                /* t_{i+1} - t_i */
  float* h;                /* [N][C] fp32 residual-stream scratch */
  int32_t chain_alone;     /* 1: this step is the only chain on the device (no concurrent lane);
                              small-M launches may then split the out_proj row-LN GEMM over K
                              (fp32 partials + a reduction pass), which pays only when the other
                              CUs are idle.  0: the lane-invariant routes only. */
} mdg_step_io;

typedef struct {
  int32_t dtype, a_mode, epi, act;
  int32_t M, N, K;
  const void* A; int32_t lda; /* PLAIN: CT [M][lda]; LNMOD: fp32 [M][lda], K == row length */
  const void* W; int32_t ldw; /* CT [N][ldw] */
  const float* bias;          /* [N] or null */
  /* LNMOD prologue: y = LN(a; eps) (*ln_w + ln_b); y = y*(1+scale) + shift with
     shift = mods[(m / rows_per_mod)*mod_stride + shift_off + k] (mods may be null) */
  const float* mods; int32_t mod_stride, rows_per_mod, shift_off, scale_off;
  const float* ln_w; const float* ln_b; float ln_eps;
  /* STORE */
  void* out; int32_t ldo, out_f32;
  /* GATE_RES: resid[m][n] += gate[(m/rows_per_mod)*mod_stride + gate_off + n] * v
     (gate null: += v) */
  float* resid; int32_t ldr; const float* gate; int32_t gate_off;
  /* QKV: N == 3*H*D; q scaled by qscale; RoPE on q,k at pos l (spatial) or t (temporal).
     TEMPORAL: [3][B*L][H][T][MDG_HEAD_STRIDE(D)] planes (pad columns left as they are);
     TEMPORAL_PACKED (D % 8 == 0, D < 32): the same planes with row stride D (no pad columns in
     memory: the attention synthesises them), read by mdg_attn_temporal_packed. */
  int32_t qkv_layout; void* qkv_out; int32_t H, D, T, L; float qscale;
  const float* rope; int32_t rope_rows; /* cos [rope_rows][D/2] then sin; null = no RoPE */
  /* EULER: x_out (= out, row stride ldo) = x_in + dt * v, v_out = v, for columns < n_valid */
  const float* x_in; float* v_out; float dt; int32_t n_valid;
  /* GATE_RES + LayerNorm (optional, bf16, N in {128, 256, 384, 512}): with xn_out set, the
     updated residual rows are also normalised (no-affine LN, eps ln_eps) and modulated for
     the NEXT projection: xn_out[m][n] = CT(LN(resid[m])[n] * (1 + xs) + xh) with
     xh = xn_mods[(m/rows_per_mod)*xn_mod_stride + xn_shift_off + n], xs likewise. */
  void* xn_out; const float* xn_mods; int32_t xn_mod_stride, xn_shift_off, xn_scale_off;
  /* ATTN_SPATIAL (bf16, PLAIN, L == 4, D == 24, H even, N == 3*H*D, M % 4 == 0): the spatial
     q|k|v projection (W, bias packed as for QKV; qscale; rope = the spatial table, rope_rows
     >= L) fused with the 4-residue attention of each frame (latent_model.py:466-470,
     mha.py:255-397): out (CT [M][ldo], ldo >= H*D) = softmax over the bias key (kvb, as in
     mdg_layer_weights) and the frame's residues with key_mask != 0 (null = all) of q.k, times
     v.  q|k|v are never written. */
  const float* kvb; const float* key_mask;
  /* Training extensions (null / 0 = off; any of them selects the non-fused tile kernels):
     resid_in  GATE_RES reads the residual from resid_in [M][ldr] and writes resid (out of place);
     aux       STORE with act GELU: also stores CT(pre-activation) to aux [M][ldaux] (saved for
               the backward); STORE with act DGELU: out = acc * gelu'(aux) (aux = the forward's
               pre-activation, read); GATE_RES: also stores CT(acc + bias), the pre-gate value.
     ln_stats  GATE_RES + LayerNorm (xn_out set): also stores each row's (mean, rstd) as fp32
               [M][2] (ABI 22; bf16, N 384, with resid_in and aux: the training forward's row-LN
               route, one launch instead of the GEMM + mdg_ln_mod pass). */
  const float* resid_in; void* aux; int32_t ldaux;
  float* ln_stats;
} mdg_gemm_desc;

int mdg_abi_version(void);
const char* mdg_last_error_string(void);

/* Device timestamps (ABI 24; no reference counterpart: instrumentation of the data-parallel
   training step, train.GraphedStep's DP markers).  mdg_stamp enqueues one single-thread kernel
   that writes the GPU's constant-rate wall clock to dst[slot] when the stream reaches it (graph-
   capturable: the markers live inside the captured step); mdg_wall_clock_khz gives that clock's
   rate for the current device. */
int mdg_stamp(uint64_t* dst, int32_t slot, void* stream);
int mdg_wall_clock_khz(int32_t* khz);

/* Workspace (attention operand buffers, hidden activations, key-padding bias). */
size_t mdg_workspace_bytes(const mdg_dims* d);
/* Byte offsets of the workspace regions, in this order: qkv_s (spatial q|k|v), qkv_t
   (temporal q|k|v planes), o (attention output), hid (MLP hidden), xn (LayerNorm+modulate
   output), kbias (temporal key-padding bias).  For profiling / tests; 0 on success. */
int mdg_workspace_offsets(const mdg_dims* d, size_t offsets[6]);
int mdg_workspace_init(const mdg_dims* d, void* ws, void* stream);
/* key-padding additive biases from mask [B,T,L] (0 -> -inf): the temporal one ([B*L][T],
   region kbias) and the spatial one ([B*T][L], after kbias; used when L >= 16, where the
   spatial attention runs on the MFMA temporal kernel with one sequence per frame) */
int mdg_prepare_mask(const mdg_dims* d, const float* mask, void* ws, void* stream);

/* out[n][c] = sum_j x[n][j] Wt[j][c] + bias[c] + base[n][c] + pos[l][c]
               + emb[idx[n]][c] + ipa[b*L + l][c]   (every term but x.Wt optional;
               Wt is the nn.Linear weight transposed, [K][C], so channel reads coalesce)
   latent_to_emb / cond_to_emb + mask_to_emb + pos_embed (latent_model.py:242-250).
   K <= 32, C % 4 == 0, C <= 512. */
int mdg_embed(int32_t N, int32_t T, int32_t L, int32_t C, int32_t K, const float* x,
              const float* Wt, const float* bias, const float* base, const float* pos,
              const float* emb, const int64_t* idx, const float* ipa, float* out, void* stream);

/* One LatentMDGenLayer (latent_model.py:456-493) on the residual h [N][C], in place. */
int mdg_layer_fwd(const mdg_dims* d, const mdg_layer_weights* w, const float* rope_l,
                  const float* rope_t, const float* mods, const float* mask, float* h, void* ws,
                  void* stream);

/* FinalLayer (layers.py:58-75) + Euler update (integrators.py:106-113) as one LN-prologue
   GEMM; w_final / b_final padded as in mdg_model.  dtype selects the operand type. */
int mdg_final_euler(int32_t dtype, int32_t N, int32_t rows_per_b, int32_t C, int32_t latent,
                    const void* w_final, const float* b_final, const float* mods_final,
                    const float* h, const float* x_in, float dt, float* x_out, float* v_out,
                    void* stream);

/* Whole denoising step: embed -> num_layers x layer -> FinalLayer -> Euler. */
int mdg_denoise_step(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws,
                     void* stream);
/* The same step in pieces: layers [first_layer, last_layer); first_layer == 0 includes the
   embedding, last_layer == num_layers the FinalLayer + Euler update.  Calls covering
   [0, k) then [k, num_layers) on one stream equal mdg_denoise_step bit for bit; the split
   lets a caller record an event mid-step (the engine offsets concurrent lanes by it). */
int mdg_denoise_step_layers(const mdg_model* m, const mdg_step_io* io, const float* mask, void* ws,
                            int32_t first_layer, int32_t last_layer, void* stream);

/* JSON text naming the kernel path each part of a denoising step takes for these dims (the
   fused / fallback routes chosen in mdg_denoise_step), for benchmark records.  0 on success. */
int mdg_describe_plan(const mdg_dims* d, char* buf, size_t n);

/* Building blocks (exposed for unit tests and for the conditioning precompute). */
int mdg_gemm(const mdg_gemm_desc* g, void* stream);
/* The block's MLP as ONE kernel (latent_model.py:488-491): fc1 = PLAIN STORE + GELU (its out is
   not written: the hidden activation stays on chip), fc2 = PLAIN GATE_RES (+ the LayerNorm
   hand-off; its A is not read), the descriptors exactly as for mdg_gemm(fc1) then
   mdg_gemm(fc2).  bf16, C == fc1.K == fc2.N == 384, F == fc1.N == fc2.K a multiple of 128,
   fc2.rows_per_mod >= 128, no training outputs; MDG_E_SHAPE otherwise. */
int mdg_mlp_fused(const mdg_gemm_desc* fc1, const mdg_gemm_desc* fc2, void* stream);
/* The spatial attention's out_proj + gated residual + temporal LayerNorm and the temporal
   q|k|v projection as ONE kernel (latent_model.py:471-477): out_proj = PLAIN GATE_RES with
   the LN hand-off (xn_out is NOT written: LN_t(h) stays on chip), qkv = the QKV epilogue into
   MDG_QKV_TEMPORAL_PACKED planes (its A is not read), the descriptors exactly as for
   mdg_gemm(out_proj) then mdg_gemm(qkv).  bf16, C == 384, head_dim % 8 == 0 and <= 48,
   out_proj.rows_per_mod >= 128, no training outputs; MDG_E_SHAPE otherwise. */
int mdg_rowln_qkv(const mdg_gemm_desc* out_proj, const mdg_gemm_desc* qkv, void* stream);
/* The temporal attention's out_proj + gated residual + the MLP LayerNorm, then the MLP, as ONE
   kernel (latent_model.py:486-491; round 5): the descriptors exactly as for mdg_gemm(out_proj)
   then mdg_mlp_fused(fc1, fc2), with out_proj.xn_out == fc1.A and out_proj.resid == fc2.resid
   (h and xn are written and read back by the same block).  h and xn equal the three-descriptor
   form bit for bit.  bf16, C == 384, out_proj.K == 384, >= 64 row tiles of 128 (the one-pass
   MLP), out_proj.rows_per_mod == fc2.rows_per_mod >= 128; MDG_E_SHAPE otherwise. */
int mdg_rowln_mlp(const mdg_gemm_desc* out_proj, const mdg_gemm_desc* fc1, const mdg_gemm_desc* fc2, void* stream);
/* qkv: CT [n_frames*L][3][H][D] (unpadded q | k | v rows of each token) */
int mdg_attn_spatial(int32_t dtype, int32_t n_frames, int32_t L, int32_t H, int32_t D,
                     const void* qkv, const float* kvb, const float* mask, void* out,
                     void* stream);
/* qkv_t: CT [3][B*L][H][T][MDG_HEAD_STRIDE(D)] (q | k | v planes), head dim in columns < D,
   k and v rows with 1.0 in pad column D (mdg_workspace_init sets it), other pad columns 0.
   head_dim <= 31 runs the 32x32x16 bf16 kernel; 32..63 the generic 16x16 MFMA kernel. */
int mdg_attn_temporal(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D,
                      const void* qkv_t, const float* kbias, const float* kvb, void* out,
                      void* stream);
/* The same attention on PACKED planes (CT [3][B*L][H][T][D], row stride D; bf16, D % 8 == 0,
   D < 32): the k / v pad column D (softmax offset, row sum) is synthesised while staging, so
   the planes carry only the head dim (24 of 32 columns for the default model). */
int mdg_attn_temporal_packed(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D,
                             const void* qkv_t, const float* kbias, const float* kvb, void* out,
                             void* stream);
/* The same, also writing lse [B*L][H][T] = log2 of each query row's softmax normaliser in the
   planes' score units (the training backward recomputes P from it), and (bf16, optional) out_lo
   CT [N][C] = O - bf16(O), the rounding residual of out, so the backward's delta = dO . O is
   accurate where the bias key dominates a row (null = skip). */
int mdg_attn_temporal_lse(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D,
                          const void* qkv_t, const float* kbias, const float* kvb, void* out, void* out_lo,
                          float* lse, void* stream);

/* Batch preparation (NewMDGenWrapper.prep_batch, wrapper.py:283-365 with get_offsets,
   utils.py:7-14, and rot_to_quat, rigid_utils.py:191-210), per token (b, t, l):
     latents[n] = [ q, t of frame0^-1 . frame(n) (q sign-fixed to real part >= 0)
                    | TPS: the same relative to frame T-1 | torsions[n] (7 x (cos, sin)) ]
     x_cond[n]  = latents[n] where the token's frame is conditioned, else 0 (null = skip)
     cond_mask[n] = 1 / 0 (int64, null = skip)
   rots [B,T,L,3,3], trans [B,T,L,3], torsions [B,T,L,7,2] (null = zeros) fp32;
   latent must be 21 (sim) or 28 (MDG_PREP_TPS).  cond_interval > 0 also conditions every
   cond_interval-th frame (--cond_interval). */
enum {
  MDG_PREP_TPS = 1,          /* --tps_condition: offsets to the last frame appended */
  MDG_PREP_NO_OFFSETS = 2,   /* --no_offsets: absolute 7-vector instead of offsets to frame 0 */
  MDG_PREP_COND_FIRST = 4,   /* condition frame 0 (--sim_condition, --tps_condition) */
  MDG_PREP_COND_LAST = 8,    /* condition frame T-1 (--tps_condition) */
};
int mdg_prep_latents(int32_t B, int32_t T, int32_t L, int32_t latent, int32_t flags, int32_t cond_interval,
                     const float* rots, const float* trans, const float* torsions, float* latents,
                     float* x_cond, int64_t* cond_mask, void* stream);

/* Denoised latents -> atom14 coordinates (NewMDGenWrapper.inference, wrapper.py:480-505, with
   frames_torsions_to_atom14, geometry.py:62-81 / 218-317), per token n = (b, t, l):
     frame  = ref[b, l] o (normalised quaternion, translation) of samples[n][0:7]
     alpha  = samples[n][tors_off .. tors_off+14) as 7 (sin, cos) pairs (unit-normalised if renorm)
     atom14[n][a] = frame . group_frame(aatype, alpha)[group(a)] . lit(aatype, a)  (0 if absent)
   samples [B,T,L,latent] fp32; ref_rots [B,L,3,3], ref_trans [B,L,3]; aatype [B,T,L] int64;
   tables (residue_constants.npz, device copies): default_frames [21][8][4][4] f32,
   group_idx [21][14] int32, atom_mask [21][14] f32, lit [21][14][3] f32.
   out: atom14 [B,T,L,14,3]; out_rots [B,T,L,3,3] / out_trans [B,T,L,3] (null = skip). */
int mdg_latents_to_atom14(int32_t B, int32_t T, int32_t L, int32_t latent, int32_t tors_off, int32_t renorm,
                          const float* samples, const float* ref_rots, const float* ref_trans,
                          const int64_t* aatype, const float* default_frames, const int32_t* group_idx,
                          const float* atom_mask, const float* lit, float* atom14, float* out_rots,
                          float* out_trans, void* stream);


/* ---------------------------------------------------------------------------------------
   Conditioning precompute (x-independent, once per rollout window for all S time points):
     c        = TimestepEmbedder(t * time_multiplier)            layers.py:17-55, latent_model.py:252
     mods     = adaLN_modulation(c) of every LatentMDGenLayer     latent_model.py:459-461
     mods_fin = FinalLayer.adaLN_modulation(c)                    layers.py:72
     ipa      = run_ipa(c, mask[:, 0], start/end frames, aatype)  latent_model.py:179-214, 341-394
                (IPALayer: affine LN -> InvariantPointAttention ipa.py:92-255 -> gated MHA over the
                 L residues with RoPE + bias_kv -> gated MLP); TPS: two IPA stacks on the relative
                 frames start^-1 o end / end^-1 o start (rigid_utils.py Rigid.invert/compose/
                 to_tensor_7), summed.
   Everything runs in fp32 (exact-f32 MFMA / VALU), whatever the denoiser's operand type.
   Rows r = s*B + b.  Weights are fp32 (nn.Linear layout unless stated). */
typedef struct {
  int32_t S, B, L;          /* time points, trajectories, residues */
  int32_t C, H, D;          /* embed_dim, mha_heads, head_dim (the IPA layers' MHA) */
  int32_t num_layers;       /* LatentMDGenLayers (adaLN 9C rows each) */
  int32_t ipa_layers;       /* IPALayers (0 = no IPA prepend) */
  int32_t ipa_heads, ipa_c, ipa_qk, ipa_v; /* InvariantPointAttention no_heads, c_hidden, P_q, P_v */
  int32_t tps;              /* 1: TPS branch (two IPA stacks on relative frames) */
  int32_t freq_dim;         /* TimestepEmbedder frequency_embedding_size (256) */
} mdg_cond_dims;

typedef struct {
  const float* ln_w; const float* ln_b; /* ipa_norm (affine LayerNorm, eps 1e-5) [C] */
  const float* w_proj; const float* b_proj; /* [P_pad][C], [P_pad]: rows linear_q (H*c) | linear_kv
                                               (H*2c) | linear_q_points (3*H*P_q) | linear_kv_points
                                               (3*H*(P_q+P_v)), zero rows up to P_pad = round_up(P, 32) */
  const float* head_weights; /* raw ipa.head_weights [H] (softplus applied on the device) */
  const float* w_out; const float* b_out; /* linear_out [C][K_pad], K = H*(c + 4*P_v) zero-padded to 64k */
  const float* wqkv; const float* bqkv;   /* mha_l q|k|v [3C][C] / [3C] packed as mdg_layer_weights */
  const float* kvb;                        /* [H][2][MDG_HEAD_STRIDE(D)] as mdg_layer_weights (position L) */
  const float* wo; const float* bo;        /* out_proj */
  const float* w1; const float* b1; const float* w2; const float* b2; /* fc1 [4C][C], fc2 [C][4C] */
} mdg_ipa_layer_weights;

typedef struct {
  mdg_cond_dims dims;
  float time_multiplier;
  const float* t_freqs;                   /* [freq_dim/2] exp(-ln(1e4) i / half) */
  const float* t_w0; const float* t_b0;   /* t_embedder.mlp.0 [C][freq_dim] */
  const float* t_w2; const float* t_b2;   /* t_embedder.mlp.2 [C][C] */
  const float* ada_w; const float* ada_b; /* every adaLN Linear stacked: rows num_layers*9C (layers) |
                                             2C (FinalLayer) | ipa_layers*6C (IPA layers), [.][C] */
  const float* aa_emb;                    /* aatype_to_emb [21][C] (null = no aa embedding) */
  const float* l2e_f_w; const float* l2e_f_b; /* TPS latent_to_emb_f [C][7], [C] */
  const float* l2e_r_w; const float* l2e_r_b; /* TPS latent_to_emb_r */
  const float* rope_l;                    /* [L+1][D/2] cos | sin (null = no RoPE) */
  mdg_ipa_layer_weights ipa[MDG_MAX_LAYERS];
} mdg_cond_model;

typedef struct {
  const float* t;          /* [S*B] raw t (time_multiplier applied here) */
  const float* mask;       /* frame mask (the reference's mask[:, 0]): mask[b*mask_stride + l] */
  int32_t mask_stride;     /* elements between trajectories' mask rows (0 = L; T*L for a [B,T,L]
                              mask, whose frame-0 rows are then read in place) */
  const float* rots; const float* trans;         /* start frames [B][L][3][3], [B][L][3] */
  const float* end_rots; const float* end_trans; /* TPS end frames */
  const float* rel7;       /* TPS: [2][B][L][7] (start^-1 o end | end^-1 o start) 7-vectors; null =
                              computed on the device (mdg_tps_rel7) */
  const int64_t* aatype;   /* [B][L] in [0, 21) or null */
  int32_t lanes;           /* 0 / 1: mods [S][num_layers][B][9C]; n > 1 (B % n == 0): lane-major
                              [n][S][num_layers][B/n][9C], each lane's step rows contiguous (the
                              engine's concurrent sub-batch chains) */
  float* mods;             /* out, layout above */
  float* mods_final;       /* out [S][B][2C] */
  float* ipa;              /* out [S][B][L][C] (ignored when ipa_layers == 0) */
} mdg_cond_io;

size_t mdg_cond_workspace_bytes(const mdg_cond_dims* d);
int mdg_precompute_cond(const mdg_cond_model* m, const mdg_cond_io* io, void* ws, void* stream);

/* TPS relative 7-vectors on the device, per residue (b, l): out[0] = start^-1 o end, out[1] =
   end^-1 o start, each [quaternion (w,x,y,z) | translation] (Rigid.invert().compose().
   to_tensor_7(), latent_model.py:197-199).  The quaternion is the dominant eigenvector of
   rot_to_quat's K matrix (rigid_utils.py:191-210); LAPACK leaves its sign arbitrary, here it is
   fixed to w >= 0.  out [2][B][L][7]. */
int mdg_tps_rel7(int32_t B, int32_t L, const float* rots, const float* trans, const float* end_rots,
                 const float* end_trans, float* out, void* stream);

/* ---------------------------------------------------------------------------------------
   Training (Transport.training_losses -> model forward -> loss.backward(): transport.py:137-222,
   wrapper.py:367-403; the block latent_model.py:456-493 under autograd).  The forward of one
   LatentMDGenLayer runs here and keeps what its backward needs; the backward runs as the
   kernels below plus the weight / input-gradient GEMMs (mdg_gemm with DGELU for fc1's input
   gradient; the weight-gradient GEMMs dW = dY^T X are plain library GEMMs on the host side).
   Every buffer is caller-owned. */
typedef struct {
  void* xn[3];       /* CT [N][C]: LN + modulate outputs feeding the spatial q|k|v, temporal
                        q|k|v and fc1 GEMMs */
  float* stats[3];   /* [N][2] (mean, rstd) of those three LayerNorms */
  void* qkv_s;       /* L < 16: CT [N][3C] spatial q|k|v (q scaled, q / k RoPE-rotated, packed
                        order); L >= 16: CT [3][B*T][H][L][DP] planes (k, v pad column D = 1;
                        DP = MDG_HEAD_STRIDE(D) here and below) */
  float* lse_s;      /* L >= 16: [B*T][H][L] log2-sum-exp2 of the spatial softmax rows */
  void* qkv_t;       /* CT [3][B*L][H][T][DP] temporal q|k|v planes (k, v pad column D = 1) */
  float* lse_t;      /* [B*L][H][T] */
  void* o[2];        /* CT [N][C] attention outputs: spatial, temporal */
  void* o_lo[2];     /* bf16 only (else null): CT [N][C] rounding residuals O - bf16(O) of the
                        attentions that run on the temporal kernel (temporal; spatial for L >= 16),
                        null = skip (the backward then takes delta from o alone) */
  void* y[3];        /* CT [N][C] pre-gate projection outputs: spatial out_proj, temporal
                        out_proj, fc2 */
  float* h1;         /* fp32 [N][C] residual after the spatial sublayer */
  float* h2;         /* fp32 [N][C] residual after the temporal sublayer */
  void* u;           /* CT [N][F] fc1 pre-activation */
  void* act;         /* CT [N][F] gelu(u), fc2's input */
  int32_t init_planes; /* nonzero: zero the plane buffers and set their pad columns first
                          (fresh allocations); 0: the pads are already in place */
  int32_t skip_temporal; /* nonzero: the temporal sublayer is left out (h2 = h1; the IPA layers'
                            MHA + MLP tail on this block, latent_model.py:341-394, whose temporal
                            gate is 0): qkv_t / lse_t / o[1] / y[1] / h2 are not written */
  /* Layer-to-layer LayerNorm hand-off (ABI 22): */
  int32_t xn0_given;     /* nonzero: xn[0] / stats[0] already hold LN_s(h_in) (the previous layer's
                            fc2 produced them); the first LayerNorm pass is skipped */
  void* xn_next;         /* non-null: also write the NEXT layer's LN_s(h_out) modulated by mods_next
                            (shift at 0, scale at C of its [B][9C] rows) to xn_next (CT [N][C]) and its
                            row statistics to stats_next ([N][2]) — fused into fc2's row-LN epilogue
                            where the bf16 row-LN GEMM takes the shape */
  float* stats_next;
  const float* mods_next;
} mdg_layer_saved;

/* Key-padding biases from mask [B,T,L] (0 -> -inf): temporal [B*L][T], spatial [B*T][L]. */
int mdg_mask_bias(int32_t B, int32_t T, int32_t L, const float* mask, float* kbias_t, float* kbias_s,
                  void* stream);

/* One LatentMDGenLayer forward for training: h_out = layer(h_in) (both fp32 [N][C], distinct),
   mods = this layer's adaLN rows [B][9C]; everything the backward needs is written to *sv.
   mask [B,T,L] (spatial key validity for L < 16), kbias_t / kbias_s from mdg_mask_bias. */
int mdg_layer_fwd_train(const mdg_dims* d, const mdg_layer_weights* w, const float* rope_l, const float* rope_t,
                        const float* mods, const float* mask, const float* kbias_t, const float* kbias_s,
                        const float* h_in, float* h_out, const mdg_layer_saved* sv, void* stream);

/* Row blocks per trajectory of mdg_ln_gate_bwd's partial sums. */
int32_t mdg_ln_gate_bwd_blocks(int32_t rows_per_b);
/* Backward of  xn = LN(h_ln)*(1 + scale) + shift  (no-affine LN, stats from the forward) and of
   the gated residual  h = h_prev + gate * y  of the sublayer below, per row m (b = m / rows_per_b):
     dh_out = dh_res + LN_bwd(dxn)                      (dxn null: dh_out = dh_res)
     dy     = CT(dh_out * gate[b])                      (y null: skipped)
   part [B][blocks][4][C] (fp32): per row block the column sums of dxn (d shift), dxn * xhat
   (d scale), dh_out * y (d gate) and dh_out * gate (the projection's bias gradient).
   mods rows [B][mod_stride]: shift at shift_off, scale at scale_off, gate at gate_off.
   dh_out may alias dh_res. */
int mdg_ln_gate_bwd(int32_t dtype, int32_t M, int32_t C, int32_t rows_per_b, const void* dxn, const float* h_ln,
                    const float* stats, const float* mods, int32_t mod_stride, int32_t shift_off, int32_t scale_off,
                    const float* dh_res, float* dh_out, const void* y, int32_t gate_off, void* dy, float* part,
                    void* stream);

/* Bias-key gradient partial slots per head of the attention backward kernels below (every slot
   is written; generic as passed to mdg_attn_temporal_bwd: the fused bf16 kernel writes one per
   sequence, ABI 21). */
int32_t mdg_attn_temporal_bwd_parts(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t generic);
int32_t mdg_attn_spatial_bwd_parts(int32_t n_frames, int32_t L, int32_t H, int32_t D);  /* (ABI 23: takes H) */
/* Scratch of mdg_attn_temporal_bwd: dO planes CT [B*L][H][T][DP], delta fp32 [B*L][H][T], and
   for bf16 with T > 256 and head_dim < 32 the fused kernel's fp32 dQ accumulator [B*L][H][T][32].
   ABI 23: takes head_dim D (the wide heads' 64-column planes); 0 for D outside 1..63. */
size_t mdg_attn_temporal_bwd_scratch(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D);
/* Temporal (and L >= 16 spatial) attention backward: from the forward's planes (qkv_t), lse,
   output o (CT [N][C]; o_lo its residual from mdg_attn_temporal_lse or null) and its gradient
   dout (CT [N][C]), writes dq | dk | dv of the linear
   projections (RoPE and the q scale undone: qscale = D^-1/2) into dqkv (CT, token-major rows of
   ld_dqkv >= 3C, packed column order); kscale = ln 2 for planes in log2 units (the forward's
   q carries log2 e).  bias_k / bias_v gradients (w.r.t. the rotated kvb rows) are written as
   per-slot partials bpart [H][parts][2][DP].  generic: 0 = the fused single-pass MFMA kernel
   (bf16 default: P / dP once per pair, one block per (sequence, head), deterministic), 2 = the
   two-pass MFMA kernels (dQ; dK / dV), 1 = the scalar kernels (the fp32 path always uses them).
   head_dim 32..63 (ABI 23): bf16 takes generic = 1 only (MDG_E_ARG otherwise). */
int mdg_attn_temporal_bwd(int32_t dtype, int32_t B, int32_t T, int32_t L, int32_t H, int32_t D, const void* qkv_t,
                          const float* kbias, const float* kvb, const void* o, const void* o_lo, const void* dout,
                          const float* lse,
                          const float* rope, int32_t rope_rows, void* scratch, void* dqkv, int32_t ld_dqkv,
                          float* bpart, float qscale, float kscale, int32_t generic, void* stream);
/* Spatial attention backward (L < 16): q|k|v [N][3C] as saved by the forward, dout CT [N][C];
   dq | dk | dv into dqkv [N][3C]; bias partials bpart [H][parts][2][DP] (every slot; columns
   >= D of a slot may be left unwritten: mdg_train_unpack_layer reads d < D only); head_dim < 64. */
int mdg_attn_spatial_bwd(int32_t dtype, int32_t n_frames, int32_t L, int32_t H, int32_t D, const void* qkv,
                         const float* kvb, const float* mask, const void* dout, const float* rope, int32_t rope_rows,
                         void* dqkv, float* bpart, float qscale, void* stream);

/* Weight / bias gradients of a linear layer from token-major operands (the nn.Linear backward
   inside LatentMDGenLayer under loss.backward(): transport.py:137-222, latent_model.py:456-493):
     dw[m][k] = sum_n dy[n][m] x[n][k]   (fp32, ld lddw; null = skip)
     db[m]    = sum_n dy[n][m]           (fp32; null = skip)
   dy CT [N][ldy] (columns 0..M-1), x CT [N][ldx] (columns 0..K-1); the reduction is split over
   token chunks whose fp32 partials (in ws) are summed in chunk order: deterministic.  bf16 needs
   N % 32 == 0 (pad the token rows with zeros); M, K, ldy, ldx multiples of 8; 16-B aligned
   operands and dw, lddw a multiple of 4.  bf16 with both outputs: the column sums ride in the
   dW blocks and one launch reduces both.  ws: mdg_wgrad_workspace_bytes(dtype, N, M, K, need_dw, need_db) bytes. */
size_t mdg_wgrad_workspace_bytes(int32_t dtype, int32_t N, int32_t M, int32_t K, int32_t need_dw, int32_t need_db);
int mdg_wgrad(int32_t dtype, int32_t N, int32_t M, int32_t K, const void* dy, int32_t ldy, const void* x, int32_t ldx,
              float* dw, int32_t lddw, float* db, void* ws, size_t ws_bytes, void* stream);

/* Few-row fp32 linears of the training step's conditioning (the TimestepEmbedder MLP,
   layers.py:17-55; every adaLN_modulation Linear of the model, latent_model.py:341-493 and
   layers.py:58-75; the IPA projections and linear_out, ipa.py:92-250), forward and backward,
   for nseg nn.Linear layers that share one input x [M][K] (ld ldx): segment i has n[i] output
   features, weight w[i] [n[i]][K] (nn.Linear layout), bias b[i] [n[i]] (null: none).
   in_act MDG_ACT_NONE: x' = x; MDG_ACT_SILU: x' = SiLU(x) (the adaLN / t-MLP nn.SiLU in front).
     fwd: y[i][m][j] = resid[i][m][j] (if non-null, ld ldr[i]) + b[i][j] + sum_k x'[m][k] w[i][j][k]
          (y ld ldy[i]; exact fp32 FMAs in ascending k).
     bwd: from dy[i] [M][lddy[i]]: dw[i] [n[i]][K] = dy^T x', db[i] = column sums of dy (either
          null: skip), and dx [M][lddx] = (sum_i dy[i] w[i]) * SiLU'(x) for SILU (null: skip),
          the weight-row reduction split into chunks of 256 rows whose partials (in ws) are
          summed in chunk order (deterministic).  K % 4 == 0, K <= 1024, x and weights 16-B aligned.
   ws: mdg_seg_linear_bwd_workspace_bytes. */
typedef struct {
  int32_t nseg;
  int32_t n[MDG_SEG_MAX];
  const float* w[MDG_SEG_MAX];
  const float* b[MDG_SEG_MAX];
  float* y[MDG_SEG_MAX];
  int32_t ldy[MDG_SEG_MAX];
  const float* resid[MDG_SEG_MAX];
  int32_t ldr[MDG_SEG_MAX];
  const float* dy[MDG_SEG_MAX];
  int32_t lddy[MDG_SEG_MAX];
  float* dw[MDG_SEG_MAX];
  float* db[MDG_SEG_MAX];
} mdg_seg_linear;
int mdg_seg_linear_fwd(int32_t M, int32_t K, const float* x, int32_t ldx, int32_t in_act, const mdg_seg_linear* s,
                       void* stream);
size_t mdg_seg_linear_bwd_workspace_bytes(int32_t M, int32_t K, const mdg_seg_linear* s);
int mdg_seg_linear_bwd(int32_t M, int32_t K, const float* x, int32_t ldx, int32_t in_act, const mdg_seg_linear* s,
                       float* dx, int32_t lddx, void* ws, size_t ws_bytes, void* stream);

/* The flow-matching plan and loss of Transport.training_losses (transport.py:137-222, velocity
   model, path.py:81-191), fp32:
     mdg_gvp_plan: for trajectory b (n_per_b contiguous elements each), t = t[b]; path 0 = GVP
       (a = sin(t pi / 2), s = cos(t pi / 2), da = pi/2 cos, ds = -pi/2 sin), 1 = Linear (a = t,
       s = 1 - t, da = 1, ds = -1): xt = a x1 + s x0, ut = da x1 + ds x0 (torch's rounding order).
     mdg_gvp_loss_fwd: loss[b] = sum (out - ut)^2 m / sum m over the [T][L][K] elements of b
       (mean_flat, transport.py:12-16), den[b] = sum m; mask element (b, t, l, k) at
       b s0 + t s1 + l s2 + k s3 (mask_strides: a broadcast view needs no copy); block partials
       summed in a fixed order.  ws: mdg_gvp_loss_workspace_bytes(B, T*L*K).
     mdg_gvp_loss_bwd: dout = 2 (out - ut) m gloss[b] / den[b]. */
int mdg_gvp_plan(int32_t B, int64_t n_per_b, int32_t path, const float* t, const float* x0, const float* x1, float* xt,
                 float* ut, void* stream);
size_t mdg_gvp_loss_workspace_bytes(int32_t B, int64_t n_per_b);
int mdg_gvp_loss_fwd(int32_t B, int32_t T, int32_t L, int32_t K, const float* out, const float* ut, const float* mask,
                     const int64_t* mask_strides, float* loss, float* den, void* ws, size_t ws_bytes, void* stream);
int mdg_gvp_loss_bwd(int32_t B, int32_t T, int32_t L, int32_t K, const float* out, const float* ut, const float* mask,
                     const int64_t* mask_strides, const float* gloss, const float* den, float* dout, void* stream);

/* The optimizer step of the graphed training step (train.py GraphedStep._update: the reference's
   Lightning loop runs clip_grad_norm_ (gradient_clip_val, train.py:52) then Adam / AdamW,
   wrapper.py:167-173), fp32, torch.optim semantics:
     norm = ||all g||_2 (chunk partials summed in a fixed order), coef = min(1, max_norm /
     (norm + 1e-6)) (1 when max_norm <= 0), g' = coef g (+ weight_decay p unless decoupled),
     step += 1, m = b1 m + (1 - b1) g', v = b2 v + (1 - b2) g'^2, p (*= 1 - lr wd when decoupled)
     -= lr / (1 - b1^step) m / (sqrt(v) / sqrt(1 - b2^step) + eps).
   g is read, not clipped in place.  One table entry per tensor; the device table image
   (tensors + chunk map) is built on the host by mdg_adam_table_build and copied by the caller,
   which may do so after a stream capture that recorded mdg_adam_step (the kernels read the table
   when they run).  ws: mdg_adam_workspace_bytes(n_chunks).  gnorm (device, may be null) gets norm.
   Hyper-parameters in double, as torch's Python floats: the bias corrections are formed in double
   per block, the element update in fp32. */
typedef struct {
  float* p;
  const float* g;
  float* m;     /* exp_avg */
  float* v;     /* exp_avg_sq */
  float* step;  /* the tensor's step count (a 0-d fp32 device tensor, torch's capturable state) */
  int64_t n;
} mdg_adam_tensor;
int32_t mdg_adam_chunks(int32_t n_tensors, const mdg_adam_tensor* tensors);
size_t mdg_adam_table_bytes(int32_t n_tensors, const mdg_adam_tensor* tensors);
int mdg_adam_table_build(int32_t n_tensors, const mdg_adam_tensor* tensors, void* table, size_t table_bytes);
size_t mdg_adam_workspace_bytes(int32_t n_chunks);
int mdg_adam_step(int32_t n_tensors, int32_t n_chunks, const void* table, double lr, double beta1, double beta2,
                  double eps, double weight_decay, int32_t decoupled, double max_norm, float* gnorm, void* ws,
                  size_t ws_bytes, void* stream);

/* Training backward of the token embedding (latent_model.py:242-255 under loss.backward()),
   from the residual gradient dh [N][C] fp32 (N = B*T*L tokens, n = (b*T + t)*L + l):
     dw1 [C][K1]    = sum_n dh[n] x1[n]^T         latent_to_emb.weight (x1 [N][K1], the noised latents)
     dw2 [C][K2]    = sum_n dh[n] x2[n]^T         cond_to_emb.weight (x2 [N][K2] = x_cond; null: skip)
     db  [C]        = sum_n dh[n]                 each embedding bias (null: skip)
     demb [E][C]    = sum_{n: idx[n] = e} dh[n]   mask_to_emb.weight (idx null: skip)
     dipa [B][L][C] = sum_t dh[b, t, l]           the IPA prepend broadcast over frames (null: skip)
   fp32; per-chunk partials in ws summed in chunk order (deterministic).  K1, K2 <= 32, E <= 4,
   L <= 8, C % 128 == 0.  ws: mdg_embed_bwd_workspace_bytes(B, T, L, C, K1, K2, E). */
size_t mdg_embed_bwd_workspace_bytes(int32_t B, int32_t T, int32_t L, int32_t C, int32_t K1, int32_t K2, int32_t E);
int mdg_embed_bwd(int32_t B, int32_t T, int32_t L, int32_t C, int32_t K1, const float* x1, int32_t K2, const float* x2,
                  const int64_t* idx, int32_t E, const float* dh, float* dw1, float* dw2, float* db, float* demb,
                  float* dipa, void* ws, size_t ws_bytes, void* stream);

/* Training FinalLayer (layers.py:58-75), fp32, C = 384, latent 21 or 28.  Row n belongs to
   trajectory b = n / rows_per_b; mods [B][2C] = (shift | scale) of its adaLN:
     fwd: xn = LN(h[n]) (1 + scale) + shift (no-affine LN, eps 1e-6); v[n] = xn w^T + bias
          (w [latent][C], the nn.Linear weight); stats [N][2] = (mean, rstd) for the backward.
     bwd: from dv [N][latent]: dh [N][C] (written), and reduced in block order (deterministic)
          dw [latent][C], dbias [latent] (null: skip), dmods [B][2C] (d shift | d scale).
   ws: mdg_final_bwd_workspace_bytes(N, rows_per_b, latent). */
int mdg_final_fwd_train(int32_t N, int32_t rows_per_b, int32_t C, int32_t latent, const float* h, const float* mods,
                        const float* w, const float* bias, float* v, float* stats, void* stream);
size_t mdg_final_bwd_workspace_bytes(int32_t N, int32_t rows_per_b, int32_t latent);
int mdg_final_bwd_train(int32_t N, int32_t rows_per_b, int32_t C, int32_t latent, const float* h, const float* stats,
                        const float* mods, const float* w, const float* dv, float* dh, float* dw, float* dbias,
                        float* dmods, void* ws, size_t ws_bytes, void* stream);

/* Invariant point attention core of the IPA prepend under autograd (reference
   src/mdgen/model/ipa.py:92-255, c_z = 0; latent_model.py:179-214), fp32, L <= 256 (33..256 on
   the long kernels since round 5: ATLAS crops), c = 32,
   8 query/key points and 8 value points (the reference's defaults; other shapes: MDG_E_SHAPE).
   Operands per token b*L + i, head h:  q [..][H][c], kv [..][H][2c] (k | v), mask [B][L], rots
   [B][L][3][3], trans [B][L][3], wc = sqrt(1 / (3c)); the points and head weights by `flags`:
     0: qp [..][H][Pq][3] and kvp [..][H][Pq + Pv][3] already in the global frame, hw [H] =
        softplus(head_weights) * sqrt(1 / (3 Pq 9/2));
     MDG_IPA_LOCAL_POINTS: qp [..][3][H*Pq] and kvp [..][3][H*(Pq + Pv)], the raw linear_q_points /
        linear_kv_points rows (x | y | z blocks, point h*P + p: ipa.py:121-140), in the residue's
        local frame; the kernel applies R p + t (rigid_utils.py:64-86) and the backward returns
        d raw = R^T d global in the same layout;
     MDG_IPA_RAW_HW: hw [H] is the raw head_weights parameter (softplus taken in the kernel),
        and dhw_part is the gradient w.r.t. it.
   fwd: out [B*L][H*c + 4*H*Pv] = [o | ol_x | ol_y | ol_z | |ol|], the linear_out input.
   bwd: from dout (same layout): dq, dkv, dqp, dkvp (the operands' layouts) and dhw_part [B][H]
   (sum over B = d hw). */
enum { MDG_IPA_LOCAL_POINTS = 1, MDG_IPA_RAW_HW = 2 };
int mdg_ipa_core_fwd(int32_t B, int32_t L, int32_t H, int32_t c, int32_t Pq, int32_t Pv, const float* q,
                     const float* kv, const float* qp, const float* kvp, const float* mask, const float* rots,
                     const float* trans, const float* hw, float wc, float* out, int32_t flags, void* stream);
int mdg_ipa_core_bwd(int32_t B, int32_t L, int32_t H, int32_t c, int32_t Pq, int32_t Pv, const float* q,
                     const float* kv, const float* qp, const float* kvp, const float* mask, const float* rots,
                     const float* trans, const float* hw, float wc, const float* dout, float* dq, float* dkv,
                     float* dqp, float* dkvp, float* dhw_part, int32_t flags, void* stream);

/* Per-step weight packing / gradient unpacking of one training layer (train_hip._HipLayerFn;
   latent_model.py:456-493 parameters, mha.py:245-247 projections, fair-esm RoPE of bias_k at
   the bias key's position S).  All sources fp32 in nn.Linear / nn.Parameter layout; the packed
   outputs are the mdg_layer_weights operands plus the transposes the input-gradient GEMMs read.
   rope_tab[i]: [rope_rows][D/2] cos then [rope_rows][D/2] sin; rope_pos[i] = S (L or T). */
typedef struct {
  int32_t C, H, D, F, rope, dtype;
  const float* wq[2]; const float* wk[2]; const float* wv[2];
  const float* bq[2]; const float* bk[2]; const float* bv[2];
  const float* wo[2]; const float* bias_k[2]; const float* bias_v[2];
  const float* w1; const float* w2;
  const float* rope_tab[2]; int32_t rope_rows[2]; int32_t rope_pos[2];
  void* wqkv[2]; void* wqkv_t[2]; float* bqkv[2]; void* wo_p[2]; void* wo_t[2]; float* kvb[2];
  void* w1_p; void* w1_t; void* w2_p; void* w2_t;
} mdg_train_pack;
/* kvb[i]: [H][2][MDG_HEAD_STRIDE(D)] (head_dim < 64).
   gwqkv / gbqkv: packed-order fp32 gradients ([3C][C], [3C]); bpart[i]: [H][parts[i]][2][DP]
   bias-key / value partials (summed here, one block per head: H <= 128); part[0..3]: the ln_gate_bwd partials [B][nblk][4][C] of the
   layer-input LN, the spatial, temporal and MLP sublayers.  Outputs fp32 in parameter layout;
   dmods [B][9C] in latent_model.py:459-461 chunk order. */
typedef struct {
  int32_t C, H, D, B, nblk, rope;
  const float* gwqkv[2]; const float* gbqkv[2];
  const float* bpart[2]; int32_t parts[2];
  const float* rope_tab[2]; int32_t rope_rows[2]; int32_t rope_pos[2];
  const float* part[4];
  float* gq[2]; float* gk[2]; float* gv[2]; float* gbq[2]; float* gbk[2]; float* gbv[2];
  float* gbias_k[2]; float* gbias_v[2];
  float* dmods; float* gbo[2]; float* gb2;
} mdg_train_unpack;
int mdg_train_pack_layer(const mdg_train_pack* p, void* stream);
int mdg_train_unpack_layer(const mdg_train_unpack* u, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MDGEN_HIP_H */
