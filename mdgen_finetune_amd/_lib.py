"""ctypes binding of libmdgen_hip.so (C ABI declared in include/mdgen_hip.h).

The library is built in-tree (mdgen_finetune_amd/libmdgen_hip.so, see csrc/Makefile) and
loaded after torch, so it binds to the HIP runtime torch already loaded (same SONAME
libamdhip64.so.7).  There is no fallback: if the library is missing or a call fails, a
RuntimeError is raised.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library is loaded)

# MDG_LIB_PATH: an alternative build of the same ABI (A/B timing of two kernel versions)
LIB_PATH = os.environ.get("MDG_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmdgen_hip.so")

MDG_F32, MDG_BF16 = 0, 1
MDG_A_PLAIN, MDG_A_LNMOD = 0, 1
MDG_EPI_STORE, MDG_EPI_GATE_RES, MDG_EPI_QKV, MDG_EPI_EULER, MDG_EPI_ATTN_SPATIAL = 0, 1, 2, 3, 4
MDG_ACT_NONE, MDG_ACT_GELU, MDG_ACT_SILU, MDG_ACT_DGELU = 0, 1, 2, 3
MDG_QKV_SPATIAL, MDG_QKV_TEMPORAL, MDG_QKV_TEMPORAL_PACKED = 0, 1, 2
MDG_PREP_TPS, MDG_PREP_NO_OFFSETS, MDG_PREP_COND_FIRST, MDG_PREP_COND_LAST = 1, 2, 4, 8
MDG_MAX_LAYERS = 16
MDG_SEG_MAX = 16
MDG_IPA_LOCAL_POINTS, MDG_IPA_RAW_HW = 1, 2
MDG_DP = 32
MDG_DP_WIDE = 64


def head_stride(D: int) -> int:
    """Row stride of the padded attention operands for head dim D (MDG_HEAD_STRIDE)."""
    return MDG_DP if D < MDG_DP else MDG_DP_WIDE

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_f32 = ctypes.c_float


class MdgDims(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("B", "T", "L", "C", "H", "D", "F", "latent", "num_layers", "dtype")]


class MdgLayerWeights(ctypes.Structure):
    _fields_ = [("wqkv", _vp * 2), ("bqkv", _vp * 2), ("wo", _vp * 2), ("bo", _vp * 2),
                ("kvb", _vp * 2), ("w1", _vp), ("b1", _vp), ("w2", _vp), ("b2", _vp)]


class MdgModel(ctypes.Structure):
    _fields_ = [("dims", MdgDims), ("w_l2e_t", _vp), ("w_final", _vp), ("b_final", _vp),
                ("rope_l", _vp), ("rope_t", _vp), ("layers", MdgLayerWeights * MDG_MAX_LAYERS)]


class MdgStepIO(ctypes.Structure):
    _fields_ = [("x_in", _vp), ("x_out", _vp), ("v_out", _vp), ("base", _vp), ("ipa", _vp),
                ("mods", _vp), ("mods_final", _vp), ("dt", _f32), ("h", _vp), ("chain_alone", _i32)]


class MdgGemmDesc(ctypes.Structure):
    _fields_ = [
        ("dtype", _i32), ("a_mode", _i32), ("epi", _i32), ("act", _i32),
        ("M", _i32), ("N", _i32), ("K", _i32),
        ("A", _vp), ("lda", _i32), ("W", _vp), ("ldw", _i32), ("bias", _vp),
        ("mods", _vp), ("mod_stride", _i32), ("rows_per_mod", _i32), ("shift_off", _i32),
        ("scale_off", _i32),
        ("ln_w", _vp), ("ln_b", _vp), ("ln_eps", _f32),
        ("out", _vp), ("ldo", _i32), ("out_f32", _i32),
        ("resid", _vp), ("ldr", _i32), ("gate", _vp), ("gate_off", _i32),
        ("qkv_layout", _i32), ("qkv_out", _vp), ("H", _i32), ("D", _i32), ("T", _i32), ("L", _i32),
        ("qscale", _f32), ("rope", _vp), ("rope_rows", _i32),
        ("x_in", _vp), ("v_out", _vp), ("dt", _f32), ("n_valid", _i32),
        ("xn_out", _vp), ("xn_mods", _vp), ("xn_mod_stride", _i32), ("xn_shift_off", _i32), ("xn_scale_off", _i32),
        ("kvb", _vp), ("key_mask", _vp),
        ("resid_in", _vp), ("aux", _vp), ("ldaux", _i32),
        ("ln_stats", _vp),
    ]


class MdgLayerSaved(ctypes.Structure):
    _fields_ = [("xn", _vp * 3), ("stats", _vp * 3), ("qkv_s", _vp), ("lse_s", _vp), ("qkv_t", _vp),
                ("lse_t", _vp), ("o", _vp * 2), ("o_lo", _vp * 2), ("y", _vp * 3), ("h1", _vp), ("h2", _vp), ("u", _vp), ("act", _vp),
                ("init_planes", _i32), ("skip_temporal", _i32),
                ("xn0_given", _i32), ("xn_next", _vp), ("stats_next", _vp), ("mods_next", _vp)]


class MdgCondDims(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("S", "B", "L", "C", "H", "D", "num_layers", "ipa_layers", "ipa_heads", "ipa_c",
                                    "ipa_qk", "ipa_v", "tps", "freq_dim")]


class MdgIpaLayerWeights(ctypes.Structure):
    _fields_ = [(n, _vp) for n in ("ln_w", "ln_b", "w_proj", "b_proj", "head_weights", "w_out", "b_out", "wqkv",
                                   "bqkv", "kvb", "wo", "bo", "w1", "b1", "w2", "b2")]


class MdgCondModel(ctypes.Structure):
    _fields_ = [("dims", MdgCondDims), ("time_multiplier", _f32)] + [
        (n, _vp) for n in ("t_freqs", "t_w0", "t_b0", "t_w2", "t_b2", "ada_w", "ada_b", "aa_emb", "l2e_f_w", "l2e_f_b",
                           "l2e_r_w", "l2e_r_b", "rope_l")] + [("ipa", MdgIpaLayerWeights * MDG_MAX_LAYERS)]


class MdgCondIO(ctypes.Structure):
    _fields_ = [("t", _vp), ("mask", _vp), ("mask_stride", _i32)] + [
        (n, _vp) for n in ("rots", "trans", "end_rots", "end_trans", "rel7", "aatype")] + [
        ("lanes", _i32), ("mods", _vp), ("mods_final", _vp), ("ipa", _vp)]


class MdgTrainPack(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("C", "H", "D", "F", "rope", "dtype")] + [
        (n, _vp * 2) for n in ("wq", "wk", "wv", "bq", "bk", "bv", "wo", "bias_k", "bias_v")] + [
        ("w1", _vp), ("w2", _vp), ("rope_tab", _vp * 2), ("rope_rows", _i32 * 2), ("rope_pos", _i32 * 2)] + [
        (n, _vp * 2) for n in ("wqkv", "wqkv_t", "bqkv", "wo_p", "wo_t", "kvb")] + [
        (n, _vp) for n in ("w1_p", "w1_t", "w2_p", "w2_t")]


class MdgTrainUnpack(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("C", "H", "D", "B", "nblk", "rope")] + [
        ("gwqkv", _vp * 2), ("gbqkv", _vp * 2), ("bpart", _vp * 2), ("parts", _i32 * 2), ("rope_tab", _vp * 2),
        ("rope_rows", _i32 * 2), ("rope_pos", _i32 * 2), ("part", _vp * 4)] + [
        (n, _vp * 2) for n in ("gq", "gk", "gv", "gbq", "gbk", "gbv", "gbias_k", "gbias_v")] + [
        ("dmods", _vp), ("gbo", _vp * 2), ("gb2", _vp)]


class MdgSegLinear(ctypes.Structure):
    _fields_ = [("nseg", _i32), ("n", _i32 * MDG_SEG_MAX), ("w", _vp * MDG_SEG_MAX), ("b", _vp * MDG_SEG_MAX),
                ("y", _vp * MDG_SEG_MAX), ("ldy", _i32 * MDG_SEG_MAX), ("resid", _vp * MDG_SEG_MAX),
                ("ldr", _i32 * MDG_SEG_MAX), ("dy", _vp * MDG_SEG_MAX), ("lddy", _i32 * MDG_SEG_MAX),
                ("dw", _vp * MDG_SEG_MAX), ("db", _vp * MDG_SEG_MAX)]


class MdgAdamTensor(ctypes.Structure):
    _fields_ = [("p", _vp), ("g", _vp), ("m", _vp), ("v", _vp), ("step", _vp), ("n", ctypes.c_int64)]


# (name, restype, argtypes) of every exported entry point — the test suite checks that the
# built library exports exactly these and that include/mdgen_hip.h declares them.
SIGNATURES = [
    ("mdg_abi_version", _i32, []),
    ("mdg_last_error_string", ctypes.c_char_p, []),
    ("mdg_stamp", _i32, [_vp, _i32, _vp]),
    ("mdg_wall_clock_khz", _i32, [ctypes.POINTER(_i32)]),
    ("mdg_workspace_bytes", ctypes.c_size_t, [ctypes.POINTER(MdgDims)]),
    ("mdg_workspace_offsets", _i32, [ctypes.POINTER(MdgDims), ctypes.POINTER(ctypes.c_size_t)]),
    ("mdg_workspace_init", _i32, [ctypes.POINTER(MdgDims), _vp, _vp]),
    ("mdg_prepare_mask", _i32, [ctypes.POINTER(MdgDims), _vp, _vp, _vp]),
    ("mdg_embed", _i32, [_i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_layer_fwd", _i32, [ctypes.POINTER(MdgDims), ctypes.POINTER(MdgLayerWeights), _vp, _vp, _vp,
                             _vp, _vp, _vp, _vp]),
    ("mdg_final_euler", _i32, [_i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp]),
    ("mdg_denoise_step", _i32, [ctypes.POINTER(MdgModel), ctypes.POINTER(MdgStepIO), _vp, _vp, _vp]),
    ("mdg_denoise_step_layers", _i32, [ctypes.POINTER(MdgModel), ctypes.POINTER(MdgStepIO), _vp, _vp, _i32, _i32,
                                       _vp]),
    ("mdg_describe_plan", _i32, [ctypes.POINTER(MdgDims), ctypes.c_char_p, ctypes.c_size_t]),
    ("mdg_gemm", _i32, [ctypes.POINTER(MdgGemmDesc), _vp]),
    ("mdg_mlp_fused", _i32, [ctypes.POINTER(MdgGemmDesc), ctypes.POINTER(MdgGemmDesc), _vp]),
    ("mdg_rowln_qkv", _i32, [ctypes.POINTER(MdgGemmDesc), ctypes.POINTER(MdgGemmDesc), _vp]),
    ("mdg_rowln_mlp", _i32, [ctypes.POINTER(MdgGemmDesc), ctypes.POINTER(MdgGemmDesc), ctypes.POINTER(MdgGemmDesc),
                             _vp]),
    ("mdg_attn_spatial", _i32, [_i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_attn_temporal", _i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_attn_temporal_packed", _i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_attn_temporal_lse", _i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_prep_latents", _i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_latents_to_atom14", _i32, [_i32, _i32, _i32, _i32, _i32, _i32] + [_vp] * 12),
    ("mdg_cond_workspace_bytes", ctypes.c_size_t, [ctypes.POINTER(MdgCondDims)]),
    ("mdg_precompute_cond", _i32, [ctypes.POINTER(MdgCondModel), ctypes.POINTER(MdgCondIO), _vp, _vp]),
    ("mdg_tps_rel7", _i32, [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_mask_bias", _i32, [_i32, _i32, _i32, _vp, _vp, _vp, _vp]),
    ("mdg_layer_fwd_train", _i32, [ctypes.POINTER(MdgDims), ctypes.POINTER(MdgLayerWeights), _vp, _vp, _vp, _vp, _vp,
                                   _vp, _vp, _vp, ctypes.POINTER(MdgLayerSaved), _vp]),
    ("mdg_ln_gate_bwd_blocks", _i32, [_i32]),
    ("mdg_ln_gate_bwd", _i32, [_i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _vp, _vp, _vp, _i32,
                               _vp, _vp, _vp]),
    ("mdg_attn_temporal_bwd_parts", _i32, [_i32, _i32, _i32, _i32, _i32]),
    ("mdg_attn_spatial_bwd_parts", _i32, [_i32, _i32, _i32, _i32]),
    ("mdg_attn_temporal_bwd_scratch", ctypes.c_size_t, [_i32, _i32, _i32, _i32, _i32, _i32]),
    ("mdg_attn_temporal_bwd", _i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32,
                                     _vp, _vp, _i32, _vp, _f32, _f32, _i32, _vp]),
    ("mdg_attn_spatial_bwd", _i32, [_i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _f32,
                                    _vp]),
    ("mdg_wgrad_workspace_bytes", ctypes.c_size_t, [_i32, _i32, _i32, _i32, _i32, _i32]),
    ("mdg_wgrad", _i32, [_i32, _i32, _i32, _i32, _vp, _i32, _vp, _i32, _vp, _i32, _vp, _vp, ctypes.c_size_t, _vp]),
    ("mdg_ipa_core_fwd", _i32, [_i32] * 6 + [_vp] * 8 + [_f32, _vp, _i32, _vp]),
    ("mdg_ipa_core_bwd", _i32, [_i32] * 6 + [_vp] * 8 + [_f32] + [_vp] * 6 + [_i32, _vp]),
    ("mdg_train_pack_layer", _i32, [ctypes.POINTER(MdgTrainPack), _vp]),
    ("mdg_train_unpack_layer", _i32, [ctypes.POINTER(MdgTrainUnpack), _vp]),
    ("mdg_embed_bwd_workspace_bytes", ctypes.c_size_t, [_i32] * 7),
    ("mdg_embed_bwd", _i32, [_i32] * 5 + [_vp, _i32, _vp, _vp, _i32] + [_vp] * 6 + [_vp, ctypes.c_size_t, _vp]),
    ("mdg_final_fwd_train", _i32, [_i32] * 4 + [_vp] * 7),
    ("mdg_final_bwd_workspace_bytes", ctypes.c_size_t, [_i32] * 3),
    ("mdg_final_bwd_train", _i32, [_i32] * 4 + [_vp] * 9 + [_vp, ctypes.c_size_t, _vp]),
    ("mdg_gvp_plan", _i32, [_i32, ctypes.c_int64, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("mdg_gvp_loss_workspace_bytes", ctypes.c_size_t, [_i32, ctypes.c_int64]),
    ("mdg_gvp_loss_fwd", _i32, [_i32] * 4 + [_vp] * 7 + [ctypes.c_size_t, _vp]),
    ("mdg_gvp_loss_bwd", _i32, [_i32] * 4 + [_vp] * 8),
    ("mdg_seg_linear_fwd", _i32, [_i32, _i32, _vp, _i32, _i32, ctypes.POINTER(MdgSegLinear), _vp]),
    ("mdg_seg_linear_bwd_workspace_bytes", ctypes.c_size_t, [_i32, _i32, ctypes.POINTER(MdgSegLinear)]),
    ("mdg_seg_linear_bwd", _i32, [_i32, _i32, _vp, _i32, _i32, ctypes.POINTER(MdgSegLinear), _vp, _i32, _vp,
                                  ctypes.c_size_t, _vp]),
    ("mdg_adam_chunks", _i32, [_i32, ctypes.POINTER(MdgAdamTensor)]),
    ("mdg_adam_table_bytes", ctypes.c_size_t, [_i32, ctypes.POINTER(MdgAdamTensor)]),
    ("mdg_adam_table_build", _i32, [_i32, ctypes.POINTER(MdgAdamTensor), _vp, ctypes.c_size_t]),
    ("mdg_adam_workspace_bytes", ctypes.c_size_t, [_i32]),
    ("mdg_adam_step", _i32, [_i32, _i32, _vp] + [ctypes.c_double] * 5 + [_i32, ctypes.c_double, _vp, _vp,
                                                                          ctypes.c_size_t, _vp]),
]

ABI_VERSION = 24
_LIB = None


def load():
    """Load (once) and return the ctypes library; raise if it is missing or mismatched."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: build it with `make -C mdgen_finetune_amd/csrc` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` (there is no non-HIP fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.mdg_abi_version()
    if v != ABI_VERSION:
        raise RuntimeError(f"libmdgen_hip ABI {v} != expected {ABI_VERSION}; rebuild")
    _LIB = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().mdg_last_error_string().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


WS_REGIONS = ("qkv_s", "qkv_t", "o", "hid", "xn", "kbias")


def workspace_offsets(dims) -> dict:
    """Byte offsets of the workspace regions (mdg_workspace_offsets)."""
    arr = (ctypes.c_size_t * 6)()
    check(load().mdg_workspace_offsets(ctypes.byref(dims), arr), "mdg_workspace_offsets")
    return dict(zip(WS_REGIONS, list(arr)))


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream
