"""The C-ABI library: builds, loads on a GPU-less host, and exports exactly the entry points
include/mdgen_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "mdgen_hip.h")


def _declared():
    src = open(HEADER).read()
    return set(re.findall(r"^\s*(?:int|int32_t|size_t|const char\*)\s+(mdg_\w+)\s*\(", src, re.M))


def test_header_declares_binding_signatures():
    from mdgen_finetune_amd import _lib

    assert _declared() == {n for n, _, _ in _lib.SIGNATURES}


def test_library_loads_and_exports_every_declared_symbol():
    from mdgen_finetune_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        # a fresh checkout: build it the way __graft_entry__.build() does (hipcc cross-compiles
        # gfx950 without a GPU)
        import subprocess

        subprocess.run(["make", "-C", os.path.join(REPO, "mdgen_finetune_amd", "csrc"), "-j8"], check=False,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600)
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail(f"{_lib.LIB_PATH} is not built (run __graft_entry__.build())")
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.mdg_abi_version() == _lib.ABI_VERSION


def test_struct_layouts_match_header():
    """ctypes mirrors of the C structs: sizes/offsets checked against a C compile of the header."""
    import subprocess
    import tempfile

    from mdgen_finetune_amd import _lib

    prog = r"""
#include <stdio.h>
#include <stddef.h>
#include "mdgen_hip.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu\n", sizeof(mdg_dims), sizeof(mdg_layer_weights), sizeof(mdg_model),
        sizeof(mdg_step_io), sizeof(mdg_gemm_desc), sizeof(mdg_layer_saved));
 printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(mdg_cond_dims), sizeof(mdg_ipa_layer_weights),
        sizeof(mdg_cond_model), sizeof(mdg_cond_io), offsetof(mdg_cond_model, time_multiplier),
        offsetof(mdg_cond_model, t_freqs), offsetof(mdg_cond_model, ipa));
 printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(mdg_train_pack), offsetof(mdg_train_pack, rope_rows),
        offsetof(mdg_train_pack, w1_t), sizeof(mdg_train_unpack), offsetof(mdg_train_unpack, part),
        offsetof(mdg_train_unpack, gb2), offsetof(mdg_step_io, chain_alone));
 printf("%zu %zu %zu %zu\n", sizeof(mdg_seg_linear), offsetof(mdg_seg_linear, w), offsetof(mdg_seg_linear, resid),
        offsetof(mdg_seg_linear, db));
 printf("%zu %zu %zu %zu %zu %zu %zu\n", offsetof(mdg_step_io, dt), offsetof(mdg_step_io, h),
        offsetof(mdg_gemm_desc, qscale), offsetof(mdg_gemm_desc, rope_rows), offsetof(mdg_gemm_desc, aux),
        offsetof(mdg_gemm_desc, ldaux), offsetof(mdg_layer_saved, skip_temporal));
 return 0; }
"""
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(td, "t")
        subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), c, "-o", exe])
        out = subprocess.check_output([exe]).decode().split()
    sizes = [int(v) for v in out[:6]]
    cond = [int(v) for v in out[6:13]]
    train = [int(v) for v in out[13:20]]
    seg = [int(v) for v in out[20:24]]
    offs = [int(v) for v in out[24:]]
    S = _lib.MdgSegLinear
    assert seg == [ctypes.sizeof(S), S.w.offset, S.resid.offset, S.db.offset]
    assert train == [ctypes.sizeof(_lib.MdgTrainPack), _lib.MdgTrainPack.rope_rows.offset, _lib.MdgTrainPack.w1_t.offset,
                     ctypes.sizeof(_lib.MdgTrainUnpack), _lib.MdgTrainUnpack.part.offset,
                     _lib.MdgTrainUnpack.gb2.offset, _lib.MdgStepIO.chain_alone.offset]
    assert cond == [ctypes.sizeof(_lib.MdgCondDims), ctypes.sizeof(_lib.MdgIpaLayerWeights),
                    ctypes.sizeof(_lib.MdgCondModel), ctypes.sizeof(_lib.MdgCondIO),
                    _lib.MdgCondModel.time_multiplier.offset, _lib.MdgCondModel.t_freqs.offset,
                    _lib.MdgCondModel.ipa.offset]
    assert sizes == [ctypes.sizeof(s) for s in (_lib.MdgDims, _lib.MdgLayerWeights, _lib.MdgModel,
                                                 _lib.MdgStepIO, _lib.MdgGemmDesc, _lib.MdgLayerSaved)]
    assert offs == [_lib.MdgStepIO.dt.offset, _lib.MdgStepIO.h.offset, _lib.MdgGemmDesc.qscale.offset,
                    _lib.MdgGemmDesc.rope_rows.offset, _lib.MdgGemmDesc.aux.offset, _lib.MdgGemmDesc.ldaux.offset,
                    _lib.MdgLayerSaved.skip_temporal.offset]


def test_shape_validation_without_gpu():
    """Host-side argument checks reject bad dims before any launch (no device needed)."""
    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    d = _lib.MdgDims(B=1, T=1000, L=4, C=384, H=16, D=24, F=1536, latent=21, num_layers=5, dtype=1)
    assert lib.mdg_workspace_bytes(ctypes.byref(d)) > 0
    wide = _lib.MdgDims(B=1, T=10, L=4, C=384, H=12, D=32, F=1536, latent=21, num_layers=5, dtype=1)
    assert lib.mdg_workspace_bytes(ctypes.byref(wide)) > 0  # head_dim 32: 64-column operand rows
    bad = _lib.MdgDims(B=1, T=10, L=4, C=512, H=8, D=64, F=2048, latent=21, num_layers=5, dtype=1)
    assert lib.mdg_workspace_bytes(ctypes.byref(bad)) == 0
    assert b"head_dim" in lib.mdg_last_error_string()
    offs = _lib.workspace_offsets(d)
    vals = [offs[k] for k in _lib.WS_REGIONS]
    assert vals == sorted(vals) and vals[0] == 0 and all(v % 256 == 0 for v in vals)
    assert offs["kbias"] < lib.mdg_workspace_bytes(ctypes.byref(d))


def test_attention_backward_sizes_without_gpu():
    """ABI 23 host-side sizes: the temporal backward's scratch scales with the head stride (32 ->
    64 columns at head_dim 32..63) and is 0 outside 1..63; bias-slot counts per variant (the fused
    kernel one per sequence, the scalar kernels one per 256 queries); the spatial backward's slot
    count takes H (the L = 4 grid-stride kernel: at most 256 blocks)."""
    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    B, T, L, H = 8, 1000, 4, 16
    narrow = lib.mdg_attn_temporal_bwd_scratch(_lib.MDG_F32, B, T, L, H, 24)
    wide = lib.mdg_attn_temporal_bwd_scratch(_lib.MDG_F32, B, T, L, H, 48)
    rows = B * L * H * T
    assert narrow >= rows * 32 * 4 + rows * 4 and wide >= rows * 64 * 4 + rows * 4 and wide > narrow
    assert lib.mdg_attn_temporal_bwd_scratch(_lib.MDG_F32, B, T, L, H, 64) == 0
    assert lib.mdg_attn_temporal_bwd_parts(_lib.MDG_BF16, B, T, L, 0) == B * L
    assert lib.mdg_attn_temporal_bwd_parts(_lib.MDG_BF16, B, T, L, 1) == B * L * 4
    assert lib.mdg_attn_temporal_bwd_parts(_lib.MDG_F32, B, T, L, 1) == B * L * 4
    assert lib.mdg_attn_spatial_bwd_parts(B * T, 4, 16, 24) == 256
    assert lib.mdg_attn_spatial_bwd_parts(2, 4, 16, 24) == 1
    assert lib.mdg_attn_spatial_bwd_parts(B * T, 6, 8, 48) == (B * T * 8 + 127) // 128


def test_adam_table_image_without_gpu():
    """mdg_adam_table_build (host only): the tensor entries, then chunk -> (tensor, chunk index)
    for chunks of 16384 elements; tensors without elements and null pointers are refused."""
    import struct

    from mdgen_finetune_amd import _lib

    lib = _lib.load()
    sizes = [1, 16384, 16385, 40000]
    tab = (_lib.MdgAdamTensor * len(sizes))()
    for i, n in enumerate(sizes):
        base = 0x1000 * (i + 1)
        tab[i] = _lib.MdgAdamTensor(base, base + 16, base + 32, base + 48, base + 64, n)
    nc = lib.mdg_adam_chunks(len(sizes), tab)
    assert nc == 1 + 1 + 2 + 3
    nbytes = lib.mdg_adam_table_bytes(len(sizes), tab)
    assert nbytes == len(sizes) * ctypes.sizeof(_lib.MdgAdamTensor) + 8 * nc
    buf = (ctypes.c_uint8 * nbytes)()
    assert lib.mdg_adam_table_build(len(sizes), tab, buf, nbytes) == 0
    raw = bytes(buf)
    head = len(sizes) * ctypes.sizeof(_lib.MdgAdamTensor)
    assert raw[:head] == bytes(tab)
    ct = struct.unpack(f"<{nc}i", raw[head:head + 4 * nc])
    ci = struct.unpack(f"<{nc}i", raw[head + 4 * nc:])
    assert list(ct) == [0, 1, 2, 2, 3, 3, 3] and list(ci) == [0, 0, 0, 1, 0, 1, 2]
    assert lib.mdg_adam_table_build(len(sizes), tab, buf, nbytes - 1) != 0  # short table
    tab[1].n = 0
    assert lib.mdg_adam_chunks(len(sizes), tab) < 0
    tab[1].n, tab[2].step = 5, None
    assert lib.mdg_adam_table_build(len(sizes), tab, buf, nbytes) != 0
    assert b"null" in lib.mdg_last_error_string()
