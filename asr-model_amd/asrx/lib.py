"""ctypes binding of the C-ABI library ``libasrx.so`` (declared in ``include/asrx.h``).

The library is built in-tree by ``make -C asr-model_amd`` (``__graft_entry__.build()``).  There is
no fallback: if the library is missing, or a call is made without a GPU, the call raises.

Every entry point returns 0 on success; a nonzero code is turned into ``RuntimeError`` carrying
``asrx_last_error()`` (SURVEY.md §8(b) "Errors").
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime first so libasrx binds to the same instance)

_HERE = os.path.dirname(os.path.abspath(__file__))
# ASRX_LIB: an alternative build of the same library (tools/exp A/B experiments only)
LIB_PATH = os.environ.get("ASRX_LIB") or os.path.join(_HERE, "libasrx.so")

_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_f32 = ctypes.c_float
_p = ctypes.c_void_p
_u32 = ctypes.c_uint32

# name -> (restype, argtypes).  Kept in the order of include/asrx.h.
SIGNATURES = {
    "asrx_last_error": (ctypes.c_char_p, []),
    "asrx_abi_version": (_i32, []),
    "asrx_noise_hash": (_u32, [_u32, _u32]),
    "asrx_set_noise_epoch": (_i32, [_u32, _p]),
    "asrx_set_gemm_variant": (_i32, [_i32]),
    "asrx_set_attn_variant": (_i32, [_i32]),
    "asrx_set_wgrad_variant": (_i32, [_i32]),
    "asrx_mel_frames": (_i32, [_i64]),
    "asrx_logmel_ws_bytes": (_i64, [_i64, _i64]),
    "asrx_flac_info": (_i32, [_p, _i64, _p, _p, _p, _p, _p]),
    "asrx_flac_decode": (_i32, [_p, _i64, _p, _i64]),
    "asrx_pcm_normalize": (_i32, [_p, _i32, _i64, _i64, _i64, _p, _p, _p, _i64, _i32, _p]),
    "asrx_logmel": (_i32, [_p, _i64, _i64, _i64, _p, _p, _p, _p, _i32, _i64, _p, _p, _i64, _p]),
    "asrx_gemm": (
        _i32,
        [_i32, _p, _i64, _i64, _i32, _i32, _p, _i64, _i64, _i32, _i32, _p, _i64, _i64, _p, _p,
         _i64, _i64, _i64, _i64, _f32, _f32, _i32, _i64, _i64, _i32, _p],
    ),
    "asrx_abby_fwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _u32, _i32, _p]),
    "asrx_abby_fwd_logits": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _u32, _i32, _p]),
    "asrx_abby_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_attn_fwd": (_i32, [_i32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i32, _f32, _p]),
    "asrx_attn_bwd": (_i32, [_i32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                             _i64, _i64, _i64, _i64, _i64, _i32, _f32, _p]),
    "asrx_layernorm_fwd": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i64, _f32, _p]),
    "asrx_layernorm_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_layernorm_bwd_acc": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i32, _p]),
    "asrx_small_linear_fwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _i32, _p]),
    "asrx_small_linear_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i32, _f32, _p]),
    "asrx_rownorm": (_i32, [_p, _p, _i64, _i64, _p]),
    "asrx_rownorm_bwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_row_normalize": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "asrx_row_normalize_bwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _i32, _p]),
    "asrx_softmax_small": (_i32, [_p, _p, _i64, _i64, _p]),
    "asrx_softmax_small_bwd": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "asrx_zero": (_i32, [_p, _i64, _p]),
    "asrx_rotary_fwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "asrx_rotary_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "asrx_abby_bwd2": (_i32, [_p] * 10 + [_i64, _i64, _i32, _p]),
    "asrx_rownorm_bwd2": (_i32, [_p, _p, _p, _p, _i64, _i64, _i32, _p]),
    "asrx_colsum_ld": (_i32, [_p, _i64, _p, _i64, _i64, _p]),
    "asrx_ce_fwd1": (_i32, [_p] * 6 + [_i64, _i64, _p]),
    "asrx_ce_bwd2": (_i32, [_p] * 6 + [_i64, _i64, _p]),
    "asrx_bn_running": (_i32, [_p] * 5 + [_i64, _i64, _i64, _f32, _f32, _p]),
    "asrx_rsqrt_eps": (_i32, [_p, _p, _i64, _f32, _p]),
    "asrx_conv3_weight": (_i32, [_p, _p, _i64, _i64] + [_p] * 6),
    "asrx_conv3_weight_bwd": (_i32, [_p] * 4 + [_i64, _i64] + [_p] * 3),
    "asrx_blend_fwd": (_i32, [_p] * 4 + [_i64, _p]),
    "asrx_blend_bwd": (_i32, [_p] * 7 + [_i64, _p]),
    "asrx_add_segments": (_i32, [_p, _i64, _p, _p, _p, _i64, _p]),
    "asrx_cat3": (_i32, [_p] * 3 + [_i64, _p, _p]),
    "asrx_layernorm_fwd2": (_i32, [_p] * 10 + [_i32, _i64, _i64, _f32, _p]),
    "asrx_vgate_weights": (_i32, [_p] * 7 + [_i64, _i64, _i64, _p]),
    "asrx_msheath_row_fwd": (_i32, [_p] * 6 + [_i64] + [_p] * 14 + [_i64] * 4 + [_f32, _f32, _p, _i64, _i64, _p]),
    "asrx_msheath_row_bwd": (_i32, [_p] * 11 + [_i64] + [_p] * 18 + [_i64] * 4 + [_f32, _p, _i64, _i64, _p]),
    "asrx_gemm_wn_rows": (_i32, [_p, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _f32, _f32, _i32, _i32, _p,
                                 _p, _p]),
    "asrx_row_tiles_max": (_i64, [_i64]),
    "asrx_wgrad_bf16": (_i32, [_p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p]),
    "asrx_pitch_dio": (_i32, [_p, _i64, _i64, _i64] + [ctypes.c_double] * 5 + [_p, _i64, _p, _p, _p, _p, _i64]
                       + [_p] * 4 + [_i64] + [_p] * 4 + [_i64, _p]),
    "asrx_pitch_stonemask": (_i32, [_p, _i64, _i64, _i64, ctypes.c_double, _p, ctypes.c_double, _i64, _p, _p]),
    "asrx_wconv_entry_bytes": (_i64, []),
    "asrx_weights_to_bf16": (_i32, [_p, _i64, _i64, _p]),
    "asrx_row_tiles": (_i32, [_p, _i64, _i64, _i64, _p, _p, _p]),
    "asrx_msheath_ctrl_fwd3": (_i32, [_p, _p, _i64, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _p] + [_i64] * 5 + [_p] * 8),
    "asrx_mem_chunks": (_i64, [_i64]),
    "asrx_seg_colsum_det": (_i32, [_p, _p, _p, _i64, _i64, _i64, _f32, _p]),
    "asrx_msheath_ctrl_bwd3": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _p, _p, _p] + [_i64] * 4 + [_p, _i32] + [_p] * 8),
    "asrx_axpy_row2_colsum": (_i32, [_p] * 6 + [_i64] * 3 + [_p, _i64, _p]),
    "asrx_vgate_fwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _f32, _p]),
    "asrx_vgate_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                              _i64, _i64, _i64, _f32, _p]),
    "asrx_tgate_fwd": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "asrx_tgate_bwd": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_axpy_row": (_i32, [_p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_axpy_row_bwd": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_axpy_row_bwd2": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_jump_select": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_jump_select_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_seg_colsum": (_i32, [_p, _p, _i64, _i64, _i64, _f32, _i32, _p]),
    "asrx_msheath_ctrl_fwd": (_i32, [_p, _p, _i64, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64,
                                     _p, _p, _p, _p, _p, _p, _p, _p]),
    "asrx_msheath_ctrl_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _p, _p, _p, _p,
                                     _p]),
    "asrx_msheath_rec_bytes": (_i64, []),
    "asrx_msheath_ctrl_fwd2": (_i32, [_p, _p, _i64, _p, _p, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _i64,
                                      _p, _p, _p, _p, _p, _p, _p, _p]),
    "asrx_msheath_ctrl_bwd2": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _i32,
                                      _p, _p, _p, _p, _p, _p]),
    "asrx_jump_select4_bwd_acc": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_jump_bwd_part_floats": (_i64, [_i64, _i64, _i64]),
    "asrx_jump_select4_bwd_part": (_i32, [_p] * 11 + [_i64, _i64, _i64, _p]),
    "asrx_msheath_ctrl_bwd4": (_i32, [_p, _i64, _p, _p, _p, _i64, _p, _p, _p, _i64, _i64, _i64, _i64, _p, _i32]
                               + [_p] * 8),
    "asrx_axpy_row2_bwd_acc": (_i32, [_p, _p, _f32, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_msheath_dx_final": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_axpy_row2": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_axpy_row2_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_jump_select4": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_jump_select4_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_colsum": (_i32, [_p, _p, _i64, _i64, _p]),
    "asrx_add_rows": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_lincomb": (_i32, [_p, _p, _p, _f32, _f32, _f32, _p, _i64, _p]),
    "asrx_act_fwd": (_i32, [_p, _p, _i64, _i32, _p]),
    "asrx_act_bwd": (_i32, [_p, _p, _p, _i64, _i32, _p]),
    "asrx_glu_fwd": (_i32, [_p, _p, _i64, _i64, _p]),
    "asrx_glu_bwd": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "asrx_dropout": (_i32, [_p, _p, _i64, _i64, _i64, _i64, _u32, _f32, _p]),
    "asrx_act_dropout_fwd": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64, _u32, _f32, _i32, _i32, _p]),
    "asrx_act_dropout_bwd": (_i32, [_p, _p, _p, _i64, _i64, _i64, _i64, _u32, _f32, _i32, _i32, _p]),
    "asrx_dwconv_fwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "asrx_dwconv_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "asrx_bn_fwd": (_i32, [_p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _f32, _i32, _p]),
    "asrx_bn_bwd": (_i32, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_stem1_fwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_stem1_bwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _i64, _p]),
    "asrx_embed_fwd": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "asrx_embed_bwd": (_i32, [_p, _p, _p, _i64, _i64, _p]),
    "asrx_ce_fwd": (_i32, [_p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_ce_bwd": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _p]),
    "asrx_policy_noise": (_i32, [_p, _i64, _i64, _i64, _u32, _p]),
    "asrx_weight_to_bf16": (_i32, [_p, _p, _i64, _i64, _i64, _i32, _p]),
    "asrx_gemm_wn_router": (_i32, [_p, _i64, _p, _i64, _p, _p, _p, _i64, _p, _i64, _i64, _i64, _p]),
    "asrx_gemm_wn": (_i32, [_p, _i64, _i32, _i64, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _f32, _f32,
                            _i32, _i32, _p]),
    "asrx_gemm_wn_ex": (_i32, [_p, _i32, _i64, _i32, _i64, _i64, _p, _i64, _p, _i32, _i64, _p, _p, _i64, _i64, _i64,
                               _f32, _f32, _i32, _i32, _p, _p, _p]),
    "asrx_wgrad_bf16_ex": (_i32, [_p, _i64, _p, _i32, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p]),
    "asrx_abby_fwd2": (_i32, [_p, _p, _p, _p, _p, _i32, _p, _p, _i64, _i64, _i64, _i64, _i64, _u32, _i32, _p, _p, _p,
                              _p]),
    "asrx_gemm_wn_gact": (_i32, [_p, _i32, _i64, _p, _i64, _p, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i32, _i32,
                                 _p]),
    "asrx_rotary_table": (_i32, [_p, _p, _i64, _i64, _p]),
    "asrx_rotary_fwd2": (_i32, [_p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "asrx_rotary_bwd2": (_i32, [_p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _f32, _p]),
    "asrx_abby_fwd3": (_i32, [_p, _p, _p, _p, _p, _p, _i32, _p, _p, _i64, _i64, _i64, _i64, _i64, _u32, _i32, _p, _p,
                               _p, _p, _p]),
    "asrx_abby_fwd_logits2": (_i32, [_p, _p, _p, _p, _i32, _p, _p, _i64, _i64, _i64, _i64, _i64, _u32, _i32, _p, _p,
                                     _p, _p]),
    "asrx_attn_fwd2": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _i64, _i64, _i64, _i32, _f32,
                              _p]),
    "asrx_attn_bwd2": (_i32, [_i32, _i32, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                              _i64, _i64, _i64, _i64, _i64, _i32, _f32, _p]),
    "asrx_small_linear_fwd2": (_i32, [_p, _i32, _p, _p, _p, _i64, _i64, _i64, _i32, _p]),
    "asrx_small_linear_bwd2": (_i32, [_p, _p, _p, _i32, _p, _p, _p, _p, _i64, _i64, _i64, _i32, _f32, _p]),
    "asrx_tgate_fwd2": (_i32, [_p, _p, _p, _i32, _i64, _i64, _p]),
    "asrx_msheath_row_fwd2": (_i32, [_p] * 6 + [_i64] + [_p] * 7 + [_i32] + [_p] * 7 + [_i64] * 4
                                    + [_f32, _f32, _p, _i64, _i64, _p]),
    "asrx_msheath_row_fwd3": (_i32, [_p] * 6 + [_i64] + [_p] * 16 + [_i64] * 4 + [_f32, _f32, _p, _i64, _i64, _p]),
    "asrx_layernorm_fwd3": (_i32, [_p, _p, _p, _p, _i32] + [_p] * 6 + [_i32, _i64, _i64, _f32, _p]),
    "asrx_jump_axpy_inplace": (_i32, [_p] * 10 + [_i64, _i64, _i64, _p]),
    "asrx_wave_pool": (_i32, [_p, _i64, _i64, _i64, _i64, _p, _p]),
    "asrx_maxfactor_param_bytes": (_i32, []),
    "asrx_maxfactor_step": (_i32, [_p, _i32, _i64, _i64, _i64, _i64, _i64, _p, _p]),
    "asrx_abby_record_cond": (_i32, [_p]),
    "asrx_gemm_wn_ce": (_i32, [_p, _i64, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i32, _p]),
    "asrx_gemm_wn_ce_f32": (_i32, [_p, _i64, _p, _i64, _p, _i64, _p, _i64, _i64, _i64, _i32, _p]),
    "asrx_ce_part_fwd": (_i32, [_p, _i64] + [_p] * 6 + [_i64, _i64, _p]),
    "asrx_ce_part_fwd_f32": (_i32, [_p, _i64] + [_p] * 6 + [_i64, _i64, _p]),
    "asrx_ce_bwd_bf16": (_i32, [_p] * 6 + [_i64, _i64, _p]),
    "asrx_ce_bwd_f32in": (_i32, [_p] * 6 + [_i64, _i64, _p]),
    "asrx_wgrad_bf16_ab": (_i32, [_p, _i64, _p, _i32, _i64, _p, _i64, _i64, _i64, _i64, _i64, _p]),
    "asrx_wgrad_bias": (_i32, [_p, _i32, _i64, _p, _i32, _i64, _p, _i64, _p, _i64, _i64, _i64, _i64, _p]),
    "asrx_act_bwd_bias": (_i32, [_p, _p, _p, _p, _i64, _i64, _i32, _p]),
    "asrx_abby_fwd_res": (_i32, [_p] * 9 + [_i64] * 5 + [_u32, _i32, _p]),
    "asrx_gemm_wn_res": (_i32, [_p, _i64, _p, _i64, _p, _i64, _p, _p, _i64, _i64, _i64, _i64, _i32, _p]),
    "asrx_gemm_wn_rot": (_i32, [_p, _i32, _i64, _p, _i64, _p, _p, _i64, _p, _p, _p, _i64, _i64, _f32, _i64, _i64,
                                _i64, _i32, _p]),
    "asrx_msheath_plan_bytes": (_i64, []),
    "asrx_msheath_layer_bytes": (_i64, []),
    "asrx_msheath_fwd_ws_bytes": (_i64, [_p, _i64, _i64, _i64]),
    "asrx_msheath_fwd": (_i32, [_p, _p, _p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p]),
    "asrx_gemm_lt": (_i32, [_p, _i64, _p, _i64, _p, _i32, _i64, _p, _i64, _i64, _i64, _f32, _f32, _p]),
}

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"asrx native library not found at {LIB_PATH}; build it with `make -C asr-model_amd`"
            )
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("ASRX_LIB") and not hasattr(lib, name):
                continue  # an older A/B build lacks entry points added since: bind what it has
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        _bind_fast(lib)
    return _lib


def _bind_fast(lib) -> None:
    """call() goes through asrx/_asrxcall.so (gen_fastcall.py: one METH_FASTCALL wrapper per entry point, bound
    to the addresses of THIS ctypes handle's functions) when it was built; ctypes otherwise.  Same C-ABI, same
    library instance -- only the Python-side argument conversion differs (~1 us instead of ~10 us per launch)."""
    if os.environ.get("ASRX_CTYPES"):
        return
    try:
        from . import _asrxcall
    except ImportError:
        return
    for name in SIGNATURES:
        if not hasattr(lib, name):
            continue
        if _asrxcall.bind(name, ctypes.cast(getattr(lib, name), ctypes.c_void_p).value):
            _FN[name] = getattr(_asrxcall, name)


def exported_symbols() -> list[str]:
    return list(SIGNATURES)


def check(rc: int, name: str) -> None:
    if rc != 0:
        msg = load().asrx_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")


# launch census (tools/call_census.py): when a Counter is installed here, every call is counted by
# (entry point, calling file:line) with the sum of its integer arguments' largest value (a size proxy)
CENSUS = None


def call(name: str, *args) -> None:
    if CENSUS is not None:
        import sys as _sys

        f = _sys._getframe(1)
        g = f.f_back
        site = f"{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}"
        if g is not None:
            site += f" <- {os.path.basename(g.f_code.co_filename)}:{g.f_lineno}"
        key = (name, site)
        CENSUS[key + ("n",)] += 1
        CENSUS[key + ("size",)] += max((a for a in args if isinstance(a, int) and a < 1 << 40), default=0)
    fn = _FN.get(name)
    if fn is None:
        lib = load()  # binds the FASTCALL wrappers into _FN on first use
        fn = _FN.get(name) or _FN.setdefault(name, getattr(lib, name))
    rc = fn(*args)
    if rc:
        check(rc, name)


_FN: dict = {}  # entry point name -> callable (FASTCALL wrapper, or the bound ctypes function)
_raw_stream = torch._C._cuda_getCurrentRawStream
_get_device = torch._C._cuda_getDevice


def stream() -> int:
    """The current HIP stream of the current device as a raw pointer (what torch.cuda.current_stream().cuda_stream
    returns, without building a Stream object per launch -- the step issues ~4000 launches, and the eager step is
    close to host-bound)."""
    return _raw_stream(_get_device())


def ptr(t) -> int | None:
    """Device address of a tensor; an int is an address already (per-call workspaces hand out offsets into one
    allocation instead of a tensor view per buffer)."""
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def require_gpu(*tensors) -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("asrx kernels take device tensors (got a CPU tensor); there is no CPU path")
