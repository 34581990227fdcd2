"""ctypes binding of libmirec.so (the C-ABI declared in include/mirec.h).

The library is loaded AFTER ``import torch`` so that its NEEDED
``libamdhip64.so.7`` resolves to the HIP runtime torch already mapped (same
soname): one HIP runtime per process, and ``torch.cuda.current_stream().cuda_stream``
is a valid ``hipStream_t`` for every entry point.

There is no fallback: if the shared library is missing the import of any op
raises, so a GPU run can never silently take a CPU / PyTorch path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_int32, c_int64, c_size_t, c_void_p, c_char_p

import torch  # noqa: F401  (must be imported before the library is dlopen'ed)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MIREC_LIB", os.path.join(_HERE, "_lib", "libmirec.so"))

_P = c_void_p


class RowsRef(ctypes.Structure):
    """struct mirec_rows_ref (include/mirec.h)."""
    _fields_ = [('lo', _P), ('hi', _P), ('split', c_int64)]


class SpmmEpilogue(ctypes.Structure):
    """struct mirec_spmm_epilogue (include/mirec.h)."""
    _fields_ = [('add', RowsRef), ('add_scale', c_float), ('y', RowsRef), ('acc_in', RowsRef),
                ('acc_out', RowsRef), ('acc_scale', c_float)]


class CtxField(ctypes.Structure):
    """struct mirec_ctx_field (include/mirec.h)."""
    _fields_ = [('kind', c_int32), ('seq_len', c_int32), ('ids', _P), ('vals', _P),
                ('offset', c_int64), ('table', _P), ('table1', _P), ('n_rows', c_int64),
                ('grad', _P), ('grad1', _P), ('keys', _P), ('grad_ld', c_int64),
                ('grad1_ld', c_int64)]


MLP_MAX_LAYERS = 6


class MlpDesc(ctypes.Structure):
    """struct mirec_mlp (include/mirec.h, K10)."""
    _L = MLP_MAX_LAYERS
    _fields_ = [('n_layers', c_int32), ('dims', c_int32 * (_L + 1)), ('dropout', c_int32 * _L),
                ('relu', c_int32 * _L), ('tile_start', c_int32 * _L),
                ('keep_threshold', ctypes.c_uint32), ('scale', c_float),
                ('seed', ctypes.c_uint64), ('counter', _P), ('arrive', _P),
                ('W', _P * _L), ('b', _P * _L), ('xs', _P * _L), ('mask0', _P),
                ('gz', _P * _L), ('dW', _P * _L), ('db', _P * _L), ('wscratch', _P),
                ('wcount', _P)]


class FlatParam(ctypes.Structure):
    """struct mirec_flat_param (include/mirec.h)."""
    _fields_ = [('p', _P), ('m', _P), ('v', _P), ('g', _P), ('n', c_int64)]


class AdamTable(ctypes.Structure):
    """struct mirec_adam_table (include/mirec.h)."""
    _fields_ = [('p', _P), ('m', _P), ('v', _P), ('n_rows', c_int64), ('rows', _P),
                ('perm', _P), ('uniq', _P), ('seg', _P), ('n_uniq', _P), ('dense_grad', _P),
                ('last', _P), ('ahead_uniq', _P), ('ahead_n_uniq', _P), ('p_alt', _P)]


class ChunkPrep(ctypes.Structure):
    """struct mirec_chunk_prep (include/mirec.h)."""
    _fields_ = [('users', _P), ('items', _P), ('s0', c_int64),
                ('n_batches', c_int64), ('Bc', c_int64), ('T', c_int64),
                ('user_keys', _P), ('item_keys', _P),
                ('random_list', _P), ('L', c_int64), ('pr_dev', _P),
                ('used_ptr', _P), ('used_cols', _P), ('used_bits', _P), ('n_bits', c_int64),
                ('n_users', c_int64), ('n_items', c_int64), ('reject', c_int32), ('status', _P),
                ('walk_ws', _P), ('walk_ws_bytes', c_size_t), ('sort_ws', _P),
                ('sort_ws_bytes', c_size_t),
                ('u_perm', _P), ('u_uniq', _P), ('u_seg', _P), ('u_nu', _P),
                ('i_perm', _P), ('i_uniq', _P), ('i_seg', _P), ('i_nu', _P),
                ('u_ahead', _P), ('u_nah', _P), ('i_ahead', _P), ('i_nah', _P),
                ('alias_thr', _P), ('alias_idx', _P), ('n_alias', c_int64),
                ('alias_seed', ctypes.c_uint64), ('alias_counter', ctypes.c_uint64),
                ('u_rec', _P), ('u_crec', _P), ('i_rec', _P), ('i_crec', _P),
                ('spec_ws', _P), ('spec_ws_bytes', c_size_t), ('r_mean', c_double),
                ('r_sd', c_double)]


# Every symbol include/mirec.h declares: name -> (restype, argtypes)
SIGNATURES = {
    "mirec_abi_version": (c_int, []),
    "mirec_last_error": (c_char_p, []),
    "mirec_sample_walk_workspace_size": (c_size_t, [c_int64, c_int64]),
    "mirec_sample_walk": (c_int, [_P, c_int64, _P, _P, c_int64, c_int64, c_int64, c_int64,
                                  _P, _P, _P, c_int64, c_int64, c_int, _P, c_int64, _P, _P,
                                  c_size_t, _P]),
    "mirec_sample_walk_segments": (c_int, [_P, c_int64, _P, _P, _P, c_int64, c_int64, c_int64,
                                           _P, _P, _P, c_int64, c_int64, c_int, _P, _P, _P,
                                           c_size_t, _P]),
    "mirec_sample_walk_spec_workspace_size": (c_size_t, [c_int64, c_int64, c_int64, c_double,
                                                         c_double]),
    "mirec_sample_walk_spec": (c_int, [_P, c_int64, _P, _P, _P, c_int64, c_int64, c_int64, _P, _P,
                                       _P, c_int64, c_int64, c_int, c_double, c_double, _P,
                                       c_int64, _P, _P, c_int64, _P, _P, c_size_t, _P]),
    "mirec_used_bitmap_bytes": (c_size_t, [c_int64, c_int64]),
    "mirec_alias_build": (c_int, [_P, c_int64, _P, _P]),
    "mirec_host_counting_order": (c_int, [_P, c_int64, c_int64, _P]),
    "mirec_host_csr_build": (c_int64, [_P, _P, c_int64, c_int64, _P, _P]),
    "mirec_sample_alias": (c_int, [_P, _P, c_int64, ctypes.c_uint64, ctypes.c_uint64, _P, c_int64,
                                   c_int64, c_int64, _P, _P, _P, c_int64, c_int64, c_int, _P,
                                   c_int64, _P, _P]),
    "mirec_shard_keys": (c_int, [_P, c_int64, c_int32, c_int64, _P, _P]),
    "mirec_shard_plan": (c_int, [_P, _P, c_int64, c_int64, c_int64, c_int32, c_int32, c_int32,
                                 c_int64, _P, _P, _P, _P, _P, _P]),
    "mirec_shard_own": (c_int, [_P, _P, _P, _P, c_int64, c_int64, _P, _P, _P, c_int64, c_int64,
                                c_int64, c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "mirec_shard_next": (c_int, [_P, _P, _P, _P, c_int64, c_int64, _P, _P, _P]),
    "mirec_shard_select": (c_int, [_P, c_int64, c_int64, c_int32, c_int64, c_int32, c_int64, _P,
                                   _P, _P, _P]),
    "mirec_shard_own_sel": (c_int, [_P, _P, _P, _P, c_int64, c_int64, _P, _P, _P, c_int64,
                                    c_int64, c_int64, c_int32, _P, c_int64, _P, _P, _P, _P, _P,
                                    _P, _P]),
    "mirec_shard_gather_f32": (c_int, [_P, _P, c_int32, _P, c_int64, _P, _P]),
    "mirec_used_bitmap_build": (c_int, [_P, _P, c_int64, c_int64, _P, _P]),
    "mirec_gather_rows": (c_int, [_P, c_int64, c_int64, _P, c_int64, _P, _P]),
    "mirec_window_gather": (c_int, [_P, c_int32, _P, _P, c_int64, c_int32, _P, _P]),
    "mirec_gather_rows_i32idx": (c_int, [_P, c_int64, c_int64, _P, c_int64, _P, _P]),
    "mirec_bpr_fwd_bwd_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P, _P, c_int64,
                                      c_int32, c_float, c_float, _P, _P, _P, _P, _P, _P]),
    "mirec_bpr_fwd_coef_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P, _P, c_int64,
                                       c_int32, c_float, c_float, _P, _P, _P]),
    "mirec_bpr_contrib_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P, _P, c_int64,
                                      c_int32, _P, c_int64, c_int64, _P, _P, _P]),
    "mirec_dot_rows_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P, c_int64, _P, _P]),
    "mirec_sum_f32": (c_int, [_P, c_int64, _P, _P]),
    "mirec_segment_sort_workspace_size": (c_size_t, [c_int64, c_int64]),
    "mirec_segment_sort": (c_int, [_P, c_int64, c_int64, _P, _P, _P, _P, _P, c_size_t, _P]),
    "mirec_segment_sort_batched": (c_int, [_P, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P,
                                           c_size_t, _P]),
    "mirec_uniq_ahead_diff": (c_int, [_P, _P, c_int64, c_int64, _P, _P, _P]),
    "mirec_segment_sort_blocks_workspace_size": (c_size_t, [c_int64, c_int64]),
    "mirec_segment_sort_onesweep_status_words": (c_int64, [c_int64]),
    "mirec_segment_sort_onesweep": (c_int, [_P, c_int64, c_int64, _P, _P, _P, _P, _P, _P,
                                            c_size_t, _P, c_int64, _P]),
    "mirec_segment_sort_fields_chained": (c_int, [_P, _P, c_int32, c_int64, c_int64, _P, _P, _P,
                                                  _P, _P, _P, c_int64, _P, _P]),
    "mirec_segment_sort_blocks": (c_int, [_P, c_int64, c_int64, c_int64, _P, _P, _P, _P, _P,
                                          c_size_t, _P]),
    "mirec_segment_sort_blocks_chained": (c_int, [_P, c_int64, c_int64, c_int64, _P, _P, _P, _P,
                                                  _P, c_int64, _P, _P]),
    "mirec_prepare_chunk": (c_int, [_P, _P]),
    "mirec_prepare_chunk_walk": (c_int, [_P, _P]),
    "mirec_prepare_chunk_group": (c_int, [_P, _P]),
    "mirec_write_bytes": (c_int, [_P, _P, c_size_t, _P]),
    "mirec_linear_shape_ok": (c_int, [c_int32, c_int32]),
    "mirec_linear_fwd_f32": (c_int, [_P, c_int64, c_int32, c_int32, _P, _P, _P, _P]),
    "mirec_linear_bwd_data_acc_f32": (c_int, [_P, c_int64, c_int32, c_int32, _P, _P, _P, _P]),
    "mirec_linear_bwd_data_f32": (c_int, [_P, c_int64, c_int32, c_int32, _P, _P, c_int32, _P]),
    "mirec_add_ln_drop_fwd_f32": (c_int, [_P, _P, c_int64, c_int32, _P, _P, c_float, c_float,
                                          ctypes.c_uint64, _P, _P, _P, _P, _P, _P]),
    "mirec_add_ln_drop_bwd_f32": (c_int, [_P, _P, c_int64, c_int32, _P, _P, _P, _P, c_float,
                                          ctypes.c_uint64, _P, _P, _P, _P, _P, _P, _P]),
    "mirec_attn_fwd_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int32, c_int32, c_float,
                                   ctypes.c_uint64, _P, _P, _P, _P, _P]),
    "mirec_attn_bwd_f32": (c_int, [_P, _P, _P, _P, _P, _P, _P, _P, c_int64, c_int32, c_int32,
                                   c_float, _P, _P, _P, _P]),
    "mirec_seq_attn_mask_f32": (c_int, [_P, c_int64, c_int32, _P, _P]),
    "mirec_gelu_fwd_f32": (c_int, [_P, c_int64, _P, _P]),
    "mirec_gelu_bwd_f32": (c_int, [_P, _P, c_int64, _P, _P]),
    "mirec_add_ln_fwd_f32": (c_int, [_P, _P, c_int64, c_int32, _P, _P, c_float, _P, _P, _P, _P]),
    "mirec_add_ln_bwd_f32": (c_int, [_P, _P, c_int64, c_int32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mirec_copy_many": (c_int, [_P, _P, _P, c_int, _P]),
    "mirec_selftest_adam_math": (c_int, [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, _P, _P]),
    "mirec_segment_reduce_f32": (c_int, [_P, c_int32, _P, _P, _P, _P, c_int64, _P, _P, c_size_t,
                                         _P]),
    "mirec_segment_reduce_pos_seg_f32": (c_int, [_P, c_int32, _P, _P, _P, _P, _P, c_int64, _P,
                                                 _P, c_size_t, _P]),
    "mirec_segment_merge2_f32": (c_int, [_P, _P, c_int64, _P, _P, _P, c_int64, _P, c_int32,
                                         c_int32, _P, _P, _P, _P, c_size_t, _P, c_int64, _P]),
    "mirec_segment_reduce2_f32": (c_int, [_P, c_int32, _P, _P, _P, _P, _P, c_int64, _P, _P, _P,
                                          c_size_t, _P]),
    "mirec_segment_reduce2_pos_seg_f32": (c_int, [_P, c_int32, _P, _P, _P, _P, _P, _P, c_int64,
                                                  _P, _P, _P, c_size_t, _P]),
    "mirec_segment_scatter_add_workspace_size": (c_size_t, [c_int64, c_int32]),
    "mirec_segment_scatter_add_f32": (c_int, [_P, c_int32, _P, _P, _P, _P, c_int64, _P,
                                              c_int64, _P, c_size_t, _P]),
    "mirec_adam_sparse_grad_f32": (c_int, [_P, _P, _P, c_int64, c_int32, _P, _P, _P, _P, _P,
                                           c_int64, _P, _P, _P, c_double, c_double, c_double,
                                           c_double, _P]),
    "mirec_adam_flat_multi_f32": (c_int, [ctypes.POINTER(FlatParam), c_int32, _P, _P, c_double,
                                          c_double, c_double, c_double, _P]),
    "mirec_adam_flat_multi_advance_f32": (c_int, [ctypes.POINTER(FlatParam), c_int32, _P, _P, _P,
                                                  c_double, c_double, c_double, c_double, _P]),
    "mirec_adam_flat_f32": (c_int, [_P, _P, _P, c_int64, _P, _P, _P, c_double, c_double,
                                    c_double, c_double, _P]),
    "mirec_adam_multi_f32": (c_int, [ctypes.POINTER(AdamTable), c_int32, c_int32, _P, _P,
                                     c_int32, c_double, c_double, c_double, c_double, _P]),
    "mirec_adam_deferred_f32": (c_int, [ctypes.POINTER(AdamTable), c_int32, _P, c_int32, _P,
                                        _P, c_int32, c_double, c_double, c_double, c_double,
                                        _P]),
    "mirec_adam_deferred_pair_f32": (c_int, [ctypes.POINTER(AdamTable), _P, c_int32, _P, _P,
                                             c_int32, c_double, c_double, c_double, c_double,
                                             _P]),
    "mirec_adam_flush_f32": (c_int, [ctypes.POINTER(AdamTable), c_int32, c_int32, _P, _P,
                                     c_int32, c_double, c_double, c_double, c_double, _P]),
    "mirec_adam_flush_rows_f32": (c_int, [ctypes.POINTER(AdamTable), c_int32, c_int32, _P, _P,
                                          _P, c_int32, c_double, c_double, c_double, c_double,
                                          _P]),
    "mirec_bpr_adam_step_f32": (c_int, [ctypes.POINTER(AdamTable), _P, c_int32, _P, c_int64,
                                        c_int32, ctypes.c_float, ctypes.c_float, _P, _P, _P,
                                        _P, _P, _P, _P, _P, _P, _P, _P, c_int32, c_double,
                                        c_double, c_double, c_double, _P]),
    "mirec_step_record_ints": (c_int64, [c_int64]),
    "mirec_colsum_multi_f32": (c_int, [_P, _P, _P, _P, c_int32, _P]),
    "mirec_offset_keys": (c_int, [_P, _P, c_int32, c_int64, _P, _P]),
    "mirec_bpr_fwd_bwd_at_ids_f32": (c_int, [_P, c_int64, c_int32, _P, _P, _P, c_int64, c_int32,
                                             ctypes.c_float, ctypes.c_float, _P, _P, _P]),
    "mirec_chunk_group_fits": (c_int, [c_int64, c_int32, c_int64, c_int64, c_int32]),
    "mirec_chunk_group": (c_int, [_P, _P, c_int64, c_int64, c_int32, c_int64, c_int64] + [_P] * 16
                          + [_P]),
    "mirec_step_records": (c_int, [_P, _P, c_int64, c_int64, c_int32, c_int64, c_int64, _P, _P,
                                   _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _P]),
    "mirec_step_finish": (c_int, [_P, c_int64, c_float, _P, _P, _P]),
    "mirec_chunk_finish": (c_int, [_P, c_int64, c_int64, c_int32, c_float, _P, _P, _P, _P]),
    "mirec_fullsort_topk_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P, _P, _P,
                                        c_int32, _P, _P, _P, _P]),
    "mirec_fullsort_topk_split_workspace_size": (ctypes.c_size_t, [c_int64, c_int32, c_int32]),
    "mirec_fullsort_topk_split_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P, _P, _P,
                                              c_int32, c_int32, _P, ctypes.c_size_t, _P, _P, _P,
                                              _P]),
    "mirec_score_matrix_f32": (c_int, [_P, c_int64, _P, c_int64, c_int32, _P, _P]),
    "mirec_spmm_csr_f32": (c_int, [_P, _P, _P, c_int64, c_int32, _P, _P, _P, c_int64, c_int32,
                                   _P, _P, c_int64, _P, ctypes.POINTER(RowsRef),
                                   ctypes.POINTER(SpmmEpilogue), _P]),
    "mirec_ctx_fm_work_floats": (c_size_t, [c_int64, c_int32, c_int32]),
    "mirec_ctx_fm_fwd_f32": (c_int, [_P, c_int32, c_int64, c_int32, _P, _P, _P, _P, _P]),
    "mirec_ctx_fm_bwd_f32": (c_int, [_P, c_int32, c_int64, c_int32, _P, _P, _P, _P, _P]),
    "mirec_sigmoid_bce_mean_f32": (c_int, [_P, _P, _P, c_int64, c_float, _P, _P, _P, _P]),
    "mirec_sigmoid_bce_f32": (c_int, [_P, _P, _P, c_int64, c_float, _P, _P, _P, _P]),
    "mirec_colsum_f32": (c_int, [_P, c_int64, c_int64, _P, _P]),
    "mirec_mlp_fwd_f32": (c_int, [_P, _P, c_int64, _P, c_int32, _P]),
    "mirec_mlp_bwd_f32": (c_int, [_P, _P, _P, c_int64, _P, _P]),
    "mirec_mlp_bwd_workspace": (c_int, [_P, c_int64, _P, _P]),
    "mirec_linear_grad_finish_scratch": (c_int64, [c_int64, c_int32]),
    "mirec_comm_init": (c_int, [ctypes.c_int, ctypes.c_int, _P, _P]),
    "mirec_comm_handle_bytes": (c_int64, []),
    "mirec_comm_window": (c_int, [_P, c_int64, c_int32, _P, _P]),
    "mirec_comm_connect": (c_int, [_P, _P]),
    "mirec_comm_layout": (c_int, [_P, _P, _P, _P]),
    "mirec_comm_destroy": (c_int, [_P]),
    "mirec_comm_status": (c_int, [_P, _P]),
    "mirec_comm_wait": (c_int, [_P, c_int32, _P]),
    "mirec_comm_config": (c_int, [_P, c_int32]),
    "mirec_comm_push_rows_f32": (c_int, [_P, _P, _P, _P, c_int64, _P]),
    "mirec_comm_bpr_f32": (c_int, [_P, _P, _P, _P, c_int64, c_int32, c_float, c_float, _P,
                                   c_int64, _P]),
    "mirec_comm_adam_deferred_f32": (c_int, [_P, ctypes.POINTER(AdamTable), c_int32, _P, c_int32,
                                             _P, _P, c_int32, c_double, c_double, c_double,
                                             c_double, _P, _P, _P, c_int64, _P]),
    "mirec_alltoallv_rows_f32": (c_int, [_P, _P, _P, _P, _P, c_int32, _P]),
    "mirec_allreduce_sum_f32": (c_int, [_P, _P, c_int64, _P]),
    "mirec_linear_grad_finish_f32": (c_int, [_P, c_int32, c_int64, _P, _P, c_int64, c_int32, _P,
                                             _P, _P, _P]),
    "mirec_seq_embed_ln_fwd_f32": (c_int, [_P, c_int64, _P, _P, c_int64, c_int32, c_int32, _P,
                                           _P, c_float, _P, _P, _P, _P]),
    "mirec_seq_embed_ln_partials": (c_int64, [c_int64]),
    "mirec_seq_embed_ln_bwd_f32": (c_int, [_P, c_int64, _P, _P, c_int64, c_int32, c_int32, _P,
                                           _P, _P, _P, _P, _P, _P, _P, _P]),
    "mirec_seq_embed_ln_drop_fwd_f32": (c_int, [_P, c_int64, _P, _P, c_int64, c_int32, c_int32,
                                                _P, _P, c_float, c_float, ctypes.c_uint64, _P,
                                                _P, _P, _P, _P, _P]),
    "mirec_seq_embed_ln_drop_bwd_f32": (c_int, [_P, c_int64, _P, _P, c_int64, c_int32, c_int32,
                                                _P, _P, _P, _P, c_float, ctypes.c_uint64, _P,
                                                _P, _P, _P, _P, _P, _P]),
    "mirec_scale_by_f32": (c_int, [_P, c_int64, _P, _P]),
    "mirec_sampled_softmax_f32": (c_int, [_P, _P, c_int64, c_int32, _P, _P, c_int64, c_int32,
                                          c_float, _P, _P, _P, _P]),
    "mirec_rank_of_pos_f32": (c_int, [_P, _P, c_int64, c_int32, _P, _P, c_int64, c_int32, _P,
                                      _P]),
    "mirec_gather_sqnorm_f32": (c_int, [_P, c_int64, c_int32, _P, c_int64, _P, _P]),
    "mirec_gather_scale_rows_f32": (c_int, [_P, c_int64, c_int32, _P, c_int64, _P, _P, _P]),
}

ABI_VERSION = 18


class NativeError(RuntimeError):
    pass


_lib = None


def lib():
    """Return the loaded library (loads it on first use); raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            f"libmirec.so not found at {LIB_PATH}: build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
    handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if handle.mirec_abi_version() != ABI_VERSION:
        raise NativeError("libmirec.so ABI version mismatch; rebuild it")
    _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().mirec_last_error()
        raise NativeError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    """hipStream_t of the current stream of `device` (default: the current device).
    The raw-stream query skips torch.cuda.current_stream's Python device
    resolution (≈ 10 µs per call on the launch path)."""
    if device is None:
        return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())
    if isinstance(device, torch.device):
        device = device.index if device.index is not None else torch._C._cuda_getDevice()
    return torch._C._cuda_getCurrentRawStream(int(device))
