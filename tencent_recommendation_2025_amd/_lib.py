"""ctypes binding of libgrk.so (the C ABI declared in include/grk.h).

The library is built in-tree (``make`` at the repo root, or
``__graft_entry__.build()``) and loaded from this package directory.  There is
no fallback: if the library is missing or fails to load, every op raises.
torch is imported first so that the HIP runtime libgrk.so links against
(``libamdhip64.so.7``) resolves to the one torch already loaded -- one runtime,
shared streams.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL: shares torch's HIP runtime)

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
# GRK_LIB: an alternative build of the same library (A/B experiments, scripts/)
LIB_PATH = Path(os.environ.get('GRK_LIB', PKG_DIR / 'libgrk.so'))

GRK_OK, GRK_EINVAL, GRK_EHIP, GRK_EUNSUPPORTED = 0, 1, 2, 3
GRK_F32, GRK_BF16, GRK_F16 = 0, 1, 2
GRK_F32_BF16 = 3  # pair logits: fp32 h, bf16 item embeddings
GRK_FP8_E4M3 = 4  # attention q/k/v: OCP fp8 e4m3
GRK_I32, GRK_I64 = 0, 1
FEAT_SKIP_ROW0 = 1   # GRK_FEAT_SKIP_ROW0
GRK_GEMM_EP_NONE, GRK_GEMM_EP_RELU = 0, 1
BWD_ORDERED, BWD_CHUNKED, BWD_DENSE_BF16 = 0, 1, 2  # grk_embedding_backward flags (bf16 dense: | with CHUNKED)
IDX_PLAIN, IDX_ITEM_MASK, IDX_USER_MASK, IDX_POSITION = 0, 1, 2, 3
ADAM_DENSE, ADAM_LAZY = 0, 1
MAX_FEATURES = 48


class GrkFeature(C.Structure):
    _fields_ = [('table', C.c_void_p), ('idx', C.c_void_p), ('num_rows', C.c_int64), ('idx_ld', C.c_int64),
                ('bag', C.c_int32), ('out_col', C.c_int32), ('idx_mode', C.c_int32), ('flags', C.c_int32)]


class GrkLookup(C.Structure):
    _fields_ = [('idx', C.c_void_p), ('grad', C.c_void_p), ('num_tokens', C.c_int64), ('idx_ld', C.c_int64),
                ('grad_ld', C.c_int64), ('row_offset', C.c_int64), ('table_rows', C.c_int64), ('bag', C.c_int32),
                ('grad_col', C.c_int32), ('idx_mode', C.c_int32), ('pad_', C.c_int32)]


class GrkAdamwHparams(C.Structure):
    _fields_ = [('lr', C.c_float), ('beta1', C.c_float), ('beta2', C.c_float), ('eps', C.c_float),
                ('weight_decay', C.c_float), ('step_size', C.c_float), ('bias_corr2_sqrt', C.c_float),
                ('pad_', C.c_float)]


class GrkAttnArgs(C.Structure):
    _fields_ = [('kind', C.c_int32), ('batch', C.c_int32), ('heads', C.c_int32), ('seq_len', C.c_int32),
                ('head_dim', C.c_int32), ('num_buckets', C.c_int32), ('q', C.c_void_p), ('k', C.c_void_p),
                ('v', C.c_void_p), ('ldq', C.c_int64), ('ldk', C.c_int64), ('ldv', C.c_int64),
                ('key_valid', C.c_void_p), ('rab', C.c_void_p), ('scale', C.c_float), ('inv_n', C.c_float),
                ('dropout_p', C.c_float), ('precise', C.c_int32), ('seed', C.c_uint64), ('out_dtype', C.c_int32),
                ('act', C.c_int32), ('seq_range', C.c_void_p), ('seed_dev', C.c_void_p), ('qkv_dtype', C.c_int32),
                ('timestamps', C.c_void_p), ('rab_t', C.c_void_p), ('num_time_buckets', C.c_int32),
                ('drab_t', C.c_void_p), ('drab_t_ws', C.c_void_p), ('row_base', C.c_void_p),
                ('num_rows', C.c_void_p), ('capacity', C.c_int64)]


class GrkGradRange(C.Structure):
    _fields_ = [('row_start', C.c_int64), ('row_end', C.c_int64), ('grad', C.c_void_p), ('grad_ld', C.c_int64),
                ('grad_dtype', C.c_int32), ('pad_', C.c_int32)]


class GrkRowCopy(C.Structure):
    _fields_ = [('src', C.c_void_p), ('dst', C.c_void_p), ('row_bytes', C.c_int64), ('src_ld', C.c_int64),
                ('dst_ld', C.c_int64)]


class GrkIndexBlock(C.Structure):
    _fields_ = [('src', C.c_void_p), ('src_ld', C.c_int64), ('width', C.c_int64), ('out_col', C.c_int64),
                ('offset', C.c_int64)]


class GrkColumnBlock(C.Structure):
    _fields_ = [('src', C.c_void_p), ('src_ld', C.c_int64), ('width', C.c_int32), ('out_col', C.c_int32),
                ('src_dtype', C.c_int32), ('pad_', C.c_int32)]


class GrkPackRange(C.Structure):
    _fields_ = [('src', C.c_void_p), ('count', C.c_int64), ('dst_offset', C.c_int64), ('src_dtype', C.c_int32),
                ('pad_', C.c_int32)]


class GrkRemapRole(C.Structure):
    _fields_ = [('inv', C.c_void_p), ('out', C.c_void_p), ('ids', C.c_void_p), ('tt', C.c_void_p),
                ('tt_want', C.c_int64), ('n', C.c_int64)]


class GrkGemmGroup(C.Structure):
    _fields_ = [('a', C.c_void_p), ('lda', C.c_int64), ('b', C.c_void_p), ('ldb', C.c_int64), ('c', C.c_void_p),
                ('ldc', C.c_int64), ('rows', C.c_int64), ('b_rows', C.c_int64)]


class GrkStoreView(C.Structure):
    _fields_ = [('sparse', C.c_void_p), ('arr', C.c_void_p), ('arr_len', C.c_void_p), ('mm', C.c_void_p),
                ('tokens', C.c_int64), ('f_sparse', C.c_int32), ('f_array', C.c_int32), ('a_cap', C.c_int32),
                ('f_mm', C.c_int32)]


class GrkStoreCol(C.Structure):
    _fields_ = [('kind', C.c_int32), ('src_col', C.c_int32), ('width', C.c_int32), ('pad_', C.c_int32),
                ('mm_rows', C.c_int64), ('mm_table', C.c_void_p), ('out', C.c_void_p)]


STORE_SPARSE, STORE_ARRAY, STORE_MM = 0, 1, 2
ATTN_SOFTMAX, ATTN_HSTU = 0, 1
ATTN_BWD_DQ, ATTN_BWD_DKDV = 1, 2
ATTN_BWD_WS_CLEAN, ATTN_BWD_DRAB_SET = 4, 8   # grk.h: clean drab scratch kept by the caller; drab written
ACT_NONE, ACT_SILU = 0, 1


class GrkError(RuntimeError):
    pass


_P, _I, _I64, _SZ, _F = C.c_void_p, C.c_int, C.c_int64, C.c_size_t, C.c_float

# name -> (restype, argtypes).  Kept in sync with include/grk.h; the CPU test
# suite checks that every symbol the header declares is exported and listed.
SIGNATURES = {
    'grk_last_error': (C.c_char_p, []),
    'grk_version': (C.c_char_p, []),
    'grk_stream_create': (_I, [C.POINTER(C.c_void_p)]),
    'grk_stream_create_priority': (_I, [C.POINTER(C.c_void_p), _I]),
    'grk_stream_destroy': (_I, [_P]),
    'grk_embedding_gather': (_I, [C.POINTER(GrkFeature), _I, _I, _I, _I, _I64, _P, C.c_int32, _P, _I64, _P, _P]),
    'grk_silu_fp8': (_I, [_P, _I64, _I64, _I, _P, _I64, _P]),
    'grk_dsilu_mul': (_I, [_P, _I64, _P, _I64, _I64, _I, _P]),
    'grk_emb_combine_fwd': (_I, [_P, _I64, _P, _I64, _P, _I64, _F, _I, _I64, _I, _F, C.c_uint64, _P, _P, _I64, _P]),
    'grk_emb_combine_bwd': (_I, [_P, _I64, _P, _I64, _P, _I64, _F, _I, _I64, _I, _F, C.c_uint64, _P, _P, _I64, _P,
                                 _I64, _P, _I64, _P]),
    'grk_embedding_backward_workspace': (_SZ, [_I64, _I64, _I]),
    'grk_embedding_chunked_size': (_I, []),
    'grk_sort_pairs_workspace': (_SZ, [_I64]),
    'grk_sort_pairs': (_I, [_P, _P, _P, _P, _P, _P, _I64, _I, _P, _SZ, _P]),
    'grk_embedding_backward': (_I, [C.POINTER(GrkLookup), _I, _I, _I, _I, _P, C.c_int32, _I64, _I64, _P, _P, _P,
                                    _P, _P, _I, _P, _SZ, _P, _P]),
    'grk_table_adamw': (_I, [_P, _I, _P, _P, _I64, _I, _P, _P, _P, _I64, _P, GrkAdamwHparams, _I, _P]),
    'grk_table_adamw_dense': (_I, [_P, _I, _P, _P, _I64, _I, _P, _I, _I64, GrkAdamwHparams, _P]),
    'grk_table_adamw_catchup': (_I, [_P, _I, _P, _P, _I64, _I, _P, _P, _I64, _P, C.c_int32, C.c_int32, _P]),
    'grk_stamp_rows': (_I, [_P, _P, _P, _I64, C.c_int32, _P]),
    'grk_table_adamw_dev': (_I, [_P, _I, _P, _P, _I64, _I, _P, _P, _P, _I64, _P, _P, C.c_int32, _P, _I, _P]),
    'grk_table_adamw_dense_dev': (_I, [_P, _I, _P, _P, _I64, _I, _P, _I, _I64, _P, C.c_int32, _P, _P]),
    'grk_table_adamw_catchup_dev': (_I, [_P, _I, _P, _P, _I64, _I, _P, _P, _I64, _P, C.c_int32, _P, _P]),
    'grk_table_adamw_catchup_slice_dev': (_I, [_P, _I, _P, _P, _I64, _I, _P, _P, C.c_int32, _P, C.c_int32, _P]),
    'grk_stamp_rows_dev': (_I, [_P, _P, _P, _I64, _P, _P]),
    'grk_table_l2_norm_workspace': (_SZ, []),
    'grk_table_adamw_ranges_dev': (_I, [_P, _I, _P, _P, _I64, _I, C.POINTER(GrkGradRange), _I, _P, C.c_int32, _P, _P,
                                       _P]),
    'grk_table_l2_norm': (_I, [_P, _I, _I64, _I, _F, _P, _P, _P, _SZ, _P]),
    'grk_table_adamw_l2_dev': (_I, [_P, _I, _P, _P, _I64, _I, _P, _P, _P, _I64, _P, _P, C.c_int32, _P, _P, _P]),
    'grk_attention_fwd': (_I, [C.POINTER(GrkAttnArgs), _P, _I64, _P, _P]),
    'grk_attention_fidelity_supported': (_I, [_I, _I]),
    'grk_attention_bwd': (_I, [C.POINTER(GrkAttnArgs), _P, _I64, _P, _I64, _I, _P, _P, _P, _I64, _P, _I64, _P, _I64,
                               _P, _P, _P]),
    'grk_attention_bwd_parts': (_I, [C.POINTER(GrkAttnArgs), _P, _I64, _P, _I64, _I, _P, _P, _P, _I64, _P, _I64,
                                     _P, _I64, _P, _P, _I, _P]),
    'grk_norm_gate_fwd': (_I, [_P, _I64, _P, _I64, _P, _P, _F, _I64, _I, _F, C.c_uint64, _P, _P, _I64, _P, _P]),
    'grk_norm_gate_bwd_workspace': (_SZ, [_I64, _I]),
    'grk_norm_gate_bwd': (_I, [_P, _I64, _P, _I64, _P, _I64, _P, _P, _P, _I64, _I, _F, C.c_uint64, _P, _P, _I64, _P,
                               _I64, _P, _P, _P, _SZ, _P]),
    'grk_seq_ranges': (_I, [_P, _I, _I, _P, _P]),
    'grk_jagged_layout': (_I, [_P, _I, _I, _I64, _P, _P, _P, _P, _P, _P, _P]),
    'grk_gather_rows': (_I, [C.POINTER(GrkRowCopy), _I, _P, _I64, _P]),
    'grk_proj_index': (_I, [C.POINTER(GrkIndexBlock), _I, _I, _I64, _P, _I64, _P]),
    'grk_write_columns': (_I, [C.POINTER(GrkColumnBlock), _I, _I64, _P, _I64, _I, _P]),
    'grk_batch_row_ids': (_I, [_P, _P, _P, _P, _I, _I64, _P, _P, _P]),
    'grk_route_workspace': (_SZ, [_I, _I64]),
    'grk_route': (_I, [_P, _I64, _I, _I64, _I64, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    'grk_flat_pack': (_I, [C.POINTER(GrkPackRange), _I, _P, _P]),
    'grk_jagged_remap': (_I, [C.POINTER(GrkRemapRole), _I, _P, _I64, _P]),
    'grk_add_norm_fwd': (_I, [_P, _I64, _P, _I64, _P, _P, _F, _I64, _I, _P, _I64, _P, _I64, _I, _P, _P]),
    'grk_add_norm_bwd_workspace': (_SZ, [_I64, _I]),
    'grk_add_norm_bwd': (_I, [_P, _I64, _I, _P, _I64, _P, _I64, _P, _P, _I64, _I, _P, _I64, _P, _P, _P, _SZ, _P]),
    'grk_gemm_tuning': (_I, [_I]),
    'grk_wgrad_workspace': (_SZ, [_I64, _I64, _I64]),
    'grk_wgrad': (_I, [_P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _I, _P, _P, _SZ, _P]),
    'grk_grouped_gemm': (_I, [C.POINTER(GrkGemmGroup), _I, _I, _I64, _I64, _I, _P]),
    'grk_grouped_wgrad_workspace': (_SZ, [C.POINTER(GrkGemmGroup), _I, _I64, _I64]),
    'grk_grouped_wgrad': (_I, [C.POINTER(GrkGemmGroup), _I, _I64, _I64, _P, _SZ, _P]),
    'grk_mips_topk_workspace': (_SZ, [_I64, _I64]),
    'grk_mips_topk': (_I, [_P, _I64, _P, _I64, _I, _I64, _I64, _I, _I, _P, _P, _P, _P, _SZ, _P]),
    'grk_sample_negatives': (_I, [_P, _P, _I64, _I, _P, _I, _I64, C.c_uint64, _I, _P, _I, _P, _P, _P, _P, _P]),
    'grk_store_features': (_I, [C.POINTER(GrkStoreView), _P, _P, _I64, C.POINTER(GrkStoreCol), _I]),
    'grk_store_array_widths': (_I, [C.POINTER(GrkStoreView), _P, _P, _I64, _P]),
    'grk_rq_assign': (_I, [_P, _I64, _P, _I64, _I, _I, _I, _P, _P, _P, _P, _P]),
    'grk_gemm': (_I, [_I, _I, _I64, _I64, _I64, _P, _I64, _P, _I64, _I, _P, _I64, _I, _P, _F, _F, _P, _I, _P]),
    'grk_gemm_ex': (_I, [_I, _I, _I64, _I64, _I64, _P, _I64, _P, _I64, _I, _P, _I64, _I, _P, _F, _F, _P, _I, _I, _P]),
    'grk_gemm_mfma_supported': (_I, [_I, _I, _I64, _I64, _I64, _I64, _I64, _I64, _I, _F, _F]),
    'grk_gemm_mfma': (_I, [_I, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _I, _P, _P, _I, _I, _P]),
    'grk_pair_logits_partials': (_SZ, [_I64]),
    'grk_sampled_softmax_workspace': (_SZ, [_I64, _I]),
    'grk_sampled_softmax_fwd': (_I, [_P, _I64, _P, _I64, _P, _P, _I64, _I, _F, _P, _P, _P, _P, _P, _SZ, _P]),
    'grk_sampled_softmax_bwd': (_I, [_P, _I64, _P, _I64, _P, _P, _I64, _I, _F, _P, _P, _P, _P, _I64, _P, _I64, _P,
                                     _SZ, _P]),
    'grk_pair_logits_fwd': (_I, [_P, _I64, _P, _I64, _P, _I64, _P, _I64, _I, _I, _P, _P, _P, _P, _P, _P]),
    'grk_pair_logits_bwd': (_I, [_P, _I64, _P, _I64, _P, _I64, _I64, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I64,
                                 _P, _I64, _P, _I64, _P]),
}

_lib = None


def build(verbose: bool = False) -> Path:
    """Compile libgrk.so in-tree with hipcc (make)."""
    jobs = str(min(16, os.cpu_count() or 4))
    r = subprocess.run(['make', '-j', jobs], cwd=REPO_DIR, capture_output=not verbose, text=True)
    if r.returncode != 0:
        raise GrkError(f'building libgrk.so failed:\n{r.stdout}\n{r.stderr}')
    return LIB_PATH


def lib():
    """The loaded library (raises if it is not built)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise GrkError(f'{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first')
        handle = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != GRK_OK:
        msg = lib().grk_last_error().decode(errors='replace')
        raise GrkError(f'{what} failed (code {rc}): {msg}')


def stream_ptr(device=None) -> int:
    """Raw hipStream_t of torch's current stream."""
    return torch.cuda.current_stream(device).cuda_stream


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return GRK_F32
    if t == torch.bfloat16:
        return GRK_BF16
    if t == torch.float16:
        return GRK_F16
    raise GrkError(f'unsupported dtype {t} (float32 / bfloat16 / float16)')


def itype_code(t: torch.dtype) -> int:
    if t == torch.int64:
        return GRK_I64
    if t == torch.int32:
        return GRK_I32
    raise GrkError(f'unsupported index dtype {t} (int32 / int64 only)')


def loaded_path() -> str | None:
    """Path of libgrk.so as mapped in this process (None if not loaded)."""
    try:
        with open('/proc/self/maps') as f:
            for line in f:
                if line.rstrip().endswith('libgrk.so'):
                    return line.split()[-1]
    except OSError:
        pass
    return None
