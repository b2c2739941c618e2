"""ctypes binding of libmsm_mi355x.so (include/msm_mi355x.h).

The library is the product: loading fails loudly if it is missing or was
built for another architecture -- there is no CPU fallback anywhere in
msm_blst_amd.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmsm_mi355x.so")

_lib = None


class MsmError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MsmError(f"{LIB_PATH} not built: run `python -m msm_blst_amd.build` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    for g in (1, 2):
        f = getattr(L, f"blst_p{g}s_mult_pippenger")
        f.argtypes = [vp, vp, sz, vp, sz, vp]
        f.restype = None
        f = getattr(L, f"blst_p{g}s_tile_pippenger")
        f.argtypes = [vp, vp, sz, vp, sz, vp, sz, sz]
        f.restype = None
        f = getattr(L, f"blst_p{g}s_mult_pippenger_scratch_sizeof")
        f.argtypes = [sz]
        f.restype = sz
        getattr(L, f"msm_p{g}_fixed_points").argtypes = [vp, sz]
        getattr(L, f"msm_p{g}_fixed_points_range").argtypes = [vp, sz, sz]
        for name in (f"msm_p{g}_to_affine", f"msm_p{g}_compress"):
            getattr(L, name).argtypes = [vp, vp]
        getattr(L, f"msm_p{g}_add").argtypes = [vp, vp, vp]
    L.msm_last_error.restype = ctypes.c_char_p
    L.msm_device_count.restype = i32
    L.msm_ctx_create.argtypes = [ctypes.POINTER(vp), i32, i32, i32]
    L.msm_ctx_set_points.argtypes = [vp, vp, sz, i32, vp]
    L.msm_ctx_mult.argtypes = [vp, vp, vp, sz, sz, i32, vp]
    L.msm_ctx_mult_batch.argtypes = [vp, vp, vp, sz, sz, sz, sz, i32, vp]
    L.msm_ctx_set_profiling.argtypes = [vp, i32]
    L.msm_ctx_phase_times.argtypes = [vp, vp]
    L.msm_ctx_destroy.argtypes = [vp]
    L.msm_ctx_destroy.restype = None
    L.msm_gen_scalars.argtypes = [vp, sz, u64]
    L.msm_test_field.argtypes = [i32, i32, vp, vp, vp, sz]
    L.msm_test_xyzz.argtypes = [i32, vp, sz, vp, i32, sz, vp]
    pp = ctypes.POINTER(vp)
    L.msm_ches_params.argtypes = [i32, i32, vp]
    L.msm_ches_ctx_create.argtypes = [pp, i32, i32, i32, i32]
    L.msm_ches_ctx_create_params.argtypes = [pp, i32, i32, vp]
    L.msm_ches_ctx_create_multi.argtypes = [pp, i32, vp, i32, i32, i32]
    L.msm_ches_ctx_shards.argtypes = [vp]
    L.msm_ches_ctx_build_table.argtypes = [vp, vp, sz, i32, vp]
    L.msm_ches_ctx_set_table.argtypes = [vp, vp, sz, i32, vp]
    L.msm_ches_ctx_get_table.argtypes = [vp, vp, sz, sz]
    L.msm_ches_ctx_mult.argtypes = [vp, vp, vp, sz, i32, vp]
    L.msm_ches_ctx_mult_batch.argtypes = [vp, vp, vp, sz, sz, sz, i32, vp]
    L.msm_ches_ctx_set_profiling.argtypes = [vp, i32]
    L.msm_ches_ctx_phase_times.argtypes = [vp, vp]
    L.msm_ches_ctx_bucket_count.argtypes = [vp]
    L.msm_ches_ctx_bucket_count.restype = sz
    L.msm_register_host_table.argtypes = [i32, vp, sz]
    L.msm_unregister_host_table.argtypes = [vp]
    L.msm_ches_ctx_batch_lanes.argtypes = [vp]
    L.msm_ches_ctx_rccl_exchange.argtypes = [vp]
    L.msm_ches_ctx_time_accumulation.argtypes = [vp, vp, sz, i32, i32, vp]
    L.msm_ches_ctx_destroy.argtypes = [vp]
    L.msm_ches_ctx_destroy.restype = None
    L.msm_ches_bucket_set.argtypes = [i32, i32, vp, sz]
    L.msm_ches_bucket_set.restype = sz
    L.msm_ches_digit_table.argtypes = [i32, i32, vp]
    for g in (1, 2):
        f = getattr(L, f"blst_p{g}s_mult_wbits_precompute_sizeof")
        f.argtypes, f.restype = [sz, sz], sz
        f = getattr(L, f"blst_p{g}s_mult_wbits_scratch_sizeof")
        f.argtypes, f.restype = [sz], sz
        f = getattr(L, f"blst_p{g}s_mult_wbits_precompute")
        f.argtypes, f.restype = [vp, sz, vp, sz], None
        f = getattr(L, f"blst_p{g}s_mult_wbits")
        f.argtypes, f.restype = [vp, vp, sz, sz, vp, sz, vp], None
    if hasattr(L, "msm_release_engine_cache"):  # (absent from older builds used in A/B runs)
        L.msm_release_engine_cache.argtypes = []
        L.msm_release_engine_cache.restype = None
        L.msm_engine_cache_stats.argtypes = [vp]
        L.msm_engine_cache_stats.restype = None
        L.msm_set_engine_cache_limit.argtypes = [sz]
        L.msm_set_engine_cache_limit.restype = sz
    L.msm_set_abort_on_error.argtypes = [i32]
    L.msm_error_pending.argtypes = []
    L.msm_wbits_ctx_create.argtypes = [pp, i32, i32, i32]
    L.msm_wbits_ctx_precompute.argtypes = [vp, vp, sz, i32, vp]
    L.msm_wbits_ctx_set_table.argtypes = [vp, vp, sz, i32, vp]
    L.msm_wbits_ctx_get_table.argtypes = [vp, vp, sz, sz]
    L.msm_wbits_ctx_mult.argtypes = [vp, vp, vp, sz, sz, i32, vp]
    L.msm_wbits_ctx_table_rows.argtypes = [vp]
    L.msm_wbits_ctx_table_rows.restype = sz
    L.msm_wbits_ctx_destroy.argtypes = [vp]
    L.msm_wbits_ctx_destroy.restype = None
    L.msm_bgmw_ctx_create.argtypes = [pp, i32, i32, i32, i32]
    L.msm_bgmw_ctx_build_table.argtypes = [vp, vp, sz, i32, vp]
    L.msm_bgmw_ctx_set_table.argtypes = [vp, vp, sz, i32, vp]
    L.msm_bgmw_ctx_get_table.argtypes = [vp, vp, sz, sz]
    L.msm_bgmw_ctx_mult.argtypes = [vp, vp, vp, sz, i32, vp]
    L.msm_bgmw_ctx_set_profiling.argtypes = [vp, i32]
    L.msm_bgmw_ctx_phase_times.argtypes = [vp, vp]
    L.msm_bgmw_ctx_bucket_count.argtypes = [vp]
    L.msm_bgmw_ctx_bucket_count.restype = sz
    L.msm_bgmw_ctx_destroy.argtypes = [vp]
    L.msm_bgmw_ctx_destroy.restype = None
    cp = ctypes.c_char_p
    for f in ("msm_ches_ctx_save_table", "msm_ches_ctx_load_table", "msm_bgmw_ctx_save_table",
              "msm_bgmw_ctx_load_table"):
        getattr(L, f).argtypes = [vp, cp]
    for g in (1, 2):
        getattr(L, f"blst_p{g}s_add").argtypes = [vp, vp, sz]
        getattr(L, f"blst_p{g}s_add").restype = None
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise MsmError(f"msm_mi355x error {rc}: {lib().msm_last_error().decode(errors='replace')}")
    return rc
