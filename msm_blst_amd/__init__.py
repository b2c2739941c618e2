"""msm_blst_amd -- MI355X-native BLS12-381 multi-scalar multiplication.

Host-side Python mirror of the reference's MSM interface (LuoGuiwen/MSM_blst,
a blst v0.3.10 fork).  The compute runs in hand-written HIP kernels for
gfx950 inside libmsm_mi355x.so (include/msm_mi355x.h); this module only
moves bytes and calls the C ABI.

Mirrors:
  blst_p1s_mult_pippenger / blst_p2s_mult_pippenger  (ref bindings/blst.h:238-246, :377-384)
  MSMContext                                          device-resident points (extension)
  ches.CHESContext                                    ref main_p1.cpp CHES driver (see ches.py)
  bgmw.BGMWContext                                    ref main_p1.cpp BGMW95 driver (see bgmw.py)
  wbits.WbitsContext, wbits.precompute / wbits.mult   blst_p{1,2}s_mult_wbits[_precompute] (see wbits.py)
"""
import ctypes

from ._ffi import MsmError, check, lib
from .bgmw import BGMWContext
from .ches import CHESContext
from .wbits import WbitsContext

__all__ = ["MsmError", "MSMContext", "CHESContext", "BGMWContext", "WbitsContext", "p1s_mult_pippenger", "p2s_mult_pippenger", "ps_add", "fixed_points", "gen_scalars",
           "compress", "to_affine", "device_count", "lib"]

POINT_BYTES = {1: 96, 2: 192}
JAC_BYTES = {1: 144, 2: 288}


def device_count():
    return lib().msm_device_count()


def engine_cache_stats():
    """(engines alive, idle, device bytes of idle engines) of the pool behind the
    blst-named entry points (include/msm_mi355x.h msm_engine_cache_stats)."""
    out = (ctypes.c_size_t * 3)()
    lib().msm_engine_cache_stats(out)
    return tuple(out)


def release_engine_cache():
    lib().msm_release_engine_cache()


def set_engine_cache_limit(nbytes):
    return lib().msm_set_engine_cache_limit(nbytes)


def _buf(data):
    if isinstance(data, (bytes, bytearray)):
        return (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data))
    return data


def gen_scalars(n, seed):
    """n 32-byte little-endian scalars < r (SplitMix64)."""
    out = (ctypes.c_uint8 * (32 * n))()
    lib().msm_gen_scalars(out, n, seed)
    return out


def fixed_points(group, n, start=0):
    """P_i = 2^(i+1) G for i in [start, start+n) (ref main_p1.cpp:52-66), blst affine layout."""
    out = (ctypes.c_uint8 * (POINT_BYTES[group] * n))()
    getattr(lib(), f"msm_p{group}_fixed_points_range")(out, start, n)
    return out


def compress(group, jac):
    out = (ctypes.c_uint8 * (48 * group))()
    getattr(lib(), f"msm_p{group}_compress")(out, _buf(jac))
    return bytes(out)


def to_affine(group, jac):
    out = (ctypes.c_uint8 * POINT_BYTES[group])()
    getattr(lib(), f"msm_p{group}_to_affine")(out, _buf(jac))
    return bytes(out)


def _mult(group, points, scalars, n, nbits):
    """blst calling convention with the {ptr, NULL} flat shortcut (multi_scalar.c:393-416)."""
    pts = _buf(points)
    sc = _buf(scalars)
    pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
    sp = (ctypes.c_void_p * 2)(ctypes.cast(sc, ctypes.c_void_p), None)
    ret = (ctypes.c_uint8 * JAC_BYTES[group])()
    getattr(lib(), f"blst_p{group}s_mult_pippenger")(ret, pp, n, sp, nbits, None)
    return bytes(ret)


def p1s_mult_pippenger(points, scalars, n, nbits=255):
    """G1 MSM; scalars packed with stride (nbits+7)//8.  Returns blst_p1 bytes (Jacobian)."""
    return _mult(1, points, scalars, n, nbits)


def p2s_mult_pippenger(points, scalars, n, nbits=255):
    return _mult(2, points, scalars, n, nbits)


def ps_add(group, points, n):
    """Sum of n affine points (blst_p1s_add / blst_p2s_add, ref bulk_addition.c:145-164), flat array."""
    pts = _buf(points)
    pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
    ret = (ctypes.c_uint8 * JAC_BYTES[group])()
    getattr(lib(), f"blst_p{group}s_add")(ret, pp, n)
    return bytes(ret)


class MSMContext:
    """Device-resident points on one GPU; repeated MSMs over new scalars.

    window_bits: Pippenger window c (bucket count 2^(c-1) per window); 0 = 16.
    """

    def __init__(self, group=1, device=0, window_bits=0):
        self.group = group
        self._ctx = ctypes.c_void_p()
        check(lib().msm_ctx_create(ctypes.byref(self._ctx), group, device, window_bits))
        self.n = 0

    def set_points(self, points, n, on_device=False, stream=None):
        ptr = points if on_device else _buf(points)
        check(lib().msm_ctx_set_points(self._ctx, ptr, n, int(bool(on_device)), stream))
        self.n = n

    def mult(self, scalars, nbits=255, stride=32, on_device=False, stream=None):
        ret = (ctypes.c_uint8 * JAC_BYTES[self.group])()
        ptr = scalars if on_device else _buf(scalars)
        check(lib().msm_ctx_mult(self._ctx, ret, ptr, stride, nbits, int(bool(on_device)), stream))
        return bytes(ret)

    def mult_batch(self, scalars, count, nbits=255, stride=32, set_stride=None, on_device=False, stream=None):
        """`count` pipelined MSMs (scalar set k at k * set_stride bytes); returns a
        list of Jacobian byte strings, equal to `count` mult() calls."""
        if set_stride is None:
            set_stride = self.n * stride
        nb = JAC_BYTES[self.group]
        rets = (ctypes.c_uint8 * (nb * count))()
        ptr = scalars if on_device else _buf(scalars)
        check(lib().msm_ctx_mult_batch(self._ctx, rets, ptr, stride, set_stride, nbits, count, int(bool(on_device)),
                                       stream))
        raw = bytes(rets)
        return [raw[k * nb:(k + 1) * nb] for k in range(count)]

    def set_profiling(self, on=True):
        check(lib().msm_ctx_set_profiling(self._ctx, int(on)))

    def phase_times(self):
        out = (ctypes.c_float * 6)()
        check(lib().msm_ctx_phase_times(self._ctx, out))
        return dict(zip(("digits", "sort", "accumulate", "reduce", "finalize", "total"), list(out)))

    def close(self):
        if self._ctx:
            lib().msm_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
