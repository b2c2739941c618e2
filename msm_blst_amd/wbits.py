"""blst's fixed-window MSM with a precomputed table of multiples.

Python mirror of ref src/multi_scalar.c:63-261 (blst.h:228-236, :367-375) and of
the C++ binding's P1_Affines / P2_Affines (ref bindings/blst.hpp:362-430):
  p{1,2}s_mult_wbits_precompute(points, n, wbits) -> table (blst layout: row i
      holds the canonical affine multiples (k+1) P_i, k < 2^(wbits-1))
  p{1,2}s_mult_wbits(table, wbits, n, scalars, nbits) -> Jacobian
  WbitsContext: the same with the table resident in HBM (msm_wbits_ctx_*).
All compute runs in libmsm_mi355x.so (HIP, gfx950).
"""
import ctypes

from ._ffi import check, lib

AFF = {1: 96, 2: 192}
JAC = {1: 144, 2: 288}


def _buf(data):
    if isinstance(data, (bytes, bytearray)):
        return (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data))
    return data


def precompute_sizeof(group, wbits, n):
    return getattr(lib(), f"blst_p{group}s_mult_wbits_precompute_sizeof")(wbits, n)


def precompute(group, points, n, wbits):
    """Table of multiples for n flat blst affine points ({ptr, NULL} convention)."""
    pts = _buf(points)
    table = (ctypes.c_uint8 * precompute_sizeof(group, wbits, n))()
    pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
    getattr(lib(), f"blst_p{group}s_mult_wbits_precompute")(table, wbits, pp, n)
    return table


def mult(group, table, wbits, n, scalars, nbits):
    """sum_i s_i P_i over flat scalars packed with stride (nbits+7)//8."""
    sc = _buf(scalars)
    sp = (ctypes.c_void_p * 2)(ctypes.cast(sc, ctypes.c_void_p), None)
    ret = (ctypes.c_uint8 * JAC[group])()
    getattr(lib(), f"blst_p{group}s_mult_wbits")(ret, _buf(table), wbits, n, sp, nbits, None)
    return bytes(ret)


class WbitsContext:
    """One GPU, one point set, table resident in HBM."""

    def __init__(self, group=1, device=0, wbits=8):
        self.group, self.wbits = group, wbits
        self._ctx = ctypes.c_void_p()
        check(lib().msm_wbits_ctx_create(ctypes.byref(self._ctx), group, device, wbits))
        self.n = 0

    def precompute(self, points, n, on_device=False, stream=None):
        check(lib().msm_wbits_ctx_precompute(self._ctx, points if on_device else _buf(points), n, int(bool(on_device)),
                                             stream))
        self.n = n

    def set_table(self, table, n, on_device=False, stream=None):
        check(lib().msm_wbits_ctx_set_table(self._ctx, table if on_device else _buf(table), n, int(bool(on_device)),
                                            stream))
        self.n = n

    def get_table(self, first=0, count=None):
        if count is None:
            count = (self.n << (self.wbits - 1)) - first
        out = (ctypes.c_uint8 * (AFF[self.group] * count))()
        check(lib().msm_wbits_ctx_get_table(self._ctx, out, first, count))
        return out

    def mult(self, scalars, nbits=255, stride=None, on_device=False, stream=None):
        stride = stride or (nbits + 7) // 8
        ret = (ctypes.c_uint8 * JAC[self.group])()
        check(lib().msm_wbits_ctx_mult(self._ctx, ret, scalars if on_device else _buf(scalars), stride, nbits,
                                       int(bool(on_device)), stream))
        return bytes(ret)

    def close(self):
        if self._ctx:
            lib().msm_wbits_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
