"""BGMW95 fixed-base MSM with the precomputed table resident in HBM.

Python mirror of the reference's BGMW95 driver path (LuoGuiwen/MSM_blst
main_p1.cpp):
  init_pippenger_BGMW95()          -> BGMWContext(...).build_table(points)   (:94-122)
  pippenger_variant_BGMW95(s[])    -> BGMWContext.mult(scalars)              (:294-398)
q = 2^EXPONENT_OF_q_BGMW95 and h_BGMW95 come from the reference's
ches_config_files (`ches.params(n_exp)["q_exp_bgmw"], ["h_bgmw"]`).  All compute
runs in libmsm_mi355x.so (HIP, gfx950).
"""
import ctypes

from ._ffi import check, lib
from .ches import AFF_BYTES, JAC_BYTES, _buf, params


class BGMWContext:
    """One GPU, one point set, table T[i h + j] = q^j P_i.

    Either pass (q_exp, h) or n_exp (the reference configuration's BGMW95 q, h).
    """

    def __init__(self, group=1, device=0, q_exp=None, h=None, n_exp=None, beta=0):
        if q_exp is None:
            p = params(n_exp, beta)
            q_exp, h = p["q_exp_bgmw"], p["h_bgmw"]
        self.group, self.q_exp, self.h = group, q_exp, h
        self._ctx = ctypes.c_void_p()
        check(lib().msm_bgmw_ctx_create(ctypes.byref(self._ctx), group, device, q_exp, h))
        self.n = 0

    def build_table(self, points, n, on_device=False, stream=None):
        ptr = points if on_device else _buf(points)
        check(lib().msm_bgmw_ctx_build_table(self._ctx, ptr, n, int(bool(on_device)), stream))
        self.n = n

    def set_table(self, table, n, on_device=False, stream=None):
        ptr = table if on_device else _buf(table)
        check(lib().msm_bgmw_ctx_set_table(self._ctx, ptr, n, int(bool(on_device)), stream))
        self.n = n

    def get_table(self, first=0, count=None):
        if count is None:
            count = self.n * self.h - first
        out = (ctypes.c_uint8 * (AFF_BYTES[self.group] * count))()
        check(lib().msm_bgmw_ctx_get_table(self._ctx, out, first, count))
        return out

    def save_table(self, path):
        """Write the table to a file (64-B header + blst affine rows)."""
        check(lib().msm_bgmw_ctx_save_table(self._ctx, str(path).encode()))

    def load_table(self, path):
        """Load a table written by save_table for the same group and parameters."""
        check(lib().msm_bgmw_ctx_load_table(self._ctx, str(path).encode()))
        self.n = self._npoints_from_file(path)

    @staticmethod
    def _npoints_from_file(path):
        import struct
        with open(path, "rb") as f:
            return struct.unpack("<8s4iQQ24x", f.read(64))[5]

    def mult(self, scalars, stride=32, on_device=False, stream=None):
        ret = (ctypes.c_uint8 * JAC_BYTES[self.group])()
        ptr = scalars if on_device else _buf(scalars)
        check(lib().msm_bgmw_ctx_mult(self._ctx, ret, ptr, stride, int(bool(on_device)), stream))
        return bytes(ret)

    def bucket_count(self):
        return lib().msm_bgmw_ctx_bucket_count(self._ctx)

    def set_profiling(self, on=True):
        check(lib().msm_bgmw_ctx_set_profiling(self._ctx, int(on)))

    def phase_times(self):
        out = (ctypes.c_float * 6)()
        check(lib().msm_bgmw_ctx_phase_times(self._ctx, out))
        return dict(zip(("digits", "sort", "accumulate", "reduce", "finalize", "total"), list(out)))

    def close(self):
        if self._ctx:
            lib().msm_bgmw_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
