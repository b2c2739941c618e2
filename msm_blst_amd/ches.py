"""CHES "nh + q/5" bucket-set MSM with the precomputed table resident in HBM.

Python mirror of the reference's CHES driver (LuoGuiwen/MSM_blst main_p1.cpp):
  init_pippenger_CHES_q_over_5()         -> CHESContext(...).build_table(points)
  pippenger_variant_q_over_5_CHES(s[])   -> CHESContext.mult(scalars)
Parameters come from the reference's ches_config_files/config_file_n_exp_*.h
(`params(n_exp, beta)`).  All compute runs in libmsm_mi355x.so (HIP, gfx950).
"""
import ctypes

from ._ffi import check, lib

JAC_BYTES = {1: 144, 2: 288}
AFF_BYTES = {1: 96, 2: 192}
PARAM_KEYS = ("n_exp", "beta", "q_exp", "h", "a_h", "d_max", "b_size", "q_exp_bgmw", "h_bgmw")


def params(n_exp, beta=0):
    """The reference configuration for n = 2^n_exp as a dict (ches_config_files)."""
    out = (ctypes.c_int * 9)()
    check(lib().msm_ches_params(n_exp, beta, out))
    return dict(zip(PARAM_KEYS, list(out)))


def bucket_set(q, a_h):
    """Bucket set B (ref auxiliaryfunc.h:257-288), ascending, from the engine's host setup."""
    n = lib().msm_ches_bucket_set(q, a_h, None, 0)
    out = (ctypes.c_int * n)()
    lib().msm_ches_bucket_set(q, a_h, out, n)
    return out


class Digit(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int), ("b", ctypes.c_int), ("alpha", ctypes.c_int)]


def digit_table(q, a_h):
    """Digit hash H[0..q] (ref main_p1.cpp:140-152) as blst `digit_decomposition` records."""
    out = (Digit * (q + 1))()
    check(lib().msm_ches_digit_table(q, a_h, out))
    return out


def _buf(data):
    if isinstance(data, (bytes, bytearray)):
        return (ctypes.c_uint8 * len(data)).from_buffer_copy(bytes(data))
    return data


class CHESContext:
    """One GPU, one point set, one CHES configuration.

    group: 1 (G1) or 2 (G2); n_exp/beta select the reference configuration, or
    pass `p` (a dict with PARAM_KEYS) for explicit parameters.  `devices` (a list
    of device ids, repeats allowed) shards the points over several devices in
    this process (msm_ches_ctx_create_multi); n_exp is then one shard's
    configuration and points/tables/scalars are passed in host memory.
    """

    def __init__(self, group=1, device=0, n_exp=None, beta=0, p=None, devices=None):
        self.group = group
        self._ctx = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            check(lib().msm_ches_ctx_create_multi(ctypes.byref(self._ctx), group, arr, len(devices), n_exp, beta))
            self.params = params(n_exp, beta)
        elif p is None:
            check(lib().msm_ches_ctx_create(ctypes.byref(self._ctx), group, device, n_exp, beta))
            self.params = params(n_exp, beta)
        else:
            arr = (ctypes.c_int * 9)(*[int(p[k]) for k in PARAM_KEYS])
            check(lib().msm_ches_ctx_create_params(ctypes.byref(self._ctx), group, device, arr))
            self.params = dict(p)
        self.n = 0

    def build_table(self, points, n, on_device=False, stream=None):
        ptr = points if on_device else _buf(points)
        check(lib().msm_ches_ctx_build_table(self._ctx, ptr, n, int(bool(on_device)), stream))
        self.n = n

    def set_table(self, table, n, on_device=False, stream=None):
        ptr = table if on_device else _buf(table)
        check(lib().msm_ches_ctx_set_table(self._ctx, ptr, n, int(bool(on_device)), stream))
        self.n = n

    def get_table(self, first=0, count=None):
        if count is None:
            count = 3 * self.n * self.params["h"] - first
        out = (ctypes.c_uint8 * (AFF_BYTES[self.group] * count))()
        check(lib().msm_ches_ctx_get_table(self._ctx, out, first, count))
        return out

    def save_table(self, path):
        """Write the table to a file (64-B header + blst affine rows)."""
        check(lib().msm_ches_ctx_save_table(self._ctx, str(path).encode()))

    def load_table(self, path):
        """Load a table written by save_table for the same group and parameters."""
        check(lib().msm_ches_ctx_load_table(self._ctx, str(path).encode()))
        self.n = self._npoints_from_file(path)

    @staticmethod
    def _npoints_from_file(path):
        import struct
        with open(path, "rb") as f:
            return struct.unpack("<8s4iQQ24x", f.read(64))[5]

    def mult(self, scalars, stride=32, on_device=False, stream=None):
        ret = (ctypes.c_uint8 * JAC_BYTES[self.group])()
        ptr = scalars if on_device else _buf(scalars)
        check(lib().msm_ches_ctx_mult(self._ctx, ret, ptr, stride, int(bool(on_device)), stream))
        return bytes(ret)

    def mult_batch(self, scalars, count, stride=32, set_stride=None, on_device=False, stream=None):
        """`count` MSMs over the same points (scalar set k at k * set_stride bytes;
        set_stride=0 repeats one set), pipelined on the device.  Returns a list of
        Jacobian byte strings."""
        if set_stride is None:
            set_stride = self.n * stride
        rets = (ctypes.c_uint8 * (JAC_BYTES[self.group] * count))()
        ptr = scalars if on_device else _buf(scalars)
        check(lib().msm_ches_ctx_mult_batch(self._ctx, rets, ptr, stride, set_stride, count, int(bool(on_device)),
                                            stream))
        raw = bytes(rets)
        nb = JAC_BYTES[self.group]
        return [raw[k * nb:(k + 1) * nb] for k in range(count)]

    def shards(self):
        return lib().msm_ches_ctx_shards(self._ctx)

    def bucket_count(self):
        return lib().msm_ches_ctx_bucket_count(self._ctx)

    def batch_lanes(self):
        """Accumulation lanes mult_batch runs (1: the one-lane schedule of the 2^20 headline)."""
        return lib().msm_ches_ctx_batch_lanes(self._ctx)

    def time_accumulation(self, scalars_dev, nsets, reps=5, set_stride=None):
        """Diagnostic: ms of one launch accumulating nsets device scalar sets (after their front)."""
        ms = ctypes.c_float()
        check(lib().msm_ches_ctx_time_accumulation(self._ctx, scalars_dev, set_stride or self.n * 32, nsets, reps,
                                                   ctypes.byref(ms)))
        return ms.value

    def set_profiling(self, on=True):
        check(lib().msm_ches_ctx_set_profiling(self._ctx, int(on)))

    def phase_times(self):
        out = (ctypes.c_float * 6)()
        check(lib().msm_ches_ctx_phase_times(self._ctx, out))
        return dict(zip(("digits", "sort", "accumulate", "reduce", "finalize", "total"), list(out)))

    def close(self):
        if self._ctx:
            lib().msm_ches_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
