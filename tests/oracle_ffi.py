"""ctypes bindings to oracle/liboracle.so -- the CPU parity checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the msm_blst_amd product path.
"""
import ctypes
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None


class Digit(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int), ("b", ctypes.c_int), ("alpha", ctypes.c_int)]


class ChesParams(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int) for k in ("n_exp", "beta", "q_exp", "h", "a_h", "d_max", "b_size",
                                              "q_exp_bgmw", "h_bgmw")]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "msm_oracle.c")
        if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sz = ctypes.c_size_t
        vp = ctypes.c_void_p
        L.or_gen_scalars.argtypes = [vp, sz, ctypes.c_uint64]
        for f in ("or_p1_fixed_points", "or_p2_fixed_points"):
            getattr(L, f).argtypes = [vp, sz]
        for f in ("or_p1s_mult_pippenger", "or_p2s_mult_pippenger", "or_p1s_mult_naive", "or_p2s_mult_naive"):
            getattr(L, f).argtypes = [vp, vp, sz, vp, sz]
        L.or_p1s_mult_pippenger_mt.argtypes = [vp, vp, sz, vp, sz, ctypes.c_int]
        L.or_pippenger_window.argtypes = [sz]
        L.or_pippenger_window.restype = sz
        L.or_ches_bucket_set.argtypes = [vp, ctypes.c_int, ctypes.c_int]
        L.or_ches_bucket_set.restype = sz
        L.or_ches_digit_table.argtypes = [vp, vp, vp, sz, ctypes.c_int]
        L.or_ches_mb_digits.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int]
        L.or_ches_params_for.argtypes = [ctypes.c_int, ctypes.c_int, vp]
        for f in ("or_p1_ches_table", "or_p2_ches_table", "or_p1_bgmw_table", "or_p2_bgmw_table"):
            getattr(L, f).argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_int]
        for f in ("or_p1_ches_msm", "or_p2_ches_msm"):
            getattr(L, f).argtypes = [vp, vp, sz, vp, vp, vp, vp, sz, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.or_p1_ches_reduce.argtypes = [vp, vp, vp, sz, ctypes.c_int]
        L.or_bgmw_digits.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int]
        for f in ("or_p1_bgmw_msm", "or_p2_bgmw_msm"):
            getattr(L, f).argtypes = [vp, vp, sz, vp, ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def buf(nbytes):
    return (ctypes.c_uint8 * nbytes)()


def scalars(n, seed):
    b = buf(32 * n)
    lib().or_gen_scalars(b, n, seed)
    return b


def repack(sc32, n, nbits):
    """32-byte scalars -> flat packing with stride (nbits+7)//8 (multi_scalar.c:395)."""
    nb = (nbits + 7) // 8
    raw = bytes(sc32)
    out = bytearray()
    for i in range(n):
        s = bytearray(raw[32 * i:32 * i + nb])
        if nbits % 8:
            s[-1] &= (1 << (nbits % 8)) - 1
        out += s
    return (ctypes.c_uint8 * len(out)).from_buffer_copy(bytes(out))


def fixed_points(group, n):
    b = buf((96 if group == 1 else 192) * n)
    getattr(lib(), f"or_p{group}_fixed_points")(b, n)
    return b


def compress(group, jac):
    out = buf(48 * group)
    getattr(lib(), f"or_p{group}_compress")(out, jac)
    return bytes(out).hex()


def msm(group, pts, sc, n, nbits=255, method="pippenger"):
    r = buf(144 * group)
    getattr(lib(), f"or_p{group}s_mult_{method}")(r, pts, n, sc, nbits)
    return r


def ches_params(n_exp, beta=0):
    p = ChesParams()
    if lib().or_ches_params_for(n_exp, beta, ctypes.byref(p)) != 0:
        raise KeyError(n_exp)
    return p


def bucket_set(q, a_h):
    n = lib().or_ches_bucket_set(None, q, a_h)
    B = (ctypes.c_int * n)()
    lib().or_ches_bucket_set(B, q, a_h)
    return B


def digit_table(B, q):
    H = (Digit * (q + 1))()
    v2i = (ctypes.c_int * (q // 2 + 1))()
    lib().or_ches_digit_table(H, v2i, B, len(B), q)
    return H, v2i
