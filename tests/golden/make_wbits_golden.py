#!/usr/bin/env python3
"""Golden fixtures for blst's fixed-window MSM (ref src/multi_scalar.c:63-261),
written from the REFERENCE itself: oracle/_ref/libblst_ref.so (compiled from
/root/reference/src/server.c + build/assembly.S by oracle/Makefile) is called
through ctypes -- blst_p{1,2}s_mult_wbits_precompute / _mult_wbits on the
reference's own fixed points (P_i = 2^(i+1) G via blst_p{1,2}_double) and
SplitMix64 scalars.  Runs only in the build container.

Writes tests/golden/wbits.json: per case {group, n, wbits, nbits, seed, case,
table_fnv (FNV-1a 64 of the precompute output bytes), compressed (result)}.
Test infrastructure only; data, no reference source text.

Case "inf" (an all-zero = infinity input point) hits a reference defect: the
precompute's batch to_affine (ref multi_scalar.c:94-120) multiplies the row's
Z = 0 into the shared prefix product, so every row k >= 1 of the other points in
that batch comes out wrong.  For these cases the fixture records the CORRECT
table (each row (k+1) P_i by the reference's blst_p{1,2}_mult + to_affine, the
infinity point's rows all-zero) and the correct sum (the reference's
blst_p{1,2}s_mult_pippenger, which skips infinity, ref ec_ops.h:717), plus the
reference's defective wbits outputs under ref_defective_*.
"""
import ctypes
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
R_ORDER = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
M64 = (1 << 64) - 1


def splitmix_scalars(n, seed):
    s = seed
    out = []

    def nxt():
        nonlocal s
        s = (s + 0x9e3779b97f4a7c15) & M64
        z = s
        z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
        z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
        return z ^ (z >> 31)

    for _ in range(n):
        while True:
            a = [nxt() for _ in range(4)]
            a[3] >>= 1
            v = a[0] | a[1] << 64 | a[2] << 128 | a[3] << 192
            if v < R_ORDER:
                break
        out.append(v)
    return out


def fnv(data):
    h = 1469598103934665603
    for b in data:
        h ^= b
        h = (h * 1099511628211) & M64
    return f"{h:016x}"


def main():
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libblst_ref.so"))
    cases = []
    specs = [  # (group, n, wbits, nbits, seed, case)
        (1, 16, 4, 255, 1, "rand"), (1, 64, 5, 255, 2, "rand"), (1, 1024, 8, 255, 1, "rand"),
        (1, 1000, 8, 64, 3, "rand"), (1, 256, 12, 255, 4, "rand"), (1, 100, 2, 255, 5, "rand"),
        (1, 37, 3, 128, 6, "rand"), (1, 64, 8, 256, 7, "rand"), (1, 128, 6, 255, 8, "inf"),
        (1, 512, 10, 255, 9, "rand"), (1, 2, 14, 255, 10, "rand"),
        (2, 16, 4, 255, 1, "rand"), (2, 256, 6, 255, 2, "rand"), (2, 50, 7, 64, 3, "inf"),
    ]
    for group, n, wbits, nbits, seed, case in specs:
        g = f"p{group}"
        aff, jac = 96 * group, 144 * group
        gen = getattr(L, f"blst_{g}_generator")
        gen.restype = ctypes.c_void_p
        dbl = getattr(L, f"blst_{g}_double")
        to_aff = getattr(L, f"blst_{g}_to_affine")
        acc = (ctypes.c_uint8 * jac).from_buffer_copy(ctypes.string_at(gen(), jac))
        pts = (ctypes.c_uint8 * (aff * n))()
        for i in range(n):
            dbl(acc, acc)
            to_aff(ctypes.byref(pts, i * aff), acc)
        nb = (nbits + 7) // 8
        vals = splitmix_scalars(n, seed)
        if case == "inf":  # an infinity point (all-zero affine) and a zero scalar
            ctypes.memset(ctypes.byref(pts, 3 * aff), 0, aff)
            vals[5] = 0
        sc = b"".join((v & ((1 << nbits) - 1)).to_bytes(32, "little")[:nb] for v in vals)
        S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
        sizeof = getattr(L, f"blst_{g}s_mult_wbits_precompute_sizeof")
        sizeof.restype = ctypes.c_size_t
        sizeof.argtypes = [ctypes.c_size_t, ctypes.c_size_t]
        T = (ctypes.c_uint8 * sizeof(wbits, n))()
        pp = (ctypes.c_void_p * 2)(ctypes.cast(pts, ctypes.c_void_p), None)
        pre = getattr(L, f"blst_{g}s_mult_wbits_precompute")
        pre.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        pre(T, wbits, pp, n)
        ssz = getattr(L, f"blst_{g}s_mult_wbits_scratch_sizeof")
        ssz.restype = ctypes.c_size_t
        ssz.argtypes = [ctypes.c_size_t]
        scratch = (ctypes.c_uint8 * ssz(n))()
        mult = getattr(L, f"blst_{g}s_mult_wbits")
        mult.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                         ctypes.c_size_t, ctypes.c_void_p]
        sp = (ctypes.c_void_p * 2)(ctypes.cast(S, ctypes.c_void_p), None)
        ret = (ctypes.c_uint8 * jac)()
        mult(ret, T, wbits, n, sp, nbits, scratch)
        out = (ctypes.c_uint8 * (48 * group))()
        getattr(L, f"blst_{g}_compress")(out, ret)
        rec = {"group": group, "n": n, "wbits": wbits, "nbits": nbits, "seed": seed, "case": case,
               "table_fnv": fnv(bytes(T)), "compressed": bytes(out).hex()}
        if case == "inf":
            rec["ref_defective_table_fnv"], rec["ref_defective_compressed"] = rec["table_fnv"], rec["compressed"]
            nwin = 1 << (wbits - 1)
            good = (ctypes.c_uint8 * len(T))()
            J, R = (ctypes.c_uint8 * jac)(), (ctypes.c_uint8 * jac)()
            for i in range(n):
                if i == 3:
                    continue  # infinity: all-zero rows
                getattr(L, f"blst_{g}_from_affine")(J, ctypes.byref(pts, i * aff))
                for k in range(nwin):
                    K = (ctypes.c_uint8 * 32).from_buffer_copy((k + 1).to_bytes(32, "little"))
                    getattr(L, f"blst_{g}_mult")(R, J, K, ctypes.c_size_t(16))
                    to_aff(ctypes.byref(good, (i * nwin + k) * aff), R)
            rec["table_fnv"] = fnv(bytes(good))
            psz = getattr(L, f"blst_{g}s_mult_pippenger_scratch_sizeof")
            psz.restype = ctypes.c_size_t
            psz.argtypes = [ctypes.c_size_t]
            pscr = (ctypes.c_uint8 * psz(n))()
            pm = getattr(L, f"blst_{g}s_mult_pippenger")
            pm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                           ctypes.c_void_p]
            pm(ret, pp, n, sp, nbits, pscr)
            getattr(L, f"blst_{g}_compress")(out, ret)
            rec["compressed"] = bytes(out).hex()
        cases.append(rec)
        print(cases[-1], flush=True)
    with open(os.path.join(HERE, "wbits.json"), "w") as f:
        json.dump({"source": "reference libblst (oracle/_ref/libblst_ref.so) blst_p{1,2}s_mult_wbits_precompute + "
                             "blst_p{1,2}s_mult_wbits; points 2^(i+1) G; SplitMix64 scalars masked to nbits; "
                             "case 'inf': point 3 all-zero (infinity), scalar 5 zero; its table_fnv/compressed are "
                             "the correct values (per-row blst mult, blst Pippenger), the reference's wbits "
                             "outputs (defective, see the script) under ref_defective_*",
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
