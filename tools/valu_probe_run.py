import ctypes, sys
L = ctypes.CDLL('/root/repo/msm_blst_amd/libmsm_mi355x.so')
o = (ctypes.c_double * 4)()
for r in range(2):
    rc = L.msm_valu_probe(0, o)
    print(rc, [f"{x:.4g}" for x in o], flush=True)
