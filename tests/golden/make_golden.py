#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs only in the build container (where /root/reference exists):
  1. `make -C oracle ref` compiles the reference libblst from its own sources
     (src/server.c + build/assembly.S), its n=2^10 G1 driver (main_p1.cpp,
     main renamed) and our small harnesses, all into oracle/_ref/.
  2. The harnesses are run; their outputs become the JSON fixtures below.
Every fixture is data (inputs and expected outputs); no reference source
text is stored.  Test infrastructure only.

`python make_golden.py large` only appends the large G1 seed-1 keys (LARGE_G1).

Fixtures written:
  msm_g1.json / msm_g2.json  compressed MSM results of blst_p{1,2}s_mult_pippenger
                             (seeded scalars, P_i = 2^(i+1) G), incl. edge cases
  fp_kat.json                blst_fp_mul / add / sub vectors (raw limbs)
  xyzz_kat.json              blst_p1xyzz_dadd_affine / _dadd sequences (raw limbs + compressed)
  ches_driver_n10.json       the reference's own n=2^10 G1 driver: bucket set, digit
                             table, table hashes, digits, results of all 4 methods
  ches_driver_p2_n10.json    the same for the reference's G2 driver (main_p2.cpp)
  ches_params_n{10,16,20}.json  bucket set / digit table hashes + MB / q/2 digits
  ches_configs.json          the 17 ches_config_files/*.h parameter sets (values)
"""
import json
import os
import re
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("REF", "/root/reference")
BIN = os.path.join(REPO, "oracle", "_ref")


def run(args):
    return subprocess.run(args, check=True, capture_output=True, text=True).stdout


# seed-1 keys at the strong-scaling shard sizes (2^20 / N points per rank,
# N = 8, 4, 2) and the weak-scaling totals (2^20 per rank: 2^22 at N = 4, 2^23
# at N = 8), so every multi-rank bench leg has a parity pin
LARGE_G1 = [(1 << e, 1, 255, "rand") for e in (17, 18, 19, 22, 23)]


def msm_case(group, n, seed, nbits, cas):
    t = time.time()
    res = run([os.path.join(BIN, "ref_golden"), "msm", str(group), str(n), str(seed), str(nbits), cas]).strip()
    print(f"G{group} n={n} seed={seed} nbits={nbits} {cas}: {res[:16]}.. ({time.time()-t:.1f}s)", file=sys.stderr)
    return {"group": group, "n": n, "seed": seed, "nbits": nbits, "case": cas, "compressed": res}


def add_large():
    """Append LARGE_G1 to msm_g1.json (the other cases unchanged)."""
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref", f"REF={REF}"], check=True)
    fn = os.path.join(HERE, "msm_g1.json")
    d = json.load(open(fn))
    have = {(c["n"], c["seed"], c["nbits"], c["case"]) for c in d["cases"]}
    for (n, seed, nbits, cas) in LARGE_G1:
        if (n, seed, nbits, cas) not in have:
            d["cases"].append(msm_case(1, n, seed, nbits, cas))
    json.dump(d, open(fn, "w"), indent=1)


def msm_cases():
    g1, g2 = [], []
    for n in (2, 3, 4, 5, 7, 8, 16, 31, 32, 64, 100, 128, 256, 512, 1000, 1024):
        for seed in (1, 2, 3):
            g1.append((n, seed, 255, "rand"))
    for n in (4096, 65536):
        for seed in (1, 2):
            g1.append((n, seed, 255, "rand"))
    g1 += [(1 << 20, 1, 255, "rand"), (1 << 21, 1, 255, "rand")]
    g1 += LARGE_G1
    for cas in ("zero", "ones", "rminus1", "equal", "negpairs", "ptr"):
        g1.append((64, 1, 255, cas))
    for nbits in (64, 128, 256):
        g1.append((64, 1, nbits, "rand"))
        g1.append((1000, 2, nbits, "rand"))
    g1.append((64, 1, 256, "ones"))
    for n in (2, 4, 8, 16, 64, 256, 1024):
        for seed in (1, 2):
            g2.append((n, seed, 255, "rand"))
    g2 += [(65536, 1, 255, "rand"), (1 << 20, 1, 255, "rand")]
    for cas in ("zero", "ones", "equal", "negpairs"):
        g2.append((64, 1, 255, cas))
    g2.append((64, 1, 64, "rand"))
    return g1, g2


def main():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref", f"REF={REF}"], check=True)
    g1, g2 = msm_cases()
    for group, cases, fname in ((1, g1, "msm_g1.json"), (2, g2, "msm_g2.json")):
        out = []
        for (n, seed, nbits, cas) in cases:
            out.append(msm_case(group, n, seed, nbits, cas))
        json.dump({"source": "reference libblst blst_p%ds_mult_pippenger via oracle/ref_golden.c" % group,
                   "points": "P_i = 2^(i+1) G (main_p1.cpp:52-66)",
                   "scalars": "SplitMix64(seed), 4 LE words, word3 >>= 1, reject >= r; packed flat with stride (nbits+7)/8",
                   "cases": out}, open(os.path.join(HERE, fname), "w"), indent=1)
    rows = []
    for line in run([os.path.join(BIN, "ref_golden"), "fpkat", "64", "7"]).split("\n"):
        if line.strip():
            a, b, m, ad, sb = line.split()
            rows.append({"a": a, "b": b, "mul": m, "add": ad, "sub": sb})
    json.dump({"source": "reference blst_fp_mul/add/sub; limbs little-endian, 16 hex digits per limb, limb 0 first",
               "vectors": rows}, open(os.path.join(HERE, "fp_kat.json"), "w"), indent=1)
    rows = []
    for line in run([os.path.join(BIN, "ref_golden"), "xyzz", "24"]).split("\n"):
        if not line.strip():
            continue
        ops, raw, comp = line.split(" | ")
        ops = [tuple(int(v) for v in o.split(":")) for o in ops.split()[1:]]
        x, y, zzz, zz = raw.split()
        c1, c2 = comp.split()
        rows.append({"ops": ops, "x": x, "y": y, "zzz": zzz, "zz": zz, "compressed": c1, "compressed_double": c2})
    json.dump({"source": "reference blst_p1xyzz_dadd_affine sequences on P_0..P_2, then acc+acc via blst_p1xyzz_dadd",
               "sequences": rows}, open(os.path.join(HERE, "xyzz_kat.json"), "w"), indent=1)
    drivers()
    for c in (10, 16, 20):
        d = json.loads(run([os.path.join(BIN, f"ref_ches_{c}")]))
        d["source"] = f"reference auxiliaryfunc.h under config_file_n_exp_{c}.h via oracle/ref_ches_params.cpp"
        json.dump(d, open(os.path.join(HERE, f"ches_params_n{c}.json"), "w"), indent=1)
    cfgs = []
    cdir = os.path.join(REF, "ches_config_files")
    for f in sorted(os.listdir(cdir)):
        m = re.match(r"config_file_n_exp_(\d+)(_beta)?\.h$", f)
        if not m:
            continue
        txt = open(os.path.join(cdir, f)).read()
        def val(k):
            return int(re.search(k + r"\s*=\s*(\d+)", txt).group(1))
        cfgs.append({"file": f, "n_exp": val("N_EXP"), "beta": int(bool(m.group(2))), "q_exp": val("EXPONENT_OF_q"),
                     "h": val("h_LEN_SCALAR"), "a_h": val("a_LEADING_TERM"), "d_max": val("d_MAX_DIFF"),
                     "b_size": val("B_SIZE"), "q_exp_bgmw": val("EXPONENT_OF_q_BGMW95"), "h_bgmw": val("h_BGMW95")})
    json.dump({"source": "values of /root/reference/ches_config_files/config_file_n_exp_*.h", "configs": cfgs},
              open(os.path.join(HERE, "ches_configs.json"), "w"), indent=1)


def drivers():
    """The reference's own n=2^10 drivers (main_p1.cpp -> ches_driver_n10.json,
    main_p2.cpp -> ches_driver_p2_n10.json) through oracle/ref_driver.cpp."""
    for g, fname in ((1, "ches_driver_n10.json"), (2, "ches_driver_p2_n10.json")):
        s = run([os.path.join(BIN, f"ref_driver_p{g}")])
        d = json.loads(s[s.index('{"group"'):])
        d["source"] = f"reference main_p{g}.cpp (config_file.h = n_exp_10) via oracle/ref_driver.cpp (GROUP={g})"
        json.dump(d, open(os.path.join(HERE, fname), "w"))


if __name__ == "__main__":
    if sys.argv[1:] == ["large"]:
        add_large()
    elif sys.argv[1:] == ["drivers"]:
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref", f"REF={REF}"], check=True)
        drivers()
    else:
        main()
