"""The reference-driver executables (msm_blst_amd/bin/msm_driver_p{1,2}, the
rebuild of ref main_p1.cpp / main_p2.cpp on the C ABI): all four methods
(CHES nh+q/5, CHES integral conversion, BGMW95, blst Pippenger) must agree on
every scalar array (ref test_pippengers, main_p1.cpp:438-610) and equal the
reference's golden result for the last array's seed."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _golden(golden, group, n, seed):
    return [c for c in golden(f"msm_g{group}.json")["cases"]
            if c["n"] == n and c["seed"] == seed and c["case"] == "rand" and c["nbits"] == 255][0]["compressed"]


@pytest.mark.parametrize("group,config,tests", [(1, 10, 3), (2, 10, 2), (1, 16, 1)])
def test_driver_four_methods_agree_with_reference(golden, group, config, tests):
    exe = os.path.join(REPO, "msm_blst_amd", "bin", f"msm_driver_p{group}")
    assert os.path.exists(exe), "build the driver: python -m msm_blst_amd.build"
    r = subprocess.run([exe, f"config={config}", f"tests={tests}", "loops=1"], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["agree"] is True
    want = _golden(golden, group, 1 << config, tests)
    for name, meth in rec["methods"].items():
        assert meth["last_compressed"] == want, name
