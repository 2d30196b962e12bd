"""The large-batch kernels the default per-launch choice does not pick
(plan_common.h launch_cfg), each in a child process whose environment forces
it: the register-direct forward / backward GEMMs (OAC_FWD2=0 OAC_BWDP=0:
gemm_big.hip, gemm_bwd.hip), the pipelined forward on 128x128 tiles with a
3-stage ring (OAC_FWD2_TILE=128,128) and the pipelined backward on 128x64 /
128x128 tiles (OAC_BWDP_CFG=9 / 11).  Each runs the ragged large-batch parity
cases (tests/alt_kernels_check.py) against the fp32 CPU oracle at 1e-5."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

VARIANTS = {
    "register_direct": {"OAC_FWD2": "0", "OAC_BWDP": "0"},
    "fwd_128x128_bwd_128x64": {"OAC_FWD2_TILE": "128,128", "OAC_BWDP_CFG": "9"},
    "fwd_64x64_nb3_bwd_128x128": {"OAC_FWD2_TILE": "64,64", "OAC_FWD2_NB": "3", "OAC_BWDP_CFG": "11"},
}


@pytest.mark.parametrize("name", list(VARIANTS))
def test_alternative_large_batch_kernels_match_oracle(name):
    env = dict(os.environ, **VARIANTS[name])
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "alt_kernels_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{name}: rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    assert r.stdout.count("ok ") == 8, r.stdout
