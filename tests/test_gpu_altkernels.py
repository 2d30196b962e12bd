"""The large-batch kernels the default per-launch choice does not pick
(plan_common.h launch_cfg), each in a child process that forces it through
oac_tuning_set (OAC_TEST_TUNING="key=value,..." read by the child script):
the pipelined forward on 128x128 tiles with a 3-stage ring and the pipelined
backward on 128x64 / 128x128 tiles (3-stage and 2-stage rings) or 64x64 on a
3-stage ring (bwdp_cfg 9 / 11 / 13 / 14 / 10), 16-deep stages on a 4-stage
ring (15), the software-pipelined loop (17), and the step-structure
fallbacks (one Adam launch per group, the P-OAC rank-K dX as a GEMM).  Each
runs the ragged large-batch parity cases (tests/alt_kernels_check.py) against
the fp32 CPU oracle at 1e-5."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

VARIANTS = {
    "fwd_128x128_bwd_128x64": "fwd_tile_m=128,fwd_tile_n=128,bwdp_cfg=9",
    "fwd_64x64_nb3_bwd_128x128": "fwd_tile_m=64,fwd_tile_n=64,fwd_nb=3,bwdp_cfg=11",
    # the backward 64x64 tiles on the 3-stage ring (the default is the 2-stage one, cfg 12)
    "bwd_64x64_nb3": "bwdp_cfg=10",
    # the backward 128x128 / 128x64 tiles on the 2-stage ring
    "bwd_128x128_nb2": "bwdp_cfg=13",
    "bwd_128x64_nb2": "bwdp_cfg=14",
    # 64x64 tiles: 16-deep stages on a 4-stage ring; the software-pipelined
    # loop on the 2-stage ring
    "bwd_64x64_fk16": "bwdp_cfg=15",
    "bwd_64x64_swp": "bwdp_cfg=17",
    # the step-structure fallbacks: one Adam launch per group, the P-OAC
    # rank-K dX as its own GEMM launch
    "adam_launches_dh2_gemm": "split_adam=-1,dh2_targets=-1",
    # the SAC policy layer 0's Adam by the last arrival of each dW tile
    "last_arrival_adam": "la_adam=1",
    # the policy-head dX in the dL/da launch's epilogue at large batch too
    # (the small-batch default; at large batch it is a launch of its own)
    "head_dx_epilogue": "head_dh2=2",
}


@pytest.mark.parametrize("name", list(VARIANTS))
def test_alternative_large_batch_kernels_match_oracle(name):
    env = dict(os.environ, OAC_TEST_TUNING=VARIANTS[name])
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "alt_kernels_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"{name}: rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    assert r.stdout.count("ok ") == 8, r.stdout


def test_head_dx_launch_small_batch_matches_oracle():
    """The small-batch step with the policy-head dX in a launch of its own
    (head_dh2=-1; the default runs it in the dL/da launch's epilogue and the
    head dW beside the policy layer-1 backward), on the ragged small-batch SAC
    shapes against the oracle."""
    env = dict(os.environ, OAC_TEST_TUNING="head_dh2=-1", OAC_TEST_SHAPES="small")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "alt_kernels_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, f"rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    assert r.stdout.count("ok ") == 4, r.stdout


def test_side_workgroup_adam_is_bitwise_the_adam_launch(tmp_path):
    """Large-batch side-workgroup Adam (GemmBatch::side_adam; the SAC step)
    against one Adam launch per group, and the policy head's column-chunk
    count, child processes: params, targets and Adam moments bit for bit after
    three steps (the P-OAC step, one Adam launch per group either way, rides
    along as a control)."""
    import numpy as np
    outs = {}
    for name, spec in {"side": "split_adam=1,dh2_targets=-1",
                       "launch": "split_adam=-1,dh2_targets=-1",
                       # and the policy head on two 128-column chunks per row
                       # block (recomputed heads, 2 pairs per wave): the same
                       # arithmetic per output, so bitwise too
                       "head_cc2": "split_adam=1,dh2_targets=-1,head_cc=2",
                       # and the policy layer 0's Adam by the last arrival of
                       # each of its dW tiles (no Adam launch): the same sums
                       # in the same order, the same update
                       "last_arrival": "split_adam=1,dh2_targets=-1,la_adam=1"}.items():
        out = str(tmp_path / f"{name}.npz")
        r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "split_adam_check.py"), out],
                           env=dict(os.environ, OAC_TEST_TUNING=spec), capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, f"{name}: rc {r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
        outs[name] = np.load(out)
        if name == "last_arrival":   # the path was taken (OAC_TRACE_LA_ADAM) at both sizes
            bits = [int(w.split("=")[1]) for w in r.stdout.split("trace", 1)[1].split()]
            assert len(bits) == 2 and all(b & 256 for b in bits), r.stdout
    a = outs["side"]
    assert len(a.files) == 16
    for other in ("launch", "head_cc2", "last_arrival"):
        b = outs[other]
        assert sorted(a.files) == sorted(b.files)
        for k in a.files:
            assert np.isfinite(a[k]).all(), k
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"{other}: {k}")
