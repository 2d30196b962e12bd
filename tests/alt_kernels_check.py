"""Run by tests/test_gpu_altkernels.py in a child process that selects a
non-default large-batch kernel (OAC_TEST_TUNING -> oac_tuning_set): the
ragged large-batch parity cases of test_gpu_ragged.py (B = 1029
/ 1100, hidden 48 / 80) for all four trainers against the fp32 CPU oracle
(OAC_TEST_SHAPES=small: the small-batch SAC cases instead, for a
small-batch step choice)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "oac-explore_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import test_gpu_ragged as tr  # noqa: E402
from oac_amd import _lib  # noqa: E402

# the kernel / schedule choice of this child (oac_tuning_set), from the parent
_lib.set_tuning_spec(os.environ.get("OAC_TEST_TUNING", ""))


def main():
    # OAC_TEST_SHAPES=small: the small-batch SAC shapes (a small-kernel step choice)
    small = os.environ.get("OAC_TEST_SHAPES") == "small"
    shapes = [s for s in tr.SHAPES if (s[3] < 1024) == small]
    fns = (tr.test_sac_ragged,) if small else (tr.test_sac_ragged, tr.test_particle_oac_ragged,
                                               tr.test_goac_ragged, tr.test_ptrain_ragged)
    for fn in fns:
        for s in shapes:
            fn(*s)
            print(f"ok {fn.__name__}{s}", flush=True)


if __name__ == "__main__":
    main()
