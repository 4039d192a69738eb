"""apply_kernel's C staging stride against the ds_read_b128 banking model
(tools/lds_banks.py, MI355X_MICROARCH.md LDS table).  The model reproduces the
round-2 counters (ACS = 57: 4 conflict cycles per read; r02_pmc_legs.json
apply1m measured 3.97 per LDS instruction) and the stride in the source is
conflict-free."""
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def test_model_matches_round2_counters():
    import lds_banks
    assert lds_banks.apply_read(57) - 4 == 4


def test_source_stride_conflict_free():
    import lds_banks
    src = open(os.path.join(REPO, "80211parallelestimation_amd", "csrc", "wce_kernels.hip")).read()
    acs = int(re.search(r"constexpr int ACS = (\d+);", src).group(1))
    assert acs >= 56 and lds_banks.apply_read(acs) == 4
