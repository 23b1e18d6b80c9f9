"""The switch kernels' A/B hooks against the oracle (gpu).  Each hook is read
once per process, so every variant runs tests/switch_variant_child.py in a child
process of its own (one at a time): plain instead of non-temporal stores, the
LDS-staged ICRC kernels, two ICRC pairs per pass, the generic egress kernel and
other apply geometries.  The child runs the ICRC tests (golden, random, every
length, odd counts, unaligned rows) and switch batches (fan-in 2, 3, 5, 8;
16-byte and 4-byte rows; graph replay) exactly as tests/test_gpu_switch.py does."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
CHILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "switch_variant_child.py")

VARIANTS = {
    "plain_stores": {"INCCL_EGRESS_NT": "0", "INCCL_APPLY_NT": "0"},
    "icrc_pair_lds": {"INCCL_ICRC_DIRECT": "0"},
    "icrc_one_frame_per_wave": {"INCCL_ICRC_DIRECT": "0", "INCCL_ICRC_PAIR": "0"},
    "icrc_two_pairs_per_pass": {"INCCL_ICRC_PAIRS_PER_PASS": "2"},
    "icrc_mask_valu": {"INCCL_ICRC_MASK_LDS": "0"},
    "icrc_mask_table_byte_zeroing": {"INCCL_ICRC_MASK_LDS": "1"},
    "egress_generic": {"INCCL_EGRESS_GENERIC": "1"},
    "apply_4_frames_8_waves": {"INCCL_APPLY_FRAMES": "4", "INCCL_APPLY_WPB": "8"},
}


@pytest.mark.parametrize("name", sorted(VARIANTS))
def test_switch_variant(gpu, name):
    env = dict(os.environ)
    env.update(VARIANTS[name])
    r = subprocess.run([sys.executable, "-u", CHILD], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (name, r.stdout[-3000:], r.stderr[-3000:])
    assert "variant ok" in r.stdout, (name, r.stdout[-3000:])
