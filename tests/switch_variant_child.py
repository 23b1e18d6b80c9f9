"""Child process of tests/test_gpu_switch_variants.py (not collected by pytest):
runs a selection of the switch / ICRC GPU tests as plain functions under the
environment it was started with, so that a kernel-selection hook read once per
process ($INCCL_ICRC_DIRECT, $INCCL_EGRESS_NT, ...) is exercised against the
oracle exactly as the default path is."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import torch  # noqa: E402

import container_inc_amd as cia  # noqa: E402

cia.load()
from oracle import oracle as O  # noqa: E402

O.build()
import test_gpu_switch as T  # noqa: E402

dev = torch.device("cuda:0")
T.test_icrc_golden_frame(dev)
T.test_icrc_random_frames(dev, O)
T.test_icrc_any_length(dev, O)
for stride, count in [(1100, 7), (1152, 5)]:
    T.test_icrc_row_strides_odd_counts(dev, O, stride, count)
for fan_in, stride in [(2, 1152), (2, 1100), (3, 1152), (8, 1152), (5, 1100)]:
    T.test_switch_batches(dev, O, fan_in, stride)
T.test_switch_batch_graph_replay(dev, O)
print("variant ok", flush=True)
