"""The root switch's ACK batch alone (bench.switch_batch(acks=True): an ACK after
every data frame, 262 144 frames), for rocprofv3 kernel traces and counter
passes: python tools/ack_probe.py"""
import json
import sys

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench  # noqa: E402

print(json.dumps(bench.switch_batch(torch.device("cuda:0"), acks=True)), flush=True)
