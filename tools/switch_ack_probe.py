"""bench.py's switch_batch (one fan-in-2 batch of 131 072 data frames through
inccl_switch_batch), with SW_ACKS=1 every data frame followed by its sender's
ACK: one JSON line, for a rocprofv3 kernel trace of either variant."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    print(json.dumps(bench.switch_batch(dev, acks=os.environ.get("SW_ACKS") == "1")), flush=True)


if __name__ == "__main__":
    main()
