import json, sys
sys.path.insert(0, ".")
import torch
import bench
d = torch.device("cuda:0")
print(json.dumps({"root": bench.switch_batch(d), "nonroot": bench.switch_nonroot_round(d)}), flush=True)
