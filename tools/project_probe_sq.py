"""gat_project at the cfg3 shape, 20 launches: the command the SQ counter passes profile."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from graphneuralnetwork_amd.ops import gat_project  # noqa: E402

dev = torch.device("cuda:0")
x = torch.randn(1_000_000, 64, device=dev)
w = torch.randn(64, 64, device=dev)
s, d = torch.randn(64, device=dev), torch.randn(64, device=dev)
for _ in range(20):
    gat_project(x, w, 8, 8, s, d)
torch.cuda.synchronize()
