"""Debug: the K=300 failing median columns 192 / 196 as one column pair (0, 4)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import byzantine_aircomp_amd as bz
from oracle import aggregators as orc
K, d = 300, 513
g = torch.Generator().manual_seed(K * 7 + d)
X = torch.randn(K, d, generator=g)
X[:, ::5] = torch.round(4 * X[:, ::5]) / 4
X[:, 3] = 1.5
Y = torch.zeros(K, 16)
Y[:, 0] = X[:, 192]
Y[:, 4] = X[:, 196]
a = bz.median(Y.cuda()).cpu().numpy()
torch.cuda.synchronize()
print("got", a[[0, 4]], "want", orc.median(Y).numpy()[[0, 4]])
