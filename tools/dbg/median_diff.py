"""Print the columns where the GPU median differs from the oracle (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import byzantine_aircomp_amd as bz
from oracle import aggregators as orc

for K, d in [(300, 513), (1000, 200), (513, 130)]:
    g = torch.Generator().manual_seed(K * 7 + d)
    X = torch.randn(K, d, generator=g)
    X[:, ::5] = torch.round(4 * X[:, ::5]) / 4
    X[:, 3] = 1.5
    a = bz.median(X.cuda()).cpu().numpy()
    b = orc.median(X).numpy()
    bad = np.nonzero(a != b)[0]
    print(K, d, "bad", len(bad), bad[:10])
    for j in bad[:4]:
        col = np.sort(X[:, j].numpy())
        r = (K - 1) // 2
        print("  col", j, "got", a[j], "want", b[j], "around", col[r - 3:r + 4], "nuniq", len(np.unique(col)))
