import torch, sys
sys.path.insert(0, ".")
import byzantine_aircomp_amd as bz
from byzantine_aircomp_amd.aggregators import Context
from byzantine_aircomp_amd import _lib
K, d = 2, 64
X = torch.zeros(K, d).cuda()
full = X.clone(); bz.OMA(full, 1e-2, seed=5)
lo, hi = 5, 40
ctx = Context(0); ctx.set_shard(d, lo)
part = X[:, lo:hi].contiguous()
_lib.check(ctx.lib.gm_oma_philox_f32(ctx.handle, part.data_ptr(), K, hi - lo, hi - lo, 1e-2, 5, None), "x")
torch.cuda.synchronize()
f = full[:, lo:hi]
for k in range(K):
    for j in range(hi - lo):
        a, b = float(part[k, j]), float(f[k, j])
        if a != b:
            print(k, j, lo + j, a, b)
print("full row0", full[0, :12].tolist())
print("part row0", part[0, :8].tolist())
