"""The Gram-space path (north_star's second design) pinned to the oracle at a
realistic K x d, past 2^31 elements (round 6; the C3 streaming kernel's counterpart is
tests/test_gpu_c3_oracle.py).

K = 256 on the C4 recipe (gm_fill_clients_f32: honest N(0, 0.05^2), the last 51 rows
N(0.25, 0.5^2), guess N(0, 0.01^2); C4 = 256 x 125M d-sharded, 15.6M per GPU) at

* d = 4,194,304 (1.07e9 elements);
* d = 8,400,000 (2.15e9 elements > 2^31: the Gram producer's row and panel offsets and
  the closing pass's tile offsets past 32 bits);

through AUTO — the guarded scaled-f16 split Gram on v_mfma_f32_16x16x32_f16, the K-space
Weiszfeld in fp64, one closing streaming pass — on the row-major [K, d]
stack and on ClientPanels, against ``oracle.gm2`` (op for op M:162-184, fp32, host):

* the Gram path actually ran (algo "gram", its guard accepted the result);
* relative L2 <= 1e-5 (north_star);
* iterations within +-1 of the oracle's on an input whose count window
  (``oracle.gm2_count_window``, exact fp64 iteration, 2-ulp movement floor) is determined
  and at most 1 wide (asserted).
"""
import pytest
import torch

from conftest import assert_iter_count, rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu

K, B = 256, 51
OPTS = {"maxiter": 1000, "tol": 1e-5}
_CACHE = {}


def _reference(d):
    if d in _CACHE:
        return _CACHE[d]
    _CACHE.clear()
    import byzantine_aircomp_amd as bz
    ctx = bz.context()
    s = torch.cuda.current_stream().cuda_stream
    X = torch.empty(K, d, device="cuda")
    bz._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, B, 0.0, 0.05,
                                              0.25, 0.5, 20211, s), "fill")
    g0 = torch.empty(d, device="cuda")
    bz._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, 20212, s),
                  "fill")
    torch.cuda.synchronize()
    win = orc.gm2_count_window(X, g0, OPTS["maxiter"], OPTS["tol"], chunk_rows=32)
    Xh, gh = X.cpu(), g0.cpu()
    want, tr = orc.gm2(Xh, dict(OPTS, guess=gh))
    del Xh
    _CACHE[d] = (X, g0, want, tr, win)
    return _CACHE[d]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("d,layout", [(4_194_304, "rows"), (4_194_304, "panels"),
                                      (8_400_000, "rows"), (8_400_000, "panels")])
def test_gram_path_vs_oracle_large(d, layout):
    import byzantine_aircomp_amd as bz
    X, g0, want, tr, win = _reference(d)
    assert win.determined and win.width <= 1, win
    assert win.early - 1 <= tr.iters <= win.late + 1, (tr, win)
    Xin = bz.ClientPanels.from_rows(X) if layout == "panels" else X
    got = bz.gm2(Xin, dict(OPTS, guess=g0))
    torch.cuda.synchronize()
    res = bz.aggregators.last_result
    del Xin
    assert res.algo == "gram" and res.guard in ("accepted", "accepted_floor"), res
    err = rel_l2(got.cpu().numpy(), want.numpy())
    print(f"gram K={K} d={d} {layout}: iters {res.iters} (oracle {tr.iters}, window "
          f"[{win.early}, {win.late}]), guard {res.guard}, rel L2 {err:.3e}")
    assert err <= 1e-5, err
    assert_iter_count(res.iters, tr.iters, win)
