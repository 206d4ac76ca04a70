"""The reference's other aggregators on the GPU (row f3) vs its golden outputs and the oracle."""
import numpy as np
import pytest
import torch

from conftest import golden_case, rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu


def test_golden_other_aggregators():
    import byzantine_aircomp_amd as bz
    meta, arr = golden_case("other_aggregators_K20_d640")
    X = torch.from_numpy(arr["X"]).cuda()
    assert np.array_equal(bz.median(X).cpu().numpy(), arr["median"])          # exact element
    assert np.array_equal(bz.Krum(X, {"honestSize": 16}).cpu().numpy(), arr["Krum"])  # a row
    assert rel_l2(bz.mean(X).cpu().numpy(), arr["mean"]) <= 1e-6
    assert rel_l2(bz.trimmed_mean(X).cpu().numpy(), arr["trimmed_mean"]) <= 1e-6


@pytest.mark.parametrize("K,d", [(1, 5), (2, 100), (7, 333), (50, 7850), (64, 1000), (65, 257),
                                 (256, 300)])
def test_coordinate_aggregators_vs_oracle(K, d):
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K + d)
    X = torch.randn(K, d, generator=g)
    X[:, ::7] = torch.round(X[:, ::7])            # ties in some columns
    Xc = X.cuda()
    assert np.array_equal(bz.median(Xc).cpu().numpy(), orc.median(X).numpy())
    assert rel_l2(bz.mean(Xc).cpu().numpy(), orc.mean(X).numpy()) <= 1e-6
    if K >= 3:
        assert rel_l2(bz.trimmed_mean(Xc).cpu().numpy(), orc.trimmed_mean(X).numpy()) <= 1e-6


@pytest.mark.parametrize("K,honest", [(10, 8), (50, 45), (50, 40), (120, 100)])
def test_krum_vs_oracle(K, honest):
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K * 3 + honest)
    X = 0.05 * torch.randn(K, 2000, generator=g)
    X[honest:] += 0.5 * torch.randn(K - honest, 2000, generator=g)
    out = bz.Krum(X.cuda(), {"honestSize": honest})
    want = orc.krum(X, {"honestSize": honest})
    assert torch.equal(out.cpu(), want)
    assert bz.aggregators.Krum.last_index < honest


def test_other_aggregators_cpu_input_roundtrip():
    import byzantine_aircomp_amd as bz
    X = torch.randn(11, 99, generator=torch.Generator().manual_seed(11))
    assert bz.median(X).device.type == "cpu"
    assert torch.equal(bz.median(X), orc.median(X))


@pytest.mark.parametrize("K,d", [(129, 77), (300, 513), (513, 130), (1000, 200), (1025, 33),
                                 (2048, 17)])
def test_coordinate_aggregators_large_K(K, d):
    """Bit-wise selection at every LDS tile shape (K up to 2048), ties included."""
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K * 7 + d)
    X = torch.randn(K, d, generator=g)
    X[:, ::5] = torch.round(4 * X[:, ::5]) / 4        # heavy ties
    X[:, 3] = 1.5                                      # a constant column
    Xc = X.cuda()
    assert np.array_equal(bz.median(Xc).cpu().numpy(), orc.median(X).numpy())
    assert rel_l2(bz.trimmed_mean(Xc).cpu().numpy(), orc.trimmed_mean(X).numpy()) <= 1e-6


def test_coordinate_aggregators_special_values():
    """torch semantics: median propagates NaN; topk ranks NaN above +inf, so a NaN in
    the trimmed top b is dropped and one in the middle makes the mean NaN; -0 == +0."""
    import byzantine_aircomp_amd as bz
    K, d = 20, 9
    g = torch.Generator().manual_seed(5)
    X = torch.randn(K, d, generator=g)
    X[0, 0] = float("nan")                             # one NaN: trimmed (top 2) drops it
    X[:3, 1] = float("nan")                            # three NaNs: one reaches the middle
    X[:, 2] = 0.0
    X[::2, 2] = -0.0
    X[0, 3], X[1, 3] = float("inf"), float("-inf")
    X[:, 4] = -X[:, 4].abs()                           # all negative
    Xc = X.cuda()
    m = bz.median(Xc).cpu()
    want = orc.median(X)
    assert torch.equal(torch.isnan(m), torch.isnan(want))
    ok = ~torch.isnan(want)
    assert torch.equal(m[ok], want[ok])
    t = bz.trimmed_mean(Xc).cpu()
    tw = orc.trimmed_mean(X)
    assert torch.equal(torch.isnan(t), torch.isnan(tw))
    ok = ~torch.isnan(tw)
    assert rel_l2(t[ok].numpy(), tw[ok].numpy()) <= 1e-6


@pytest.mark.parametrize("K", [129, 200, 256, 257, 512, 513, 1000, 1024])
def test_staged_selection_special_values(K):
    """The staged-transpose kernels (median K <= 1024, trimmed mean K <= 512) and the
    branch-free slot keys at the tile boundaries: NaN columns (median NaN; trimmed mean per
    torch's topk order), -0 / +0, infinities, all-negative columns, a ragged last tile."""
    import byzantine_aircomp_amd as bz
    d = 37
    g = torch.Generator().manual_seed(K)
    X = torch.randn(K, d, generator=g)
    X[K // 2, 0] = float("nan")
    X[: K // 3, 1] = float("nan")                      # NaNs reach the trimmed middle
    X[:, 2] = 0.0
    X[::2, 2] = -0.0
    X[0, 3], X[1, 3] = float("inf"), float("-inf")
    X[:, 4] = -X[:, 4].abs()
    X[:, 5] = torch.round(X[:, 5])                      # ties
    Xc = X.cuda()
    m, want = bz.median(Xc).cpu(), orc.median(X)
    assert torch.equal(torch.isnan(m), torch.isnan(want))
    ok = ~torch.isnan(want)
    assert torch.equal(m[ok], want[ok])
    t, tw = bz.trimmed_mean(Xc).cpu(), orc.trimmed_mean(X)
    assert torch.equal(torch.isnan(t), torch.isnan(tw))
    ok = ~torch.isnan(tw)
    assert rel_l2(t[ok].numpy(), tw[ok].numpy()) <= 1e-6


@pytest.mark.parametrize("K,d,honest", [(129, 1001, 100), (300, 4096, 240), (260, 77, 200)])
def test_krum_multi_tile_vs_oracle(K, d, honest):
    """Pair tiles of 128 rows: K spanning 2-3 row tiles, ragged d (scalar column tail)."""
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K + d + honest)
    X = 0.05 * torch.randn(K, d, generator=g)
    X[honest:] += 0.5 * torch.randn(K - honest, d, generator=g)
    perm = torch.randperm(K, generator=g)            # Byzantine rows anywhere
    X = X[perm].contiguous()
    out = bz.Krum(X.cuda(), {"honestSize": honest})
    assert torch.equal(out.cpu(), orc.krum(X, {"honestSize": honest}))


def test_krum_strided_rows():
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(9)
    base = torch.randn(40, 530, generator=g)
    X = base[:, 3:520]                                # ldx = 530, unaligned start
    out = bz.Krum(X.cuda(), {"honestSize": 30})
    assert torch.equal(out.cpu(), orc.krum(X.contiguous(), {"honestSize": 30}))


@pytest.mark.parametrize("K,d", [(20, 640), (50, 7850), (65, 257), (256, 300), (300, 513),
                                 (1000, 200), (1025, 33)])
def test_coordinate_aggregators_on_panels(K, d):
    """mean / median / trimmed_mean / Krum on a ClientPanels == on the row-major matrix
    (the same kernels with panel addressing: bit-identical)."""
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K * 11 + d)
    X = torch.randn(K, d, generator=g)
    X[:, ::5] = torch.round(4 * X[:, ::5]) / 4
    Xc = X.cuda()
    P = bz.ClientPanels.from_rows(Xc)
    for f in (bz.mean, bz.median, bz.trimmed_mean):
        assert torch.equal(f(P, {}), f(Xc, {})), f.__name__
    if K <= 1024:
        honest = max(2, int(0.8 * K))
        a = bz.Krum(Xc, {"honestSize": honest})
        ia = bz.aggregators.Krum.last_index
        b = bz.Krum(P, {"honestSize": honest})
        assert bz.aggregators.Krum.last_index == ia and torch.equal(a, b)


@pytest.mark.parametrize("K,d", [(1000, 300), (513, 130), (300, 77), (1024, 64)])
def test_median_value_histogram_edge_columns(K, d):
    """The median's value-linear histogram (coordinate.hip median_vhist, K > 512) and its
    fall-backs to the bitwise selection: spread columns; a column with a few huge outliers
    (the rank's bin holds nearly every key: more than the compaction takes); clustered
    columns; +-inf (an infinite range); a tiny and a subnormal range (the bin scale
    overflows); an all-equal and a +-0 column; heavy ties.  Every result equals torch's."""
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K + 3 * d)
    X = torch.randn(K, d, generator=g)
    X[:5, 0] = 1e30
    X[:, 1] = 0.03 + 1e-3 * torch.randn(K, generator=g)
    X[0, 2] = float("inf")
    X[1, 3] = float("-inf")
    X[:, 4] = 1.0 + torch.arange(K, dtype=torch.float32) * 1e-7
    X[:, 5] = 1e-40 * torch.randint(0, 3, (K,), generator=g).float()
    X[:, 6] = 2.5
    X[:, 7] = 0.0
    X[::2, 7] = -0.0
    X[:, 8] = torch.round(X[:, 8] * 2)
    X[:, 9] = -X[:, 9].abs()
    X[K // 2:, 10] = 1e4 * X[K // 2:, 10]
    X[:K // 2 + 5, 11] = float("inf")                  # the median is +inf
    X[:K // 2 + 5, 12] = 3e38                          # ... a huge finite value
    assert np.array_equal(bz.median(X.cuda()).cpu().numpy(), orc.median(X).numpy())
