"""getVarience (M:127-129) as one HIP streaming pass (gm_honest_variance_f32)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(X, H):
    h = X[:H].double()
    return float(((h - h.mean(dim=0)) ** 2).sum(dim=1).mean())


def _ref_fp32(X, H):            # the reference's own fp32 expression (M:128-129)
    h = X[:H]
    return float(torch.mean(((h - h.mean(dim=0)) ** 2).sum(dim=1)))


@pytest.mark.parametrize("K,H,d,offset", [(50, 40, 7850, 0.0), (50, 50, 7852, 0.0),
                                          (7, 3, 333, 0.0), (1000, 800, 65_536, 0.0),
                                          (64, 60, 4096, 100.0), (1, 1, 9, 0.0)])
def test_honest_variance_rows(K, H, d, offset):
    from byzantine_aircomp_amd.training import getVarience
    g = torch.Generator().manual_seed(K + d)
    X = offset + 0.05 * torch.randn(K, d, generator=g)
    X[H:] += 0.3
    got = getVarience(X.cuda(), H)
    assert got.dtype == torch.float32 and got.dim() == 0
    want = _ref(X, H)
    assert abs(float(got) - want) <= 1e-6 * max(want, 1e-30) + 1e-30
    # and within fp32 rounding of the reference's own expression (not at a large offset,
    # where the reference's fp32 mean loses digits that the fp64 pass keeps)
    if offset == 0.0:
        assert abs(float(got) - _ref_fp32(X, H)) <= 1e-5 * want


def test_honest_variance_strided_and_panels():
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.training import getVarience
    g = torch.Generator().manual_seed(3)
    big = torch.randn(300, 5000, generator=g)
    X = big[:, :4096]                      # ldx 5000 > d
    want = _ref(X, 250)
    assert abs(float(getVarience(X.cuda(), 250)) - want) <= 1e-6 * want
    P = bz.ClientPanels.from_rows(X.contiguous().cuda())
    assert abs(float(getVarience(P, 250)) - want) <= 1e-6 * want
