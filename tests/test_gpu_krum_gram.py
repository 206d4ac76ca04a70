"""Krum through the Gram MFMA kernel (row f3, round 5; coordinate.hip krum_gram_bounds).

The Gram path bounds every pairwise distance, keeps the rows whose score bounds reach the
smallest upper bound, and recomputes those rows with the exact path's arithmetic, so its
index and row must EQUAL the exact pair-distance path's (GMAGG_KRUM=0) — and through it the
oracle's (M:197-204) — bit for bit, on spread data, exact ties, Byzantine rows anywhere,
panels, and the inputs that send it back to the exact path (non-finite Gram, too many
candidates)."""
import pytest
import torch

from oracle import aggregators as orc

pytestmark = pytest.mark.gpu


def _recipe(K, d, honest, seed, perm=True):
    """The C3 recipe shape: honest N(0, 0.05^2), Byzantine rows shifted N(0.25, 0.5^2)."""
    g = torch.Generator().manual_seed(seed)
    X = 0.05 * torch.randn(K, d, generator=g)
    X[honest:] = 0.25 + 0.5 * torch.randn(K - honest, d, generator=g)
    if perm:
        X = X[torch.randperm(K, generator=g)].contiguous()
    return X


def _both(X, honest, monkeypatch):
    import byzantine_aircomp_amd as bz
    Krum = bz.aggregators.Krum
    monkeypatch.setenv("GMAGG_KRUM", "1")
    a = bz.Krum(X, {"honestSize": honest})
    ia, info = Krum.last_index, dict(Krum.last_info)
    monkeypatch.setenv("GMAGG_KRUM", "0")
    b = bz.Krum(X, {"honestSize": honest})
    ib = Krum.last_index
    assert Krum.last_info["algo"] == "exact" and Krum.last_info["reason"] == "not_chosen"
    return a, ia, info, b, ib


@pytest.mark.parametrize("K,d,honest", [(64, 4096, 52), (100, 20_000, 80), (128, 65_536, 103),
                                        (200, 12_288, 160), (256, 262_144, 205), (33, 1000, 30)])
def test_gram_krum_equals_exact(K, d, honest, monkeypatch):
    X = _recipe(K, d, honest, K + d).cuda()
    a, ia, info, b, ib = _both(X, honest, monkeypatch)
    assert info["algo"] == "gram" and info["reason"] == "ok", info
    assert 1 <= info["candidates"] <= 128, info
    assert ia == ib and torch.equal(a, b)


@pytest.mark.parametrize("K,d,honest", [(64, 3000, 50), (120, 2048, 100)])
def test_gram_krum_vs_oracle(K, d, honest, monkeypatch):
    import byzantine_aircomp_amd as bz
    X = _recipe(K, d, honest, 7 * K + d)
    monkeypatch.setenv("GMAGG_KRUM", "1")
    out = bz.Krum(X.cuda(), {"honestSize": honest})
    assert bz.aggregators.Krum.last_info["algo"] == "gram"
    assert torch.equal(out.cpu(), orc.krum(X, {"honestSize": honest}))


def test_gram_krum_exact_ties(monkeypatch):
    """Rows 5..14 identical (equal scores): both paths take the first index."""
    X = _recipe(96, 8192, 80, 3, perm=False)
    X[5:15] = X[5]
    a, ia, info, b, ib = _both(X.cuda(), 80, monkeypatch)
    assert info["algo"] == "gram"
    assert ia == ib and torch.equal(a, b)


def test_gram_krum_byzantine_centre(monkeypatch):
    """Row 0 Byzantine: bounds from that centre are too loose for the honest rows' near-equal
    scores (too many candidates), so the Gram is recomputed around the row of the smallest
    upper bound; the result still equals the exact path's."""
    X = _recipe(256, 1 << 20, 205, 17, perm=False)
    X[[0, 230]] = X[[230, 0]]
    a, ia, info, b, ib = _both(X.cuda(), 205, monkeypatch)
    assert info["algo"] == "gram" and info["reason"] == "ok", info
    assert ia == ib and torch.equal(a, b)


def test_gram_krum_panels(monkeypatch):
    import byzantine_aircomp_amd as bz
    X = _recipe(160, 30_000, 128, 11).cuda()
    P = bz.ClientPanels.from_rows(X)
    monkeypatch.setenv("GMAGG_KRUM", "1")
    a = bz.Krum(P, {"honestSize": 128})
    ia, info = bz.aggregators.Krum.last_index, dict(bz.aggregators.Krum.last_info)
    monkeypatch.setenv("GMAGG_KRUM", "0")
    b = bz.Krum(X, {"honestSize": 128})
    assert info["algo"] == "gram", info
    assert bz.aggregators.Krum.last_index == ia and torch.equal(a, b)


def test_gram_krum_nonfinite_falls_back(monkeypatch):
    """An element far beyond the f16 headroom of its (row, block) scale — set by the block's
    first 128 columns, where row 3 sits 1e-6 from the centre row 0 — makes the Gram
    non-finite: the exact path answers.  (d = 65,536: blocks of 256 columns.)"""
    X = _recipe(64, 65_536, 50, 5, perm=False)
    X[3, :128] = X[0, :128] + 1e-6
    X[3, 200] = 1e6
    a, ia, info, b, ib = _both(X.cuda(), 50, monkeypatch)
    assert info["algo"] == "exact" and info["reason"] == "gram_nonfinite", info
    assert ia == ib and torch.equal(a, b)


def test_gram_krum_too_many_candidates_falls_back(monkeypatch):
    """200 identical rows: every score 0, every row a candidate (> 128)."""
    g = torch.Generator().manual_seed(2)
    X = torch.randn(1, 4096, generator=g).repeat(200, 1)
    a, ia, info, b, ib = _both(X.cuda(), 180, monkeypatch)
    assert info["algo"] == "exact" and info["reason"] == "candidates", info
    assert ia == ib and torch.equal(a, b)


def test_gram_krum_not_eligible(monkeypatch):
    """d % 4 != 0 (the Gram kernel's float4 stages) and K > 256 stay on the exact path."""
    import byzantine_aircomp_amd as bz
    monkeypatch.setenv("GMAGG_KRUM", "1")
    for K, d in ((64, 4099), (300, 4096)):
        X = _recipe(K, d, int(0.8 * K), K + d).cuda()
        bz.Krum(X, {"honestSize": int(0.8 * K)})
        assert bz.aggregators.Krum.last_info == {"algo": "exact", "candidates": 0,
                                                 "reason": "not_eligible"}


def test_gram_krum_auto_choice(monkeypatch):
    import byzantine_aircomp_amd as bz
    monkeypatch.delenv("GMAGG_KRUM", raising=False)
    for (K, d), want in (((64, 1 << 17), "gram"), ((50, 7850), "exact"), ((256, 1 << 13), "gram"),
                         ((64, 1 << 16), "exact"), ((128, 1 << 18), "gram")):
        X = _recipe(K, d, int(0.8 * K), K + d, perm=False).cuda()
        bz.Krum(X, {"honestSize": int(0.8 * K)})
        assert bz.aggregators.Krum.last_info["algo"] == want, (K, d)


@pytest.mark.parametrize("K,d", [(64, 4), (70, 60), (96, 1028), (255, 3000)])
def test_gram_krum_small_and_ragged(K, d, monkeypatch):
    """One Gram stage or less (d = 4, 60), a column count off the 64-column stage, K just
    under the 256-row tile: still the exact path's row."""
    X = _recipe(K, d, int(0.8 * K), 3 * K + d).cuda()
    a, ia, info, b, ib = _both(X, int(0.8 * K), monkeypatch)
    assert info["algo"] == "gram" or info["reason"] == "candidates", info
    assert ia == ib and torch.equal(a, b)


def test_gram_krum_panels_ragged(monkeypatch):
    """Panels whose last panel is partial (d = 1000 at W = 64)."""
    import byzantine_aircomp_amd as bz
    X = _recipe(200, 1000, 160, 21).cuda()
    P = bz.ClientPanels.from_rows(X)
    monkeypatch.setenv("GMAGG_KRUM", "1")
    a = bz.Krum(P, {"honestSize": 160})
    ia, info = bz.aggregators.Krum.last_index, dict(bz.aggregators.Krum.last_info)
    monkeypatch.setenv("GMAGG_KRUM", "0")
    b = bz.Krum(X, {"honestSize": 160})
    assert info["algo"] == "gram" or info["reason"] == "candidates", info
    assert bz.aggregators.Krum.last_index == ia and torch.equal(a, b)


@pytest.mark.parametrize("scale", [1e3, 1e6])
def test_gram_krum_huge_byzantine_rows(scale, monkeypatch):
    """Byzantine rows `scale` x the honest spread: the Gram kernel's f16 scale is
    one power of two per column block, set by the block's largest |x - p| — a Byzantine row —
    so the honest rows' elements sit scale-times lower in f16 (near or in the subnormal
    range at 1e6).  The bounds carry that absolute error (krum_gram_bounds' A term, from the
    exported block exponents): the Gram path either returns the exact path's row or, when
    the bounds leave too many candidates, hands the call to the exact path."""
    g = torch.Generator().manual_seed(int(scale) % 1000 + 5)
    K, d, honest = 128, 65_536, 103
    X = 0.05 * torch.randn(K, d, generator=g)
    X[honest:] = scale * (0.25 + 0.5 * torch.randn(K - honest, d, generator=g))
    X = X[torch.randperm(K, generator=g)].contiguous()
    if bool(torch.all(X[0].abs() > 1.0)):            # keep an honest centre row
        X[[0, 1]] = X[[1, 0]]
    a, ia, info, b, ib = _both(X.cuda(), honest, monkeypatch)
    assert info["algo"] == "gram" or info["reason"] in ("candidates", "gram_nonfinite"), info
    assert ia == ib and torch.equal(a, b), (ia, ib, info)
