"""ClientPanels host logic on CPU tensors (layout round trips; no kernels)."""
import torch

from byzantine_aircomp_amd.panels import ClientPanels


def test_round_trips_and_partial_last_panel():
    for K, d in [(1, 1), (3, 31), (50, 7850), (1000, 100), (7, 257)]:
        X = torch.randn(K, d)
        P = ClientPanels.from_rows(X, device="cpu")
        assert P.data.shape == (-(-d // P.W), K, P.W)
        assert torch.equal(P.to_rows(), X)
        Q = ClientPanels(K, d, device="cpu")
        for k in range(K):
            Q.store(k, X[k])
        assert torch.equal(Q.data, P.data)
        assert torch.equal(P.row(K - 1), X[K - 1])
        assert torch.allclose(P.mean(), X.mean(dim=0), rtol=1e-6, atol=1e-7)
        # element (k, j) at data[j // W, k, j % W]; padding columns are zero
        j = d - 1
        assert P.data[j // P.W, K - 1, j % P.W] == X[K - 1, j]
        if d % P.W:
            assert torch.count_nonzero(P.data[-1, :, d % P.W:]) == 0
