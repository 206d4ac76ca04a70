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


def test_problem_panels_layout():
    """batched.ProblemPanels: problem p is one ClientPanels block (element (p, k, j) at
    data[p, j // W, k, j % W]); strides as the batched C ABI takes them."""
    from byzantine_aircomp_amd.batched import ProblemPanels
    for P, K, d in [(1, 5, 7), (3, 50, 300), (2, 200, 1001)]:
        X = torch.randn(P, K, d)
        B = ProblemPanels(P, K, d, device="cpu")
        for p in range(P):
            B.data[p].copy_(ClientPanels.from_rows(X[p], device="cpu").data)
        assert B.W == ClientPanels(K, d, device="cpu").W
        assert torch.equal(B.to_rows(), X)
        assert B.panel_stride == K * B.W and B.problem_stride == B.npan * K * B.W
        assert B.data.stride(0) == B.problem_stride and B.data.stride(1) == B.panel_stride
        p, k, j = P - 1, K - 1, d - 1
        assert B.data[p, j // B.W, k, j % B.W] == X[p, k, j]
