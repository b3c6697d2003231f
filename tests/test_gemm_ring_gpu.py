"""gemm4p's ring pipeline for NT products (EPI_RING: gemm4r_kernel, a 4-slot ring of 32-deep
K stages) — the same MFMA accumulation order as the two-buffer kernel, so results must be
bitwise equal to it (bias, GELU + pre-activation aux, batched items, ragged M / N tails), and
close to an fp32 torch product."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _r(*s, g):
    return (torch.rand(*s, device="cuda", generator=g) * 2 - 1).bfloat16()


@pytest.mark.parametrize("M,N,K", [(4096, 2048, 1024), (1000, 2056, 640), (264, 136, 128), (2048, 6144, 192),
                                   (520, 776, 256)])
@pytest.mark.parametrize("bias", [False, True])
def test_ring_bitwise_equals_two_buffer_kernel(M, N, K, bias):
    from paddle_hackathon_amd.ops import gemm as G
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a, bt = _r(M, K, g=g), _r(N, K, g=g)
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    ref = G.gemm_p(a, bt, bias=b, epi_extra=G.EPI_EARLY)
    got = G.gemm_p(a, bt, bias=b, epi_extra=G.EPI_EARLY | G.EPI_RING)
    assert torch.equal(got, ref)
    f32 = a.float() @ bt.float().t() + (b if bias else 0)
    assert ((got.float() - f32).norm() / f32.norm()).item() < 1e-2


def test_ring_gelu_aux_and_batched():
    from paddle_hackathon_amd.ops import gemm as G
    g = torch.Generator(device="cuda").manual_seed(7)
    M, N, K = 2048, 4096, 512
    a, bt = _r(M, K, g=g), _r(N, K, g=g)
    b = torch.randn(N, device="cuda", generator=g)
    aux0, aux1 = (torch.empty(M, N, dtype=torch.bfloat16, device="cuda") for _ in range(2))
    ref = G.gemm_p(a, bt, bias=b, gelu_aux=aux0, epi_extra=G.EPI_EARLY)
    got = G.gemm_p(a, bt, bias=b, gelu_aux=aux1, epi_extra=G.EPI_EARLY | G.EPI_RING)
    assert torch.equal(got, ref) and torch.equal(aux1, aux0)
    # batched items share one persistent grid
    x, y = _r(3, 520, 256, g=g), _r(3, 264, 256, g=g)
    out = G.bmm_p(x, y)   # NT
    ring = torch.empty_like(out)
    L = G._L()
    rc = L.pha_gemm4p_batched(G._DT[x.dtype], G._ptr(x), G._ptr(y), G._ptr(ring), 520, 264, 256, x.stride(1),
                              y.stride(1), ring.stride(1), 0, 0, 0, G.EPI_EARLY | G.EPI_RING, None,
                              G._num_cus(x.device), 0, None, 1, G._stream(x), None, 3, x.stride(0), y.stride(0),
                              ring.stride(0))
    assert rc == 0 and torch.equal(ring, out)


@pytest.mark.parametrize("M,N,K", [(4096, 2048, 1024), (1000, 2056, 640), (2048, 6144, 256), (520, 776, 320),
                                   (8192, 2048, 8192)])
def test_adeep_bitwise_equals_two_buffer_kernel(M, N, K, monkeypatch):
    """EPI_ADEEP (3 A + 2 B LDS slots): same MFMA order, bitwise equal to the two-buffer kernel"""
    from paddle_hackathon_amd.ops import gemm as G
    monkeypatch.setenv("PHA_G4P_ADEEP", "0")   # the reference: the default would pick A-deep at K >= 4096
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 1)
    a, bt = _r(M, K, g=g), _r(N, K, g=g)
    ref = G.gemm_p(a, bt, epi_extra=G.EPI_EARLY)
    got = G.gemm_p(a, bt, epi_extra=G.EPI_EARLY | G.EPI_ADEEP)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("lv", [40, 72, 104])
@pytest.mark.parametrize("M,N,K,bias", [(4096, 2048, 1024, True), (1000, 2056, 640, False), (520, 776, 4096, True),
                                        (2048, 6144, 128, True)])
def test_spread_dma_placement_bitwise(lv, M, N, K, bias, monkeypatch):
    """SPREAD (gemm4p.hip sp_na / sp_gb: the next-next K-tile's DMAs over 24-28 MFMA groups) only
    moves LDS-DMA issue points: bitwise equal to the shipped LV 8 schedule, incl. the first K-tile's
    counted wait with the previous tile's stores in flight"""
    from paddle_hackathon_amd.ops import gemm as G
    monkeypatch.setenv("PHA_G4P_ADEEP", "0")
    g = torch.Generator(device="cuda").manual_seed(M + N + K + lv)
    a, bt = _r(M, K, g=g), _r(N, K, g=g)
    b = torch.randn(N, device="cuda", generator=g) if bias else None
    monkeypatch.setenv("PHA_G4P_LV", "8")
    ref = G.gemm_p(a, bt, bias=b)
    monkeypatch.setenv("PHA_G4P_LV", str(lv))
    got = G.gemm_p(a, bt, bias=b)
    assert torch.equal(got, ref)
