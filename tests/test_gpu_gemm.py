"""bf16 MFMA GEMM (csrc/gemm_bf16.hip) vs the fp32 PyTorch reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16).cuda()


@pytest.mark.parametrize("M,N,K,tile", [(256, 256, 128, (128, 128)), (512, 1024, 1024, (128, 128)),
                                        (128, 192, 64, (64, 64)), (4096, 64, 1024, (128, 64)),
                                        (1024, 1024, 4096, (64, 64)), (512, 256, 256, (256, 128)),
                                        (256, 256, 128, (128, 128, 4)), (512, 1024, 1024, (128, 128, 3)),
                                        (256, 512, 64, (128, 128, 3)), (512, 256, 1024, (128, 128, 4))])
def test_gemm_f32_epilogue(native_built, M, N, K, tile):
    from sharetrade.ops.gemm import EPI_F32, gemm_nt

    A, B = _bf((M, K), 1), _bf((N, K), 2)
    out = torch.empty(M, N, dtype=torch.float32, device="cuda")
    gemm_nt(A, B, out, EPI_F32, tile=tile, alpha=0.5)
    ref = 0.5 * (A.float() @ B.float().t())
    torch.cuda.synchronize()
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
    # accumulate
    gemm_nt(A, B, out, EPI_F32, tile=tile, alpha=0.5, accumulate=True)
    assert torch.allclose(out, 2 * ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("tile", [(128, 128), (64, 64), (256, 128), (128, 128, 3), (128, 128, 4)])
def test_gemm_bf16_bias_relu_and_transposed_out(native_built, tile):
    from sharetrade.ops.gemm import EPI_BF16, gemm_nt

    M, N, K = 512, 256, 320
    A, B = _bf((M, K), 3), _bf((N, K), 4)
    bias = torch.randn(N, device="cuda")
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    outT = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
    gemm_nt(A, B, out, EPI_BF16, tile=tile, outT=outT, bias=bias, relu=True)
    ref = torch.relu(A.float() @ B.float().t() + bias)
    torch.cuda.synchronize()
    assert torch.allclose(out.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    assert torch.equal(outT, out.t().contiguous())


@pytest.mark.parametrize("tile", [(128, 128), (64, 64), (128, 64), (256, 128), (128, 128, 3)])
def test_gemm_bf16_qhead_partials(native_built, tile):
    """qhead: the next layer's head (nq <= 4 rows) folded into the bf16 epilogue -- the per-row partial sums over
    each wave's BN / 2 columns add up to the stored bf16 output times the head rows (fp32 reference); the output
    itself is unchanged; two problems of one batched launch write their own partials."""
    from sharetrade.ops.gemm import EPI_BF16, gemm_nt, gemm_nt_batched

    M, N, K = 512, 256, 320
    A, B = _bf((M, K), 13), _bf((N, K), 14)
    bias = torch.randn(N, device="cuda")
    Wq = _bf((3, N), 15, 0.1)
    wn = tile[1] // 2
    qp = torch.full((N // wn, M, 4), float("nan"), device="cuda")
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    out0 = torch.empty_like(out)
    gemm_nt(A, B, out0, EPI_BF16, tile=tile, bias=bias, relu=True)
    gemm_nt(A, B, out, EPI_BF16, tile=tile, bias=bias, relu=True, qhead=(Wq, qp))
    torch.cuda.synchronize()
    assert torch.equal(out, out0)
    ref = out.float() @ Wq.float().t()
    got = qp.sum(0)
    assert torch.allclose(got[:, :3], ref, rtol=1e-4, atol=1e-4 * float(ref.abs().max()))
    assert float(got[:, 3].abs().max()) == 0.0
    with pytest.raises(RuntimeError):   # a partial buffer of the wrong part count is refused, not overrun
        gemm_nt(A, B, out, EPI_BF16, tile=tile, bias=bias, relu=True, qhead=(Wq, qp[:1].contiguous()))
    if len(tile) == 2:
        A2 = _bf((M, K), 16)
        qp2 = torch.zeros_like(qp)
        out2 = torch.empty_like(out)
        qp.zero_()
        gemm_nt_batched([(A, B, out, dict(bias=bias, relu=True, qhead=(Wq, qp))),
                         (A2, B, out2, dict(bias=bias, relu=True, qhead=(Wq, qp2)))], EPI_BF16, tile=tile)
        torch.cuda.synchronize()
        assert torch.allclose(qp.sum(0)[:, :3], ref, rtol=1e-4, atol=1e-4 * float(ref.abs().max()))
        ref2 = out2.float() @ Wq.float().t()
        assert torch.allclose(qp2.sum(0)[:, :3], ref2, rtol=1e-4, atol=1e-4 * float(ref2.abs().max()))


@pytest.mark.parametrize("tile", [(64, 64), (256, 128), (128, 128, 4)])
def test_gemm_relu_grad_epilogue(native_built, tile):
    from sharetrade.ops.gemm import EPI_RELU_GRAD, gemm_nt

    M, N, K = 256, 128, 64
    A, B = _bf((M, K), 5), _bf((N, K), 6)
    act = torch.relu(torch.randn(M, N, device="cuda")).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    outT = torch.empty(N, M, dtype=torch.bfloat16, device="cuda")
    gemm_nt(A, B, out, EPI_RELU_GRAD, tile=tile, outT=outT, auxT=act.t().contiguous())
    ref = (A.float() @ B.float().t()) * (act.float() > 0)
    torch.cuda.synchronize()
    assert torch.allclose(out.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    assert torch.equal(outT, out.t().contiguous())


def test_gemm_rejects_bad_shapes(native_built):
    from sharetrade.ops.gemm import EPI_F32, gemm_nt

    A, B = _bf((100, 64), 1), _bf((128, 64), 2)
    with pytest.raises(ValueError):
        gemm_nt(A, B, torch.empty(100, 128, device="cuda"), EPI_F32)


@pytest.mark.parametrize("M,N,K,tile,sk", [(1024, 1024, 4096, (128, 128), "auto"), (768, 256, 16384, (64, 64), 8),
                                           (768, 64, 16384, (64, 64), "auto"),
                                           (1024, 1024, 4096, (128, 128, 3), "auto")])
def test_gemm_split_k(native_built, M, N, K, tile, sk):
    from sharetrade.ops.gemm import EPI_F32, gemm_nt, pick_splitk

    A, B = _bf((M, K), 7), _bf((N, K), 8)
    bias = torch.randn(N, device="cuda")
    out = torch.full((M, N), float("nan"), dtype=torch.float32, device="cuda")   # zeroed by the wrapper
    gemm_nt(A, B, out, EPI_F32, tile=tile, splitk=sk, bias=bias)
    ref = A.float() @ B.float().t() + bias
    torch.cuda.synchronize()
    if sk == "auto":
        assert pick_splitk(M, N, K, tile) > 1
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
    gemm_nt(A, B, out, EPI_F32, tile=tile, splitk=sk, accumulate=True)   # bias not re-added
    assert torch.allclose(out, 2 * ref - bias, rtol=1e-4, atol=1e-3 * float(ref.abs().max()))


@pytest.mark.parametrize("M,N,K", [(512, 256, 320), (1024, 512, 1024), (256, 1024, 64)])
def test_gemm_256x256_tile(native_built, M, N, K):
    """256x256 tile (4 waves of 128x128 accumulators): every epilogue but the transposed output,
    which the tile refuses (its C^T staging would not fit in LDS)."""
    from sharetrade.ops.gemm import EPI_BF16, EPI_F32, EPI_RELU_GRAD, gemm_nt

    A, B = _bf((M, K), 7), _bf((N, K), 8)
    bias = torch.randn(N, device="cuda")
    ref = A.float() @ B.float().t()
    out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    gemm_nt(A, B, out, EPI_BF16, tile=(256, 256), bias=bias, relu=True)
    r = torch.relu(ref + bias)
    torch.cuda.synchronize()
    assert torch.allclose(out.float(), r, rtol=1e-2, atol=1e-2 * float(r.abs().max()))
    o32 = torch.empty(M, N, device="cuda")
    gemm_nt(A, B, o32, EPI_F32, tile=(256, 256), alpha=0.5)
    torch.cuda.synchronize()
    assert torch.allclose(o32, 0.5 * ref, rtol=1e-4, atol=1e-3)
    act = torch.relu(torch.randn(M, N, device="cuda")).to(torch.bfloat16)
    gemm_nt(A, B, out, EPI_RELU_GRAD, tile=(256, 256), auxT=act.t().contiguous())
    r = ref * (act.float() > 0)
    torch.cuda.synchronize()
    assert torch.allclose(out.float(), r, rtol=1e-2, atol=1e-2 * float(r.abs().max()))
    with pytest.raises(RuntimeError):
        gemm_nt(A, B, out, EPI_BF16, tile=(256, 256), outT=torch.empty(N, M, dtype=torch.bfloat16, device="cuda"))


@pytest.mark.parametrize("epi,tile,sk", [(0, (128, 128), 1), (2, (64, 64), 1), (2, (128, 128), 4), (1, (128, 64), 1)])
def test_gemm_batched_equals_single_launches(native_built, epi, tile, sk):
    """gemm_nt_batched: 3 same-shape problems in one grid == 3 single launches, bit for bit."""
    from sharetrade.ops.gemm import EPI_BF16, EPI_F32, EPI_RELU_GRAD, gemm_nt, gemm_nt_batched

    M, N, K = 512, 256, 1024
    probs, outs1, outs2 = [], [], []
    for i in range(3):
        A, B = _bf((M, K), 20 + i), _bf((N, K), 30 + i)
        kw = {}
        if epi == EPI_BF16:
            kw = dict(bias=torch.randn(N, device="cuda"), relu=True,
                      outT=torch.empty(N, M, dtype=torch.bfloat16, device="cuda"))
        elif epi == EPI_RELU_GRAD:
            kw = dict(auxT=torch.relu(torch.randn(N, M, device="cuda")).to(torch.bfloat16),
                      outT=torch.empty(N, M, dtype=torch.bfloat16, device="cuda"))
        else:
            kw = dict(splitk=sk, bias=torch.randn(N, device="cuda"))
        dt = torch.float32 if epi == EPI_F32 else torch.bfloat16
        o1, o2 = torch.empty(M, N, dtype=dt, device="cuda"), torch.empty(M, N, dtype=dt, device="cuda")
        kw2 = dict(kw)
        if "outT" in kw:
            kw2["outT"] = torch.empty_like(kw["outT"])
        gemm_nt(A, B, o1, epi, tile=tile, **kw)
        probs.append((A, B, o2, kw2))
        outs1.append((o1, kw.get("outT")))
        outs2.append((o2, kw2.get("outT")))
    gemm_nt_batched(probs, epi, tile=tile)
    torch.cuda.synchronize()
    for (o1, t1), (o2, t2) in zip(outs1, outs2):
        if sk > 1:
            assert torch.allclose(o1, o2, rtol=1e-5, atol=1e-4)   # split-K: atomic summation order
        else:
            assert torch.equal(o1, o2)
        if t1 is not None:
            assert torch.equal(t1, t2)


def test_gemm_grouped_mixed_shapes(native_built):
    """gemm_nt_batched with different shapes per problem (grouped GEMM) == single launches."""
    from sharetrade.ops.gemm import EPI_BF16, gemm_nt, gemm_nt_batched

    shapes = [(1024, 256, 512), (256, 512, 128), (512, 128, 1024)]
    probs, refs = [], []
    for i, (M, N, K) in enumerate(shapes):
        A, B = _bf((M, K), 50 + i), _bf((N, K), 60 + i)
        bias = torch.randn(N, device="cuda")
        r = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        gemm_nt(A, B, r, EPI_BF16, tile=(128, 128), bias=bias, relu=True)
        o = torch.empty_like(r)
        probs.append((A, B, o, dict(bias=bias, relu=True)))
        refs.append(r)
    gemm_nt_batched(probs, EPI_BF16, tile=(128, 128))
    torch.cuda.synchronize()
    for (_, _, o, _), r in zip(probs, refs):
        assert torch.equal(o, r)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 256, 128), (256, 512, 192), (1024, 768, 1024),
                                   (2048, 1024, 512)])
def test_gemm_pingpong_matches_128_tile(native_built, M, N, K):
    """256x256 ping-pong kernel (8 waves, two groups one barrier interval apart, LDS-DMA staging with
    counted waits): bit-identical to the 128x128 kernel (same k order per output), both epilogues;
    nk = 1, 2, 3 cover the pipeline fill / drain paths.  Repeated launches: a staging race would show
    as a mismatch on some run."""
    from sharetrade.ops.gemm import EPI_BF16, EPI_F32, gemm_nt

    A, B = _bf((M, K), 11), _bf((N, K), 12)
    bias = torch.randn(N, device="cuda")
    ref = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
    gemm_nt(A, B, ref, EPI_BF16, tile=(128, 128), bias=bias, relu=True)
    out = torch.empty_like(ref)
    for t in ((256, 256, "pp"), (256, 256, "ppp"), (256, 256, "w4")):
        for _ in range(3):
            out.fill_(7)
            gemm_nt(A, B, out, EPI_BF16, tile=t, bias=bias, relu=True)
            torch.cuda.synchronize()
            assert torch.equal(out, ref), t
    o32w = torch.full((M, N), float("nan"), device="cuda")
    r32 = torch.empty(M, N, device="cuda")
    gemm_nt(A, B, r32, EPI_F32, tile=(128, 128), bias=bias, alpha=0.5)
    o32 = torch.full((M, N), float("nan"), device="cuda")
    gemm_nt(A, B, o32, EPI_F32, tile=(256, 256, "pp"), bias=bias, alpha=0.5)
    gemm_nt(A, B, o32w, EPI_F32, tile=(256, 256, "w4"), bias=bias, alpha=0.5)
    torch.cuda.synchronize()
    assert torch.equal(o32, r32) and torch.equal(o32w, r32)
    gemm_nt(A, B, o32, EPI_F32, tile=(256, 256, "pp"), alpha=0.5, accumulate=True)
    full = 0.5 * (A.float() @ B.float().t())
    torch.cuda.synchronize()
    assert torch.allclose(o32, r32 + full, rtol=1e-4, atol=1e-3 * float(full.abs().max()))
    with pytest.raises(RuntimeError):   # no transposed output
        gemm_nt(A, B, out, EPI_BF16, tile=(256, 256, "pp"), outT=torch.empty(N, M, dtype=torch.bfloat16, device="cuda"))


@pytest.mark.parametrize("sk", [1, 4])
def test_gemm_dual_equals_two_launches(native_built, sk):
    """gemm_dual: a relu-grad product (with C^T) and a differently shaped f32 product (split-K) in one
    grid == the two single launches."""
    from sharetrade.ops.gemm import EPI_F32, EPI_RELU_GRAD, gemm_dual, gemm_nt

    M0, N0, K0 = 512, 256, 256
    M1, N1, K1 = 256, 384, 1024
    A0, B0 = _bf((M0, K0), 41), _bf((N0, K0), 42)
    A1, B1 = _bf((M1, K1), 43), _bf((N1, K1), 44)
    aux = torch.relu(torch.randn(N0, M0, device="cuda")).to(torch.bfloat16)
    r0 = torch.empty(M0, N0, dtype=torch.bfloat16, device="cuda")
    r0T = torch.empty(N0, M0, dtype=torch.bfloat16, device="cuda")
    r1 = torch.empty(M1, N1, device="cuda")
    gemm_nt(A0, B0, r0, EPI_RELU_GRAD, tile=(128, 128), outT=r0T, auxT=aux)
    gemm_nt(A1, B1, r1, EPI_F32, tile=(128, 128), splitk=sk)
    o0, o0T, o1 = torch.empty_like(r0), torch.empty_like(r0T), torch.full_like(r1, float("nan"))
    gemm_dual((A0, B0, o0, dict(outT=o0T, auxT=aux)), EPI_RELU_GRAD, (A1, B1, o1, dict(splitk=sk)), EPI_F32)
    torch.cuda.synchronize()
    assert torch.equal(o0, r0) and torch.equal(o0T, r0T)
    if sk == 1:
        assert torch.equal(o1, r1)
    else:
        assert torch.allclose(o1, r1, rtol=1e-5, atol=1e-4)
