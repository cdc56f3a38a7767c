"""Grouped MFMA GEMMs of the projected feature tables (grk_grouped_gemm /
grk_grouped_wgrad, csrc/grk_ggemm.hip) against torch fp32 GEMMs of the same bf16
operands, and the model's grouped projection (functional.project_blocks) against
the torch.bmm projection it replaces, from identical parameters."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'

# C2's projected tables: 3 x 10001, 3 x 1001, 4 x 101, 4 x 11 (item), 8 x 1001 (user);
# plus row counts at and around the 128-row tile edge
ROWS = [11, 101, 1001, 10001, 1, 127, 128, 129, 64]


def _bf(shape, gen, scale=1.0):
    return (scale * torch.randn(shape, generator=gen, device=DEV)).bfloat16()


@pytest.mark.parametrize('b_layout', [0, 1])
@pytest.mark.parametrize('out', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('d', [512, 64])
def test_grouped_gemm_matches_fp32_matmul(b_layout, out, d):
    """C_g = A_g . B_g^T (layout 0, the forward P = E W^T) or A_g . B_g (layout 1, the
    backward dE = dP W), B_g a column block of one wide weight (strided view): fp32
    output within 1e-5 normwise of the fp32 product of the bf16 operands (both
    accumulate in fp32, in different orders), bf16 output within one bf16 rounding
    of it elementwise."""
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(0)
    nb = len(ROWS) + 1
    W = _bf((d, nb * d), g, 0.05)
    groups, refs = [], []
    for i, rows in enumerate(ROWS):
        A = _bf((rows, d), g)
        blk = W[:, (i + 1) * d:(i + 2) * d]
        C = torch.full((rows, d), float('nan'), dtype=out, device=DEV)
        groups.append((A, blk, C))
        refs.append(A.float() @ (blk.float().t() if b_layout == 0 else blk.float()))
    K.grouped_gemm(groups, n=d, k=d, b_layout=b_layout)
    torch.cuda.synchronize()
    for (A, _, C), ref in zip(groups, refs):
        got = C.float()
        assert torch.isfinite(got).all()
        if out == torch.float32:
            assert float((got - ref).norm() / ref.norm()) < 1e-5, A.shape
        else:
            assert ((got - ref).abs() <= ref.abs() * 2 ** -8 + 1e-6).all(), A.shape


@pytest.mark.parametrize('d', [512, 64])
def test_grouped_wgrad_matches_fp32_matmul(d):
    """C_g = A_g^T B_g over each group's rows padded to 32 with zero A rows (B's rows
    past b_rows read its last row: exact zeros), written into column blocks of one
    fp32 gradient; groups above 1024 rows are split over K and summed in slice order.
    Within 1e-5 normwise of the fp32 product, untouched columns unchanged."""
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(1)
    nb = len(ROWS)
    dW = torch.full((d, nb * d), 7.0, device=DEV)
    groups, refs = [], []
    for i, rows in enumerate(ROWS):
        pad = -(-rows // 32) * 32
        A = torch.zeros(pad + 8, d, dtype=torch.bfloat16, device=DEV)
        A[:rows] = _bf((rows, d), g)
        B = _bf((rows, d), g)
        groups.append((A, B, dW[:, i * d:(i + 1) * d], pad, rows))
        refs.append(A[:rows].float().t() @ B.float())
    K.grouped_wgrad(groups[:-1], m=d, n=d)       # the last block is left alone
    torch.cuda.synchronize()
    for (A, B, C, _, _), ref in zip(groups[:-1], refs[:-1]):
        assert float((C - ref).norm() / ref.norm()) < 1e-5, B.shape
    assert (dW[:, (nb - 1) * d:] == 7.0).all()


def test_grouped_wgrad_is_deterministic():
    """Split-K slices summed in slice order: two launches give the same bits."""
    from tencent_recommendation_2025_amd import kernels as K
    g = torch.Generator(device=DEV).manual_seed(2)
    A = _bf((10016, 512), g)
    A[10001:] = 0
    B = _bf((10001, 512), g)
    outs = []
    for _ in range(2):
        C = torch.empty(512, 512, device=DEV)
        K.grouped_wgrad([(A, B, C, 10016, 10001)], m=512, n=512)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_grouped_projection_matches_bmm_projection():
    """The fused model's projections on the grouped GEMMs vs torch.bmm, from identical
    parameters and batch: the same loss (1e-5; the projected rows differ by bf16
    roundings of different summation orders), and every gradient -- dnn weights
    (fp32 here, bf16 through the bmm path), feature-table rows, all others -- within
    1e-2 normwise (the bmm path's bf16 weight gradient: ~2^-9 per element)."""
    from tencent_recommendation_2025_amd import synthetic as S
    from tencent_recommendation_2025_amd.model import BaselineModel
    from tencent_recommendation_2025_amd.optim import FusedAdamW
    from tencent_recommendation_2025_amd.train import Trainer
    cfg = S.SyntheticConfig(batch_size=16, maxlen=40, num_items=3000, num_users=400, min_len=6)
    stats, types = S.feature_schema(cfg)
    out = {}
    for grouped in (False, True):
        args = S.make_args(hidden_units=128, maxlen=40, num_blocks=2, num_heads=2, grouped_proj=grouped)
        torch.manual_seed(0)
        m = BaselineModel(cfg.num_users, cfg.num_items, stats, types, args).to(DEV)
        opt = FusedAdamW(m, lr=1e-3)
        tr = Trainer(m, opt, loss='bce')
        batch = S.make_batch(cfg, torch.Generator(device=DEV).manual_seed(3), DEV)
        if grouped:
            assert m._grouped_proj('item') is not None and m._grouped_proj('user') is not None
        opt.zero_grad()
        opt.begin_step(batch)
        loss = tr.compute_loss(batch)
        loss.backward()
        grads = {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}
        for grp in opt.groups:
            if grp.dense_grads:   # the bmm path collects per equal-row-count stack, the grouped one per table
                full = torch.zeros(grp.rows, grp.dim, device=DEV)
                for off, gd in grp.dense_grads.items():
                    full[off:off + gd.shape[0]] += gd.float()
                grads[f'table group {grp.name}'] = full
        out[grouped] = (loss.item(), grads)
    (l0, g0), (l1, g1) = out[False], out[True]
    assert abs(l0 - l1) < 1e-5 * abs(l0), (l0, l1)
    assert 'table group small' in g0 and set(g0) == set(g1)
    for k in g0:
        a, b = g0[k], g1[k]
        assert float((a - b).norm() / a.norm().clamp(min=1e-30)) < 1e-2, k
