"""Packed per-head projection weights (packing.py) and their gradient paths on CPU:
the one-add accumulation into a bucket laid out in pack order must give exactly
the per-parameter autograd gradients, across accumulation micro-steps."""
import torch

from differential_transformer_replication_amd import control as C
from differential_transformer_replication_amd.dp import BucketedAllReduce


def _model(seed=0):
    torch.manual_seed(seed)
    return C.StandardTransformer(97, 64, 4, 2, 24, 0.0)


def test_packed_grad_accumulation_matches_autograd():
    ref, m = _model(), _model()
    sync = BucketedAllReduce(m, bucket_cap_mb=0.05)          # several buckets, world size 1
    holders = [blk.attn._pack for blk in m.blocks] if hasattr(m.blocks[0], "attn") else \
        [mod._pack for mod in m.modules() if isinstance(mod, C.MultiHeadAttention)]
    assert holders and all("grad" in h for h in holders)
    calls = []
    for h in holders:                                        # count the one-add path's reports
        h["on_ready"] = (lambda f: (lambda p: (calls.append(p), f(p))))(h["on_ready"])
    g = torch.Generator().manual_seed(1)
    for _ in range(2):                                       # two micro-steps accumulate
        idx = torch.randint(0, 97, (2, 24), generator=g)
        tgt = torch.randint(0, 97, (2, 24), generator=g)
        ref(idx, tgt)[1].backward()
        m(idx, tgt)[1].backward()
    for (n, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
        assert torch.equal(a.grad, b.grad), n
    n_packed = sum(len(mod.packed_params()) for mod in m.modules() if isinstance(mod, C.MultiHeadAttention))
    assert len(calls) == 2 * n_packed                        # every packed weight, both micro-steps
    # the bucket views are intact and zero_grad keeps them
    sync.zero_grad()
    for mod in m.modules():
        if isinstance(mod, C.MultiHeadAttention):
            pp = mod.packed_params()
            base = pp[0].grad.data_ptr()
            off = 0
            for p in pp:
                assert p.grad.data_ptr() == base + 4 * off and float(p.grad.abs().sum()) == 0.0
                off += p.numel()


def test_unbound_grads_fall_back_to_autograd():
    """set_to_none (or any replaced .grad) silently returns to per-parameter grads."""
    ref, m = _model(), _model()
    BucketedAllReduce(m)
    for p in m.parameters():
        p.grad = None
    idx = torch.randint(0, 97, (2, 24), generator=torch.Generator().manual_seed(2))
    ref(idx, idx)[1].backward()
    m(idx, idx)[1].backward()
    for (n, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
        assert torch.equal(a.grad, b.grad), n


def test_lambda_pack_grads_match_per_head_reference():
    """MultiHeadDiffAttention / MultiHeadAlternatingDiffAttention coefficients from the
    packed lambda vectors: same values and gradients as the per-head reference
    formula (diff_transformer.py:41-48, Ndiff_transformer.py:79-93), unbound and
    bound to a DP bucket (one-add path)."""
    from differential_transformer_replication_amd import diff_transformer as D
    from differential_transformer_replication_amd import Ndiff_transformer as ND
    for bound in (False, True):
        torch.manual_seed(0)
        m = D.MultiHeadDiffAttention(3, 8, 48, 0.0, 16)
        nd = ND.MultiHeadAlternatingDiffAttention(2, 8, 32, 0.0, 16, 3)
        for mod in (m, nd):
            for p in mod.parameters():
                if p.dim() == 1 and p.numel() == 8:
                    p.data.normal_(0, 0.1)
            if bound:
                BucketedAllReduce(mod)
        w = torch.randn(3, 2, generator=torch.Generator().manual_seed(1))
        (m.coefficients(2) * w).sum().backward()
        for h, head in enumerate(m.heads):
            ps = [head.lambda_q1, head.lambda_k1, head.lambda_q2, head.lambda_k2]
            c = [q.detach().clone().requires_grad_(True) for q in ps]
            lam = (torch.exp(c[0] * c[1]) - torch.exp(c[2] * c[3]) + head.lambda_init).mean()
            (-lam * w[h, 1]).backward()
            for q, r in zip(ps, c):
                assert torch.allclose(q.grad, r.grad, rtol=1e-6, atol=1e-7)
        w2 = torch.randn(2, 3, generator=torch.Generator().manual_seed(2))
        (nd.coefficients(2) * w2).sum().backward()
        for h, head in enumerate(nd.heads):
            lq = [q.detach().clone().requires_grad_(True) for q in head.lambda_qs]
            lk = [q.detach().clone().requires_grad_(True) for q in head.lambda_ks]
            e = [torch.exp(a * b) for a, b in zip(lq, lk)]
            lams = [(e[i] - (e[i - 1] if i else 0) + head.lambda_init).mean() for i in range(3)]
            sum(l * (1 if i % 2 == 0 else -1) * w2[h, i] for i, l in enumerate(lams)).backward()
            for q, r in zip(list(head.lambda_qs) + list(head.lambda_ks), lq + lk):
                assert torch.allclose(q.grad, r.grad, rtol=1e-6, atol=1e-7)
