"""GPU parity of the Block-level kernels around the attention path: the block-per-row
LayerNorm backward on many rows, the Blocks' ``LayerNorm`` (ln1/ln2/ln_f) on the HIP
LN kernels, and the fused SwiGLU -- each against a float64 PyTorch reference of the
reference model's op (diff_transformer.py SwiGLU / nn.LayerNorm)."""
import pytest
import torch
from torch.nn import functional as F

from conftest import rel_err
from oracle import diffattn_oracle as orc
from test_gpu_parity import TOL, DEV, _ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,C", [(4099, 1024), (2051, 2048), (9000, 384), (1, 8192)])
def test_ln_backward_many_rows(dtype, rows, C):
    """Many rows per workgroup (odd counts: both parities of the double-buffered row
    slot), the per-block partials and their ordered reduction."""
    ops = _ops()
    g = torch.Generator().manual_seed(rows + C)
    x = torch.randn(rows, C, generator=g) * 2 + 0.5
    w = 1 + 0.1 * torch.randn(C, generator=g)
    b = 0.1 * torch.randn(C, generator=g)
    dy = torch.randn(rows, C, generator=g)
    xq = x.to(dtype).double().requires_grad_(True)
    w64, b64 = w.double().requires_grad_(True), b.double().requires_grad_(True)
    ref = orc.group_layer_norm(xq, w64, b64) * 0.2
    ref.backward(dy.to(dtype).double())
    xg = x.to(dtype).to(DEV).requires_grad_(True)
    wg, bg = w.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    out = ops.group_ln_scale(xg, wg, bg, 1e-5, 0.2)
    out.backward(dy.to(dtype).to(DEV))
    tol = TOL[dtype]
    assert rel_err(out.float().cpu(), ref) < tol
    assert rel_err(xg.grad.float().cpu(), xq.grad) < tol
    assert rel_err(wg.grad.cpu(), w64.grad) < tol
    assert rel_err(bg.grad.cpu(), b64.grad) < tol


@pytest.mark.parametrize("autocast", [False, True])
def test_block_layernorm_matches_torch(autocast):
    ops = _ops()
    torch.manual_seed(3)
    C = 768
    ln = ops.LayerNorm(C).to(DEV)
    with torch.no_grad():
        ln.weight.normal_(1.0, 0.1)
        ln.bias.normal_(0.0, 0.1)
    ref = torch.nn.LayerNorm(C).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in ln.state_dict().items()})
    x = torch.randn(4, 300, C) * 3
    dy = torch.randn(4, 300, C)
    xg = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        y = ln(xg)
    assert y.dtype == torch.float32                     # fp32 statistics and output, as F.layer_norm
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    r = ref(x64)
    r.backward(dy.double())
    assert rel_err(y.cpu(), r) < 1e-5
    assert rel_err(xg.grad.cpu(), x64.grad) < 1e-5
    assert rel_err(ln.weight.grad.cpu(), ref.weight.grad) < 1e-5
    assert rel_err(ln.bias.grad.cpu(), ref.bias.grad) < 1e-5


@pytest.mark.parametrize("ydt", [torch.bfloat16, torch.float16])
def test_block_layernorm_autocast_out(ydt):
    """ln1/ln2/ln_f under autocast write the autocast dtype directly (fp32 statistics,
    one rounding -- what the consuming GEMM's cast would produce) and take that
    dtype's gradient back (dta_ln_args.io_dtype)."""
    ops = _ops()
    torch.manual_seed(4)
    C = 1024
    ln = ops.LayerNorm(C, autocast_out=True).to(DEV)
    with torch.no_grad():
        ln.weight.normal_(1.0, 0.1)
        ln.bias.normal_(0.0, 0.1)
    ref = torch.nn.LayerNorm(C).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in ln.state_dict().items()})
    x = torch.randn(3, 257, C) * 2
    dy = torch.randn(3, 257, C).to(ydt)
    xg = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=ydt):
        y = ln(xg)
    assert y.dtype == ydt
    y.backward(dy.to(DEV))
    x64 = x.double().requires_grad_(True)
    r = ref(x64)
    r.backward(dy.double())
    assert rel_err(y.float().cpu(), r) < 1e-2
    # the output is the fp32 result rounded once
    assert rel_err(y.float().cpu(), r.to(ydt).double()) < 1e-2
    assert rel_err(xg.grad.cpu(), x64.grad) < 1e-5
    assert rel_err(ln.weight.grad.cpu(), ref.weight.grad) < 1e-5
    assert rel_err(ln.bias.grad.cpu(), ref.bias.grad) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_swiglu_matches_torch(dtype):
    ops = _ops()
    g = torch.Generator().manual_seed(7)
    a = torch.randn(3, 129, 1536, generator=g) * 3
    b = torch.randn(3, 129, 1536, generator=g)
    d = torch.randn(3, 129, 1536, generator=g)
    a64 = a.to(dtype).double().requires_grad_(True)
    b64 = b.to(dtype).double().requires_grad_(True)
    r = F.silu(a64) * b64
    r.backward(d.to(dtype).double())
    ag = a.to(dtype).to(DEV).requires_grad_(True)
    bg = b.to(dtype).to(DEV).requires_grad_(True)
    out = ops.swiglu(ag, bg)
    assert out.dtype == dtype
    out.backward(d.to(dtype).to(DEV))
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert rel_err(out.float().cpu(), r) < tol
    assert rel_err(ag.grad.float().cpu(), a64.grad) < tol
    assert rel_err(bg.grad.float().cpu(), b64.grad) < tol


def test_swiglu_module_uses_fused_kernel():
    """The Block's SwiGLU module routes through dta_swiglu over one packed GEMM
    (autograd node _PackedSwiGLU)."""
    from differential_transformer_replication_amd import diff_transformer as D
    m = D.SwiGLU(64, 256).to(DEV)
    y = m(torch.randn(2, 5, 64, device=DEV))
    assert type(y.grad_fn).__name__ == "_PackedSwiGLUBackward"


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_packed_swiglu_matches_two_linears(mode):
    """SwiGLU with gate/xform as one packed GEMM vs the reference module's two
    nn.Linear + silu * (diff_transformer.py:95-105), in fp64 on the CPU: output, input
    grad and every weight / bias grad (fp32 1e-4; bf16 autocast 2e-2)."""
    from differential_transformer_replication_amd import diff_transformer as D
    torch.manual_seed(3)
    m = D.SwiGLU(96, 256)
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0, 0.1)
    ref = {k: v.double().requires_grad_(True) for k, v in m.state_dict().items()}
    x = torch.randn(3, 37, 96)
    x64 = x.double().requires_grad_(True)
    g = torch.randn(3, 37, 256)
    r = F.silu(F.linear(x64, ref["linear_gate.weight"], ref["linear_gate.bias"])) * \
        F.linear(x64, ref["linear_xform.weight"], ref["linear_xform.bias"])
    r.backward(g.double())
    mg = m.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "bf16"):
        y = mg(xg)
    assert type(y.grad_fn).__name__ == "_PackedSwiGLUBackward"
    y.backward(g.to(DEV).to(y.dtype))
    tol = 1e-4 if mode == "fp32" else 2e-2
    assert rel_err(y.float().cpu(), r) < tol
    assert rel_err(xg.grad.float().cpu(), x64.grad) < tol
    for n, p in mg.named_parameters():
        assert p.grad.dtype == torch.float32
        assert rel_err(p.grad.cpu(), ref[n].grad) < tol, n
    # the parameters are row views of the packs; state_dict keys are the reference's
    assert set(mg.state_dict()) == set(ref)
    assert mg.linear_xform.weight.data_ptr() == mg.linear_gate.weight.data_ptr() + 256 * 96 * 4


@pytest.mark.parametrize("arch", ["diff", "ndiff"])
def test_bound_gradients_equal_autograd(arch):
    """The DP buckets' one-add paths (packed projection weights, packed lambda
    vectors, LayerNorm / GroupLayerNorm dw-db accumulated in place) give bitwise the
    gradients plain autograd gives, over two accumulation micro-steps."""
    from differential_transformer_replication_amd import diff_transformer as D, Ndiff_transformer as ND
    from differential_transformer_replication_amd.dp import BucketedAllReduce

    def build():
        torch.manual_seed(0)
        if arch == "diff":
            return D.DiffTransformer(97, 64, 2, 2, 32, 0.0).to(DEV)
        return ND.AlternatingDiffTransformer(97, 64, 2, 2, 32, 0.0, n_terms=3).to(DEV)

    ref, m = build(), build()
    for mod in (ref, m):
        for p in mod.parameters():
            if p.dim() == 1 and p.numel() == 16:
                with torch.no_grad():
                    p.copy_(torch.linspace(-0.2, 0.2, 16, device=DEV))
    BucketedAllReduce(m, bucket_cap_mb=0.5)
    g = torch.Generator().manual_seed(5)
    for _ in range(2):
        idx = torch.randint(0, 97, (2, 32), generator=g).to(DEV)
        tgt = torch.randint(0, 97, (2, 32), generator=g).to(DEV)
        ref(idx, tgt)[1].backward()
        m(idx, tgt)[1].backward()
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
        assert torch.equal(a.grad, b.grad), n


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("n", [8, 1000, 1 << 20, (1 << 20) + 5])
def test_accumulate_f32(dtype, n):
    """dta_accumulate_f32 (packing.accumulate): fp32 g += d for the packed-gradient
    buckets, bitwise equal to torch's fp32 add of the upcast gradient (tail included)."""
    from differential_transformer_replication_amd import packing
    gen = torch.Generator().manual_seed(n)
    g = torch.randn(n, generator=gen).to(DEV)
    d = torch.randn(n, generator=gen).to(dtype).to(DEV)
    ref = g + d.float()
    packing.accumulate(g, d)
    torch.cuda.synchronize()
    assert torch.equal(g, ref)


@pytest.mark.parametrize("O,I", [(1024, 1024), (3072, 1024), (512, 256), (96, 40)])
def test_weight_grad_split_k(O, I):
    """packing.weight_grad (dW = dy^T x, fp32 output, split over tokens for small
    outputs) against an fp64 product of the same bf16 operands."""
    from differential_transformer_replication_amd import packing
    K = 4096
    gen = torch.Generator().manual_seed(O + I)
    dy = torch.randn(K, O, generator=gen).to(torch.bfloat16)
    x = torch.randn(K, I, generator=gen).to(torch.bfloat16)
    ref = dy.double().t() @ x.double()
    dw = packing.weight_grad(dy.to(DEV), x.to(DEV))
    assert dw.dtype == torch.float32 and dw.shape == (O, I)
    assert rel_err(dw.cpu(), ref) < 1e-5


@pytest.mark.parametrize("mode", ["fp32", "bf16"])
def test_linear_op_matches_nn_linear(mode):
    """ops.linear (the MHA output projection and FFN output Linear) vs nn.Linear in fp64:
    output, input grad, weight and bias grads (fp32 1e-4; bf16 autocast 2e-2)."""
    from differential_transformer_replication_amd import ops as O_
    torch.manual_seed(4)
    lin = torch.nn.Linear(256, 128)
    ref = torch.nn.Linear(256, 128).double()
    ref.load_state_dict({k: v.double() for k, v in lin.state_dict().items()})
    x = torch.randn(2, 300, 256)
    x64 = x.double().requires_grad_(True)
    g = torch.randn(2, 300, 128)
    ref(x64).backward(g.double())
    lg = lin.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode == "bf16"):
        y = O_.linear(xg, lg)
    y.backward(g.to(DEV).to(y.dtype))
    tol = 1e-4 if mode == "fp32" else 2e-2
    assert rel_err(y.float().cpu(), ref(x64).detach()) < tol
    assert rel_err(xg.grad.float().cpu(), x64.grad) < tol
    assert lg.weight.grad.dtype == torch.float32
    assert rel_err(lg.weight.grad.cpu(), ref.weight.grad) < tol
    assert rel_err(lg.bias.grad.cpu(), ref.bias.grad) < tol


def test_add_layer_norm_fused_equals_unfused():
    """ops.add_layer_norm (a Block's residual add + ln2 in one pass, fp32 stream, bf16
    branch output, bf16 LN output under autocast) gives bitwise the outputs and
    gradients of x + a followed by the LayerNorm, and matches fp64 within bf16 tolerance."""
    from differential_transformer_replication_amd import ops as O_
    torch.manual_seed(6)
    C = 1024
    ln = O_.LayerNorm(C, autocast_out=True).to(DEV)
    with torch.no_grad():
        ln.weight.normal_(1.0, 0.1)
        ln.bias.normal_(0.0, 0.1)
    x0 = torch.randn(3, 77, C, device=DEV)
    a0 = torch.randn(3, 77, C, device=DEV).to(torch.bfloat16)
    gx = torch.randn(3, 77, C, device=DEV)
    gy = torch.randn(3, 77, C, device=DEV).to(torch.bfloat16)
    outs = []
    for fused in (True, False):
        O_._RES_FUSE = fused
        x = x0.clone().requires_grad_(True)
        a = a0.clone().requires_grad_(True)
        ln.weight.grad = ln.bias.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            xo, y = O_.add_layer_norm(x, a, ln)
        assert xo.dtype == torch.float32 and y.dtype == torch.bfloat16
        (xo * gx).sum().backward(retain_graph=True)
        (y.float() * gy.float()).sum().backward()
        outs.append([t.detach().clone() for t in (xo, y, x.grad, a.grad, ln.weight.grad, ln.bias.grad)])
    O_._RES_FUSE = True
    for u, v in zip(*outs):
        assert torch.equal(u, v)
    # fp64 reference of the same math
    x64 = x0.double().requires_grad_(True)
    a64 = a0.double().requires_grad_(True)
    s = x64 + a64
    y64 = F.layer_norm(s, (C,), ln.weight.double(), ln.bias.double(), ln.eps)
    ((s * gx.double()).sum() + (y64 * gy.double()).sum()).backward()
    assert rel_err(outs[0][1].float().cpu(), y64.detach().cpu()) < 2e-2
    assert rel_err(outs[0][2].cpu(), x64.grad.cpu()) < 2e-2
    assert rel_err(outs[0][3].float().cpu(), a64.grad.cpu()) < 2e-2


@pytest.mark.parametrize("rows,n", [(300, 256), (4096, 1024), (1, 64)])
def test_swiglu_bias_gradient_pass(rows, n):
    """dta_swiglu_bwd with dbias: dA | dB as the plain backward writes them, plus their
    column sums (the packed gate / xform bias gradient) summed in a fixed order."""
    from differential_transformer_replication_amd import ops as O_
    gen = torch.Generator().manual_seed(rows + n)
    y2 = (torch.randn(rows, 2 * n, generator=gen) * 2).to(torch.bfloat16).to(DEV)
    d2 = torch.randn(rows, n, generator=gen).to(torch.bfloat16).to(DEV)
    dy_ref, dy = torch.empty_like(y2), torch.empty_like(y2)
    O_._swiglu_launch(y2, n, None, d2, dy_ref)
    db = torch.empty(2 * n, device=DEV)
    O_._swiglu_launch(y2, n, None, d2, dy, db)
    torch.cuda.synchronize()
    assert torch.equal(dy, dy_ref)
    ref = dy_ref.double().sum(0)
    assert rel_err(db.cpu(), ref.cpu()) < 1e-5
