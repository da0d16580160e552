"""GPU parity of the drop-in modules against the reference's own outputs.

Every case loads the reference's state_dict from ``tests/golden/golden_modules.npz``
(produced by running the reference modules in fp64, tests/golden/make_golden.py),
runs our module on the MI355X HIP path in fp32, and compares the output, the
input gradient and EVERY parameter gradient (including the lambda_q / lambda_k
grads that flow through d(coef)), plus the lambda_init side effects.
Tolerance (north_star): fp32 max|a-b|/max|b| <= 1e-4; bf16 autocast <= 2e-2.
The loss-curve test replays the reference's cfg1 training steps
(golden_loss_curve.npz) on the GPU.
"""
import math
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, Golden, rel_err
from test_boundary_cpu import _build, _cases

from differential_transformer_replication_amd import diff_transformer as D
from differential_transformer_replication_amd import Ndiff_transformer as ND

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP32_TOL = 1e-4
BF16_TOL = 2e-2


def _layer(case, g):
    meta = [int(v) for v in g["meta"]]
    return None if case == "ctrlmha" else meta[-1]


def _run_module(case, g, dtype_ctx=None):
    m = _build(case, g).to(DEV)
    ref_sd = dict(g.state_dict(torch.float32))
    sd = m.state_dict()
    for k in sd:
        if k.endswith("tril"):
            ref_sd[k] = sd[k]
    m.load_state_dict(ref_sd, strict=True)
    x = torch.from_numpy(g["in0"]).float().to(DEV).requires_grad_(True)
    layer = _layer(case, g)
    ctx = dtype_ctx if dtype_ctx is not None else torch.autocast("cuda", enabled=False)
    with ctx:
        out = m(x) if layer is None else m(x, layer)
    gout = torch.from_numpy(g["gout"]).to(DEV)
    (out.float() * gout).sum().backward()
    return m, x, out


@pytest.mark.parametrize("prefix", ["diffhead", "mhdiff", "althead", "mhalt"])
def test_module_fp32_matches_reference(golden, prefix):
    for case in _cases(golden, prefix):
        g = Golden(golden, case)
        m, x, out = _run_module(case, g)
        assert rel_err(out, g["out"]) < FP32_TOL, (case, "out")
        assert rel_err(x.grad, g["grad_in0"]) < FP32_TOL, (case, "grad_in0")
        grads = g.grads()
        named = dict(m.named_parameters())
        assert set(grads) <= set(named), case
        for k, ref in grads.items():
            got = named[k].grad
            assert got is not None, (case, k)
            if float(np.abs(ref).max()) == 0.0:
                assert float(got.abs().max()) < 1e-6, (case, k)
            else:
                assert rel_err(got, ref) < FP32_TOL, (case, k, rel_err(got, ref))
        # lambda_init side effects (get_lambda writes the per-head buffer)
        sd = m.state_dict()
        for k, v in g.state_dict(torch.float32).items():
            if k.endswith("lambda_init"):
                assert torch.allclose(sd[k].float().cpu(), v.float(), rtol=0, atol=1e-7), (case, k)


@pytest.mark.parametrize("prefix", ["mhdiff", "mhalt"])
def test_module_bf16_autocast(golden, prefix):
    for case in _cases(golden, prefix):
        g = Golden(golden, case)
        m, x, out = _run_module(case, g, torch.autocast("cuda", dtype=torch.bfloat16))
        assert rel_err(out.float(), g["out"]) < BF16_TOL, (case, "out")
        assert rel_err(x.grad, g["grad_in0"]) < BF16_TOL, (case, "grad_in0")
        # every parameter gradient too: projections, GroupLayerNorm, and the lambda_q / lambda_k
        # grads that reach the parameters through d(coef).  A bf16 gradient that is a sum with
        # heavy cancellation (d lambda = sum <dO, A_i V>) carries the bf16 rounding of its terms,
        # so the bar is the north star's 2e-2 or, where larger, 2x the error of the reference
        # algorithm itself under the same bf16 autocast (the oracle run on the GPU): the two
        # round at different points (the reference rounds dO V^T per map element to bf16; the
        # fused path forms delta_i = <dO, O_i> from fp32 O_i but rounds P to bf16 for P V).
        ref_err = _reference_bf16_grad_errors(case, g)
        named = dict(m.named_parameters())
        log = []
        for k, ref in g.grads().items():
            got = named[k].grad
            assert got is not None, (case, k)
            if float(np.abs(ref).max()) == 0.0:
                assert float(got.abs().max()) < 1e-4, (case, k)
                continue
            err = rel_err(got, ref)
            # only the lambda vectors may exceed the north star's 2e-2 (reason above): their
            # bar is 2x the reference algorithm's own bf16 error; every other gradient is held to 2e-2
            loose = any(t in k for t in BF16_LOOSE)
            bar = max(BF16_TOL, 2.0 * ref_err[k]) if loose else BF16_TOL
            log.append({"case": case, "param": k, "err": err, "ref_alg_bf16_err": ref_err[k], "bar": bar,
                        "over_2e-2": err >= BF16_TOL})
            assert err < bar, (case, k, err, ref_err[k])
        _log_errors(f"bf16_grad_errors_{prefix}", log)


# parameter-name fragments whose bf16 gradient may exceed 2e-2 (test_module_bf16_autocast):
# d lambda_* = exp(lq*lk) lk / hs * d(coef), and d(coef) = sum over (b, t) of <dO, O_i>, a sum
# with heavy cancellation whose terms carry bf16 rounding
BF16_LOOSE = ("lambda_q", "lambda_k")


def _log_errors(name, rows):
    """Every gradient's error and bar, for the run record (DTA_TEST_LOG_DIR, when set)."""
    import json
    d = os.environ.get("DTA_TEST_LOG_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


def _reference_bf16_grad_errors(case, g):
    """Relative error vs the fp64 fixture of every parameter gradient when the
    reference algorithm (oracle restatement, eager ATen) runs under bf16 autocast
    on the GPU with the same weights and inputs."""
    from oracle import diffattn_oracle as orc
    meta = [int(v) for v in g["meta"]]
    sd = {k: v.to(DEV).requires_grad_(True) for k, v in g.state_dict(torch.float32).items()
          if v.is_floating_point() and "lambda_init" not in k}
    x = torch.from_numpy(g["in0"]).float().to(DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        if case.startswith("mhdiff"):
            H, hs, Cm, T, blk, layer = meta
            out = orc.multihead_diff_attention(x, sd, H, layer, blk)
        else:
            N, H, hs, Cm, T, blk, layer = meta
            out = orc.multihead_alternating_diff_attention(x, _with_freqs(sd, g, H), H, N, layer, blk)
    (out.float() * torch.from_numpy(g["gout"]).to(DEV)).sum().backward()
    return {k: rel_err(sd[k].grad, ref) if float(np.abs(ref).max()) > 0 else 0.0
            for k, ref in g.grads().items()}


def _with_freqs(sd, g, H):
    full = g.state_dict(torch.float32)
    for h in range(H):
        k = f"heads.{h}.freqs_cis"
        if k in full:
            sd[k] = full[k].to(DEV)
    return sd


@pytest.mark.parametrize("case,ctor", [
    ("modeldiff", lambda: D.DiffTransformer(97, 64, 2, 2, 24, 0.0)),
    ("modelalt", lambda: ND.AlternatingDiffTransformer(97, 64, 2, 2, 24, 0.0, n_terms=3)),
])
def test_tiny_model_matches_reference(golden, case, ctor):
    g = Golden(golden, case)
    m = ctor().to(DEV)
    m.load_state_dict(g.state_dict(torch.float32), strict=True)
    idx = torch.from_numpy(g["idx"]).to(DEV)
    tgt = torch.from_numpy(g["tgt"]).to(DEV)
    logits, loss = m(idx, tgt)
    loss.backward()
    assert rel_err(logits, g["logits"]) < FP32_TOL
    assert abs(float(loss) - float(g["loss"])) / abs(float(g["loss"])) < FP32_TOL
    for k, p in m.named_parameters():
        ref = g[f"grad::{k}"]
        if float(np.abs(ref).max()) == 0.0:
            assert float(p.grad.abs().max()) < 1e-6, k
        else:
            assert rel_err(p.grad, ref) < FP32_TOL, (k, rel_err(p.grad, ref))


def test_generate_runs_on_gpu():
    torch.manual_seed(0)
    m = D.DiffTransformer(97, 64, 2, 2, 24, 0.0).to(DEV).eval()
    out = m.generate(torch.zeros(1, 1, dtype=torch.long, device=DEV), 30)   # crops to block_size
    assert out.shape == (1, 31)


def test_cfg1_loss_curve_matches_reference(golden_curve):
    """cfg1 DiffTransformer(12000, 384, 6, 6, 256), fp32, seed 1337, AdamW(3.2e-4,
    (0.9, 0.95), wd 0.1), cosine warmup 4/12, clip 1.0, micro-batch 2: the same
    12 steps the reference took (train.py:236-268 semantics, fp32)."""
    z = golden_curve
    torch.manual_seed(1337)
    model = D.DiffTransformer(12000, 384, 6, 6, 256, 0.0).to(DEV)
    opt = torch.optim.AdamW(model.parameters(), lr=3.2e-4, betas=(0.9, 0.95), weight_decay=0.1)
    toks = torch.from_numpy(z["curve/toks"]).to(DEV)
    offs = z["curve/offs"]
    T = 256
    model.train()
    losses, gnorms = [], []
    for s in range(offs.shape[0]):
        X = torch.stack([toks[o:o + T] for o in offs[s].tolist()])
        Y = torch.stack([toks[o + 1:o + T + 1] for o in offs[s].tolist()])
        for grp in opt.param_groups:
            grp["lr"] = float(z["curve/lrs"][s])
        _, loss = model(X, Y)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
        gnorms.append(float(gn))
    ref_l, ref_g = z["curve/losses"], z["curve/gnorms"]
    for s, (a, b) in enumerate(zip(losses, ref_l)):
        assert abs(a - b) / abs(b) < FP32_TOL, (s, a, b)
    for s, (a, b) in enumerate(zip(gnorms, ref_g)):
        assert abs(a - b) / abs(b) < 1e-3, (s, a, b)
    assert all(math.isfinite(v) for v in losses)


@pytest.mark.parametrize("model,dtype", [("diff", "bf16"), ("ndiff", "bf16"), ("diff", "fp16"), ("ndiff", "fp32")])
def test_trainer_steps_on_gpu(model, dtype):
    """The DP Trainer (world 1) through the HIP path: mixed precision, clip, AdamW,
    cosine schedule; loss finite and moving on a repeated batch."""
    from differential_transformer_replication_amd.train import (ShardedWindows, Trainer, TrainingConfig,
                                                                build_model)
    cfg = TrainingConfig(model=model, n_embd=128, n_head=2, n_layer=2, block_size=64, n_terms=3,
                         vocab_size=101, micro_batch_size=4, grad_acc_steps=2, warmup_iters=1,
                         max_iters=50, learning_rate=3e-3, dtype=dtype)
    torch.manual_seed(0)
    dev = torch.device(DEV, 0)
    m = build_model(cfg).to(dev)
    toks = torch.randint(0, cfg.vocab_size, (5000,), device=dev)
    it = ShardedWindows(toks, cfg.block_size, cfg.micro_batch_size, 0, 1, 0)
    X, Y = it.next()
    tr = Trainer(cfg, m, 1, 0, dev)
    losses = [float(tr.step(lambda: (X, Y))) for _ in range(8)]
    assert all(math.isfinite(v) for v in losses), losses
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("hs,T", [(64, 97), (128, 160)])
def test_control_mha_on_fused_kernel(dtype, hs, T):
    """control.py's MultiHeadAttention (control.py:64-78) on the GPU runs the fused
    kernels' N=1, coef 1, dv=hs case; compared in fp64 on the CPU with the oracle's
    restatement (orc.control_multihead, pinned to the reference fixtures) and with the
    same module's PyTorch path: output, input gradient and every weight gradient."""
    from differential_transformer_replication_amd import control as C
    from oracle import diffattn_oracle as orc
    torch.manual_seed(3)
    H, C_ = 3, 3 * hs
    m = C.MultiHeadAttention(H, hs, C_, 0.0, 256)
    x = torch.randn(2, T, C_)
    g = torch.randn(2, T, C_)
    ref = m.double()
    x64 = x.double().requires_grad_(True)
    out64 = ref(x64)
    (out64 * g.double()).sum().backward()
    grads64 = {n: p.grad.clone() for n, p in ref.named_parameters()}
    sd = {k: (v.detach().clone().requires_grad_(True) if v.is_floating_point() else v)
          for k, v in ref.state_dict().items()}
    xo = x.double().requires_grad_(True)
    out_orc = orc.control_multihead(xo, sd, H, 256)
    (out_orc * g.double()).sum().backward()
    mg = C.MultiHeadAttention(H, hs, C_, 0.0, 256)
    mg.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ref.state_dict().items()})
    mg = mg.to(DEV).to(dtype)
    xg = x.to(DEV, dtype).requires_grad_(True)
    assert C._fused_ok(xg, 0.0, hs)
    out = mg(xg)
    (out * g.to(DEV, dtype)).sum().backward()
    tol = FP32_TOL if dtype == torch.float32 else BF16_TOL

    def rel(a, b):
        return ((a.double().cpu() - b).abs().max() / b.abs().max()).item()

    assert rel(out, out64.detach()) < tol
    assert rel(xg.grad, x64.grad) < tol
    for n, p in mg.named_parameters():
        assert rel(p.grad, grads64[n]) < tol, n
    # the oracle (reference algorithm restated)
    assert rel(out, out_orc.detach()) < tol
    assert rel(xg.grad, xo.grad) < tol
    for n, p in mg.named_parameters():
        assert rel(p.grad, sd[n].grad) < tol, ("oracle", n)


def _replay_curve(z, prefix, fp16):
    """The reference's step (train.py:251-279) on the HIP path: same seed, data,
    AdamW, CosineWarmupScheduler, clip; fp16 adds autocast + GradScaler."""
    from differential_transformer_replication_amd.train import CosineWarmupScheduler
    mb, T, steps, warm = (int(v) for v in z[prefix + "meta"])
    torch.manual_seed(1337)
    model = D.DiffTransformer(12000, 384, 6, 6, 256, 0.0).to(DEV)
    opt = torch.optim.AdamW(model.parameters(), lr=3.2e-4, betas=(0.9, 0.95), weight_decay=0.1)
    sched = CosineWarmupScheduler(opt, warm, steps, 6e-5)
    scaler = torch.amp.GradScaler("cuda") if fp16 else None
    toks = torch.from_numpy(z[prefix + "toks"].astype(np.int64)).to(DEV)
    offs = z[prefix + "offs"]
    losses, lrs = [], []
    model.train()
    for s in range(steps):
        X = torch.stack([toks[o:o + T] for o in offs[s].tolist()])
        Y = torch.stack([toks[o + 1:o + T + 1] for o in offs[s].tolist()])
        lrs.append(opt.param_groups[0]["lr"])
        if fp16:
            with torch.autocast("cuda", dtype=torch.float16):
                _, loss = model(X, Y)
            scaler.scale(loss).backward()
            scaler.unscale_(opt)
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            scaler.step(opt)
            scaler.update()
        else:
            _, loss = model(X, Y)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
        opt.zero_grad(set_to_none=True)
        sched.step()
        losses.append(float(loss))
    np.testing.assert_allclose(lrs, z[prefix + "lrs"], rtol=1e-6)
    return np.array(losses)


def test_cfg1_long_fp32_curve_matches_reference():
    """50 optimizer steps at cfg1's micro-batch 32 (train.py defaults), fp32: every
    step's loss within 1e-4 of the reference's own curve."""
    z = np.load(os.path.join(GOLDEN, "golden_loss_curve_long.npz"))
    losses = _replay_curve(z, "curve32/", False)
    ref = z["curve32/losses"]
    rel = np.abs(losses - ref) / np.abs(ref)
    assert rel.max() < 1e-4, (int(rel.argmax()), float(rel.max()))


def test_cfg1_fp16_gradscaler_curve_overlays_reference():
    """The reference's fp16 autocast + GradScaler loop (train.py:251-279), 50 steps:
    the HIP path's curve overlays the reference's (recorded with CPU autocast, whose
    fp16 GEMMs round differently) within 2e-2 per step and 5e-3 on the mean."""
    z = np.load(os.path.join(GOLDEN, "golden_loss_curve_long.npz"))
    losses = _replay_curve(z, "curve16/", True)
    ref = z["curve16/losses"]
    rel = np.abs(losses - ref) / np.abs(ref)
    assert np.isfinite(losses).all()
    assert rel.max() < 2e-2, (int(rel.argmax()), float(rel.max()))
    assert rel.mean() < 5e-3, float(rel.mean())


@pytest.mark.parametrize("key", ["alt3", "diff"])
def test_bf16_curve_overlays_reference(key):
    """The differential models the benches train (cfg3's AlternatingDiffTransformer with
    n_terms=3, cfg4's DiffTransformer; small shapes, head size 64), 50 optimizer steps of the
    reference's loop (train.py:236-281: AdamW, CosineWarmupScheduler, clip 1.0) under bf16
    autocast on the HIP path, against the reference's fp32 curve of the same seed and data
    (tests/golden/make_curve_golden_bf16.py).  Tolerance, per step |ours - ref32| / ref32:
    max <= 2e-2 (north_star's bf16 bar), and mean <= max(5e-3, 2x the reference's own
    bf16-autocast drift from its fp32 curve, recorded in the same fixture)."""
    from differential_transformer_replication_amd.train import CosineWarmupScheduler
    z = np.load(os.path.join(GOLDEN, "golden_loss_curve_diffmodels.npz"))
    p = key + "/"
    mb, T, steps, warm = (int(v) for v in z[p + "meta"])
    torch.manual_seed(1337)
    model = (ND.AlternatingDiffTransformer(12000, 384, 3, 4, 256, 0.0, n_terms=3) if key == "alt3"
             else D.DiffTransformer(12000, 512, 4, 4, 256, 0.0))
    sd = {k: v for k, v in model.state_dict().items() if v.is_floating_point()}
    assert sorted(sd) == list(z[p + "init_keys"])
    init = np.array([[float(sd[k].double().sum()), float((sd[k].double() ** 2).sum())] for k in sorted(sd)])
    np.testing.assert_allclose(init, z[p + "init_sums"], rtol=1e-12, atol=1e-9)   # summation order
    model = model.to(DEV)
    opt = torch.optim.AdamW(model.parameters(), lr=3.2e-4, betas=(0.9, 0.95), weight_decay=0.1)
    sched = CosineWarmupScheduler(opt, warm, steps, 6e-5)
    toks = torch.from_numpy(z[p + "toks"].astype(np.int64)).to(DEV)
    offs = z[p + "offs"]
    losses, lrs = [], []
    model.train()
    for s in range(steps):
        X = torch.stack([toks[o:o + T] for o in offs[s].tolist()])
        Y = torch.stack([toks[o + 1:o + T + 1] for o in offs[s].tolist()])
        lrs.append(opt.param_groups[0]["lr"])
        with torch.autocast("cuda", dtype=torch.bfloat16):
            _, loss = model(X, Y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        sched.step()
        losses.append(float(loss))
    np.testing.assert_allclose(lrs, z[p + "lrs"], rtol=1e-6)
    losses = np.array(losses)
    ref32, ref16 = z[p + "losses"], z[p + "bf16_losses"]
    rel = np.abs(losses - ref32) / np.abs(ref32)
    ref_drift = np.abs(ref16 - ref32) / np.abs(ref32)
    log = os.environ.get("DTA_TEST_LOG_DIR")
    if log:
        import json
        with open(os.path.join(log, f"bf16_curve_{key}.json"), "w") as fh:
            json.dump({"ours_bf16": losses.tolist(), "ref_fp32": ref32.tolist(), "ref_bf16_cpu": ref16.tolist(),
                       "rel_max": float(rel.max()), "rel_mean": float(rel.mean()),
                       "ref_drift_max": float(ref_drift.max()), "ref_drift_mean": float(ref_drift.mean())}, fh)
    assert np.isfinite(losses).all()
    assert rel.max() <= 2e-2, (int(rel.argmax()), float(rel.max()))
    assert rel.mean() <= max(5e-3, 2 * ref_drift.mean()), (float(rel.mean()), float(ref_drift.mean()))
