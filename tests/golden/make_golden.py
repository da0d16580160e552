"""Generate the golden fixtures in ``tests/golden/*.npz`` by running the
REFERENCE modules (imported read-only from ``/root/reference``) on the CPU.

This script is the only thing in the repository that touches the reference,
and it only runs in the build container (the reference never travels to the
GPU box).  The outputs are data only: inputs, state dicts, outputs and
gradients, in float64 (``.double()`` modules) unless a case says fp32.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import torch

REF = os.environ.get("DTA_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import diff_transformer as ref_diff          # noqa: E402
import Ndiff_transformer as ref_ndiff        # noqa: E402
import control as ref_control                # noqa: E402

SEP = "::"


def _np(t: torch.Tensor) -> np.ndarray:
    # stored as fp32: inputs and parameters are generated fp32-representable
    # (lossless), fp64 outputs/grads keep ~6e-8 relative precision, far below
    # the 1e-6 fp64 parity bar
    t = t.detach().cpu()
    if t.is_complex():
        t = torch.view_as_real(t)
    if t.is_floating_point():
        t = t.float()
    return t.numpy().copy()


def _fp32_exact(mod: torch.nn.Module) -> torch.nn.Module:
    """Round every parameter to fp32 before the fp64 run so fixtures store them losslessly."""
    with torch.no_grad():
        for p in mod.parameters():
            p.copy_(p.float().double())
    return mod


def _randomize_lambdas(mod: torch.nn.Module, gen: torch.Generator) -> None:
    # zero-initialised lambdas sit at a saddle (SURVEY semantic 4): randomise
    with torch.no_grad():
        for name, p in mod.named_parameters():
            if "lambda_" in name:
                p.copy_(torch.randn(p.shape, generator=gen, dtype=p.dtype) * 0.1)


def _randomize_norm(mod: torch.nn.Module, gen: torch.Generator) -> None:
    with torch.no_grad():
        for name, p in mod.named_parameters():
            if "group_norm" in name or name in ("weight", "bias"):
                p.add_(torch.randn(p.shape, generator=gen, dtype=p.dtype) * 0.1)


def _state(mod: torch.nn.Module) -> dict:
    out = {}
    for k, v in mod.state_dict().items():
        if k.endswith("tril"):
            continue                         # T x T ones-lower: regenerated, never stored
        out["sd" + SEP + k] = _np(v)
    return out


def _module_case(mod, inputs, call, seed, extra=None):
    """Run forward + backward against a random upstream gradient."""
    gen = torch.Generator().manual_seed(seed + 7)
    _fp32_exact(mod)
    xs = [(x.float().double() if x.is_floating_point() else x).clone()
          .requires_grad_(x.is_floating_point()) for x in inputs]
    out = call(mod, *xs)
    g = torch.randn(out.shape, generator=gen, dtype=torch.float32).to(out.dtype)
    (out * g).sum().backward()
    rec = {"out": _np(out), "gout": _np(g)}
    for i, x in enumerate(xs):
        rec[f"in{i}"] = _np(x)
        if x.grad is not None:
            rec[f"grad_in{i}"] = _np(x.grad)
    for name, p in mod.named_parameters():
        if p.grad is not None:
            rec["grad" + SEP + name] = _np(p.grad)
    rec.update(_state(mod))            # post-forward: lambda_init side effects included
    if extra:
        rec.update(extra)
    return rec


def cases():
    torch.set_default_dtype(torch.float64)
    rec = {}

    def put(name, d):
        for k, v in d.items():
            rec[name + "/" + k] = v

    # ---- GroupLayerNorm (diff_transformer.py:5-20)
    torch.manual_seed(11)
    gen = torch.Generator().manual_seed(11)
    gln = ref_diff.GroupLayerNorm(3, 8).double()
    _randomize_norm(gln, gen)
    x = torch.randn(2, 5, 48, generator=gen) * 2 + 0.5
    put("gln", _module_case(gln, [x], lambda m, a: m(a), 11))

    # ---- DiffHead (diff_transformer.py:22-73)
    for ci, (hs, C, T, blk, layer) in enumerate([(16, 32, 7, 16, 1), (32, 64, 129, 160, 3),
                                                  (64, 64, 64, 64, 2), (16, 32, 1, 8, 5)]):
        torch.manual_seed(100 + ci)
        gen = torch.Generator().manual_seed(100 + ci)
        m = ref_diff.DiffHead(hs, C, 0.0, blk).double()
        _randomize_lambdas(m, gen)
        x = torch.randn(2, T, C, generator=gen)
        put(f"diffhead{ci}", _module_case(m, [x], lambda mm, a: mm(a, layer), 100 + ci,
                                          {"meta": np.array([hs, C, T, blk, layer])}))

    # ---- MultiHeadDiffAttention (diff_transformer.py:75-93)
    for ci, (H, hs, C, T, blk, layer) in enumerate([(2, 16, 64, 7, 8, 1), (3, 32, 96, 129, 129, 3),
                                                     (2, 64, 128, 192, 200, 6), (4, 16, 128, 64, 80, 2)]):
        torch.manual_seed(200 + ci)
        gen = torch.Generator().manual_seed(200 + ci)
        m = ref_diff.MultiHeadDiffAttention(H, hs, C, 0.0, blk).double()
        _randomize_lambdas(m, gen)
        _randomize_norm(m, gen)
        x = torch.randn(2 if T < 200 else 1, T, C, generator=gen)
        put(f"mhdiff{ci}", _module_case(m, [x], lambda mm, a: mm(a, layer), 200 + ci,
                                        {"meta": np.array([H, hs, C, T, blk, layer])}))

    # ---- AlternatingDiffHead (Ndiff_transformer.py:40-126)
    for ci, (N, hs, C, T, blk, layer) in enumerate([(1, 16, 32, 7, 8, 1), (2, 16, 32, 64, 64, 1),
                                                     (3, 32, 64, 129, 130, 3), (4, 16, 48, 33, 40, 4)]):
        torch.manual_seed(300 + ci)
        gen = torch.Generator().manual_seed(300 + ci)
        m = ref_ndiff.AlternatingDiffHead(hs, C, 0.0, blk, N).double()
        _randomize_lambdas(m, gen)
        x = torch.randn(2, T, C, generator=gen)
        put(f"althead{ci}", _module_case(m, [x], lambda mm, a: mm(a, layer), 300 + ci,
                                         {"meta": np.array([N, hs, C, T, blk, layer])}))

    # ---- MultiHeadAlternatingDiffAttention (Ndiff_transformer.py:128-146)
    for ci, (N, H, hs, C, T, blk, layer) in enumerate([(2, 2, 16, 64, 31, 32, 1),
                                                        (3, 3, 16, 96, 65, 65, 2),
                                                        (4, 2, 32, 128, 97, 160, 3)]):
        torch.manual_seed(400 + ci)
        gen = torch.Generator().manual_seed(400 + ci)
        m = ref_ndiff.MultiHeadAlternatingDiffAttention(H, hs, C, 0.0, blk, N).double()
        _randomize_lambdas(m, gen)
        _randomize_norm(m, gen)
        x = torch.randn(2, T, C, generator=gen)
        put(f"mhalt{ci}", _module_case(m, [x], lambda mm, a: mm(a, layer), 400 + ci,
                                       {"meta": np.array([N, H, hs, C, T, blk, layer])}))

    # ---- control MultiHeadAttention (control.py:24-78)
    torch.manual_seed(500)
    gen = torch.Generator().manual_seed(500)
    m = ref_control.MultiHeadAttention(4, 16, 64, 0.0, 48).double()
    x = torch.randn(2, 33, 64, generator=gen)
    put("ctrlmha", _module_case(m, [x], lambda mm, a: mm(a), 500,
                                {"meta": np.array([4, 16, 64, 33, 48])}))

    # ---- RoPE helpers (Ndiff_transformer.py:4-22)
    fc = ref_ndiff.precompute_freqs_cis(32, 40)
    gen = torch.Generator().manual_seed(600)
    xr = torch.randn(2, 17, 32, generator=gen, dtype=torch.float32)
    rec["rope/freqs"] = _np(fc)
    rec["rope/x"] = _np(xr)
    rec["rope/out"] = _np(ref_ndiff.apply_rotary_emb(xr, fc))

    # ---- whole tiny models (forward, loss, grads)
    for name, ctor, kw in [
        ("modeldiff", ref_diff.DiffTransformer, dict(vocab_size=97, n_embd=64, n_head=2, n_layer=2,
                                                      block_size=24, dropout=0.0)),
        ("modelalt", ref_ndiff.AlternatingDiffTransformer, dict(vocab_size=97, n_embd=64, n_head=2,
                                                                 n_layer=2, block_size=24, dropout=0.0,
                                                                 n_terms=3)),
        ("modelctrl", ref_control.StandardTransformer, dict(vocab_size=97, n_embd=64, n_head=4,
                                                            n_layer=2, block_size=24, dropout=0.0)),
    ]:
        torch.manual_seed(700)
        m = ctor(**kw).double()
        gen = torch.Generator().manual_seed(701)
        _randomize_lambdas(m, gen)
        _fp32_exact(m)
        idx = torch.randint(0, 97, (2, 19), generator=gen)
        tgt = torch.randint(0, 97, (2, 19), generator=gen)
        logits, loss = m(idx, tgt)
        loss.backward()
        d = {"idx": idx.numpy(), "tgt": tgt.numpy(), "logits": _np(logits), "loss": _np(loss)}
        for pn, p in m.named_parameters():
            d["grad" + SEP + pn] = _np(p.grad)
        d.update(_state(m))
        d["meta"] = np.array(list(kw.values()), dtype=np.float64)
        put(name, d)
    torch.set_default_dtype(torch.float32)
    return rec


class _CosineWarmup:
    """Restatement of train.py:95-107 (CosineWarmupScheduler.get_lr), used only to
    drive the reference model for the loss-curve fixture; its values are checked
    against the lr numbers SURVEY section 8c measured from the reference itself."""

    def __init__(self, base_lr, warmup, max_steps, min_lr):
        self.base, self.warm, self.max, self.min = base_lr, warmup, max_steps, min_lr

    def lr(self, step):
        if step < self.warm:
            return self.base * step / self.warm
        prog = (step - self.warm) / (self.max - self.warm)
        return self.min + (self.base - self.min) * 0.5 * (1.0 + math.cos(math.pi * prog))


def loss_curve():
    """cfg1 DiffTransformer(12000, 384, 6, 6, 256, 0), fp32, seed 1337, AdamW
    (train.py:236-241), cosine warmup, clip 1.0 -- 12 steps at micro-batch 2 on
    seeded synthetic tokens."""
    torch.set_num_threads(8)
    torch.manual_seed(1337)
    model = ref_diff.DiffTransformer(12000, 384, 6, 6, 256, 0.0)
    ck = np.array([float(p.detach().double().sum()) for p in model.parameters()])
    sq = np.array([float(p.detach().double().pow(2).sum()) for p in model.parameters()])
    opt = torch.optim.AdamW(model.parameters(), lr=3.2e-4, betas=(0.9, 0.95), weight_decay=0.1)
    sched = _CosineWarmup(3.2e-4, 4, 12, 6e-5)
    gen = torch.Generator().manual_seed(1337)
    toks = torch.randint(0, 12000, (4096,), generator=gen)
    steps, mb, T = 12, 2, 256
    offs = torch.randint(0, toks.numel() - T - 1, (steps, mb), generator=gen)
    losses, gnorms, lrs = [], [], []
    model.train()
    for s in range(steps):
        X = torch.stack([toks[o:o + T] for o in offs[s].tolist()])
        Y = torch.stack([toks[o + 1:o + T + 1] for o in offs[s].tolist()])
        for g in opt.param_groups:
            g["lr"] = sched.lr(s)
        _, loss = model(X, Y)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
        gnorms.append(float(gn))
        lrs.append(sched.lr(s))
        print(f"step {s}: loss {losses[-1]:.6f} gnorm {gnorms[-1]:.6f}", flush=True)
    return {"curve/losses": np.array(losses), "curve/gnorms": np.array(gnorms),
            "curve/lrs": np.array(lrs), "curve/toks": toks.numpy(), "curve/offs": offs.numpy(),
            "curve/param_sum": ck, "curve/param_sq": sq,
            "curve/lr_pins": np.array([_CosineWarmup(3.2e-4, 1000, 40000, 6e-5).lr(s)
                                       for s in (0, 1, 999, 1000, 20000, 40000)])}


def main():
    rec = cases()
    np.savez_compressed(os.path.join(OUT, "golden_modules.npz"), **rec)
    curve = loss_curve()
    np.savez_compressed(os.path.join(OUT, "golden_loss_curve.npz"), **curve)
    for fn in ("golden_modules.npz", "golden_loss_curve.npz"):
        print(fn, os.path.getsize(os.path.join(OUT, fn)) // 1024, "KiB")


if __name__ == "__main__":
    main()
