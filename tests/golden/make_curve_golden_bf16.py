"""Training-curve fixtures for the DIFFERENTIAL models the benches train, from the
REFERENCE, run on this container's CPU (the reference never travels to the GPU box):

  alt3/*   AlternatingDiffTransformer(12000, 384, 3, 4, 256, 0, n_terms=3)
           (Ndiff_transformer.py:181-230; cfg3's model class at a small shape:
           head size 384 // 6 = 64 as at cfg3, N = 3 branches, RoPE)
  diff/*   DiffTransformer(12000, 512, 4, 4, 256, 0) (diff_transformer.py:128-175;
           cfg4's model class at a small shape, head size 64)

Each: seed 1337, micro-batch 8 x 256 seeded synthetic tokens (data(): a noisy repeated motif), AdamW(3.2e-4, (0.9, 0.95),
wd 0.1) (train.py:236-241), the reference's own CosineWarmupScheduler (train.py:109-123,
warmup 10, max 50, min 6e-5), grad clip 1.0, 50 optimizer steps:
  <p>losses      the fp32 curve (the GPU bf16 replay overlays it)
  <p>bf16_losses the SAME reference loop under CPU bf16 autocast (train.py:251-256's
                 autocast with dtype bfloat16): the reference algorithm's own bf16 drift
                 from its fp32 curve, which sets the replay's tolerance
  <p>init_sums   per-entry (sum, sum of squares) of the seeded initial state, for the
                 floating state_dict keys in sorted order (<p>init_keys): the replay checks
                 it builds the same initial model
  <p>toks/offs   the data; <p>lrs the schedule; <p>meta [mb, T, steps, warmup]

train.py imports tiktoken and wandb at module level (absent here and unused by the
scheduler): empty stand-in modules satisfy those two imports.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_curve_golden_bf16.py
"""
import os
import sys
import time
import types

import numpy as np
import torch

REF = os.environ.get("DTA_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
for name in ("tiktoken", "wandb"):
    sys.modules.setdefault(name, types.ModuleType(name))

import diff_transformer as ref_diff          # noqa: E402
import Ndiff_transformer as ref_ndiff        # noqa: E402
import train as ref_train                    # noqa: E402

STEPS, T, WARM, MB = 50, 256, 10, 8
MODELS = {
    "alt3": lambda: ref_ndiff.AlternatingDiffTransformer(12000, 384, 3, 4, 256, 0.0, n_terms=3),
    "diff": lambda: ref_diff.DiffTransformer(12000, 512, 4, 4, 256, 0.0),
}


def data(key):
    """Learnable synthetic tokens (uniform random tokens leave the loss flat at ln 12000, where
    bf16 error in the gradients would not show): a 97-token motif over 256 of the 12000 ids,
    repeated, with 5% of the positions redrawn.  Every 256-token window holds 2+ periods, so
    the model can lower the loss by unigram statistics and by copying one period back."""
    gen = torch.Generator().manual_seed({"alt3": 5151, "diff": 6161}[key])
    ids = torch.randperm(12000, generator=gen)[:256]
    motif = ids[torch.randint(0, 256, (97,), generator=gen)]
    toks = motif.repeat(60_000 // 97 + 1)[:60_000].clone()
    noise = torch.rand(toks.numel(), generator=gen) < 0.05
    toks[noise] = ids[torch.randint(0, 256, (int(noise.sum()),), generator=gen)]
    offs = torch.randint(0, toks.numel() - T - 1, (STEPS, MB), generator=gen)
    return toks, offs


def run(key, bf16):
    torch.manual_seed(1337)
    model = MODELS[key]()
    sd = {k: v for k, v in model.state_dict().items() if v.is_floating_point()}
    init = (np.array(sorted(sd)), np.array([[float(sd[k].double().sum()), float((sd[k].double() ** 2).sum())]
                                            for k in sorted(sd)]))
    opt = torch.optim.AdamW(model.parameters(), lr=3.2e-4, betas=(0.9, 0.95), weight_decay=0.1)
    sched = ref_train.CosineWarmupScheduler(opt, warmup_steps=WARM, max_steps=STEPS, min_lr=6e-5)
    toks, offs = data(key)
    losses, lrs = [], []
    model.train()
    t0 = time.time()
    for s in range(STEPS):
        X = torch.stack([toks[o:o + T] for o in offs[s].tolist()])
        Y = torch.stack([toks[o + 1:o + T + 1] for o in offs[s].tolist()])
        lrs.append(opt.param_groups[0]["lr"])
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=bf16):
            _, loss = model(X, Y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        sched.step()
        losses.append(float(loss))
        print(f"{key} {'bf16' if bf16 else 'fp32'} step {s}: loss {losses[-1]:.6f} ({time.time() - t0:.0f}s)",
              flush=True)
    return np.array(losses), np.array(lrs), init, toks, offs


def main():
    torch.set_num_threads(len(os.sched_getaffinity(0)))
    rec = {}
    for key in MODELS:
        l32, lrs, init, toks, offs = run(key, False)
        l16, _, _, _, _ = run(key, True)
        p = key + "/"
        rec.update({p + "losses": l32, p + "bf16_losses": l16, p + "lrs": lrs, p + "init_keys": init[0],
                    p + "init_sums": init[1],
                    p + "toks": toks.numpy().astype(np.int32), p + "offs": offs.numpy(),
                    p + "meta": np.array([MB, T, STEPS, WARM])})
    path = os.path.join(OUT, "golden_loss_curve_diffmodels.npz")
    np.savez_compressed(path, **rec)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
