"""Long training-curve fixtures from the REFERENCE, run on
this container's CPU (the reference never travels to the GPU box):

  curve32/*   cfg1 DiffTransformer(12000, 384, 6, 6, 256, 0), fp32, seed 1337,
              micro-batch 32 x 256 (train.py:57-93 defaults), AdamW (train.py:236-241),
              the reference's own CosineWarmupScheduler (train.py:109-123, warmup 10,
              max 50), grad clip 1.0 -- 50 optimizer steps
  curve16/*   the reference's mixed-precision step (train.py:251-279): autocast fp16
              + GradScaler (init scale 2^16) + unscale_ + clip + scaler.step/update,
              same model and schedule, micro-batch 4, 50 steps.  Autocast runs on the
              CPU here, so its fp16 GEMMs round differently from a GPU's: the GPU
              replay compares with a tolerance (tests/test_gpu_modules.py).

train.py imports tiktoken and wandb at module level (absent here and unused by the
scheduler): empty stand-in modules satisfy those two imports.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_curve_golden.py
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
import train as ref_train                    # noqa: E402

STEPS, T, WARM = 50, 256, 10


def run(mb, fp16):
    torch.manual_seed(1337)
    model = ref_diff.DiffTransformer(12000, 384, 6, 6, 256, 0.0)
    opt = torch.optim.AdamW(model.parameters(), lr=3.2e-4, betas=(0.9, 0.95), weight_decay=0.1)
    sched = ref_train.CosineWarmupScheduler(opt, warmup_steps=WARM, max_steps=STEPS, min_lr=6e-5)
    scaler = torch.amp.GradScaler("cpu") if fp16 else None
    gen = torch.Generator().manual_seed(4242 + mb)
    toks = torch.randint(0, 12000, (200_000,), generator=gen)
    offs = torch.randint(0, toks.numel() - T - 1, (STEPS, mb), generator=gen)
    losses, gnorms, lrs, scales = [], [], [], []
    model.train()
    t0 = time.time()
    for s in range(STEPS):
        X = torch.stack([toks[o:o + T] for o in offs[s].tolist()])
        Y = torch.stack([toks[o + 1:o + T + 1] for o in offs[s].tolist()])
        lrs.append(opt.param_groups[0]["lr"])
        if fp16:
            with torch.autocast("cpu", dtype=torch.float16):
                _, loss = model(X, Y)
            scaler.scale(loss).backward()
            scaler.unscale_(opt)
            gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            scales.append(float(scaler.get_scale()))
            scaler.step(opt)
            scaler.update()
        else:
            _, loss = model(X, Y)
            loss.backward()
            gn = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
        opt.zero_grad(set_to_none=True)
        sched.step()
        losses.append(float(loss))
        gnorms.append(float(gn))
        print(f"{'fp16' if fp16 else 'fp32'} step {s}: loss {losses[-1]:.6f} gnorm {gnorms[-1]:.4f} "
              f"({time.time() - t0:.0f}s)", flush=True)
    p = "curve16/" if fp16 else "curve32/"
    out = {p + "losses": np.array(losses), p + "gnorms": np.array(gnorms), p + "lrs": np.array(lrs),
           p + "toks": toks.numpy().astype(np.int32), p + "offs": offs.numpy(),
           p + "meta": np.array([mb, T, STEPS, WARM])}
    if fp16:
        out[p + "scales"] = np.array(scales)
    return out


def main():
    torch.set_num_threads(len(os.sched_getaffinity(0)))
    rec = {}
    rec.update(run(32, False))
    rec.update(run(4, True))
    np.savez_compressed(os.path.join(OUT, "golden_loss_curve_long.npz"), **rec)
    print("wrote golden_loss_curve_long.npz", os.path.getsize(os.path.join(OUT, "golden_loss_curve_long.npz")) // 1024,
          "KiB")


if __name__ == "__main__":
    main()
