"""aten op counts and CUDA kernel launches of ONE cfg4 training step (torch.profiler),
to find launch-bound glue.  python tools/op_counts.py [--layers 20]"""
import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from differential_transformer_replication_amd.train import (CFG4, ShardedWindows, Trainer,  # noqa: E402
                                                            TrainingConfig, build_model)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=20)
    a = ap.parse_args()
    base = dict(CFG4)
    base["n_layer"] = a.layers
    cfg = TrainingConfig(**base, warmup_iters=100, max_iters=10_000, dtype="bf16")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = build_model(cfg).to(dev)
    toks = torch.randint(0, cfg.vocab_size, (1_000_000,)).to(dev)
    it = ShardedWindows(toks, cfg.block_size, cfg.micro_batch_size, 0, 1, 0)
    tr = Trainer(cfg, model, 1, 0, dev)
    for _ in range(2):
        tr.step(it.next)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        tr.step(it.next)
        torch.cuda.synchronize()
    cnt = collections.Counter()
    for e in prof.events():
        if e.name.startswith("aten::"):
            cnt[e.name] += 1
    for n, c in cnt.most_common(45):
        print(f"{c:6d} {n}")


if __name__ == "__main__":
    main()
