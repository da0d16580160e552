import argparse, sys, time, torch
sys.path.insert(0, '.')
from differential_transformer_replication_amd.train import train_bench
for tag, model, n in [("cfg4", "diff", 2), ("n3a", "ndiff", 3), ("n3b", "ndiff", 3), ("n4", "ndiff", 4)]:
    torch.cuda.empty_cache()
    t = time.time()
    r = train_bench(argparse.Namespace(steps=6, warmup=3, model=model, n_terms=n, device="cuda"), 1, 0)
    print(tag, r["ms_per_step"], "wall", round(time.time() - t, 1), flush=True)
