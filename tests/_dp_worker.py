"""Child process of tests/test_gpu_dp_rccl.py::test_two_rank_packed_dp_on_one_gpu.

Rank ``r`` of ``world`` gloo ranks that share cuda:0: builds the seeded
DiffTransformer, wraps it in BucketedAllReduce (packed projections, lambda packs
and LayerNorms bound to their buckets), runs one forward/backward on its batch
shard, synchronises and saves its gradients, its loss and the hook reports."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from differential_transformer_replication_amd import diff_transformer as D
        from differential_transformer_replication_amd.dp import BucketedAllReduce
        torch.manual_seed(rank + 3)                 # rank 0's init reaches every rank by broadcast
        m = D.DiffTransformer(97, 64, 2, 2, 32, 0.0).to(dev)
        with torch.no_grad():                       # lambdas off their zero-init saddle
            for n, p in m.named_parameters():
                if "lambda_" in n:
                    p.normal_(0, 0.1, generator=torch.Generator(device=dev).manual_seed(11))
        reports = {}

        class Counted(BucketedAllReduce):          # every hook call, autograd's and the bound packs'
            def _on_grad(self, p):
                reports[id(p)] = reports.get(id(p), 0) + 1
                return super()._on_grad(p)

        sync = Counted(m, bucket_cap_mb=0.05)
        g = torch.Generator().manual_seed(5)
        idx = torch.randint(0, 97, (4, 32), generator=g)
        tgt = torch.randint(0, 97, (4, 32), generator=g)
        sh = slice(2 * rank, 2 * rank + 2)
        loss = m(idx[sh].to(dev), tgt[sh].to(dev))[1]
        loss.backward()
        launched = [b.handle is not None for b in sync.buckets]
        complete = [b.pending == 0 and len(b.seen) == b.size for b in sync.buckets]
        sync.synchronize()
        torch.cuda.synchronize()
        names = {id(p): n for n, p in m.named_parameters()}
        torch.save({"loss": float(loss), "launched": launched, "complete": complete,
                    "reports": {names[k]: v for k, v in reports.items()},
                    "init": {n: p.detach().cpu() for n, p in m.named_parameters()},
                    "grads": {n: p.grad.detach().cpu() for n, p in m.named_parameters()}}, out)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
