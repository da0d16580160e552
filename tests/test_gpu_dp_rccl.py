"""The DP gradient path over RCCL on the GPU (torch.distributed backend "nccl" is
RCCL on ROCm): a 1-rank process group with BucketedAllReduce forced to launch its
bucket all-reduces from the post-accumulate-grad hooks, overlapped with backward,
then synchronize().  Sum over one rank times 1/world = the gradients themselves, so
they must equal a run without DP bitwise (train.py's step structure)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist


pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bucketed_allreduce_over_rccl_single_rank():
    from differential_transformer_replication_amd import diff_transformer as D
    from differential_transformer_replication_amd.dp import BucketedAllReduce
    dev = torch.device("cuda", 0)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        def build():
            torch.manual_seed(0)
            return D.DiffTransformer(97, 64, 2, 2, 32, 0.0).to(dev)

        ref, m = build(), build()
        sync = BucketedAllReduce(m, bucket_cap_mb=0.05, reduce_single=True)
        assert len(sync.buckets) > 1
        g = torch.Generator().manual_seed(5)
        idx = torch.randint(0, 97, (2, 32), generator=g).to(dev)
        tgt = torch.randint(0, 97, (2, 32), generator=g).to(dev)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            lr = ref(idx, tgt)[1]
            lm = m(idx, tgt)[1]
        lr.backward()
        lm.backward()
        launched = sum(b.handle is not None for b in sync.buckets)
        assert launched == len(sync.buckets)          # every bucket reduced from the hooks
        sync.synchronize()
        torch.cuda.synchronize()
        for (n, a), (_, b) in zip(ref.named_parameters(), m.named_parameters()):
            assert torch.equal(a.grad, b.grad), n
        sync.clip_grad_norm_(1.0)
        sync.zero_grad()
        assert all(float(b.flat.abs().max()) == 0.0 for b in sync.buckets)
    finally:
        dist.destroy_process_group()
