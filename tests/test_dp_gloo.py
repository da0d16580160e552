"""Data-parallel gradient sync (dp.BucketedAllReduce) on CPU with gloo,
world_size 2: DP-averaged gradients equal the single-process full-batch
gradients; no_sync accumulation; multiple buckets; unused parameters."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from differential_transformer_replication_amd.dp import BucketedAllReduce


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 32)
        self.unused = torch.nn.Linear(4, 4)
        self.c = torch.nn.Linear(32, 1)

    def forward(self, x):
        return self.c(torch.tanh(self.b(torch.tanh(self.a(x)))))


def _data():
    g = torch.Generator().manual_seed(0)
    return torch.randn(8, 16, generator=g), torch.randn(8, 1, generator=g)


def _worker(rank, world, port, accum, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank + 100)          # different init per rank: broadcast must fix it
    net = Net()
    sync = BucketedAllReduce(net, bucket_cap_mb=0.002)   # tiny cap -> several buckets
    assert len(sync.buckets) >= 3
    x, y = _data()
    xs, ys = x.chunk(world)[rank], y.chunk(world)[rank]
    if accum:
        for i, (xm, ym) in enumerate(zip(xs.chunk(2), ys.chunk(2))):
            ctx = sync.no_sync() if i == 0 else torch.enable_grad()
            with ctx:
                (torch.nn.functional.mse_loss(net(xm), ym) / 2).backward()
    else:
        torch.nn.functional.mse_loss(net(xs), ys).backward()
    sync.synchronize()
    grads = {n: p.grad.clone() for n, p in net.named_parameters()}
    params = {n: p.detach().clone() for n, p in net.named_parameters()}
    out.put((rank, grads, params))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("accum", [False, True])
def test_dp_matches_full_batch(accum):
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, accum, out)) for r in range(world)]
    for p in procs:
        p.start()
    res = [out.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    # reference: rank 0's (broadcast) initial weights, full batch, one process
    torch.manual_seed(100)
    ref = Net()
    ref.load_state_dict(res[0][2])
    x, y = _data()
    torch.nn.functional.mse_loss(ref(x), y).backward()
    for _, grads, params in res:
        for n, p in ref.named_parameters():
            assert torch.equal(params[n], res[0][2][n]), n
            want = p.grad if p.grad is not None else torch.zeros_like(p)
            assert torch.allclose(grads[n], want, atol=1e-6, rtol=1e-5), n
