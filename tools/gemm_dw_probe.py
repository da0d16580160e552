"""Weight-gradient GEMM layouts at the cfg4 shapes (K = 32768 tokens): time the
bf16 dW = dY^T X the training step runs, its fp32-output fused-accumulate form
(torch.addmm(..., out_dtype=float32)) and operand-order variants.  GPU only."""
import json
import torch

dev = torch.device("cuda", 0)
K = 32768


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


res = {}
for O, I in [(8192, 1024), (3072, 1024), (1024, 4096), (1024, 1024)]:
    dy = torch.randn(K, O, device=dev, dtype=torch.bfloat16)
    x = torch.randn(K, I, device=dev, dtype=torch.bfloat16)
    g = torch.zeros(O, I, device=dev)
    fl = 2.0 * O * I * K
    r = {}
    r["dyT_x_bf16"] = timeit(lambda: dy.t() @ x)
    r["xT_dy_bf16_T"] = timeit(lambda: (x.t() @ dy).t())
    r["dyT_contig_x"] = timeit(lambda: dy.t().contiguous() @ x)
    r["acc_add_"] = timeit(lambda: g.add_(dy.t() @ x))
    try:
        r["addmm_f32_out"] = timeit(lambda: torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g))
        ref = (dy.t() @ x).float()
        g.zero_()
        torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)
        r["addmm_vs_bf16_maxrel"] = float((g - ref).abs().max() / ref.abs().max())
    except Exception as e:  # noqa: BLE001
        r["addmm_f32_out"] = "ERR " + str(e)[:120]
    try:
        r["mm_f32"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    except Exception as e:  # noqa: BLE001
        r["mm_f32"] = "ERR " + str(e)[:120]
    r["tflops_dyT_x"] = fl / r["dyT_x_bf16"] / 1e6
    res[f"{O}x{I}"] = r
    print(f"{O}x{I}", json.dumps(r), flush=True)
