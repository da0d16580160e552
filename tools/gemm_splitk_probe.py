"""Split-K weight-gradient GEMMs at the cfg4 shapes: dW = dY^T X as S batched GEMMs
over K/S tokens each (fp32 partials) plus one sum, vs the single GEMM.  GPU only."""
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


def splitk(dy, x, S, f32):
    Kc = dy.shape[0] // S
    a = dy.view(S, Kc, -1).transpose(1, 2)
    b = x.view(S, Kc, -1)
    p = torch.bmm(a, b, out_dtype=torch.float32) if f32 else torch.bmm(a, b)
    return p.sum(0, dtype=torch.float32)


for O, I in [(8192, 1024), (3072, 1024), (1024, 4096), (1024, 1024), (12000, 1024)]:
    dy = torch.randn(K, O, device=dev, dtype=torch.bfloat16)
    x = torch.randn(K, I, device=dev, dtype=torch.bfloat16)
    ref = torch.mm(dy.t(), x, out_dtype=torch.float32)
    r = {"mm_f32": timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32)),
         "mm_bf16": timeit(lambda: dy.t() @ x),
         "swap_bf16": timeit(lambda: (x.t() @ dy).t())}
    for S in (2, 4, 8):
        for f32 in (True, False):
            k = f"split{S}_{'f32' if f32 else 'bf16'}"
            try:
                r[k] = timeit(lambda: splitk(dy, x, S, f32))
                r[k + "_err"] = float((splitk(dy, x, S, f32) - ref).abs().max() / ref.abs().max())
            except Exception as e:  # noqa: BLE001
                r[k] = "ERR " + str(e)[:100]
    print(f"{O}x{I}", json.dumps({k: (round(v, 1) if isinstance(v, float) and v > 1e-2 else v) for k, v in r.items()}),
          flush=True)
