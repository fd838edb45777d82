import sys, time
sys.path.insert(0, "tensorrt-model-optimizer_amd"); sys.path.insert(0, ".")
import torch
from scripts.ptq_llama import build_model
m = build_model(4, torch.device("cuda"), "mixtral-8x7b")
ids = torch.randint(0, 32000, (16, 512), device="cuda")
outs = {}
for impl in ["eager", "grouped_mm", "batched_mm"]:
    try:
        m.config._experts_implementation = impl
        with torch.no_grad():
            m(ids); torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                o = m(ids).logits
            torch.cuda.synchronize()
        outs[impl] = o.float()
        print(impl, "ms/fwd(4 layers)", (time.perf_counter() - t0) / 3 * 1e3, flush=True)
    except Exception as e:
        print(impl, "FAILED", repr(e)[:300], flush=True)
for k, v in outs.items():
    print(k, "max|diff| vs eager", (v - outs["eager"]).abs().max().item())
x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(8, 2048, 4096, device="cuda", dtype=torch.bfloat16)
offs = torch.tensor([512 * (i + 1) for i in range(8)], device="cuda", dtype=torch.int32)
try:
    y = torch._grouped_mm(x, w.transpose(-2, -1), offs=offs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        y = torch._grouped_mm(x, w.transpose(-2, -1), offs=offs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print("grouped_mm 4096x4096x(8x2048): %.3f ms, %.1f TFLOP/s" % (dt * 1e3, 2 * 4096 * 4096 * 2048 / dt / 1e12))
    ref = torch.cat([x[512 * i:512 * (i + 1)] @ w[i].T for i in range(8)])
    print("grouped vs loop max diff", (y.float() - ref.float()).abs().max().item())
except Exception as e:
    print("grouped_mm direct FAILED", repr(e)[:300])
