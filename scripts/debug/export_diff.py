import sys, json, tempfile, copy
sys.path.insert(0, "tensorrt-model-optimizer_amd"); sys.path.insert(0, ".")
import torch
from safetensors.torch import load_file
from tests.test_gpu_export import _tiny, _cfg, META, G
import modelopt_amd.torch.quantization as mtq
from modelopt_amd.torch.export import export_hf_checkpoint
t = load_file(str(G / "export.safetensors"))
for case in sys.argv[1:]:
    ids = t["calib_ids"].cuda()
    model = _tiny().cuda()
    mtq.quantize(model, _cfg(mtq, META[case]["preset"]), lambda m: [m(b) for b in ids])
    state = {k[len(case) + 7:]: v for k, v in t.items() if k.startswith(case + ".state.")}
    print(case, "our keys not in ref:", [k for k in model.state_dict() if k not in state][:6])
    model.load_state_dict(state, strict=False)
    d = tempfile.mkdtemp()
    try:
        export_hf_checkpoint(model, export_dir=d)
    except Exception as e:
        import traceback; traceback.print_exc(); continue
    got = load_file(d + "/model.safetensors")
    want = {k[len(case) + 8:]: v for k, v in t.items() if k.startswith(case + ".export.")}
    n = 0
    for k, v in want.items():
        g = got.get(k)
        if g is None: continue
        a = g.view(torch.uint8) if g.element_size() == 1 else g
        b = v.view(torch.uint8) if v.element_size() == 1 else v
        if g.shape != v.shape or not torch.equal(a, b):
            print("  ", k, g.dtype, tuple(g.shape), v.dtype, tuple(v.shape))
            print("     got ", g.float().flatten()[:6].tolist())
            print("     want", v.float().flatten()[:6].tolist())
            n += 1
            if n > 6: break
