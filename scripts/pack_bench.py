"""es_pack_weights at ViT-S (the F1 engine): median ms of 20 launches.  python scripts/pack_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "endoscopy-image-classification_amd"))
import torch  # noqa: E402

from endossl.vit import NativeViT, ViTConfig  # noqa: E402

m = NativeViT(ViTConfig(num_classes=23), seed=0).to("cuda")
eng = m.engine()
eng.pack(m.flat)
ts = []
for _ in range(20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.pack(m.flat)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
sd = m.state_dict()
ok = all(torch.equal(wb, sd[n].reshape(wb.shape[0], -1).bfloat16()) for n, wb in eng.wb.items())
okT = all(torch.equal(eng.wt[n], sd[n].reshape(eng.wb[n].shape[0], -1).t().contiguous().bfloat16()) for n in eng.wt)
print(f"pack median {sorted(ts)[10]:.4f} ms, W exact {ok}, W^T exact {okT}")
