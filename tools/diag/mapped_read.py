"""Is the wrong region of a small qk_out_alloc mapping unwritten, or misread by the D2H copy?
Compares first.cpu() with first.clone().cpu() (a device-side copy first) and with a device-side
comparison against the reference uploaded to a torch buffer."""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
import torch
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd import VirtualCircuit, engine
from hardwareawareoptimalquantumcircuitcuttingandknitting_amd.pipeline import KnitPipeline
import circuits
from oracle import dense

engine.OUT_MAPPED_MIN_BYTES = int(sys.argv[1]) if len(sys.argv) > 1 else 0
cut = circuits.two_fragment("cx", 8, 8, n_cuts=4)[1]
pipe = KnitPipeline(VirtualCircuit(cut), factored=True)
ref = dense.run_dense(cut)
ref_d = torch.from_numpy(ref).cuda()
for _ in range(2):
    pipe.step().cpu()
stats = {"d2h": 0, "clone": 0, "device": 0}
for it in range(40):
    first = pipe.take_out()
    pipe.run_into(first)
    torch.cuda.synchronize()
    dev_bad = int(((first - ref_d).abs() > 1e-12).sum().item())
    c = first.clone()
    torch.cuda.synchronize()
    a = first.cpu().numpy()
    b = c.cpu().numpy()
    ba, bb = np.count_nonzero(np.abs(a - ref) > 1e-12), np.count_nonzero(np.abs(b - ref) > 1e-12)
    stats["d2h"] += ba > 0; stats["clone"] += bb > 0; stats["device"] += dev_bad > 0
    if ba or bb or dev_bad:
        print(f"it {it}: d2h wrong {ba}, clone->d2h wrong {bb}, device compare wrong {dev_bad}, ptr {first.data_ptr():#x}", flush=True)
    del first, c
print("min bytes", engine.OUT_MAPPED_MIN_BYTES, "runs with wrong entries (of 40):", stats, flush=True)
