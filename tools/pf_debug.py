"""GPU debug: how many instances the product-form kernel hands to qp_wg_kernel."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from model_predictive_control_amd import batched
import bench


class A:
    pass


for cfg in (5, 3):
    a = A(); a.batch = 2048; a.slots = 1; a.horizon = 0; a.reps = 1
    w = bench.CONFIGS[cfg](a, torch.device("cuda"), 0)
    w.step(0)
    torch.cuda.synchronize()
    for key, ws in batched._WS.items():
        nbytes = ws.numel()
        n = w.n
        m = getattr(w, "m", 0) if cfg == 3 else 0
        print(cfg, key, nbytes)
    # counter sits after the dense swept matrices
    nt = w.n + (120 if cfg == 3 else 0)
    off = ((a.batch * nt * nt * 4 + 255) // 256) * 256
    for key, ws in batched._WS.items():
        if ws.numel() >= off + 4:
            cnt = ws[off:off + 4].view(torch.int32).item()
            print("cfg", cfg, "nt", nt, "retry count", cnt, "of", a.batch)
    batched._WS.clear()
