"""Debug: the ill-conditioned QR test, per line errors."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np, torch
from gflownet_spai_amd import PreconditionerEnv, kernels
for nb in (4, 13, 40):
    w = 5
    n = nb * w
    g = torch.Generator().manual_seed(5)
    blocks = 1.0 + 1e-5 * torch.randn(nb, w, w, generator=g, dtype=torch.float64)
    bi = torch.arange(nb).view(nb, 1, 1) * w
    rows = (bi + torch.arange(w).view(1, w, 1)).expand(nb, w, w).reshape(-1)
    cols = (bi + torch.arange(w).view(1, 1, w)).expand(nb, w, w).reshape(-1)
    A = torch.sparse_coo_tensor(torch.stack([rows, cols]), blocks.reshape(-1), (n, n))
    env = PreconditionerEnv(n, A, A, side="AM", fill="qr", keep_m=True)
    bits = torch.zeros(1, (env.init_nnz + 31) // 32, dtype=torch.int32, device="cuda")
    env.fill_partial(bits)
    m = env.last_m[0].cpu().numpy()
    errs = []
    for j in range(n):
        B0 = blocks[j // w].numpy()
        ref = np.linalg.inv(B0)[:, j % w]
        errs.append(np.linalg.norm(m[j] - ref) / np.linalg.norm(ref))
    errs = np.array(errs)
    bad = np.flatnonzero(errs > 1e-8)
    print(nb, "max err", errs.max(), "bad lines", bad[:20], len(bad))
    print(" pattern idx line 0..2", env.pattern.idx[:3].cpu().numpy().tolist(), "a idx", env.a_lines.idx[:3].cpu().numpy().tolist())
