"""Debug: QR fill on a block-diagonal ill-conditioned matrix, fp64 vs fp32-rounded values."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
from gflownet_spai_amd import PreconditionerEnv, kernels
nb, w = 4, 5
n = nb * w
g = torch.Generator().manual_seed(5)
for scale in (1e-5, 0.5):
    for f32 in (False, True):
        blocks = 1.0 + scale * torch.randn(nb, w, w, generator=g, dtype=torch.float64)
        if f32:
            blocks = blocks.float().double()
        bi = torch.arange(nb).view(nb, 1, 1) * w
        rows = (bi + torch.arange(w).view(1, w, 1)).expand(nb, w, w).reshape(-1)
        cols = (bi + torch.arange(w).view(1, 1, w)).expand(nb, w, w).reshape(-1)
        A = torch.sparse_coo_tensor(torch.stack([rows, cols]), blocks.reshape(-1), (n, n))
        for fill in ("qr", "lsq"):
            env = PreconditionerEnv(n, A, A, side="AM", fill=fill, keep_m=True)
            bits = torch.zeros(1, (env.init_nnz + 31) // 32, dtype=torch.int32, device="cuda")
            r2 = env.fill_partial(bits)
            m = env.last_m[0].cpu().numpy()
            B0 = blocks[0].numpy()
            ref = np.linalg.inv(B0)  # column j of M (AM side): D^-1 e_j, D = block
            err = max(np.linalg.norm(m[j] - ref[:, j]) / np.linalg.norm(ref[:, j]) for j in range(w))
            print(f"scale {scale} f32vals {f32} fill {fill} a_dtype {kernels.narrow_values(env.a_lines).dtype} "
                  f"rows {env.qr_rows} err {err:.3e} res2 {float(r2[0]):.3e}")
            if err > 1e-6 and fill == "qr":
                print(" m[0]", m[0], "\n ref", ref[:, 0])
