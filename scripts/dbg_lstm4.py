"""Debug: H=4 LSTM forward on tiny cases vs nn.LSTM (fp32, CPU)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gflownet_spai_amd import kernels
torch.manual_seed(4)
lstm = torch.nn.LSTM(1, 4, batch_first=True)
P = [lstm.weight_ih_l0, lstm.weight_hh_l0, lstm.bias_ih_l0, lstm.bias_hh_l0]
Pd = [p.detach().cuda() for p in P]
for lens in ([1], [2], [5], [16], [17], [48], [49], [100]):
    T = max(lens)
    x = np.random.default_rng(0).integers(0, 100, size=(len(lens), T))
    h, st = kernels.lstm_forward(torch.tensor(x).cuda(), torch.tensor(lens, dtype=torch.int32).cuda(), *Pd, keep_states=True)
    with torch.no_grad():
        _, (hr, _) = lstm(torch.tensor(x, dtype=torch.float32).unsqueeze(-1))
    print(lens, h.cpu().numpy().ravel(), hr[0].numpy().ravel(), float((h.cpu() - hr[0]).abs().max()))
