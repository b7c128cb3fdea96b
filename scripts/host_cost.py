import sys, time, torch, os
sys.path.insert(0, os.getcwd())
import bench
from gflownet_spai_amd import GFlowNet, PreconditionerEnv, poisson_2d
A = poisson_2d(1024, torch.float32); n = A.shape[0]
dev = torch.device("cuda", 0)
env = PreconditionerEnv(n, A, A, side="AM", fill="lsq", keep_m=True, device=dev)
E = env.num_actions - 1
g = torch.Generator().manual_seed(123)
logits = torch.randn(E + 1, generator=g); logits[E] = bench.terminal_logit(logits[:E].numpy(), 0.2)
model = GFlowNet(bench.SyntheticLogits(logits.to(dev)), None, env, mode="throughput", seed=1234)
s0 = [A] * 8
for _ in range(5): model.sample_states(s0, return_log=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20): model.sample_states(s0, return_log=True)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {1e3*(t1-t0)/20:.3f} ms/step, wall {1e3*(t2-t0)/20:.3f} ms/step")
