import copy, os, sys, torch
sys.path.insert(0, os.getcwd())
import bench
from penroz.models.executor import GPTExecutor
from penroz.models.mapper import Mapper
from penroz.models.model import NeuralNetworkModel
from penroz.ops import _ext
torch.manual_seed(0)
m = NeuralNetworkModel("p", Mapper(bench.gpt2_layers(), {"adamw": {"lr": 6e-4, "betas": [0.9, 0.95], "eps": 1e-8}})).cuda()
ref = copy.deepcopy(m)
B, T = 4, 1024
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.randint(0, 50304, (B, T), device="cuda", generator=g)
y = torch.randint(0, 50304, (B, T), device="cuda", generator=g)
_ext.FORCE_TORCH = True
_, loss_ref = ref(x, y, skip_softmax=True); loss_ref.backward()
_ext.FORCE_TORCH = False
ex = GPTExecutor(m, torch.device("cuda")); ex.setup_training(False); ex.zero_grad()
loss = ex.train_micro_step(x, y, 1.0)
torch.cuda.synchronize()
print("loss", loss.item(), loss_ref.item())
bad = []
for (n, p), (_, r) in zip(m.named_parameters(), ref.named_parameters()):
    gg = ex.grad(p)
    rel = ((gg - r.grad).norm() / (r.grad.norm() + 1e-12)).item()
    print(f"{n:30s} rel {rel:.4f} |g| {gg.norm().item():.4e} |ref| {r.grad.norm().item():.4e}")
