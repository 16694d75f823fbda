import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from penroz.ops import gemm
print("loaded", gemm.load_tuned_gemms())
import torch.cuda.tunable as t
print("enabled", t.is_enabled(), "tuning", t.tuning_is_enabled(), "file", t.get_filename())
print("results", t.get_results()[:3])
x = torch.randn(65536, 768, device="cuda", dtype=torch.bfloat16)
w = torch.randn(50304, 768, device="cuda", dtype=torch.bfloat16)
y = torch.empty(65536, 50304, device="cuda", dtype=torch.bfloat16)
for en in (True, False, True):
    t.enable(en)
    for _ in range(3): torch.mm(x, w.t(), out=y)
    torch.cuda.synchronize(); t0=time.perf_counter()
    for _ in range(10): torch.mm(x, w.t(), out=y)
    torch.cuda.synchronize(); print("enabled", en, (time.perf_counter()-t0)/10*1e3, "ms")
