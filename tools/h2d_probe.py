"""Does a pageable 512-B H2D .to() block the host behind queued GPU work?  (Q.calculate_loss's torch.rand(B).to(dev))"""
import time
import torch
dev = torch.device("cuda:0")
a = torch.randn(4096, 4096, device=dev)
for _ in range(3):
    (a @ a).sum().item()
def q():
    for _ in range(20):
        a @ a
for name, fn in (("pageable", lambda: torch.rand(128).to(dev)),
                 ("pinned non_blocking", lambda: torch.rand(128).pin_memory().to(dev, non_blocking=True)),
                 ("none", lambda: torch.rand(128))):
    for _ in range(3):
        torch.cuda.synchronize()
        q()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("%-20s host %.3f ms (queue drained %.3f ms later)" % (name, (t1 - t0) * 1e3, (t2 - t1) * 1e3))
