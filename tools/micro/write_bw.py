"""HBM write / copy bandwidth of plain torch kernels at the RVQ output sizes (a roof for the
fused RVQ's z_q_is stream): fill_ of 91 MB / 365 MB / 1.4 GB and copy_ of the same."""
import torch

dev = torch.device("cuda:0")
for mb in (91.2, 365, 1460):
    n = int(mb * 1e6 / 4)
    a = torch.empty(n, device=dev)
    b = torch.empty(n, device=dev)
    for name, fn, byt in (("fill", lambda: a.fill_(1.0), n * 4),
                          ("copy", lambda: b.copy_(a), n * 8)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        print(f"{name} {mb:7.1f} MB: {us:8.1f} us  {byt / us / 1e6:6.2f} TB/s")
