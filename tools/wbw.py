import torch, time
x = torch.empty(4 * 64**3 * 32, device="cuda")
y = torch.empty_like(x)
for name, fn in [("fill", lambda: x.fill_(1.0)), ("copy", lambda: y.copy_(x))]:
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20): fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    nb = x.numel() * 4 * (1 if name == "fill" else 2)
    print(f"{name}: {dt*1e6:.1f} us, {nb/dt/1e12:.2f} TB/s")
