import torch, time
q = torch.randn(1024, 768, device="cuda"); x = torch.randn(1024, 768, device="cuda")
for dt in (torch.float32,):
    torch.backends.cuda.matmul.allow_tf32 = False
    for _ in range(10): y = q @ x.T
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(200): y = q @ x.T
    torch.cuda.synchronize(); print("fp32 mm 1024x1024x768:", (time.perf_counter() - t) / 200 * 1e6, "us")
