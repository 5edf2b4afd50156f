import torch
x = torch.tensor([1.0, 448.0, 464.0, 470.0, 480.0, 500.0, 1e6, -1e6, 0.0013, -464.1, 2**-10], dtype=torch.float32)
a = x.to(torch.float8_e4m3fn).view(torch.uint8)
b = x.cuda().to(torch.float8_e4m3fn).view(torch.uint8).cpu()
print("cpu", a.tolist()); print("gpu", b.tolist()); print("equal", torch.equal(a, b))
