import sys, torch
sys.path.insert(0, "/root/repo/build/spike")
import _spike
x = torch.randn(1000, device="cuda")
y = _spike.scale(x, 3.0)
torch.cuda.synchronize()
print("spike ext ok:", torch.allclose(y, 3 * x))
