import sys
sys.path[:0] = ["/root/repo", "/root/repo/cmu-11785-idl-1.58bit-asr_amd"]
import torch
from onebit_asr.layernorm import layer_norm, layer_norm_fork
gpu = torch.device("cuda:0")
torch.manual_seed(9)
w = torch.randn(144, device=gpu, requires_grad=True)
b = torch.randn(144, device=gpu, requires_grad=True)
x = torch.randn(3, 77, 144, device=gpu, requires_grad=True)
gy = torch.randn(3, 77, 144, device=gpu)
gr = torch.randn(3, 77, 144, device=gpu)
y, xr = layer_norm_fork(x, w, b)
(y * gy + xr * gr).sum().backward()
g_fork = x.grad.clone(); x.grad = None
y0 = layer_norm(x, w, b)
(y0 * gy).sum().backward()
g_ln = x.grad.clone(); x.grad = None
y0 = layer_norm(x, w, b)
(y0 * gy + x * gr).sum().backward()
g_ref = x.grad.clone()
print("fork vs ln+gr", (g_fork - (g_ln + gr)).abs().max().item())
print("ref vs ln+gr", (g_ref - (g_ln + gr)).abs().max().item())
print("fork vs ref", (g_fork - g_ref).abs().max().item())
