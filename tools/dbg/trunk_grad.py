import sys, torch
sys.path.insert(0, '.')
import torch.nn.functional as F
from adaptive_amd.trunk import resnet_conv
print("allow_tf32 cudnn", torch.backends.cudnn.allow_tf32, "matmul", torch.backends.cuda.matmul.allow_tf32)
torch.manual_seed(0)
t = resnet_conv()
with torch.no_grad():
    for mod in t.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.weight.uniform_(0.2, 0.4)
x = torch.rand(2, 3, 224, 224, generator=torch.Generator().manual_seed(3))
w = torch.randn(2, 2048, 7, 7, generator=torch.Generator().manual_seed(4))
def run(dev, tf32):
    torch.backends.cudnn.allow_tf32 = tf32
    m = resnet_conv(); m.load_state_dict(t.state_dict()); m = m.to(dev).train()
    y = m(x.to(dev)); loss = (y * w.to(dev)).sum(); loss.backward()
    return y.detach().cpu(), m[7][2].conv3.weight.grad.cpu(), m[5][0].conv1.weight.grad.cpu()
ref = run("cpu", False)
for tf in (False, True):
    g = run("cuda", tf)
    print("tf32", tf, [ (torch.linalg.norm(a-b)/torch.linalg.norm(b)).item() for a, b in zip(g, ref)])
