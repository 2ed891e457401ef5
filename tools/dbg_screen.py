"""Debug: inspect the vocab-screen summaries left in the decode workspace after one sampler call."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from adaptive_amd import Config, Encoder2Decoder, synth
dev = torch.device("cuda:0")
m = Encoder2Decoder(Config()).to(dev).load_synthetic(123)
B, E, H, V, C, P = 512, 256, 512, 10123, 2048, 49
T = int(sys.argv[1]) if len(sys.argv) > 1 else 1
Vp = (V + 127) // 128 * 128
feats = torch.from_numpy(synth.make_features(B)).to(dev)
ids, _, _ = m.sampler(feats, max_len=T)
torch.cuda.synchronize()
ws = m._ws
off = 0
def take(nbytes):
    global off
    o = off
    off = (off + nbytes + 255) // 256 * 256
    return o
o = {}
o["a_g"] = take(B * C * 4); o["V"] = take(B * P * H * 4); o["vwv"] = take(B * P * 64 * 4); o["vg"] = take(B * E * 4)
o["xg"] = take(B * 5 * H * 4)
for i in range(2):
    o[f"h{i}"] = take(B * H * 4); o[f"c{i}"] = take(B * H * 4)
o["s"] = take(B * H * 4); o["u"] = take(B * H * 4); o["unorm"] = take(B * 4); o["part"] = take(B * (H // 16) * 128 * 4)
o["ub"] = take(B * H * 2); o["summ"] = take(B * (Vp // 128) * 16)
f = lambda k, n: ws[o[k]: o[k] + n * 4].view(torch.float32).cpu().numpy()
u = f("u", B * H).reshape(B, H)
un = f("unorm", B)
print("unorm", un[:4], "vs", np.linalg.norm(u[:4], axis=1))
ub = ws[o["ub"]: o["ub"] + B * H * 2].view(torch.int16).cpu().numpy().reshape(B, H).astype(np.uint16)
ubf = (ub.astype(np.uint32) << 16).view(np.float32)
print("ub vs u max abs rel", np.abs(ubf - u).max())
sm = f("summ", B * (Vp // 128) * 4).reshape(B, Vp // 128, 4)
print("summ row0 first tiles", sm[0, :3])
W = m.decoder.adaptive.mlp.weight.detach().cpu().numpy(); bb = m.decoder.adaptive.mlp.bias.detach().cpu().numpy()
L = u @ W.T + bb
print("true max row0", L[0].max(), "argmax", L[0].argmax(), "ids", ids[0, 0].item())
mlb = sm[:, :, 0].max(1)
nc = ((sm[:, :, 1] >= mlb[:, None]).sum(1) + 128 * (sm[:, :, 2] >= mlb[:, None]).sum(1))
print("mlb row0", mlb[0], "candidates per row: mean", nc.mean(), "max", nc.max())
bad = np.argsort(-nc)[:5]
print("worst rows", bad, nc[bad])
r = bad[0]
print("row", r, "mlb", mlb[r], "top tiles ub1/ub2", np.sort(sm[r, :, 1])[-5:], np.sort(sm[r, :, 2])[-5:])
print("u row norm", un[r], "L max", L[r].max(), "sorted top", np.sort(L[r])[-5:])
